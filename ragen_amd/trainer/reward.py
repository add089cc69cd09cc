"""Reward plumbing of the StarPO loop — drop-in for DummyRewardManager (train.py:16-91).

RAGEN's rollout already carries the rule rewards (``rm_scores``, placed by
get_masks_and_scores on the device), so the manager passes them through unchanged
(train.py:31-37) and ``token_level_scores = token_level_rewards = rm_scores`` in fit
(agent_trainer.py:572-617, no KL in the reward by default).  The fallback for batches without
``rm_scores`` places each row's ``non_tensor_batch['reward']`` at its last valid response token
(train.py:39-62), vectorised over the rows."""
import numpy as np
import torch

from ..protocol import DataProto


class DummyRewardManager:
    def __init__(self, tokenizer=None, num_examine: int = 0, compute_score=None):
        self.tokenizer = tokenizer
        self.num_examine = num_examine
        self.compute_score = compute_score

    def __call__(self, data: DataProto, return_dict: bool = False):
        if "rm_scores" in data.batch.keys():
            t = data.batch["rm_scores"]
            return {"reward_tensor": t} if return_dict else t
        responses = data.batch["responses"]
        prompt_length = data.batch["prompts"].shape[-1]
        valid = data.batch["attention_mask"][:, prompt_length:].sum(-1)
        reward = torch.zeros_like(responses, dtype=torch.float32)
        score = torch.tensor(np.asarray(data.non_tensor_batch["reward"], dtype=np.float64), dtype=torch.float32)
        rows = torch.arange(responses.shape[0])
        # reward_tensor[i, valid_response_length - 1] = score (an empty response writes column -1)
        reward[rows, (valid - 1) % responses.shape[1]] = score
        return {"reward_tensor": reward} if return_dict else reward


def compute_reward(data: DataProto, reward_fn):
    """verl trainer.ppo.reward.compute_reward as fit calls it (agent_trainer.py:575):
    -> (reward_tensor, reward_extra_infos_dict)."""
    out = reward_fn(data, return_dict=True)
    return out["reward_tensor"], out.get("reward_extra_info", {})
