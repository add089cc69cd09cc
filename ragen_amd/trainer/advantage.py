"""compute_advantage and the rollout filter — drop-ins for agent_trainer.py:60-137 and
agent_trainer.py:461-500, running on the GPU engine."""
import torch

from .. import ops
from ..protocol import DataProto
from . import core_algos


class AdvantageEstimator:
    GAE = "gae"
    GRPO = "grpo"
    REINFORCE_PLUS_PLUS = "reinforce_plus_plus"
    REINFORCE_PLUS_PLUS_BASELINE = "reinforce_plus_plus_baseline"
    REMAX = "remax"
    RLOO = "rloo"


def compute_advantage(data: DataProto, adv_estimator, gamma=1.0, lam=1.0, num_repeat=1, multi_turn=False,
                      norm_adv_by_std_in_grpo=True, bi_level_gae=False, high_level_gamma=1.0):
    """agent_trainer.py:60-137 for the estimators of RAGEN's StarPO loop (GAE, bi-level GAE,
    GRPO).  REINFORCE++/REMAX/RLOO are verl estimators outside this engine's scope."""
    if "response_mask" not in data.batch:
        data.batch["response_mask"] = data.batch["loss_mask"]
    est = getattr(adv_estimator, "value", adv_estimator)
    if est == AdvantageEstimator.GAE:
        if bi_level_gae:
            adv, ret = core_algos.compute_bi_level_gae_advantage_return(
                data.batch["token_level_rewards"], data.batch["values"], data.batch["response_mask"], gamma, lam,
                high_level_gamma)
        else:
            adv, ret = core_algos.compute_gae_advantage_return(
                data.batch["token_level_rewards"], data.batch["values"], data.batch["response_mask"], gamma, lam)
    elif est == AdvantageEstimator.GRPO:
        mask = data.batch["response_mask"]
        if multi_turn:
            mask = data.batch["loss_mask"][:, -mask.size(1):]
        adv, ret = core_algos.compute_grpo_outcome_advantage(data.batch["token_level_rewards"], mask,
                                                             data.non_tensor_batch["uid"],
                                                             norm_adv_by_std_in_grpo=norm_adv_by_std_in_grpo)
    else:
        raise NotImplementedError(f"advantage estimator {est!r} is not part of the StarPO hot path")
    data.batch["advantages"] = adv
    data.batch["returns"] = ret
    return data


def filter_rollout(batch: DataProto, num_groups: int, group_size: int, ratio: float, ftype: str):
    """_filter_rollout (agent_trainer.py:461-500): returns (filtered batch, metrics).

    Tie order among equal in-group std values: ascending group index (documented deviation:
    torch.topk's choice among ties is implementation-defined)."""
    dev = torch.device("cuda", torch.cuda.current_device())
    rm = batch.batch["original_rm_scores"].to(dev, torch.float32).contiguous()
    rows = ops.row_sum(rm)
    keep, met, _ = ops.filter_groups(rows, num_groups, group_size, ratio, ftype)
    metrics = dict(zip(["rollout/in_group_std", "rollout/in_group_max", "rollout/in_group_mean",
                        "rollout/chosen_in_group_std", "rollout/chosen_in_group_max",
                        "rollout/chosen_in_group_mean"], met.cpu().tolist()))
    if ratio == 1:
        return batch, metrics
    mask = keep.bool().unsqueeze(1).expand(-1, group_size).flatten().cpu()
    return batch.select_rows(mask), metrics
