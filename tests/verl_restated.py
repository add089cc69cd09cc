"""verl's outcome-advantage estimators as published in verl.trainer.ppo.core_algos (the v0.3
line; verl is an empty submodule in the reference, agent_trainer.py:102-134 calls these),
restated on CPU torch.  Test infrastructure only: the checker for the device kernels and the
C oracle, run with the reference's own numerics (torch CPU f32 ops, cumsum's double
accumulator, torch.mean over per-group score lists).  Parity beyond this restatement is
unpinned: no reference vectors exist for these functions."""
from collections import defaultdict

import torch


def masked_mean(values, mask, axis=None):
    return (values * mask).sum(axis=axis) / mask.sum(axis=axis)


def masked_var(values, mask, unbiased=True):
    mean = masked_mean(values, mask)
    centered_values = values - mean
    variance = masked_mean(centered_values ** 2, mask)
    if unbiased:
        mask_sum = mask.sum()
        if mask_sum == 0:
            raise ValueError("At least one element in the mask has to be 1.")
        if mask_sum == 1:
            raise ValueError("The sum of the mask is one, which can cause a division by zero.")
        bessel_correction = mask_sum / (mask_sum - 1)
        variance = variance * bessel_correction
    return variance


def masked_whiten(values, mask, shift_mean=True):
    mean, var = masked_mean(values, mask), masked_var(values, mask)
    whitened = (values - mean) * torch.rsqrt(var + 1e-8)
    if not shift_mean:
        whitened += mean
    return whitened


def compute_reinforce_plus_plus_outcome_advantage(token_level_rewards, response_mask, gamma):
    with torch.no_grad():
        returns = torch.zeros_like(token_level_rewards)
        running_return = 0
        for t in reversed(range(token_level_rewards.shape[1])):
            running_return = token_level_rewards[:, t] + gamma * running_return
            returns[:, t] = running_return
            running_return = running_return * response_mask[:, t]
        advantages = masked_whiten(returns, response_mask)
        advantages = advantages * response_mask
    return advantages, returns


def _id2mean(scores, index):
    id2score = defaultdict(list)
    id2mean = {}
    for i in range(scores.shape[0]):
        id2score[index[i]].append(scores[i])
    for idx in id2score:
        if len(id2score[idx]) == 1:
            id2mean[idx] = torch.tensor(0.0)
        elif len(id2score[idx]) > 1:
            id2mean[idx] = torch.mean(torch.tensor(id2score[idx]))
        else:
            raise ValueError(f"no score in prompt index: {idx}")
    return id2score, id2mean


def compute_reinforce_plus_plus_baseline_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6):
    response_length = token_level_rewards.shape[-1]
    scores = token_level_rewards.sum(dim=-1)
    with torch.no_grad():
        _, id2mean = _id2mean(scores, index)
        for i in range(scores.shape[0]):
            scores[i] = scores[i] - id2mean[index[i]]
        scores = scores.unsqueeze(-1).tile([1, response_length]) * response_mask
        scores = masked_whiten(scores, response_mask) * response_mask
    return scores, scores


def compute_rloo_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6):
    scores = token_level_rewards.sum(dim=-1)
    with torch.no_grad():
        id2score, id2mean = _id2mean(scores, index)
        for i in range(scores.shape[0]):
            response_num = len(id2score[index[i]])
            if response_num > 1:
                scores[i] = scores[i] * response_num / (response_num - 1) - id2mean[index[i]] * response_num / (
                    response_num - 1)
        scores = scores.unsqueeze(-1) * response_mask
    return scores, scores


def compute_remax_outcome_advantage(token_level_rewards, reward_baselines, response_mask):
    with torch.no_grad():
        returns = (token_level_rewards * response_mask).flip(dims=[-1]).cumsum(dim=-1).flip(dims=[-1])
        advantages = returns - reward_baselines.unsqueeze(-1) * response_mask
    return advantages, returns
