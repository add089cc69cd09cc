from .advantage import AdvantageEstimator, compute_advantage, compute_response_mask, filter_rollout
from .core_algos import (compute_bi_level_gae_advantage_return, compute_gae_advantage_return,
                         compute_grpo_outcome_advantage, masked_whiten)
from .reward import DummyRewardManager, compute_reward

__all__ = ["AdvantageEstimator", "compute_advantage", "compute_response_mask", "filter_rollout", "DummyRewardManager",
           "compute_reward", "compute_bi_level_gae_advantage_return",
           "compute_gae_advantage_return", "compute_grpo_outcome_advantage", "masked_whiten"]
