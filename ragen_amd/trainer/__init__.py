from .advantage import AdvantageEstimator, compute_advantage, filter_rollout
from .core_algos import (compute_bi_level_gae_advantage_return, compute_gae_advantage_return,
                         compute_grpo_outcome_advantage, masked_whiten)

__all__ = ["AdvantageEstimator", "compute_advantage", "filter_rollout", "compute_bi_level_gae_advantage_return",
           "compute_gae_advantage_return", "compute_grpo_outcome_advantage", "masked_whiten"]
