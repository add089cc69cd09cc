"""compute_advantage and the rollout filter — drop-ins for agent_trainer.py:60-137 and
agent_trainer.py:461-500, running on the GPU engine."""
import torch

from .. import distributed as rd
from ..protocol import DataProto
from ..torch_ops import FILTER
from . import core_algos


_WARNED = set()


def _warn_rank_local(what: str, process_group):
    """Once per call site: torch.distributed is up with more than one rank but no process_group
    was passed, so `what` runs over this rank's shard only (batch-global is opt-in)."""
    if process_group is not None or what in _WARNED or not rd.initialized() or rd.world()[0] <= 1:
        return
    import warnings
    _WARNED.add(what)
    warnings.warn(f"{what}: torch.distributed has {rd.world()[0]} ranks but process_group=None, so it runs over "
                  "this rank's rows only; pass process_group= for the whole sharded batch", RuntimeWarning,
                  stacklevel=3)


class AdvantageEstimator:
    GAE = "gae"
    GRPO = "grpo"
    REINFORCE_PLUS_PLUS = "reinforce_plus_plus"
    REINFORCE_PLUS_PLUS_BASELINE = "reinforce_plus_plus_baseline"
    REMAX = "remax"
    RLOO = "rloo"


def compute_response_mask(data: DataProto) -> torch.Tensor:
    """verl compute_response_mask (the fallback of agent_trainer.py:61-62): the attention mask
    over the response columns."""
    response_length = data.batch["responses"].size(1)
    return data.batch["attention_mask"][:, -response_length:]


def compute_advantage(data: DataProto, adv_estimator, gamma=1.0, lam=1.0, num_repeat=1, multi_turn=False,
                      norm_adv_by_std_in_grpo=True, bi_level_gae=False, high_level_gamma=1.0, process_group=None,
                      shard_rows=None):
    """agent_trainer.py:60-137: GAE (verl, or RAGEN's bi-level), GRPO, REINFORCE++ (and its
    baseline form), REMAX and RLOO, each on the engine's kernels; an unknown estimator raises
    NotImplementedError as the reference does.  ``process_group``: the batch is this rank's
    shard and whitening uses the statistics of the whole sharded batch (core_algos); ``shard_rows``
    (every rank's row count) makes that gather free of host synchronisation."""
    pg = {"process_group": process_group, "shard_rows": shard_rows}
    _warn_rank_local("compute_advantage whitening", process_group)
    if "response_mask" not in data.batch:
        data.batch["response_mask"] = compute_response_mask(data)
    est = getattr(adv_estimator, "value", adv_estimator)
    if est == AdvantageEstimator.GAE:
        if bi_level_gae:
            adv, ret = core_algos.compute_bi_level_gae_advantage_return(
                data.batch["token_level_rewards"], data.batch["values"], data.batch["response_mask"], gamma, lam,
                high_level_gamma, **pg)
        else:
            adv, ret = core_algos.compute_gae_advantage_return(
                data.batch["token_level_rewards"], data.batch["values"], data.batch["response_mask"], gamma, lam, **pg)
    elif est == AdvantageEstimator.GRPO:
        mask = data.batch["response_mask"]
        if multi_turn:
            mask = data.batch["loss_mask"][:, -mask.size(1):]
        adv, ret = core_algos.compute_grpo_outcome_advantage(data.batch["token_level_rewards"], mask,
                                                             data.non_tensor_batch["uid"],
                                                             norm_adv_by_std_in_grpo=norm_adv_by_std_in_grpo)
    elif est == AdvantageEstimator.REINFORCE_PLUS_PLUS_BASELINE:
        adv, ret = core_algos.compute_reinforce_plus_plus_baseline_outcome_advantage(
            data.batch["token_level_rewards"], data.batch["response_mask"], data.non_tensor_batch["uid"], **pg)
    elif est == AdvantageEstimator.REINFORCE_PLUS_PLUS:
        adv, ret = core_algos.compute_reinforce_plus_plus_outcome_advantage(
            data.batch["token_level_rewards"], data.batch["response_mask"], gamma, **pg)
    elif est == AdvantageEstimator.REMAX:
        adv, ret = core_algos.compute_remax_outcome_advantage(
            data.batch["token_level_rewards"], data.batch["reward_baselines"], data.batch["response_mask"])
    elif est == AdvantageEstimator.RLOO:
        adv, ret = core_algos.compute_rloo_outcome_advantage(
            data.batch["token_level_rewards"], data.batch["response_mask"], data.non_tensor_batch["uid"])
    else:
        raise NotImplementedError
    data.batch["advantages"] = adv
    data.batch["returns"] = ret
    return data


FILTER_METRICS = ("rollout/in_group_std", "rollout/in_group_max", "rollout/in_group_mean",
                  "rollout/chosen_in_group_std", "rollout/chosen_in_group_max", "rollout/chosen_in_group_mean")


def filter_rollout(batch: DataProto, num_groups: int, group_size: int, ratio: float, ftype: str,
                   process_group=None):
    """_filter_rollout (agent_trainer.py:461-500): returns (filtered batch, metrics).

    Tie order among equal in-group std values: ascending group index (documented deviation:
    torch.topk's choice among ties is implementation-defined).  With ``process_group`` the
    batch is this rank's shard: the groups are ranked over every rank's scores
    (ragen_amd.distributed.global_filter), so the kept set equals the 1-GPU run's and
    ``num_groups`` is the GLOBAL count (es_manager.train.env_groups), as in the reference."""
    _warn_rank_local("filter_rollout", process_group)
    rm = batch.batch["original_rm_scores"]
    dev = rm.device if rm.is_cuda else torch.device("cuda", torch.cuda.current_device())
    rows = torch.ops.ragen_amd.row_sum(rm.to(dev, torch.float32).contiguous())

    def select(scores, G):
        if G != num_groups:
            raise RuntimeError(f"shape '[{num_groups}, {group_size}]' is invalid for input of size {scores.numel()}")
        if ftype not in FILTER:
            raise ValueError(f"Invalid rollout filter type: {ftype}")
        keep, met, _, _, _ = torch.ops.ragen_amd.filter_groups(scores, G, group_size, float(ratio), FILTER[ftype])
        return keep, met

    if process_group is not None:
        keep, met = rd.global_filter(rows, group_size, select, group=process_group)
    else:
        keep, met = select(rows, rows.numel() // group_size if rows.numel() % group_size == 0 else -1)
    metrics = dict(zip(FILTER_METRICS, met.cpu().tolist()))
    if ratio == 1:
        return batch, metrics
    mask = keep.bool().unsqueeze(1).expand(-1, group_size).flatten().cpu()
    return batch.select_rows(mask), metrics
