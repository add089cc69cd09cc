"""Advantage estimators on the GPU engine — drop-ins for ragen/trainer/core_algos.py:4-92 and
the verl functions RAGEN imports from it (App. A.4): same names, signatures and return
values.  Tensors may arrive on the CPU (as in the reference trainer, whose batch lives on the
driver) and go back there; GPU tensors stay on their own device.

Errors are raised where verl / RAGEN raise them (mask sum 0 or 1 -> ValueError; bi-level
IndexError, core_algos.py:79): the kernels write a status word and per-row error bits, and
the estimator reads them once (``check=True``, the default) — for a CPU caller after the copy
of the results back, for a GPU caller with one small device -> host read.  ``check=False``
leaves GPU results unchecked and the estimator free of host synchronisation.

Batch-global whitening over a sharded batch is opt-in: ``process_group=<group>`` makes every
rank all-gather the per-row fp64 partials and reduce them in global row order, so the shards
whiten exactly like the whole batch; the error flags are then reduced over the group before
anything is raised, so every rank raises together.  Without it the statistics are this
process's rows only, whatever torch.distributed state exists.  ``shard_rows=[n_0, .., n_W-1]``
(every rank's row count, e.g. ``distributed.shard_rows`` of the shard plan) lets the gather skip
its size exchange: with ``check=False`` a sharded estimator then never synchronises the host.
"""
from collections import OrderedDict

import numpy as np
import torch

from .. import distributed as rd
from .. import ops
from ..torch_ops import VARIANT


def _device(*xs):
    for x in xs:
        if isinstance(x, torch.Tensor) and x.is_cuda:
            return x.device
    return torch.device("cuda", torch.cuda.current_device())


def _dev(x, device):
    return x.to(device, non_blocking=True).contiguous()


def _whiten(adv, mask, row_stats, group=None, sizes=None):
    """In place; -> device status i32[1] (0 ok; 1 / 2 = verl's ValueError cases).  With a
    process group the statistics are the whole sharded batch's (opt-in, module docstring)."""
    if group is not None:
        return torch.ops.ragen_amd.masked_whiten_stats_(adv, rd.global_whiten_stats(row_stats, group, sizes))
    return torch.ops.ragen_amd.masked_whiten_(adv, mask, row_stats)


def _back(out_device, tensors, status=None, err=None, check=True, group=None):
    """Results to the caller's device, then the error flags the kernels wrote (one small read;
    for a CPU caller it follows the copy).  Under a process group the flags are reduced over it
    first, so a bad row on one rank raises on every rank instead of stranding the others."""
    res = [t.to(out_device) for t in tensors]
    if not check and out_device.type == "cuda":
        return res
    flags = []
    if status is not None:
        flags.append(status.reshape(-1)[:1].to(torch.int64))
    if err is not None:
        flags.append(err.any().reshape(1).to(torch.int64))
    if not flags:
        return res
    f = torch.cat(flags)
    if group is not None:
        f = rd.all_reduce_max(f, group)
    f = f.cpu().tolist()
    if status is not None:
        ops.raise_whiten_status(int(f[0]))
    if err is not None and f[-1]:
        raise IndexError("index out of range: last loss-mask position of a row carries no reward "
                         "(reference core_algos.py:79)")
    return res


def masked_whiten(values: torch.Tensor, mask: torch.Tensor, shift_mean: bool = True, check: bool = True,
                  process_group=None, shard_rows=None) -> torch.Tensor:
    """verl masked_whiten; ValueError for a mask sum of 0 or 1 like verl's masked_var."""
    if not shift_mean:
        raise NotImplementedError("shift_mean=False is not used by RAGEN")
    dev = _device(values, mask)
    x = _dev(values.float(), dev).clone()
    m = _dev(mask, dev)
    stats = torch.ops.ragen_amd.whiten_row_stats(x, m)
    status = _whiten(x, m, stats, process_group, shard_rows)
    return _back(values.device, [x], status, check=check, group=process_group)[0]


def compute_gae_advantage_return(token_level_rewards, values, response_mask, gamma, lam, variant="legacy",
                                 check=True, process_group=None, shard_rows=None):
    """verl compute_gae_advantage_return (legacy form by default)."""
    dev = _device(token_level_rewards, values, response_mask)
    r, v, m = _dev(token_level_rewards.float(), dev), _dev(values.float(), dev), _dev(response_mask, dev)
    stats = torch.empty(r.shape[0], 3, dtype=torch.float64, device=dev)
    if variant not in VARIANT:
        raise ValueError(f"GAE variant must be 'legacy' or 'masked', got {variant!r}")
    adv, ret = torch.ops.ragen_amd.gae(r, v, m, float(gamma), float(lam), VARIANT[variant], stats)
    status = _whiten(adv, m, stats, process_group, shard_rows)
    return tuple(_back(token_level_rewards.device, [adv, ret], status, check=check, group=process_group))


def compute_bi_level_gae_advantage_return(token_level_rewards, values, loss_mask, gamma, lam, high_level_gamma,
                                          check=True, process_group=None, shard_rows=None):
    """core_algos.py:4-92 (IndexError where the reference raises it, core_algos.py:79)."""
    dev = _device(token_level_rewards, values, loss_mask)
    r, v, m = _dev(token_level_rewards.float(), dev), _dev(values.float(), dev), _dev(loss_mask, dev)
    stats = torch.empty(r.shape[0], 3, dtype=torch.float64, device=dev)
    err = torch.empty(r.shape[0], dtype=torch.uint8, device=dev)
    adv, ret = torch.ops.ragen_amd.bilevel_gae(r, v, m, float(gamma), float(lam), float(high_level_gamma), stats, err)
    status = _whiten(adv, m, stats, process_group, shard_rows)
    return tuple(_back(token_level_rewards.device, [adv, ret], status, err, check=check, group=process_group))


def _grouped(r, m, index, dev, run):
    """Rows grouped by ``index`` (any hashable ids, first-seen order, as verl's id2score dict):
    permute to contiguous groups if needed, run(rows, mask, seg) -> adv, scatter back."""
    groups = OrderedDict()
    for i, k in enumerate(index):
        groups.setdefault(k, []).append(i)
    perm = np.concatenate([np.asarray(v, np.int64) for v in groups.values()]) if groups else np.zeros(0, np.int64)
    seg = np.zeros(len(groups) + 1, np.int32)
    seg[1:] = np.cumsum([len(v) for v in groups.values()])
    ident = np.array_equal(perm, np.arange(len(perm)))
    p = None if ident else torch.from_numpy(perm).to(dev)
    rr = r if ident else r[p].contiguous()
    mm = m if ident else m[p].contiguous()
    adv = run(rr, mm, ops.segments(seg, rr.shape[0], dev))
    if not ident:
        out = torch.empty_like(adv)
        out[p] = adv
        adv = out
    return adv


def compute_grpo_outcome_advantage(token_level_rewards, response_mask, index, epsilon: float = 1e-6,
                                   norm_adv_by_std_in_grpo: bool = True):
    """verl compute_grpo_outcome_advantage: rows grouped by ``index`` (any hashable ids).
    Groups are rank-local under sharding (RAGEN's uids are unique per row, so every group has
    one member, agent_trainer.py:551-552)."""
    dev = _device(token_level_rewards, response_mask)
    r, m = _dev(token_level_rewards.float(), dev), _dev(response_mask, dev)
    adv = _grouped(r, m, index, dev, lambda rr, mm, seg: torch.ops.ragen_amd.grpo_outcome(
        rr, mm, seg, float(epsilon), bool(norm_adv_by_std_in_grpo))[0])
    adv = _back(token_level_rewards.device, [adv])[0]
    return adv, adv


# The verl estimators agent_trainer.compute_advantage dispatches to besides GAE / GRPO
# (agent_trainer.py:102-134).  verl is an empty submodule in the reference: restated from
# verl's published core_algos (the v0.3 line RAGEN pins through vllm 0.8.2); parity unpinned
# beyond that restatement (tests/verl_restated.py runs it on CPU torch as the checker).

def compute_reinforce_plus_plus_outcome_advantage(token_level_rewards, response_mask, gamma, check=True,
                                                  process_group=None, shard_rows=None):
    """verl: returns = right-to-left running = r + gamma * running, reset by the mask;
    advantages = masked_whiten(returns, mask) * mask."""
    dev = _device(token_level_rewards, response_mask)
    r, m = _dev(token_level_rewards.float(), dev), _dev(response_mask, dev)
    stats = torch.empty(r.shape[0], 3, dtype=torch.float64, device=dev)
    adv, ret = torch.ops.ragen_amd.reinforce_pp_returns(r, m, float(gamma), stats)
    status = _whiten(adv, m, stats, process_group, shard_rows)
    torch.ops.ragen_amd.mask_mul_(adv, m)
    return tuple(_back(token_level_rewards.device, [adv, ret], status, check=check, group=process_group))


def compute_reinforce_plus_plus_baseline_outcome_advantage(token_level_rewards, response_mask, index,
                                                           epsilon: float = 1e-6, check=True, process_group=None,
                                                           shard_rows=None):
    """verl: score = sum_t r minus its group's mean (0 for a single-row group), tiled over the
    mask, then masked_whiten(., mask) * mask.  -> (adv, adv)."""
    dev = _device(token_level_rewards, response_mask)
    r, m = _dev(token_level_rewards.float(), dev), _dev(response_mask, dev)
    adv = _grouped(r, m, index, dev, lambda rr, mm, seg: torch.ops.ragen_amd.grpo_outcome(
        rr, mm, seg, float(epsilon), False)[0])
    stats = torch.ops.ragen_amd.whiten_row_stats(adv, m)
    status = _whiten(adv, m, stats, process_group, shard_rows)
    torch.ops.ragen_amd.mask_mul_(adv, m)
    adv = _back(token_level_rewards.device, [adv], status, check=check, group=process_group)[0]
    return adv, adv


def compute_rloo_outcome_advantage(token_level_rewards, response_mask, index, epsilon: float = 1e-6):
    """verl: leave-one-out baseline, s * n/(n-1) - mean * n/(n-1) for groups of n > 1, tiled
    over the mask.  -> (adv, adv)."""
    dev = _device(token_level_rewards, response_mask)
    r, m = _dev(token_level_rewards.float(), dev), _dev(response_mask, dev)
    adv = _grouped(r, m, index, dev, lambda rr, mm, seg: torch.ops.ragen_amd.rloo_outcome(rr, mm, seg)[0])
    adv = _back(token_level_rewards.device, [adv])[0]
    return adv, adv


def compute_remax_outcome_advantage(token_level_rewards, reward_baselines, response_mask):
    """verl: returns = reverse cumsum of r * mask; advantages = returns - baseline * mask."""
    dev = _device(token_level_rewards, reward_baselines, response_mask)
    r, m = _dev(token_level_rewards.float(), dev), _dev(response_mask, dev)
    b = _dev(reward_baselines.float(), dev)
    adv, ret = torch.ops.ragen_amd.remax(r, m, b)
    return tuple(_back(token_level_rewards.device, [adv, ret]))
