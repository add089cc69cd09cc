"""Multi-GPU sharding of the rollout: one process per GPU, torch.distributed
("nccl" = RCCL over xGMI on ROCm; "gloo" in CPU tests).

Partitioning: contiguous, group-aligned — rank r of W owns env groups
[r*G/W, (r+1)*G/W); global env ids, group ids and seeds (base + global group id) are kept,
so a rank's envs are bit-identical to the same envs of a 1-GPU run.  The rollout itself
needs no collective.  The real exchange steps after it are:
  * the rollout filter (agent_trainer.py:461-500) ranks groups GLOBALLY: all-gather the
    per-group trajectory scores, then every rank runs the identical deterministic top-k;
  * masked whitening (verl masked_whiten) uses batch-global mean/var: all-gather the
    per-row (sum, sum_sq, count) partials and reduce them in global row order, so the
    statistics are identical for every world size;
  * reassembly of the trajectory record before the PPO update: every rank's episode arena
    (``EpisodeState``: counters, flags, penalties, per-turn rewards / info / exec counts — one
    contiguous buffer by construction) in ONE all-gather (``gather_episode``), plus optional
    fixed-shape per-env rows (``gather_rollout``).
"""
from typing import Callable, Dict, Tuple

import numpy as np
import torch
import torch.distributed as dist


def initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def world() -> Tuple[int, int]:
    if initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def shard_groups(n_groups: int, world_size: int, rank: int) -> Tuple[int, int]:
    """-> (first global group, number of local groups); contiguous and group-aligned."""
    lo = (n_groups * rank) // world_size
    hi = (n_groups * (rank + 1)) // world_size
    return lo, hi - lo


def _staged(x: torch.Tensor, group=None) -> torch.Tensor:
    """gloo moves host memory: a GPU tensor goes through a host copy (RCCL takes it directly)."""
    if x.is_cuda and dist.get_backend(group) == "gloo":
        return x.cpu()
    return x


def all_reduce_max(x: torch.Tensor, group=None) -> torch.Tensor:
    """Element-wise max over the ranks of ``group`` (the default group if None); the local
    tensor without a process group."""
    if not initialized():
        return x
    xs = _staged(x.contiguous().clone(), group)
    dist.all_reduce(xs, op=dist.ReduceOp.MAX, group=group)
    return xs.to(x.device)


def shard_rows(n_groups: int, group_size: int, world_size: int):
    """Every rank's row count under the group-aligned shard plan (shard_groups), in rank order:
    known on every host without communication, so a gather given it needs no host sync."""
    return [shard_groups(n_groups, world_size, r)[1] * group_size for r in range(world_size)]


def all_gather_rows(x: torch.Tensor, with_offset: bool = False, group=None, sizes=None):
    """Concatenate every rank's [n_r, ...] rows in rank order (n_r may differ by rank).
    Whenever a process group exists the collective runs (also at world size 1, so the one-GPU
    tests exercise the RCCL path); without one the local rows are returned.
    sizes: every rank's n_r in rank order when the caller knows them (e.g. ``shard_rows``): the
    size exchange and its device -> host read are skipped, so the gather is stream-ordered.
    Without it the sizes are all-gathered and read back (one host synchronisation).
    with_offset: -> (rows, this rank's first row in the result)."""
    if not initialized():
        return (x, 0) if with_offset else x
    W, rank = dist.get_world_size(group), dist.get_rank(group)
    xs = _staged(x.contiguous(), group)
    if sizes is None:
        n = torch.tensor([xs.shape[0]], dtype=torch.int64, device=xs.device)
        gathered = [torch.zeros_like(n) for _ in range(W)]
        dist.all_gather(gathered, n, group=group)
        sizes = [int(s) for s in torch.cat(gathered).cpu().tolist()]
    else:
        sizes = [int(s) for s in sizes]
        if len(sizes) != W or sizes[rank] != xs.shape[0]:
            raise ValueError(f"sizes {sizes} do not match world size {W} / this rank's {xs.shape[0]} rows")
    m = max(sizes)
    if all(s == m for s in sizes):  # equal shards: one all-gather straight into the result
        out = torch.empty((W * m,) + tuple(xs.shape[1:]), dtype=xs.dtype, device=xs.device)
        dist.all_gather_into_tensor(out, xs, group=group)
        out = out.to(x.device)
    else:
        pad = torch.zeros((m,) + tuple(xs.shape[1:]), dtype=xs.dtype, device=xs.device)
        pad[:xs.shape[0]] = xs
        bufs = [torch.empty_like(pad) for _ in range(W)]
        dist.all_gather(bufs, pad, group=group)
        out = torch.cat([b[:s] for b, s in zip(bufs, sizes)], dim=0).to(x.device)
    return (out, sum(sizes[:rank])) if with_offset else out


def global_whiten_stats(row_stats: torch.Tensor, group=None, sizes=None) -> torch.Tensor:
    """[n_local, 3] f64 (sum, sum_sq, count) -> [n_global, 3] in global row order; with
    ``sizes`` (every rank's row count) free of host synchronisation."""
    return all_gather_rows(row_stats, group=group, sizes=sizes)


def gather_group_scores(scores: torch.Tensor, group_size: int, with_offset: bool = False, group=None):
    """Per-env trajectory scores of the local groups -> all groups' scores (global order);
    with_offset also returns the first global GROUP index of this rank."""
    assert scores.shape[0] % group_size == 0
    rows, off = all_gather_rows(scores.view(-1, group_size), with_offset=True, group=group)
    return (rows.reshape(-1), off) if with_offset else rows.reshape(-1)


def global_filter(local_scores: torch.Tensor, group_size: int, select: Callable, group=None):
    """The rollout filter over the GLOBAL batch (agent_trainer.py:461-500 ranks groups across all
    of them): every rank gathers every group's scores, runs the same deterministic
    ``select(all_scores, num_groups) -> (keep u8[G], metrics)`` and keeps its own slice.
    -> (keep of the local groups, metrics)."""
    all_scores, g0 = gather_group_scores(local_scores, group_size, with_offset=True, group=group)
    G = all_scores.numel() // group_size
    keep, metrics = select(all_scores, G)
    n_local = local_scores.shape[0] // group_size
    return keep[g0:g0 + n_local], metrics


def gather_bytes(buf: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """Every rank's contiguous u8 buffer (same size on all ranks) -> u8[W, numel] in rank order,
    one all-gather.  ``out`` (u8, W*numel, preallocated) makes the call graph-capturable.
    Without a process group the local buffer is returned as a view."""
    flat = buf.reshape(-1)
    if not initialized():
        return flat.view(1, -1)
    W = dist.get_world_size()
    n = flat.numel()
    if out is None:
        out = torch.empty(W * n, dtype=torch.uint8, device=buf.device)  # flat: gloo and RCCL both take it
    assert buf.dtype == torch.uint8 and buf.is_contiguous()
    assert out.dtype == torch.uint8 and out.numel() == W * n and out.is_contiguous()
    dist.all_gather_into_tensor(out.view(-1), flat)
    return out.view(W, n)


def gather_episode(ep, out: torch.Tensor = None) -> torch.Tensor:
    """Every rank's episode arena -> u8[W, nbytes] in rank order, one collective.  All ranks
    must hold the same (B, T) shard shape; ``episode_views`` re-types a rank's row.  Several
    rollouts' arenas from ``EpisodeState.pool`` move together with ``gather_bytes``."""
    return gather_bytes(ep.arena, out)


def episode_views(gathered: torch.Tensor, B: int, T: int):
    """u8[W, nbytes] from gather_episode -> one EpisodeState (views) per rank."""
    from .ops import EpisodeState
    fields, total = EpisodeState.layout(B, T)
    assert gathered.shape[1] == max(total, 1)
    return [EpisodeState(arena=row, **{n: EpisodeState.view(row, dt, sh, off) for n, dt, sh, off in fields})
            for row in gathered]


def gather_rollout(tensors: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Reassemble fixed-shape per-env trajectory tensors [n_local, ...] from every rank."""
    return {k: all_gather_rows(v) for k, v in tensors.items()}


def all_reduce_max_int(v: int, group=None, device=None) -> int:
    """max of a Python int over the ranks (the local value without a process group)."""
    if not initialized():
        return int(v)
    t = torch.tensor([int(v)], dtype=torch.int64, device=device if device is not None else "cpu")
    return int(all_reduce_max(t, group).cpu()[0])


def left_pad(x: torch.Tensor, width: int, value) -> torch.Tensor:
    """[B, w] -> [B, width] with `value` columns added on the left (w <= width)."""
    w = x.shape[1]
    if w == width:
        return x
    out = torch.full((x.shape[0], width), value, dtype=x.dtype, device=x.device)
    out[:, width - w:] = x
    return out


def gather_formulated(dp, pad_id: int, group=None, sizes=None):
    """Token-level reassembly of formulate_rollouts' batch over the ranks: the
    reference builds ONE left-padded batch (ctx_manager.py:278-306), so every rank pads its
    shard to the global width S (an all-reduce of max S), then the rows are all-gathered in
    rank order — the global env order, since shards are contiguous (``sizes``: every rank's
    row count when known, e.g. EnvStateManager.shard_sizes: no size exchange).  Token tensors [B, S],
    masks / scores [B, S-1]; responses = input_ids[:, 1:]; original_rm_scores keeps aliasing
    rm_scores.  env_ids / group_ids are gathered too (messages_list stays with its rank).
    -> a DataProto of the whole batch, identical on every rank."""
    from .protocol import DataProto
    b = dp.batch
    ids = b["input_ids"]
    S = all_reduce_max_int(ids.shape[1], group, ids.device)
    spec = {"input_ids": (S, int(pad_id)), "attention_mask": (S, 0), "position_ids": (S, 0),
            "loss_mask": (S - 1, False), "rm_scores": (S - 1, 0.0)}
    out = {}
    for k, (w, v) in spec.items():
        if k in b.keys():
            out[k] = all_gather_rows(left_pad(b[k], w, v).contiguous(), group=group, sizes=sizes)
    out["responses"] = out["input_ids"][:, 1:]
    if "original_rm_scores" in b.keys():
        out["original_rm_scores"] = out["rm_scores"]
    nt = {}
    for k in ("env_ids", "group_ids"):
        if k in dp.non_tensor_batch:  # a LazyDataProto makes these two without building its messages
            loc = torch.tensor(np.asarray(dp.non_tensor_batch[k], np.int64), device=ids.device)
            nt[k] = np.array(all_gather_rows(loc, group=group, sizes=sizes).cpu().tolist(), dtype=object)
    return DataProto(out, nt, dict(dp.meta_info))
