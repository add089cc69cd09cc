"""Advantage estimators on the GPU engine — drop-ins for ragen/trainer/core_algos.py:4-92 and
the verl functions RAGEN imports from it (App. A.4): same names, signatures and return
values; tensors may arrive on the CPU (as in the reference) and are moved to the device.
"""
from collections import OrderedDict

import numpy as np
import torch

from .. import ops


def _dev(x, device):
    return x.to(device).contiguous()


def _device():
    return torch.device("cuda", torch.cuda.current_device())


def masked_whiten(values: torch.Tensor, mask: torch.Tensor, shift_mean: bool = True) -> torch.Tensor:
    """verl masked_whiten; raises ValueError for a mask sum of 0 or 1 like verl's masked_var."""
    if not shift_mean:
        raise NotImplementedError("shift_mean=False is not used by RAGEN")
    dev = _device()
    x = _dev(values.float(), dev).clone()
    m = _dev(mask, dev)
    n = int((m != 0).sum().item())
    if n == 0:
        raise ValueError("At least one element in the mask has to be 1.")
    if n == 1:
        raise ValueError("The sum of the mask is one, which can cause a division by zero.")
    ops.masked_whiten_(x, m)
    return x.to(values.device)


def compute_gae_advantage_return(token_level_rewards, values, response_mask, gamma, lam, variant="legacy"):
    """verl compute_gae_advantage_return (legacy form by default)."""
    dev = _device()
    r, v, m = _dev(token_level_rewards.float(), dev), _dev(values.float(), dev), _dev(response_mask, dev)
    B = r.shape[0]
    stats = torch.zeros(B, 3, dtype=torch.float64, device=dev)
    adv, ret = ops.gae(r, v, m, gamma, lam, variant, row_stats=stats)
    _check_mask_sum(stats)
    ops.masked_whiten_(adv, m, stats)
    return adv.to(token_level_rewards.device), ret.to(token_level_rewards.device)


def compute_bi_level_gae_advantage_return(token_level_rewards, values, loss_mask, gamma, lam, high_level_gamma):
    """core_algos.py:4-92 (IndexError where the reference raises it, core_algos.py:79)."""
    dev = _device()
    r, v, m = _dev(token_level_rewards.float(), dev), _dev(values.float(), dev), _dev(loss_mask, dev)
    stats = torch.zeros(r.shape[0], 3, dtype=torch.float64, device=dev)
    adv, ret = ops.bilevel_gae(r, v, m, gamma, lam, high_level_gamma, row_stats=stats)
    _check_mask_sum(stats)
    ops.masked_whiten_(adv, m, stats)
    return adv.to(token_level_rewards.device), ret.to(token_level_rewards.device)


def _check_mask_sum(stats):
    n = float(stats[:, 2].sum().item())
    if n == 0:
        raise ValueError("At least one element in the mask has to be 1.")
    if n == 1:
        raise ValueError("The sum of the mask is one, which can cause a division by zero.")


def compute_grpo_outcome_advantage(token_level_rewards, response_mask, index, epsilon: float = 1e-6,
                                   norm_adv_by_std_in_grpo: bool = True):
    """verl compute_grpo_outcome_advantage: rows grouped by ``index`` (any hashable ids)."""
    dev = _device()
    r, m = _dev(token_level_rewards.float(), dev), _dev(response_mask, dev)
    groups = OrderedDict()
    for i, k in enumerate(index):
        groups.setdefault(k, []).append(i)
    perm = np.concatenate([np.asarray(v, np.int64) for v in groups.values()])
    seg = np.zeros(len(groups) + 1, np.int32)
    seg[1:] = np.cumsum([len(v) for v in groups.values()])
    ident = np.array_equal(perm, np.arange(len(perm)))
    p = torch.from_numpy(perm).to(dev)
    rr = r if ident else r[p].contiguous()
    mm = m if ident else m[p].contiguous()
    adv, _ = ops.grpo_outcome(rr, mm, torch.from_numpy(seg).to(dev), epsilon, norm_adv_by_std_in_grpo)
    if not ident:
        out = torch.empty_like(adv)
        out[p] = adv
        adv = out
    adv = adv.to(token_level_rewards.device)
    return adv, adv
