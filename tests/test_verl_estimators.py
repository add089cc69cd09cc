"""The verl estimators compute_advantage dispatches to besides GAE / GRPO
(agent_trainer.py:102-134): REINFORCE++, REINFORCE++-baseline, REMAX, RLOO.
CPU: the C oracle == verl restated on CPU torch (tests/verl_restated.py).
GPU: the kernels (rmi_reinforce_pp_returns, rmi_remax, rmi_rloo_outcome, rmi_mask_mul, with
the whitening kernels) == the oracle, and compute_advantage on each estimator == verl.
Returns bit-exact; whitened advantages within 1e-5 (fp64 statistics vs torch's f32 sums)."""
from collections import OrderedDict

import numpy as np
import pytest
import torch

import oracle
import verl_restated as verl


def _batch(B=96, L=57, seed=0, groups=12):
    rng = np.random.default_rng(seed)
    r = (rng.standard_normal((B, L)) * (rng.random((B, L)) < 0.2)).astype(np.float32)
    lens = rng.integers(1, L + 1, B)
    m = (np.arange(L)[None, :] >= (L - lens)[:, None]).astype(np.uint8)  # left-padded responses
    m[rng.random((B, L)) < 0.05] = 0  # holes (env-observation tokens)
    m[:, -1] = 1
    uid = [f"u{int(g)}" for g in rng.integers(0, groups, B)]  # shuffled, uneven groups, some singletons
    uid[0] = "solo"
    base = rng.standard_normal(B).astype(np.float32)
    return r, m, uid, base


def _perm(uid):
    groups = OrderedDict()
    for i, k in enumerate(uid):
        groups.setdefault(k, []).append(i)
    perm = np.concatenate([np.asarray(v) for v in groups.values()])
    seg = np.zeros(len(groups) + 1, np.int32)
    seg[1:] = np.cumsum([len(v) for v in groups.values()])
    return perm, seg


def _unperm(x, perm):
    out = np.empty_like(x)
    out[perm] = x
    return out


@pytest.mark.parametrize("gamma", [1.0, 0.95])
def test_oracle_reinforce_pp_equals_verl(gamma):
    r, m, _, _ = _batch()
    adv, ret = oracle.reinforce_pp(r, m, gamma)
    vadv, vret = verl.compute_reinforce_plus_plus_outcome_advantage(torch.from_numpy(r), torch.from_numpy(m).bool(),
                                                                    gamma)
    assert np.array_equal(ret, vret.numpy())
    np.testing.assert_allclose(adv, vadv.numpy(), rtol=1e-5, atol=1e-5)


def test_oracle_remax_equals_verl():
    r, m, _, base = _batch(seed=1)
    adv, ret = oracle.remax(r, m, base)
    vadv, vret = verl.compute_remax_outcome_advantage(torch.from_numpy(r), torch.from_numpy(base),
                                                      torch.from_numpy(m).bool())
    assert np.array_equal(ret, vret.numpy())
    assert np.array_equal(adv, vadv.numpy())


def test_oracle_rloo_and_baseline_equal_verl():
    r, m, uid, _ = _batch(seed=2)
    perm, seg = _perm(uid)
    adv, _ = oracle.rloo(r[perm], m[perm], seg)
    vadv, _ = verl.compute_rloo_outcome_advantage(torch.from_numpy(r), torch.from_numpy(m).bool(), uid)
    np.testing.assert_allclose(_unperm(adv, perm), vadv.numpy(), rtol=1e-6, atol=1e-6)
    adv, _ = oracle.reinforce_pp_baseline(r[perm], m[perm], seg)
    vadv, _ = verl.compute_reinforce_plus_plus_baseline_outcome_advantage(torch.from_numpy(r),
                                                                          torch.from_numpy(m).bool(), uid)
    np.testing.assert_allclose(_unperm(adv, perm), vadv.numpy(), rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("gamma", [1.0, 0.95])
def test_reinforce_pp_kernel_vs_oracle(device, gamma):
    from ragen_amd import ops
    r, m, _, _ = _batch(B=1031, L=333, seed=3)  # ragged: B % 4, L % 4 != 0
    st = torch.empty(r.shape[0], 3, dtype=torch.float64, device=device)
    adv, ret = ops.reinforce_pp_returns(torch.from_numpy(r).to(device), torch.from_numpy(m).to(device), gamma, st)
    _, oret = oracle.reinforce_pp(r, m, gamma, whiten=False)
    assert np.array_equal(ret.cpu().numpy(), oret)
    assert np.array_equal(adv.cpu().numpy(), oret)


@pytest.mark.gpu
def test_remax_rloo_kernels_vs_oracle(device):
    from ragen_amd import ops
    r, m, uid, base = _batch(B=1031, L=333, seed=4, groups=200)
    td = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(device)  # noqa: E731
    adv, ret = ops.remax(td(r), td(m), td(base))
    oadv, oret = oracle.remax(r, m, base)
    assert np.array_equal(ret.cpu().numpy(), oret) and np.array_equal(adv.cpu().numpy(), oadv)
    perm, seg = _perm(uid)
    adv, _ = ops.rloo_outcome(td(r[perm]), td(m[perm]), seg)
    oadv, _ = oracle.rloo(r[perm], m[perm], seg)
    np.testing.assert_allclose(adv.cpu().numpy(), oadv, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("est", ["reinforce_plus_plus", "reinforce_plus_plus_baseline", "remax", "rloo"])
def test_compute_advantage_verl_estimators(device, est):
    """agent_trainer.compute_advantage's dispatch (advantage.py) on a CPU batch == verl."""
    from ragen_amd.protocol import DataProto
    from ragen_amd.trainer.advantage import compute_advantage
    r, m, uid, base = _batch(B=512, L=200, seed=5, groups=60)
    tr, tm, tb = torch.from_numpy(r), torch.from_numpy(m).bool(), torch.from_numpy(base)
    data = DataProto.from_dict({"token_level_rewards": tr.clone(), "response_mask": tm.clone(),
                                "reward_baselines": tb.clone()}, non_tensors={"uid": np.array(uid, dtype=object)})
    out = compute_advantage(data, est, gamma=0.97)
    adv, ret = out.batch["advantages"], out.batch["returns"]
    assert adv.device.type == "cpu" and ret.device.type == "cpu"
    if est == "reinforce_plus_plus":
        vadv, vret = verl.compute_reinforce_plus_plus_outcome_advantage(tr, tm, 0.97)
        assert torch.equal(ret, vret)
    elif est == "reinforce_plus_plus_baseline":
        vadv, vret = verl.compute_reinforce_plus_plus_baseline_outcome_advantage(tr.clone(), tm, uid)
    elif est == "remax":
        vadv, vret = verl.compute_remax_outcome_advantage(tr, tb, tm)
        assert torch.equal(ret, vret) and torch.equal(adv, vadv)
    else:
        vadv, vret = verl.compute_rloo_outcome_advantage(tr.clone(), tm, uid)
    torch.testing.assert_close(adv, vadv, rtol=1e-5, atol=1e-5)
