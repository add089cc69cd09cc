"""GPU parity of BASELINE.json configs[3] and configs[4] at their full sizes.

configs[4] — Countdown, 16 384 envs x 4 turns, mixed-length trajectories: the turn kernel
against oracle.countdown_turn (es_manager.py:149-169 over countdown/env.py:58-62, pinned to
the reference-run trace in tests/test_oracle.py) on every field of the record each turn, then
the resulting mixed-length token rows through GAE (gamma = 1, lambda = 1 and 0.95) and
bi-level GAE against the oracle.

configs[3] — the N>1 exchange (the RCCL all-gather of the rollout record before the PPO
update), run through a real 1-rank RCCL group on this GPU: the gather of a pool of episode
arenas captured in a HIP graph and replayed, and the batch-global whitening path.

Bar: bit-exact record, rewards and returns; whitened advantages within 1e-5.
"""
import os
import socket

import numpy as np
import pytest
import torch

import oracle
from ragen_amd import distributed as rd
from ragen_amd import ops, synthetic
from ragen_amd.env import CountdownBatch, SokobanBatch
from ragen_amd.env.configs import CountdownEnvConfig, SokobanEnvConfig
from ragen_amd.env.countdown import synthetic_instances

pytestmark = pytest.mark.gpu

EP_FIELDS = ("num_actions", "flags", "n_turns", "penalty", "turn_reward", "turn_info", "turn_exec")


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _countdown_rollout(device, B=16384, T=4):
    inst = synthetic_instances(1024, 7)
    env = CountdownBatch(CountdownEnvConfig(data=inst), B, T, 1, device)
    env.reset(synthetic.env_seeds(B))
    mine = [inst[int(i)] for i in env.index]
    answers = synthetic.countdown_answers(mine, T)  # SURVEY §8(d) mix: 50 % empty turns
    nums = [list(m["nums"]) for m in mine]
    targets = [int(m["target"]) for m in mine]
    oep = oracle.Episode(B, T)
    zeros = torch.zeros(B, 1, dtype=torch.int8, device=device)
    for t in range(T):
        lists = [[a] if a is not None else [] for a in answers[t]]
        buf, lens = env.encode_answers(lists)
        n = np.array([len(x) for x in lists], np.uint8)
        err = torch.zeros(B, dtype=torch.uint8, device=device)
        env.step_turn(t, zeros, _t(n, device), None, 1, -0.1, err, answers=_t(buf, device), answer_len=_t(lens, device))
        oracle.countdown_turn(lists, nums, targets, oep, t, None, 1, -0.1)
        torch.cuda.synchronize()
        assert not err.any(), "an answer left the evaluator's grammar"
        for k in EP_FIELDS:
            np.testing.assert_array_equal(getattr(env.ep, k).cpu().numpy(), getattr(oep, k), err_msg=f"turn {t} {k}")
    return env, oep


@pytest.mark.parametrize("use_has_input", [False, True])
def test_countdown_multi_slot_cap_vs_oracle(device, use_has_input):
    """The turn kernel's single-step form (countdown.hip: at most one step per turn, on slot 0)
    against the oracle's general loop with K = 3 answer slots, 0..3 answers per turn, cap 2, and
    (has_input) envs stepped again after they are done, so turns with no room left under the
    cap (left <= 0) and turns after a done episode both occur."""
    B, T, K, cap = 2048, 5, 3, 2
    inst = synthetic_instances(256, 11)
    env = CountdownBatch(CountdownEnvConfig(data=inst), B, T, K, device)
    env.reset(synthetic.env_seeds(B))
    mine = [inst[int(i)] for i in env.index]
    nums = [list(m["nums"]) for m in mine]
    targets = [int(m["target"]) for m in mine]
    oep = oracle.Episode(B, T)
    rng = np.random.default_rng(5)
    zeros = torch.zeros(B, K, dtype=torch.int8, device=device)
    has = np.ones(B, np.uint8)
    has[rng.random(B) < 0.2] = 0
    for t in range(T):
        per_turn = [synthetic.countdown_answers(mine, 1, seed=100 * t + k, p_empty=0.0)[0] for k in range(K)]
        lists = [[per_turn[k][b] for k in range(int(rng.integers(0, K + 1)))] for b in range(B)]
        buf, lens = env.encode_answers(lists)
        n = np.array([len(x) for x in lists], np.uint8)
        err = torch.zeros(B, dtype=torch.uint8, device=device)
        hi = _t(has, device) if use_has_input else None
        env.step_turn(t, zeros, _t(n, device), hi, cap, -0.1, err, answers=_t(buf, device), answer_len=_t(lens, device))
        oracle.countdown_turn(lists, nums, targets, oep, t, has if use_has_input else None, cap, -0.1)
        torch.cuda.synchronize()
        assert not err.any()
        for k in EP_FIELDS:
            np.testing.assert_array_equal(getattr(env.ep, k).cpu().numpy(), getattr(oep, k), err_msg=f"turn {t} {k}")
    assert (oep.turn_exec <= 1).all() and (oep.turn_exec == 1).any()
    if use_has_input:  # stepped again after done: the cap is reached, then turns with left <= 0
        assert (oep.num_actions == cap).any()


def test_countdown_config4_vs_oracle(device):
    env, oep = _countdown_rollout(device)
    B = env.B
    # mixed lengths: every episode length 1..4 occurs, and some envs never answered
    lengths = np.bincount(oep.n_turns, minlength=5)
    assert (lengths[1:] > 0).all(), lengths
    assert ((oep.flags & oracle.FLAG_DONE) == 0).any()
    np.testing.assert_array_equal(ops.rollout_metrics(env.ep).cpu().numpy(), oracle.rollout_metrics(oep))
    s, p = ops.trajectory_scores(env.ep)
    os_, op_ = oracle.trajectory_scores(oep)
    np.testing.assert_array_equal(s.cpu().numpy(), os_)
    np.testing.assert_array_equal(p.cpu().numpy(), op_)
    seg = np.arange(0, B + 1, 16, dtype=np.int32)
    norm = ops.group_normalize(s, p, seg, "mean_std")
    np.testing.assert_allclose(norm.cpu().numpy(), oracle.group_normalize(os_, op_, seg, "mean_std"), rtol=0,
                               atol=1e-5)
    # the segmented-scan stress: token rows of these trajectories (score at the last column)
    r, v, m = synthetic.token_rows(oep.n_turns, os_ + op_, seed=21)
    tr, tv, tm = _t(r, device), _t(v, device), _t(m, device)
    for lam in (1.0, 0.95):
        stats = torch.zeros(B, 3, dtype=torch.float64, device=device)
        adv, ret = ops.gae(tr, tv, tm, 1.0, lam, row_stats=stats)
        oadv, oret = oracle.gae(r, v, m, 1.0, lam)
        np.testing.assert_array_equal(ret.cpu().numpy(), oret)
        np.testing.assert_array_equal(adv.cpu().numpy(), oadv)
        ops.masked_whiten_(adv, tm, stats)
        np.testing.assert_allclose(adv.cpu().numpy(), oracle.masked_whiten(oadv, m), rtol=0, atol=1e-5)
    # bi-level GAE with each turn's reward on its last response token (the turn-score variant)
    ts = oep.turn_reward.T.astype(np.float32).copy()
    rb, vb, mb = synthetic.token_rows(oep.n_turns, os_, seed=22, turn_scores=ts)
    err = torch.zeros(B, dtype=torch.uint8, device=device)
    adv, ret = ops.bilevel_gae(_t(rb, device), _t(vb, device), _t(mb, device), 1.0, 0.95, 0.95, check_errors=False,
                               err=err)
    oadv, oret, oerr = oracle.bilevel_gae(rb, vb, mb, 1.0, 0.95, 0.95)
    ok = oerr == 0
    np.testing.assert_array_equal(err.cpu().numpy() != 0, ~ok)
    assert ok.sum() > B // 4 and (~ok).sum() > 0  # zero-reward last turns raise in the reference
    np.testing.assert_array_equal(ret.cpu().numpy()[ok], oret[ok])
    np.testing.assert_array_equal(adv.cpu().numpy()[ok], oadv[ok])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def rccl_group(device):
    """A real 1-rank RCCL ('nccl') process group on this GPU: the N>1 exchange code path."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=device)
    try:
        yield dist
    finally:
        dist.destroy_process_group()


def test_rccl_arena_gather_graph(device, rccl_group):
    """configs[3]'s exchange: the episode arenas of G rollouts (one pool, contiguous) gathered
    by ONE all-gather captured in a HIP graph; the replay's views equal the local arenas."""
    B, T, K, G = 8192, 5, 5, 4
    env = SokobanBatch(SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100), B, T, K, device)
    env.reset(synthetic.env_seeds(B))
    pool, eps = ops.EpisodeState.pool(G, B, T, device)
    st = env.struct()
    for j, ep in enumerate(eps):  # different actions per arena, so the arenas differ
        ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=50 + j)
        ids, n = _t(ids, device), _t(n, device)
        env.restore()
        for t in range(T):
            ops.sokoban_step_turn(st, ep, ops.turn_struct(t, ids[t], n[t], None, 10, -0.1))
    torch.cuda.synchronize()
    assert not torch.equal(eps[0].arena, eps[1].arena)
    W = rccl_group.get_world_size()
    out = torch.zeros(W * pool.numel(), dtype=torch.uint8, device=device)
    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(side):  # communicator setup outside the capture
        rd.gather_bytes(pool, out)
    torch.cuda.synchronize()
    out.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        rd.gather_bytes(pool, out)
    for _ in range(3):
        out.zero_()
        g.replay()
    torch.cuda.synchronize()
    views = rd.episode_views(out.view(W * G, -1), B, T)
    assert len(views) == W * G
    for v, ep in zip(views, eps):
        for k in EP_FIELDS:
            assert torch.equal(getattr(v, k), getattr(ep, k)), k


def test_rccl_global_whitening(device, rccl_group):
    """masked_whiten over gathered per-row partials (global_whiten_stats, through RCCL) ==
    the single-process whitening, bit for bit, and == the oracle within 1e-5."""
    from ragen_amd.trainer import core_algos
    rng = np.random.default_rng(3)
    n_turns = rng.integers(1, 5, size=4096)
    r, v, m = synthetic.token_rows(n_turns, rng.standard_normal(4096).astype(np.float32), seed=5)
    tr, tv, tm = _t(r, device), _t(v, device), _t(m, device)
    stats = torch.zeros(r.shape[0], 3, dtype=torch.float64, device=device)
    adv, ret = ops.gae(tr, tv, tm, 1.0, 0.95, row_stats=stats)
    gstats = rd.global_whiten_stats(stats)
    assert torch.equal(gstats, stats)
    a1 = adv.clone()
    ops.masked_whiten_stats_(a1, gstats)
    a2 = adv.clone()
    ops.masked_whiten_(a2, tm, stats)
    torch.cuda.synchronize()
    assert torch.equal(a1, a2)
    # the facade's opt-in global path (CPU inputs, as the trainer's)
    fa, fr = core_algos.compute_gae_advantage_return(torch.from_numpy(r), torch.from_numpy(v), torch.from_numpy(m),
                                                     1.0, 0.95, process_group=rccl_group.group.WORLD)
    assert torch.equal(fa, a1.cpu()) and torch.equal(fr, ret.cpu())
    oadv, _ = oracle.gae(r, v, m, 1.0, 0.95)
    np.testing.assert_allclose(fa.numpy(), oracle.masked_whiten(oadv, m), rtol=0, atol=1e-5)
