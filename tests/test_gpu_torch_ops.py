"""torch.ops.ragen_amd.* (the dispatcher path the facades use) against the raw C-ABI path
(ragen_amd.ops over ctypes structs), bit for bit, and the ops inside torch.compile."""
import numpy as np
import pytest
import torch

from ragen_amd import ops, synthetic
from ragen_amd.env import BanditBatch, CountdownBatch, FrozenLakeBatch, SokobanBatch
from ragen_amd.env.configs import BanditEnvConfig, CountdownEnvConfig, FrozenLakeEnvConfig, SokobanEnvConfig
from ragen_amd.env.countdown import synthetic_instances

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _same(a, b, names):
    for n in names:
        assert torch.equal(getattr(a, n), getattr(b, n)), n
    assert torch.equal(a.ep.arena, b.ep.arena)


def test_sokoban_op_equals_ctypes(device):
    B, T, K = 8192, 5, 5
    cfg = SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100)
    a, b = SokobanBatch(cfg, B, T, K, device), SokobanBatch(cfg, B, T, K, device)
    a.reset(synthetic.env_seeds(B))
    b.load_state(a.room_fixed.cpu().numpy(), a.init_state.cpu().numpy(), a.init_player.cpu().numpy())
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4)
    for t in range(T):
        a.step_turn(t, _t(ids[t], device), _t(n[t], device), None, 10, -0.1)
        ops.sokoban_step_turn(b.struct(), b.ep, ops.turn_struct(t, _t(ids[t], device), _t(n[t], device), None, 10,
                                                                -0.1))
    torch.cuda.synchronize()
    _same(a, b, ("room_state", "player", "num_env_steps", "boxes_on_target"))
    ra, rb = a.render_rows(), ops.sokoban_render(b.struct(), B, b.config.grid_lookup, device)
    assert ops.decode_rows(*ra) == ops.decode_rows(*rb)  # bytes past a row's length are not written


def test_frozenlake_bandit_countdown_op_equals_ctypes(device):
    B, T, K = 4096, 8, 5
    a, b = (FrozenLakeBatch(FrozenLakeEnvConfig(), B, T, K, device) for _ in range(2))
    a.reset(synthetic.env_seeds(B))
    b.load_state(a.init_desc.cpu().numpy(), a.init_s.cpu().numpy(), a.init_rng.cpu().numpy())
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=3)
    for t in range(T):
        a.step_turn(t, _t(ids[t], device), _t(n[t], device), None, 10, -0.1)
        ops.frozenlake_step_turn(b.struct(), b.ep, ops.turn_struct(t, _t(ids[t], device), _t(n[t], device), None,
                                                                   10, -0.1))
    torch.cuda.synchronize()
    _same(a, b, ("s", "rng"))
    # Bandit
    a, b = (BanditBatch(BanditEnvConfig(lo_arm_name="Phoenix", hi_arm_name="Dragon"), B, 2, 1, device)
            for _ in range(2))
    a.reset(synthetic.env_seeds(B))
    b.load_state(a.hi_is_first.cpu().numpy(), a.rng.cpu().numpy())
    for t in range(2):
        ids = _t(np.random.default_rng(t).integers(1, 3, size=(B, 1)).astype(np.int8), device)
        one = torch.ones(B, dtype=torch.uint8, device=device)
        a.step_turn(t, ids, one, None, 2, -0.1)
        ops.bandit_step_turn(b.struct(), b.ep, ops.turn_struct(t, ids, one, None, 2, -0.1))
    torch.cuda.synchronize()
    _same(a, b, ("rng",))
    # Countdown
    inst = synthetic_instances(256, 7)
    a, b = (CountdownBatch(CountdownEnvConfig(data=inst), B, 2, 1, device) for _ in range(2))
    a.reset(synthetic.env_seeds(B))
    b.reset(synthetic.env_seeds(B))
    answers = synthetic.countdown_answers([inst[int(i)] for i in a.index], 2)
    z = torch.zeros(B, 1, dtype=torch.int8, device=device)
    for t in range(2):
        lists = [[x] if x is not None else [] for x in answers[t]]
        buf, lens = a.encode_answers(lists)
        nn = _t(np.array([len(x) for x in lists], np.uint8), device)
        a.step_turn(t, z, nn, None, 1, -0.1, answers=_t(buf, device), answer_len=_t(lens, device))
        ops.countdown_step_turn(b.struct(), b.ep, ops.turn_struct(t, z, nn, None, 1, -0.1), _t(buf, device),
                                _t(lens, device))
    torch.cuda.synchronize()
    assert torch.equal(a.ep.arena, b.ep.arena)


def test_advantage_ops_equal_ctypes_and_compile(device):
    rng = np.random.default_rng(0)
    r, v, m = synthetic.token_rows(rng.integers(1, 6, 2048), rng.standard_normal(2048).astype(np.float32), seed=4)
    tr, tv, tm = _t(r, device), _t(v, device), _t(m, device)
    s1 = torch.empty(tr.shape[0], 3, dtype=torch.float64, device=device)
    s2 = torch.empty_like(s1)
    a1, r1 = torch.ops.ragen_amd.gae(tr, tv, tm, 1.0, 0.95, 0, s1)
    a2, r2 = ops.gae(tr, tv, tm, 1.0, 0.95, "legacy", s2)
    assert torch.equal(a1, a2) and torch.equal(r1, r2) and torch.equal(s1, s2)

    def fn(r, v, m):
        stats = torch.empty(r.shape[0], 3, dtype=torch.float64, device=r.device)
        adv, ret = torch.ops.ragen_amd.gae(r, v, m, 1.0, 0.95, 0, stats)
        status = torch.ops.ragen_amd.masked_whiten_(adv, m, stats)
        return adv * 1.0, ret, status

    eager = fn(tr, tv, tm)
    compiled = torch.compile(fn, backend="aot_eager", fullgraph=True)(tr, tv, tm)
    for x, y in zip(eager, compiled):
        assert torch.equal(x, y)
    assert int(eager[2]) == 0
