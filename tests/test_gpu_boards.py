"""The Sokoban turn's board cache (SokobanBatch.enable_boards; include/ragen_amd.h, the
rmi_sokoban_t boards / boards_mode fields): turns that read each room's cached bitboards instead
of decoding its grid rows == the oracle bit for bit, across rollouts (restore between), with
has_input patterns that leave envs out of the building turn, irregular rooms and action ids off
the regular path (the waves that fall back to the rows), and the bench's captured sequence
(fused first turn BUILD, plain and finalize turns USE) against the same rollout without a cache.
Launches that do not keep the cache refuse a struct carrying it."""
import numpy as np
import pytest
import torch

import oracle
from ragen_amd import _lib, ops, synthetic
from ragen_amd.env import SokobanBatch
from ragen_amd.env.configs import SokobanEnvConfig
from test_gpu_parity import _host_ep, _irregular_rooms, _t

pytestmark = pytest.mark.gpu
FIELDS = ("num_actions", "flags", "n_turns", "penalty", "turn_reward", "turn_info", "turn_exec")


def _match(env, oep, fixed, state, player, nes, bot, ok=None):
    ok = np.ones(env.B, bool) if ok is None else ok
    np.testing.assert_array_equal(env.room_state.cpu().numpy()[ok], state[ok])
    np.testing.assert_array_equal(env.room_fixed.cpu().numpy()[ok], fixed[ok])
    np.testing.assert_array_equal(env.player.cpu().numpy()[ok], player[ok])
    np.testing.assert_array_equal(env.num_env_steps.cpu().numpy()[ok], nes[ok])
    np.testing.assert_array_equal(env.boxes_on_target.cpu().numpy()[ok], bot[ok])
    h = _host_ep(env.ep)
    for k in FIELDS:
        got, want = h[k], getattr(oep, k)
        if got.ndim == 2:
            np.testing.assert_array_equal(got[:, ok], want[:, ok], err_msg=k)
        else:
            np.testing.assert_array_equal(got[ok], want[ok], err_msg=k)


@pytest.mark.parametrize("B", [8192, 20000])
def test_boards_rollouts_vs_oracle(device, B):
    T, K = 5, 5
    cfg = SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100)
    env = SokobanBatch(cfg, B, T, K, device)
    assert env.enable_boards()
    env.reset(synthetic.env_seeds(B))
    fixed0 = env.room_fixed.cpu().numpy()
    state0, player0 = env.room_state.cpu().numpy(), env.player.cpu().numpy()
    rng = np.random.default_rng(B)
    for rollout in range(3):
        if rollout:
            env.restore()
        fixed, state, player = fixed0.copy(), state0.copy(), player0.copy()
        nes, bot = np.zeros(B, np.int32), np.zeros(B, np.int32)
        oep = oracle.Episode(B, T)
        ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=100 + rollout)
        # turn 0 leaves ~30 % of the envs out (the BUILD turn writes their entries unstepped);
        # later turns feed a random 80 % of the envs, derived from the done flags on even turns
        has = (rng.random((T, B)) < np.where(np.arange(T) == 0, 0.7, 0.8)[:, None]).astype(np.uint8)
        for t in range(T):
            h_in = has[t] if (t == 0 or t % 2) else None
            env.step_turn(t, _t(ids[t], device), _t(n[t], device), None if h_in is None else _t(h_in, device), 10,
                          -0.1)
            oracle.sokoban_turn(6, 6, 1, 100, fixed, state, player, nes, bot, oep, t, ids[t], n[t], h_in, 10, -0.1)
            torch.cuda.synchronize()
            _match(env, oep, fixed, state, player, nes, bot)
        assert env._boards_valid
        tags = env.boards.cpu().numpy()[:, 13]
        assert (tags == 1).all(), "every generated room stays regular: every entry tagged"


@pytest.mark.parametrize("frac_irregular", [0.01, 0.5])
def test_boards_irregular_rooms_vs_oracle(device, frac_irregular):
    """Irregular rooms (exact LDS path: their entries untagged) mixed with regular ones, invalid
    and out-of-range action ids (waves falling back to the rows): == the oracle wherever the
    reference does not raise, and the same error flags where it does."""
    rng = np.random.default_rng(int(frac_irregular * 1000) + 7)
    B, T, K, H, W = 16500, 4, 6, 6, 6
    env = SokobanBatch(SokobanEnvConfig(dim_x=H, dim_y=W, num_boxes=1, max_steps=12), B, T, K, device)
    assert env.enable_boards()
    env.reset(synthetic.env_seeds(B))
    fixed = env.room_fixed.cpu().numpy().copy()
    state = env.room_state.cpu().numpy().copy()
    player = env.player.cpu().numpy().copy()
    idx = np.nonzero(rng.random(B) < frac_irregular)[0]
    f2, s2, p2 = fixed[idx].copy(), state[idx].copy(), player[idx].copy()
    _irregular_rooms(rng, len(idx), H, W, f2, s2, p2)
    fixed[idx], state[idx], player[idx] = f2, s2, p2
    env.load_state(fixed, state, player)
    nes, bot = np.zeros(B, np.int32), np.zeros(B, np.int32)
    oep = oracle.Episode(B, T)
    bad = np.zeros(B, bool)
    for t in range(T):
        ids = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, -1], size=(B, K),
                         p=[0.05] + [0.11] * 8 + [0.03, 0.04]).astype(np.int8)
        if t == 2:  # a turn on the regular path only: the cached waves step from their entries
            ids = np.clip(ids, 1, 8).astype(np.int8)
        n = rng.integers(0, K + 1, size=B).astype(np.uint8)
        err = torch.zeros(B, dtype=torch.uint8, device=device)
        env.step_turn(t, _t(ids, device), _t(n, device), None, 9, -0.1, err)
        oerr = oracle.sokoban_turn(H, W, 1, 12, fixed, state, player, nes, bot, oep, t, ids, n, None, 9, -0.1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(err.cpu().numpy() != 0, oerr != 0)
        bad |= oerr != 0
        _match(env, oep, fixed, state, player, nes, bot, ~bad)


def test_boards_bench_sequence_equals_uncached(device):
    """The bench's captured rollout (fused first turn = BUILD, plain turns and the fused last
    turn = USE) replayed 3 times in a HIP graph: every arena, the state and the finalize outputs
    == the same rollout without a cache."""
    import bench
    outs = []
    for boards in (False, True):
        R = bench.Rollout(device, 0, boards=boards)
        assert R.boards == boards
        g = torch.cuda.CUDAGraph()
        R.step()
        torch.cuda.synchronize()
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            R.step()
        torch.cuda.current_stream(device).wait_stream(s)
        with torch.cuda.graph(g):
            R.step()
        arenas = []
        for _ in range(3):
            g.replay()
            torch.cuda.synchronize()
            arenas.append(R.env.ep.arena.clone())
        outs.append((arenas, R.env.room_state.clone(), R.env.player.clone(), R.norm.clone(), R.metrics.clone()))
    (a0, s0, p0, n0, m0), (a1, s1, p1, n1, m1) = outs
    for x, y in zip(a0, a1):
        assert torch.equal(x, y)
    assert torch.equal(s0, s1) and torch.equal(p0, p1) and torch.equal(n0, n1)
    # (metrics hold NaN where the reference divides by zero turns: equal NaN positions, equal values)
    torch.testing.assert_close(m0, m1, rtol=0, atol=0, equal_nan=True)
    assert torch.equal(a1[0], a1[2])


def test_boards_refused_where_not_kept(device):
    cfg = SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100)
    small = SokobanBatch(cfg, 4096, 2, 5, device)
    assert not small.enable_boards()  # 4 lanes per env: the cache is not kept there
    env = SokobanBatch(cfg, 8192, 2, 5, device)
    assert env.enable_boards()
    env.reset(synthetic.env_seeds(8192))
    st = env.board_struct(_lib.BOARDS_USE)
    with pytest.raises(NotImplementedError):  # a state writer given the cache
        ops.sokoban_reset(st, env.ep, env.init_state, env.init_player)
    ids = torch.ones(8192, 5, dtype=torch.int8, device=device)
    n = torch.full((8192,), 2, dtype=torch.uint8, device=device)
    turn = ops.turn_struct(0, ids, n, None, 10, -0.1)
    obs = ops.render_buffers(8192, 6, 6, device)
    with pytest.raises(NotImplementedError):  # the render-fused turn keeps no cache
        ops.sokoban_step_turn_render(st, env.ep, turn, ops.render_struct(cfg.grid_lookup, 6, 6, *obs))
    small_st = small.struct()
    small_st.boards, small_st.boards_mode = env.boards.data_ptr(), _lib.BOARDS_BUILD
    with pytest.raises(NotImplementedError):
        ops.sokoban_step_turn(small_st, small.ep, ops.turn_struct(0, ids[:4096], n[:4096], None, 10, -0.1))


def test_boards_invalidate_after_direct_write(device):
    """A caller that rewrites the rooms directly and calls invalidate_boards(): the next turn
    rebuilds the cache from the new rows (== the oracle on the new rooms)."""
    B, T, K = 8192, 3, 5
    cfg = SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100)
    env = SokobanBatch(cfg, B, T, K, device)
    assert env.enable_boards()
    env.reset(synthetic.env_seeds(B))
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=3)
    env.step_turn(0, _t(ids[0], device), _t(n[0], device), None, 10, -0.1)
    other = SokobanBatch(cfg, B, T, K, device)
    other.reset(synthetic.env_seeds(B, first_group=B // 16))  # different rooms
    env.room_fixed.copy_(other.room_fixed)
    env.room_state.copy_(other.room_state)
    env.player.copy_(other.player)
    env.invalidate_boards()
    fixed, state, player = (x.cpu().numpy().copy() for x in (env.room_fixed, env.room_state, env.player))
    nes, bot = env.num_env_steps.cpu().numpy().astype(np.int32), env.boxes_on_target.cpu().numpy().astype(np.int32)
    oep = oracle.Episode(B, T)
    h = _host_ep(env.ep)
    for k in FIELDS:
        getattr(oep, k)[...] = h[k]
    for t in (1, 2):
        env.step_turn(t, _t(ids[t], device), _t(n[t], device), None, 10, -0.1)
        oracle.sokoban_turn(6, 6, 1, 100, fixed, state, player, nes, bot, oep, t, ids[t], n[t], None, 10, -0.1)
        torch.cuda.synchronize()
        _match(env, oep, fixed, state, player, nes, bot)


@pytest.mark.parametrize("frac_irregular", [0.0, 0.02])
def test_boards_first_turn_reads_reset_entries_vs_oracle(device, frac_irregular):
    """The fused first turn (rmi_sokoban_step_turn_first): the first rollout's under BUILD writes
    the reset state's entries (init_boards), the later rollouts' under USE read them instead of
    decoding the reset rows -- with envs left out of turn 0 (their entries are the reset's),
    irregular reset rooms (untagged: their waves decode) and off-path action ids -- == the oracle
    every turn of 3 rollouts."""
    rng = np.random.default_rng(int(frac_irregular * 100) + 3)
    B, T, K, H, W = 8192, 3, 5, 6, 6
    env = SokobanBatch(SokobanEnvConfig(dim_x=H, dim_y=W, num_boxes=1, max_steps=100), B, T, K, device)
    assert env.enable_boards()
    env.reset(synthetic.env_seeds(B))
    fixed0 = env.room_fixed.cpu().numpy().copy()
    state0 = env.room_state.cpu().numpy().copy()
    player0 = env.player.cpu().numpy().copy()
    idx = np.nonzero(rng.random(B) < frac_irregular)[0]
    if len(idx):
        f2, s2, p2 = fixed0[idx].copy(), state0[idx].copy(), player0[idx].copy()
        _irregular_rooms(rng, len(idx), H, W, f2, s2, p2)
        fixed0[idx], state0[idx], player0[idx] = f2, s2, p2
        env.load_state(fixed0, state0, player0)
    assert not env.init_boards_valid
    for rollout in range(3):
        fixed, state, player = fixed0.copy(), state0.copy(), player0.copy()
        nes, bot = np.zeros(B, np.int32), np.zeros(B, np.int32)
        oep = oracle.Episode(B, T)
        bad = np.zeros(B, bool)
        for t in range(T):
            ids = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 9], size=(B, K),
                             p=[0.05] + [0.115] * 8 + [0.03]).astype(np.int8)
            if frac_irregular == 0.0:
                ids = np.clip(ids, 1, 4).astype(np.int8)
            n = rng.integers(0, K + 1, size=B).astype(np.uint8)
            h_in = (rng.random(B) < 0.7).astype(np.uint8) if t == 0 else None
            err = torch.zeros(B, dtype=torch.uint8, device=device)
            if t == 0:
                mode = _lib.BOARDS_USE if env.init_boards_valid else _lib.BOARDS_BUILD
                keep = (_t(ids, device), _t(n, device), _t(h_in, device))  # alive through the launch
                turn = ops.turn_struct(0, *keep, 10, -0.1)
                ops.sokoban_step_turn_first(env.board_struct(mode), env.ep, turn, env.init_state, env.init_player, err)
                env.init_boards_valid = True
                env._boards_valid = True  # the first turn wrote every live env's entry
            else:
                env.step_turn(t, _t(ids, device), _t(n, device), None, 10, -0.1, err)
            oerr = oracle.sokoban_turn(H, W, 1, 100, fixed, state, player, nes, bot, oep, t, ids, n, h_in, 10, -0.1)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(err.cpu().numpy() != 0, oerr != 0)
            bad |= oerr != 0
            _match(env, oep, fixed, state, player, nes, bot, ~bad)
        if rollout == 0:
            ent = env.init_boards.cpu().numpy()
            assert (ent[:, 13] == 1).sum() >= B - len(idx)  # every regular reset room tagged
