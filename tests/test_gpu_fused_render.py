"""rmi_sokoban_step_turn_render: the turn and the next observation in one launch == the turn
launch followed by rmi_sokoban_render, bit for bit (state, episode record, error bytes, every
row's bytes and length), and the rows == the oracle's render of the state after the turn
(sokoban/env.py:53-61).  Covered: the three turn forms (plain, first fused with the reset, last
fused with the finalize), the u32 and u64 board windows of 36-cell rooms, 8x8 rooms, waves on
the exact path (irregular rooms, unknown codes), partial has_input masks, done envs, a glyph
table with absent and 4-byte glyphs, and the two-launch form of small batches."""
import numpy as np
import pytest
import torch

import oracle
from ragen_amd import ops, synthetic
from ragen_amd.env import SokobanBatch
from ragen_amd.env.configs import SokobanEnvConfig

pytestmark = pytest.mark.gpu

LK_WIDE = {0: "#", 1: "_", 2: "O", 3: "√", 4: "X", 5: "\U0001F600", 6: "S"}  # code 7+: absent -> '?'


def regular_rooms(rng, B, H, W, n_boxes):
    """Random regular rooms (border wall, interior floor / targets, boxes, one player)."""
    fixed = np.zeros((B, H, W), np.uint8)
    fixed[:, 1:H - 1, 1:W - 1] = 1
    inner = [(r, c) for r in range(1, H - 1) for c in range(1, W - 1)]
    state = fixed.copy()
    player = np.zeros((B, 2), np.int8)
    for b in range(B):
        cells = rng.permutation(len(inner))
        tg = [inner[i] for i in cells[:n_boxes]]
        bx = [inner[i] for i in cells[n_boxes:2 * n_boxes]]
        if rng.random() < 0.3:  # some boxes already on their targets
            bx[0] = tg[0]
        pl = inner[cells[2 * n_boxes]]
        for r, c in tg:
            fixed[b, r, c] = 2
        state[b] = fixed[b]
        for r, c in bx:
            state[b, r, c] = 3 if fixed[b, r, c] == 2 else 4
        state[b, pl[0], pl[1]] = 5
        player[b] = pl
    return fixed.reshape(B, -1), state.reshape(B, -1), player


def _pair(device, B, H, W, n_boxes, seed, lk=None, irregular=0):
    rng = np.random.default_rng(seed)
    cfg = SokobanEnvConfig(dim_x=H, dim_y=W, num_boxes=n_boxes, max_steps=100)
    if lk is not None:
        cfg.grid_lookup = lk
    fixed, state, player = regular_rooms(rng, B, H, W, n_boxes)
    if irregular:  # hand-made rooms: unknown codes, players anywhere (the exact path)
        state[:irregular] = rng.integers(0, 20, size=(irregular, H * W))
        fixed[:irregular] = rng.integers(0, 3, size=(irregular, H * W))
    envs = []
    for _ in range(2):
        e = SokobanBatch(cfg, B, 6, 5, device)
        e.load_state(fixed, state, player)
        envs.append(e)
    return envs, rng


def _rows_equal(a, b):
    (ra, na), (rb, nb) = a, b
    na_h, nb_h = na.cpu().numpy(), nb.cpu().numpy()
    np.testing.assert_array_equal(na_h, nb_h)
    ra_h, rb_h = ra.cpu().numpy(), rb.cpu().numpy()
    for i in range(len(na_h)):
        w = (int(na_h[i]) + 3) // 4 * 4  # the bytes written, the last dword's zero tail included
        assert ra_h[i, :w].tobytes() == rb_h[i, :w].tobytes(), i


def _state_equal(a, b, t=None):
    for k in ("room_state", "player", "num_env_steps", "boxes_on_target"):
        x, y = getattr(a, k), getattr(b, k)
        if not torch.equal(x, y):
            bad = (x != y).reshape(x.shape[0], -1).any(1).nonzero().flatten().cpu().tolist()
            raise AssertionError(f"turn {t}: {k} differs in {len(bad)} envs, first {bad[:8]}: "
                                 f"{x[bad[0]].cpu().tolist()} vs {y[bad[0]].cpu().tolist()}")
    for k in ("num_actions", "flags", "n_turns", "penalty", "turn_reward", "turn_info", "turn_exec"):
        assert torch.equal(getattr(a.ep, k), getattr(b.ep, k)), (t, k)


def _oracle_rows(env, rows, lk):
    st, fx = env.room_state.cpu().numpy(), env.room_fixed.cpu().numpy()
    out, n = rows
    got = ops.decode_rows(out, n)
    want = [oracle.sokoban_render(st[i], fx[i], env.H, env.W, lk) for i in range(env.B)]
    assert got == want


@pytest.mark.parametrize("B,H,W,nb,irregular,lk", [
    (8192, 6, 6, 1, 0, None),
    (8192, 12, 3, 1, 0, None),          # 36 cells, board window past 32 bits (u64)
    (6000, 8, 8, 2, 0, LK_WIDE),        # 64 cells, 4-byte and absent glyphs
    (8192, 6, 6, 1, 100, LK_WIDE),      # exact-path waves, unknown codes
    (1000, 6, 6, 1, 0, None),           # small batch: the turn and the render as two launches
])
def test_turn_render_equals_turn_then_render(device, B, H, W, nb, irregular, lk):
    (a, b), rng = _pair(device, B, H, W, nb, seed=B + H * 10 + W, lk=lk, irregular=irregular)
    T, K = 6, 5
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=B)
    for t in range(T):
        act, na = torch.from_numpy(ids[t]).to(device), torch.from_numpy(n[t]).to(device)
        has = None
        if t % 2 == 1:  # a partial input mask
            has = torch.from_numpy((rng.random(B) < 0.7).astype(np.uint8)).to(device)
        ea = torch.zeros(B, dtype=torch.uint8, device=device)
        eb = torch.zeros(B, dtype=torch.uint8, device=device)
        a.step_turn(t, act, na, has, 10, -0.1, ea, render=True)
        ra = a.render_rows()
        b.step_turn(t, act, na, has, 10, -0.1, eb)
        rb = b.render_rows()
        torch.cuda.synchronize()
        assert ra is a._rows  # the fused rows, no second launch
        assert torch.equal(ea, eb)
        _state_equal(a, b)
        _rows_equal(ra, rb)
        _oracle_rows(a, ra, a.config.grid_lookup)


@pytest.mark.parametrize("B", [8192, 2048])
def test_first_and_last_turn_forms(device, B):
    """The first turn fused with the reset, and the last fused with the finalize, each with the
    render in the same launch == the fused turn form then rmi_sokoban_render."""
    (a, b), _ = _pair(device, B, 6, 6, 1, seed=7)
    T, K = 3, 5
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=3)
    lk = a.config.grid_lookup
    fin_out = []
    for e in (a, b):
        norm = torch.empty(B, dtype=torch.float32, device=device)
        met = torch.empty(B, 4, dtype=torch.float64, device=device)
        fin_out.append((norm, met, ops.finalize_struct(16, "mean_std", norm, met)))
    for t in range(T):
        act, na = torch.from_numpy(ids[t]).to(device), torch.from_numpy(n[t]).to(device)  # (alive: ts points at them)
        ts = ops.turn_struct(t, act, na, None, 10, -0.1)
        obs = ops.render_buffers(B, 6, 6, device)
        r = ops.render_struct(lk, 6, 6, *obs)
        kw = {}
        if t == 0:
            kw = {"init_state": a.init_state, "init_player": a.init_player}
        elif t == T - 1:
            kw = {"fin": fin_out[0][2]}
        ops.sokoban_step_turn_render(a.struct(), a.ep, ts, r, **kw)
        if t == 0:
            ops.sokoban_step_turn_first(b.struct(), b.ep, ts, b.init_state, b.init_player)
        elif t == T - 1:
            ops.sokoban_step_turn_finalize(b.struct(), b.ep, ts, fin_out[1][2])
        else:
            ops.sokoban_step_turn(b.struct(), b.ep, ts)
        rb = ops.sokoban_render(b.struct(), B, lk, device)
        torch.cuda.synchronize()
        _state_equal(a, b, t)
        _rows_equal(obs, rb)
    for x, y in zip(fin_out[0][:2], fin_out[1][:2]):  # norm, metrics (NaN where no action ran)
        torch.testing.assert_close(x, y, rtol=0, atol=0, equal_nan=True)


@pytest.mark.parametrize("B", [8192, 65536])
def test_first_form_helper_waves_leave_other_envs_alone(device, B):
    """Pins round 4's room_state divergence of the fused first form: the render
    helper waves of a workgroup (kObsFan - 1 per turn wave) must map to no env.  When they took
    an env index from their wave number they indexed envs of the NEXT workgroups, skipped the
    turn (not a turn wave) but still ran the reset-row store of the first form, rewriting those
    envs' rows with their init rows after their own workgroup had stepped them: only room_state,
    only the first form, and only where several workgroups run -- timing-dependent, so the launch
    is repeated at two grid sizes."""
    (a, b), _ = _pair(device, B, 6, 6, 1, seed=11)
    ids, n = synthetic.rollout_actions(B, 1, 5, 1, 4, seed=5)
    act, na = torch.from_numpy(ids[0]).to(device), torch.from_numpy(n[0]).to(device)
    ts = ops.turn_struct(0, act, na, None, 10, -0.1)
    ops.sokoban_step_turn_first(b.struct(), b.ep, ts, b.init_state, b.init_player)
    torch.cuda.synchronize()
    assert not torch.equal(b.room_state, b.init_state)  # envs moved: a reset store would show
    lk = a.config.grid_lookup
    for rep in range(6):
        obs = ops.render_buffers(B, 6, 6, device)
        r = ops.render_struct(lk, 6, 6, *obs)
        ops.sokoban_step_turn_render(a.struct(), a.ep, ts, r, init_state=a.init_state, init_player=a.init_player)
        torch.cuda.synchronize()
        _state_equal(a, b, rep)


def test_render_entry_validation(device):
    """Argument errors as the separate entry points report them."""
    B = 8192
    (a, _), _ = _pair(device, B, 6, 6, 1, seed=1)
    ids, n = synthetic.rollout_actions(B, 1, 5, 1, 4, seed=1)
    act, na = torch.from_numpy(ids[0]).to(device), torch.from_numpy(n[0]).to(device)
    ts = ops.turn_struct(0, act, na, None, 10, -0.1)
    out, ln = ops.render_buffers(B, 6, 6, device)
    r = ops.render_struct(a.config.grid_lookup, 6, 6, out, ln)
    r.stride = 8  # below H*W*4 + H - 1
    with pytest.raises(ValueError):
        ops.sokoban_step_turn_render(a.struct(), a.ep, ts, r)
    r = ops.render_struct(a.config.grid_lookup, 6, 6, out, ln)
    fin = ops.finalize_struct(16, "mean", torch.empty(B, dtype=torch.float32, device=device))
    with pytest.raises(ValueError):  # first and last form together
        ops.sokoban_step_turn_render(a.struct(), a.ep, ts, r, fin=fin, init_state=a.init_state,
                                     init_player=a.init_player)
