"""rmi_sokoban_token_turn: a Sokoban turn from the generations' token ids in ONE launch (decode +
parse, the turn, the render) == rmi_detok_parse followed by the separate turn form (plain, first
fused with the reset, last fused with the finalize) and rmi_sokoban_render, bit for bit: the
decoded text and its lengths, the decode / parse error bytes, actions, n_actions, spans, the
state and the whole episode record, the turn's error bytes, every observation row and length,
and the finalize's outputs.  Covered: the three turn forms over a 5-turn rollout, partial
has_input masks, batches that end inside a workgroup, waves on the exact path with absent and
4-byte glyphs, finalize groups of 4 and 16 (fused) and 32 (the two-call form), and room layouts
the fused launch does not take (a u64 board window, 8x8 rooms), which run the two calls; and the
turn-inputs form the turn chain takes (has set: rmi_turn_inputs between the decode and the turn,
decode errors, a partial has_t), fused and through the separate launches.  And the token turn
straight against the oracle: the host decode + `_parse_response` + action mapping
(oracle/parse.py), oracle.sokoban_turn, oracle.sokoban_render and the finalize's metrics and
normalised scores (test_token_turn_against_oracle)."""
import numpy as np
import pytest
import torch

import oracle
from oracle import parse as oparse
from ragen_amd import ops, synthetic
from test_gpu_fused_render import LK_WIDE, _pair, _rows_equal, _state_equal
from test_gpu_parity import _host_ep

pytestmark = pytest.mark.gpu

NAMES = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}


def _tokens(device, B, T, K, seed):
    """Per-turn response token ids (the synthetic responses over the byte vocabulary, with some
    rows' answers cut so the parse fails), the parse config, the vocabulary and the row stride."""
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=seed)
    table, skip = synthetic.byte_vocab()
    vt = ops.VocabTable.from_bytes(table, skip, device)
    rng = np.random.default_rng(seed)
    toks, stride = [], 0
    for t in range(T):
        texts = synthetic.responses_for_actions(ids[t], n[t], NAMES, seed=seed + t)
        for i in rng.choice(B, size=B // 50, replace=False):  # no </answer>: the parse finds nothing
            texts[i] = texts[i].replace("</answer>", "")
        toks.append(torch.from_numpy(synthetic.tokenize_greedy(texts, table)).to(device))
        stride = max(stride, max(len(x.encode()) for x in texts))
    return ops.parse_config(True, K, "||", NAMES), vt, toks, (stride + 16 + 3) // 4 * 4


def _dirty(o):
    for v in o.values():
        if v is not None:
            v.fill_(0x5A if v.dtype in (torch.uint8, torch.int8) else 7)


def _run(device, B, H, W, nb, seed, T=5, gs=16, irregular=0, lk=None, has_every=0):
    (a, b), rng = _pair(device, B, H, W, nb, seed=seed, lk=lk, irregular=irregular)
    K = 5
    cfg, vt, toks, stride = _tokens(device, B, T, K, seed)
    glk = a.config.grid_lookup
    fin_out = []
    for _ in range(2):
        norm = torch.empty(B, dtype=torch.float32, device=device)
        met = torch.empty(B, 4, dtype=torch.float64, device=device)
        fin_out.append((norm, met, ops.finalize_struct(gs, "mean_std", norm, met)))
    for t in range(T):
        has = None
        if has_every and t % has_every == 1:
            has = torch.from_numpy((rng.random(B) < 0.7).astype(np.uint8)).to(device)
        # a: the token turn, into dirtied buffers
        oa = ops.detok_parse(toks[t], vt, stride, cfg)
        torch.cuda.synchronize()
        _dirty(oa)
        tok = ops.token_rows_struct(toks[t], vt, cfg, oa)
        tsa = ops.turn_struct(t, oa["actions"], oa["n_actions"], has, 10, -0.1)
        obs_a = ops.render_buffers(B, H, W, device)
        ra = ops.render_struct(glk, H, W, *obs_a)
        ea = torch.zeros(B, dtype=torch.uint8, device=device)
        kw = {}
        if t == 0:
            kw = {"init_state": a.init_state, "init_player": a.init_player}
        elif t == T - 1:
            kw = {"fin": fin_out[0][2]}
        ops.sokoban_token_turn(tok, a.struct(), a.ep, tsa, ra, err=ea, **kw)
        # b: the decode + parse launch, the turn form, the render
        ob = ops.detok_parse(toks[t], vt, stride, cfg)
        tsb = ops.turn_struct(t, ob["actions"], ob["n_actions"], has, 10, -0.1)
        eb = torch.zeros(B, dtype=torch.uint8, device=device)
        if t == 0:
            ops.sokoban_step_turn_first(b.struct(), b.ep, tsb, b.init_state, b.init_player, eb)
        elif t == T - 1:
            ops.sokoban_step_turn_finalize(b.struct(), b.ep, tsb, fin_out[1][2], eb)
        else:
            ops.sokoban_step_turn(b.struct(), b.ep, tsb, eb)
        rb = ops.sokoban_render(b.struct(), B, glk, device)
        torch.cuda.synchronize()
        for k in ("text_len", "decode_err", "actions", "n_actions", "spans", "err"):
            assert torch.equal(oa[k], ob[k]), (t, k)
        tl = ob["text_len"].cpu().numpy()
        ta, tb = oa["text"].cpu().numpy(), ob["text"].cpu().numpy()
        for i in range(B):
            w = (int(tl[i]) + 3) // 4 * 4
            assert ta[i, :w].tobytes() == tb[i, :w].tobytes(), (t, i)
        assert torch.equal(ea, eb), t
        _state_equal(a, b, t)
        _rows_equal(obs_a, rb)
    for x, y in zip(fin_out[0][:2], fin_out[1][:2]):  # norm, metrics (NaN where no action ran)
        torch.testing.assert_close(x, y, rtol=0, atol=0, equal_nan=True)
    return a


@pytest.mark.parametrize("B,has_every,gs", [(8192, 0, 16), (8192, 2, 16), (1000, 0, 8)])
def test_token_turn_equals_detok_parse_turn_render(device, B, has_every, gs):
    """(1000 envs: the last workgroup holds 8; finalize groups of 8.)"""
    a = _run(device, B, 6, 6, 1, seed=B + has_every, gs=gs, has_every=has_every)
    assert int(a.ep.turn_exec.sum().item()) > 0


def test_token_turn_exact_path_and_wide_glyphs(device):
    _run(device, 4096, 6, 6, 1, seed=3, irregular=100, lk=LK_WIDE)


@pytest.mark.parametrize("gs", [4, 32])
def test_token_turn_finalize_groups(device, gs):
    """Groups of 4 finalize inside the fused launch; groups of 32 do not fit its 16 envs and take
    the two calls (the finalize fused into the turn launch)."""
    _run(device, 2048, 6, 6, 1, seed=gs, T=3, gs=gs)


@pytest.mark.parametrize("H,W,nb", [(12, 3, 1), (8, 8, 2)])
def test_token_turn_other_layouts(device, H, W, nb):
    """Layouts outside the fused launch (a u64 board window; 64-cell rooms) run the two calls."""
    _run(device, 2048, H, W, nb, seed=H * W, T=3)


def test_token_turn_validation(device):
    B = 64
    (a, _), _ = _pair(device, B, 6, 6, 1, seed=1)
    cfg, vt, toks, stride = _tokens(device, B, 1, 5, 1)
    o = ops.detok_parse(toks[0], vt, stride, cfg)
    tok = ops.token_rows_struct(toks[0], vt, cfg, o)
    ts = ops.turn_struct(0, o["actions"][:, :4].contiguous(), o["n_actions"], None, 10, -0.1)  # K mismatch
    obs = ops.render_buffers(B, 6, 6, device)
    r = ops.render_struct(a.config.grid_lookup, 6, 6, *obs)
    with pytest.raises(ValueError):
        ops.sokoban_token_turn(tok, a.struct(), a.ep, ts, r)
    ts = ops.turn_struct(0, o["actions"], o["n_actions"], None, 10, -0.1)
    fin = ops.finalize_struct(16, "mean", torch.empty(B, dtype=torch.float32, device=device))
    with pytest.raises(ValueError):  # first and last form together
        ops.sokoban_token_turn(tok, a.struct(), a.ep, ts, r, fin=fin, init_state=a.init_state,
                               init_player=a.init_player)


@pytest.mark.parametrize("pad", [0, 600])
def test_token_turn_with_turn_inputs(device, pad):
    """has set (the turn chain's steps 2-4 in one call): == rmi_detok_parse, rmi_turn_inputs, then
    the turn with the render; rows with out-of-range ids (decode errors: those envs do not step)
    and a partial has_t.  pad widens the rows past the fused launch's LDS, so the call runs the
    separate launches itself."""
    B = 4096
    (a, b), rng = _pair(device, B, 6, 6, 1, seed=21 + pad)
    cfg, vt, toks, stride = _tokens(device, B, 2, 5, 21)
    stride += pad
    glk = a.config.grid_lookup
    for t in range(2):
        tk = toks[t].clone()
        tk[::37, 3] = 10 ** 9  # an id outside the vocabulary: RMI_ERR_INDEX in the decode
        has_t = torch.from_numpy((rng.random(B) < 0.8).astype(np.uint8)).to(device)
        kw_a = {"init_state": a.init_state, "init_player": a.init_player} if t == 0 else {}
        kw_b = {"init_state": b.init_state, "init_player": b.init_player} if t == 0 else {}
        oa = ops.detok_parse(tk, vt, stride, cfg)
        torch.cuda.synchronize()
        _dirty(oa)
        tok = ops.token_rows_struct(tk, vt, cfg, oa)
        has_a = torch.full((B,), 7, dtype=torch.uint8, device=device)
        tok.has_t, tok.has = has_t.data_ptr(), has_a.data_ptr()
        ea = torch.full((B,), 0x55, dtype=torch.uint8, device=device)  # zeroed by the turn inputs
        tsa = ops.turn_struct(t, oa["actions"], oa["n_actions"], has_a, 10, -0.1)
        obs_a = ops.render_buffers(B, 6, 6, device)
        ops.sokoban_token_turn(tok, a.struct(), a.ep, tsa, ops.render_struct(glk, 6, 6, *obs_a), err=ea, **kw_a)
        ob = ops.detok_parse(tk, vt, stride, cfg)
        has_b = torch.empty(B, dtype=torch.uint8, device=device)
        eb = torch.full((B,), 0x55, dtype=torch.uint8, device=device)
        ops.turn_inputs(has_t, ob["decode_err"], has_b, eb)
        tsb = ops.turn_struct(t, ob["actions"], ob["n_actions"], has_b, 10, -0.1)
        obs_b = ops.render_buffers(B, 6, 6, device)
        ops.sokoban_step_turn_render(b.struct(), b.ep, tsb, ops.render_struct(glk, 6, 6, *obs_b), err=eb, **kw_b)
        torch.cuda.synchronize()
        assert int(ob["decode_err"].ne(0).sum()) > 0 and int(has_b.eq(0).sum()) > 0
        for k in ("text_len", "decode_err", "actions", "n_actions", "spans", "err"):
            assert torch.equal(oa[k], ob[k]), (t, k)
        assert torch.equal(has_a, has_b) and torch.equal(ea, eb), t
        _state_equal(a, b, t)
        _rows_equal(obs_a, obs_b)


@pytest.mark.parametrize("has_every", [0, 2])
def test_token_turn_against_oracle(device, has_every):
    """The fused token turn against the oracle, not against the separate launches: every turn's
    token rows are decoded on the host (oracle.parse.detokenize over the byte vocabulary), given
    back their '<think>' prefix and parsed by the reference's `_parse_response` restatement with
    its action mapping (unknown names -> id 0); oracle.sokoban_turn steps the same rooms with
    those actions (first turn fused with the reset, plain turns, the last fused with the
    finalize), and each turn's observation rows equal oracle.sokoban_render of the oracle's state;
    the finalize's metrics and normalised scores equal oracle.rollout_metrics and
    oracle.group_normalize of the oracle's trajectory scores."""
    B, T, K, gs = 2048, 4, 5, 16
    (a, _), rng = _pair(device, B, 6, 6, 1, seed=77 + has_every)
    cfg, vt, toks, stride = _tokens(device, B, T, K, 77 + has_every)
    table, skip = synthetic.byte_vocab()
    glk = a.config.grid_lookup
    fixed = a.room_fixed.cpu().numpy().copy()
    state = a.init_state.cpu().numpy().copy()
    player = a.init_player.cpu().numpy().copy()
    nes, bot = np.zeros(B, np.int32), np.zeros(B, np.int32)
    oep = oracle.Episode(B, a.ep.T)  # (the record holds 6 turns; T of them run)
    norm = torch.empty(B, dtype=torch.float32, device=device)
    met = torch.empty(B, 4, dtype=torch.float64, device=device)
    fin = ops.finalize_struct(gs, "mean_std", norm, met)
    stepped = 0
    for t in range(T):
        has = None
        if has_every and t % has_every == 1:
            has = (rng.random(B) < 0.7).astype(np.uint8)
        # the oracle's actions: host decode, the reference's parse and action mapping
        rows = toks[t].cpu().numpy()
        ids = np.zeros((B, K), np.int8)
        n = np.zeros(B, np.uint8)
        for i in range(B):
            text = oparse.prefixed(oparse.detokenize(rows[i].tolist(), table, skip), True)
            _, acts = oparse.parse_response(text, True, K, "||")
            aid = oparse.action_ids(acts, NAMES)
            ids[i, :len(aid)] = aid
            n[i] = len(aid)
        # the token turn
        o = ops.detok_parse(toks[t], vt, stride, cfg)
        tok = ops.token_rows_struct(toks[t], vt, cfg, o)
        ts = ops.turn_struct(t, o["actions"], o["n_actions"], None if has is None else torch.from_numpy(has).to(device),
                             10, -0.1)
        obs = ops.render_buffers(B, 6, 6, device)
        kw = {}
        if t == 0:
            kw = {"init_state": a.init_state, "init_player": a.init_player}
        elif t == T - 1:
            kw = {"fin": fin}
        ops.sokoban_token_turn(tok, a.struct(), a.ep, ts, ops.render_struct(glk, 6, 6, *obs), **kw)
        oracle.sokoban_turn(6, 6, 1, 100, fixed, state, player, nes, bot, oep, t, ids, n, has, 10, -0.1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(o["n_actions"].cpu().numpy(), n)
        np.testing.assert_array_equal(o["actions"].cpu().numpy(), ids)
        np.testing.assert_array_equal(a.room_state.cpu().numpy(), state)
        np.testing.assert_array_equal(a.player.cpu().numpy(), player)
        h = _host_ep(a.ep)
        for k in ("num_actions", "flags", "n_turns", "penalty", "turn_reward", "turn_info", "turn_exec"):
            np.testing.assert_array_equal(h[k], getattr(oep, k), err_msg=f"turn {t}: {k}")
        want = [oracle.sokoban_render(state[i], fixed[i], 6, 6, glk) for i in range(B)]
        assert ops.decode_rows(*obs) == want, t
        stepped += int(oep.turn_exec[t].sum())
    assert stepped > B and (n == 0).any()
    np.testing.assert_array_equal(met.cpu().numpy(), oracle.rollout_metrics(oep))
    sc, pen = oracle.trajectory_scores(oep)
    want_norm = oracle.group_normalize(sc, pen, np.arange(0, B + 1, gs, dtype=np.int32), "mean_std")
    np.testing.assert_allclose(norm.cpu().numpy(), want_norm, rtol=0, atol=1e-5)
