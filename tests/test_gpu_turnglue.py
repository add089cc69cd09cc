"""The turn loop's reductions (csrc/turnglue.hip) against torch: rmi_turn_readback (flags copy,
actions left, the packed readback with the longest text / observation) and rmi_next_rows_stats
(longest next row, any pending host row, count) — the eight-envs-per-thread form (B % 8 == 0,
aligned arrays) and the scalar form (ragged B, or arrays at odd offsets), optional inputs absent."""
import numpy as np
import pytest
import torch

from ragen_amd import _lib, ops

pytestmark = pytest.mark.gpu


def _arrays(B, device, off, g):
    def u8(hi):
        return torch.randint(0, hi, (B + off,), generator=g, dtype=torch.int32).to(torch.uint8).to(device)[off:]

    def i32(hi):
        return torch.randint(0, hi, (B + off,), generator=g, dtype=torch.int32).to(device)[off:]
    return u8, i32


@pytest.mark.parametrize("B,off", [(8192, 0), (1000, 0), (8, 0), (4096, 1), (24, 3)])
def test_turn_readback_and_next_rows_stats(device, B, off):
    g = torch.Generator(device="cpu").manual_seed(B + off)
    u8, i32 = _arrays(B, device, off, g)
    flags, err, dec_err, num_actions = u8(8), u8(3), u8(2), u8(20)
    max_actions, text_len, obs_len = i32(40) + 10, i32(5000), i32(90)
    for tl, ol in ((text_len, obs_len), (None, None)):
        flags_copy = torch.empty(B, dtype=torch.uint8, device=device)
        left = torch.empty(B, dtype=torch.int32, device=device)
        pack = torch.full((ops.readback_bytes(B),), 0xAB, dtype=torch.uint8, device=device)
        ops.turn_readback(flags, err, dec_err, num_actions, max_actions, tl, ol, flags_copy, left, pack)
        assert torch.equal(flags_copy, flags)
        assert torch.equal(left, max_actions - num_actions.to(torch.int32))
        h = pack.cpu().numpy()
        assert (h[:B] == flags.cpu().numpy()).all() and (h[B:2 * B] == err.cpu().numpy()).all()
        assert (h[2 * B:3 * B] == dec_err.cpu().numpy()).all()
        o = (3 * B + 3) & ~3
        tail = h[o:o + 8].view(np.int32)
        assert tail[0] == (int(tl.max()) if tl is not None else 0) and tail[1] == (int(ol.max()) if ol is not None else 0)
    length, has, bad = i32(3000), u8(2), u8(2)
    for hs, bd in ((has, bad), (None, None)):
        stats = torch.empty(3, dtype=torch.int32, device=device)
        ops.next_rows_stats(length, hs, flags, bd, stats)
        nxt = ((flags & _lib.FLAG_DONE) == 0) & ((hs != 0) if hs is not None else True)
        want = [int(length[nxt].max()) if bool(nxt.any()) else 0, int(bool((bd != 0).any())) if bd is not None else 0,
                int(nxt.sum())]
        assert stats.cpu().tolist() == want


@pytest.mark.parametrize("B", [8192, 1000, 1])
def test_prompt_commit_stats_equals_the_two_launches(device, B):
    """rmi_prompt_commit_stats == rmi_prompt_commit then rmi_next_rows_stats over its bad rows."""
    g = torch.Generator(device="cpu").manual_seed(B)
    u8, i32 = _arrays(B, device, 0, g)
    bpe_err, text_err, active, flags, has = u8(2), u8(2), u8(2), u8(8), u8(2)
    mark, length = i32(900), i32(3000)
    for act, mk, hs in ((active, mark, has), (None, None, None)):
        want_upd, got_upd = (i32(50) for _ in range(2))
        got_upd.copy_(want_upd)
        want_bad, got_bad = (torch.empty(B, dtype=torch.uint8, device=device) for _ in range(2))
        want_st, got_st = (torch.empty(3, dtype=torch.int32, device=device) for _ in range(2))
        ops.prompt_commit(bpe_err, text_err, act, mk, want_upd, want_bad)
        ops.next_rows_stats(length, hs, flags, want_bad, want_st)
        ops.prompt_commit_stats(bpe_err, text_err, act, mk, got_upd, got_bad, length, hs, flags, got_st)
        assert torch.equal(got_bad, want_bad) and torch.equal(got_upd, want_upd)
        assert got_st.cpu().tolist() == want_st.cpu().tolist()


@pytest.mark.parametrize("n", [8192, 1000, 3, 1])
def test_count_nonzero_into_the_readback(device, n):
    """The generation batch's flagged-row count (ops.count_nonzero_into -> readback_pad slot)."""
    g = torch.Generator(device="cpu").manual_seed(n)
    x = (torch.rand(n, generator=g) < 0.01).to(torch.uint8) * torch.randint(1, 256, (n,), generator=g).to(torch.uint8)
    x = x.to(device)
    pack = torch.full((ops.readback_bytes(64),), 0xAB, dtype=torch.uint8, device=device)
    slot = ops.readback_pad(pack, 64)
    ops.count_nonzero_into(x, slot)
    assert int(slot.item()) == int((x != 0).sum())
    h = pack.cpu().numpy()
    o = ((3 * 64 + 3) & ~3) + 24
    assert (np.delete(h, np.arange(o, o + 4)) == 0xAB).all()  # nothing else of the pack written


@pytest.mark.parametrize("B,off", [(8192, 0), (1000, 0), (4096, 1), (24, 3)])
def test_turn_readback_pad_summary(device, B, off):
    """rmi_turn_readback_pad: rmi_turn_readback's pack plus the tail's pad count, the OR of the
    step / decode error bytes and the done count (the chain's host reads these instead of
    scanning the arrays)."""
    g = torch.Generator(device="cpu").manual_seed(7 * B + off)
    u8, i32 = _arrays(B, device, off, g)
    flags, num_actions = u8(8), u8(20)
    max_actions, text_len, obs_len = i32(40) + 10, i32(5000), i32(90)
    zero = torch.zeros(B, dtype=torch.uint8, device=device)
    for err, dec_err, pad in ((u8(3), u8(2), u8(2)), (zero, zero, None), (zero, u8(9), zero[:5])):
        flags_copy = torch.empty(B, dtype=torch.uint8, device=device)
        left = torch.empty(B, dtype=torch.int32, device=device)
        pack = torch.full((ops.readback_bytes(B),), 0xAB, dtype=torch.uint8, device=device)
        p = ops._ptr
        _call("rmi_turn_readback_pad", p(flags), p(err), p(dec_err), p(num_actions), p(max_actions), p(text_len),
              p(obs_len), B, p(flags_copy), p(left), p(pack), p(pad), 0 if pad is None else pad.numel(),
              ops._stream(device))
        h = pack.cpu().numpy()
        o = (3 * B + 3) & ~3
        tail = h[o:o + 36].view(np.int32)
        assert (h[:B] == flags.cpu().numpy()).all() and (h[2 * B:3 * B] == dec_err.cpu().numpy()).all()
        assert tail[0] == int(text_len.max()) and tail[1] == int(obs_len.max())
        assert tail[6] == (0 if pad is None else int((pad != 0).sum()))
        e_or = int(np.bitwise_or.reduce(err.cpu().numpy()))
        d_or = int(np.bitwise_or.reduce(dec_err.cpu().numpy()))
        assert ops.readback_summary(tail) == (e_or, d_or, int(((flags & _lib.FLAG_DONE) != 0).sum()))
        assert (h[o + 8:o + 24] == 0xAB).all()  # the stats and raw slots are other writers'


def _call(name, *args):
    from ragen_amd import _lib
    ops.check(getattr(_lib.lib(), name)(*args), name)


@pytest.mark.parametrize("B", [8192, 20000, 1000, 1])
def test_next_rows_list(device, B):
    """rmi_next_rows_list: the envs with has and not done, ascending, and every env's index in
    that list (-1: not in it) == numpy."""
    g = torch.Generator(device="cpu").manual_seed(B)
    u8, _ = _arrays(B, device, 0, g)
    has, flags = u8(2), u8(8)
    for hs in (has, None):
        rows = torch.full((B,), -7, dtype=torch.int64, device=device)
        src = torch.full((B,), -7, dtype=torch.int64, device=device)
        _call("rmi_next_rows_list", ops._ptr(hs), flags.data_ptr(), B, rows.data_ptr(), src.data_ptr(),
              ops._stream(device))
        h = np.ones(B, bool) if hs is None else hs.cpu().numpy() != 0
        nxt = h & ((flags.cpu().numpy() & _lib.FLAG_DONE) == 0)
        want = np.nonzero(nxt)[0]
        r = rows.cpu().numpy()
        assert np.array_equal(r[:len(want)], want) and (r[len(want):] == -7).all()
        w_src = np.full(B, -1, np.int64)
        w_src[want] = np.arange(len(want))
        assert np.array_equal(src.cpu().numpy(), w_src)


@pytest.mark.parametrize("B", [8192, 1000, 3])
def test_formulate_stats_and_tail(device, B):
    g = torch.Generator(device="cpu").manual_seed(B)
    u8, i32 = _arrays(B, device, 0, g)
    length, bad, n_turns = i32(3000), u8(2), u8(6)
    n_sc = torch.empty(B, dtype=torch.int32, device=device)
    stats = torch.empty(3, dtype=torch.int32, device=device)
    for bd in (bad, None):
        _call("rmi_formulate_stats", length.data_ptr(), ops._ptr(bd), n_turns.data_ptr(), B, n_sc.data_ptr(),
              stats.data_ptr(), ops._stream(device))
        want = [int(length.max()), int(bool((bd != 0).any())) if bd is not None else 0, int(n_turns.max())]
        assert stats.cpu().tolist() == want
        assert torch.equal(n_sc, n_turns.to(torch.int32))
    counts, err = i32(1500), u8(5) * (u8(2) != 0).to(torch.uint8)
    out = torch.empty(2, dtype=torch.int64, device=device)
    _call("rmi_formulate_tail", counts.data_ptr(), err.data_ptr(), B, out.data_ptr(), ops._stream(device))
    bits = 0
    for x in err.cpu().tolist():
        bits |= x
    assert out.cpu().tolist() == [int(counts.to(torch.int64).sum()), bits]


def test_assemble_rows_ex_counts_and_normalised_score(device):
    """rmi_assemble_rows_ex == rmi_assemble_rows, plus the response_mask row counts and the
    last score column replaced by the given scores."""
    g = torch.Generator(device="cpu").manual_seed(0)
    B, cap = 700, 900
    im_start = 151644
    tokens = torch.randint(100, 1000, (B, cap), generator=g)
    tokens[torch.rand(B, cap, generator=g) < 0.05] = im_start
    tokens = tokens.to(device)
    row_len = torch.randint(1, cap, (B,), generator=g, dtype=torch.int32).to(device)
    start = (torch.arange(B, dtype=torch.int64) * cap).to(device)
    S = int(row_len.max())
    T = 4
    scores = torch.randn(T, B, generator=g, dtype=torch.float64).to(device)
    n_sc = torch.randint(0, T + 1, (B,), generator=g, dtype=torch.int32).to(device)
    last = torch.randn(B, generator=g).to(device)
    flags = _lib.MS_RESPONSE_MASK | _lib.MS_ROLL
    outs = []
    for ex in (False, True):
        ids, am, pos = (torch.empty(B, S, dtype=torch.int64, device=device) for _ in range(3))
        sc = torch.empty(B, S - 1, dtype=torch.float32, device=device)
        lm, rm = (torch.empty(B, S - 1, dtype=torch.uint8, device=device) for _ in range(2))
        err = torch.empty(B, dtype=torch.uint8, device=device)
        cnt = torch.empty(B, dtype=torch.int32, device=device)
        common = (tokens.data_ptr(), start.data_ptr(), row_len.data_ptr(), B, S, 151643, im_start, 151645,
                  scores.data_ptr(), n_sc.data_ptr(), T, T, flags)
        tail = (ids.data_ptr(), am.data_ptr(), pos.data_ptr(), sc.data_ptr(), lm.data_ptr(), rm.data_ptr())
        if ex:
            _call("rmi_assemble_rows_ex", *common, last.data_ptr(), *tail, cnt.data_ptr(), err.data_ptr(),
                  ops._stream(device))
        else:
            _call("rmi_assemble_rows", *common, *tail, err.data_ptr(), ops._stream(device))
        outs.append((ids, am, pos, sc, lm, rm, err, cnt))
    a, b = outs
    for x, y in zip(a[:7], b[:7]):
        if x.dtype == torch.float32:
            assert torch.equal(x[:, :-1], y[:, :-1])
        else:
            assert torch.equal(x, y)
    assert torch.equal(b[3][:, -1], last)
    assert torch.equal(b[7], a[5].to(torch.int32).sum(1).to(torch.int32))
