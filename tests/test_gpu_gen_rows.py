"""rmi_gen_rows (csrc/parse.hip): the turn's generations onto the env batch ahead of the fused
decode + parse — against the torch formulation it replaced in ContextManager._device_env_inputs:
the rows scattered onto a zeroed [n_envs, R] batch, n_ids = R for the envs given (0 else), and
the has-input mask, and the longest given row's raw bytes = the sum of VocabTable.raw_len over its ids clamped to
[0, V) (skipped tokens 0) — every env, a subset, none, ids outside the vocabulary."""
import numpy as np
import pytest
import torch

from ragen_amd import ops

pytestmark = pytest.mark.gpu


def _vocab(dev, V=300, seed=3):
    rng = np.random.default_rng(seed)
    table = [bytes(rng.integers(32, 127, rng.integers(0, 20)).astype(np.uint8)) for _ in range(V)]
    skip = (rng.random(V) < 0.1).astype(np.uint8)
    return ops.VocabTable.from_bytes(table, skip, dev)


def _want(resp, env_rows, n, vocab):
    R = resp.shape[1]
    V = vocab.raw_len.numel()
    ids = torch.zeros(n, R, dtype=torch.int64, device=resp.device)
    n_ids = torch.zeros(n, dtype=torch.int32, device=resp.device)
    ids[env_rows] = resp
    n_ids[env_rows] = R
    raw = vocab.raw_len[resp.clamp(0, V - 1)].sum(1)
    return ids, n_ids, int(raw.max()) if resp.numel() else 0


@pytest.mark.parametrize("R", [1, 63, 64, 200])
def test_gen_rows_equals_torch(device, R):
    vocab = _vocab(device)
    V = vocab.raw_len.numel()
    rng = np.random.default_rng(R)
    n = 1000
    for which in ("all", "subset", "one"):
        rows = {"all": np.arange(n), "subset": np.sort(rng.choice(n, 437, replace=False)),
                "one": np.array([n - 1])}[which]
        resp = torch.from_numpy(rng.integers(-2, V + 3, (len(rows), R))).to(device)
        rows_t = torch.from_numpy(rows).to(device)
        ids_w, n_w, raw_w = _want(resp, rows_t, n, vocab)
        raw = torch.empty(1, dtype=torch.int32, device=device)
        if which == "all":
            torch.ops.ragen_amd.gen_rows(resp, None, n, vocab.packed, None, None, raw)
        else:
            src = np.full(n, -1, np.int64)
            src[rows] = np.arange(len(rows))
            ids = torch.full((n, R), 7, dtype=torch.int64, device=device)  # garbage: every row is written
            n_ids = torch.full((n,), 7, dtype=torch.int32, device=device)
            has = torch.full((n,), 7, dtype=torch.uint8, device=device)
            torch.ops.ragen_amd.gen_rows(resp, torch.from_numpy(src).to(device), n, vocab.packed, ids, n_ids, raw,
                                         has)
            assert torch.equal(ids, ids_w) and torch.equal(n_ids, n_w), which
            assert torch.equal(has, (n_w > 0).to(torch.uint8)), which
        assert int(raw) == raw_w, which


def test_gen_rows_no_rows(device):
    vocab = _vocab(device)
    n, R = 64, 16
    resp = torch.empty(0, R, dtype=torch.int64, device=device)
    ids = torch.full((n, R), 7, dtype=torch.int64, device=device)
    n_ids = torch.full((n,), 7, dtype=torch.int32, device=device)
    raw = torch.full((1,), 7, dtype=torch.int32, device=device)
    torch.ops.ragen_amd.gen_rows(resp, torch.full((n,), -1, dtype=torch.int64, device=device), n, vocab.packed,
                                 ids, n_ids, raw)
    assert not ids.any() and not n_ids.any() and int(raw) == 0


def test_gen_rows_chained(device):
    """rmi_gen_rows_chained (the device turn loop's form, two alternating raw slots): the same
    rows and raw max as rmi_gen_rows when raw_max starts at 0, no zeroing of raw_max, and
    raw_next zeroed; alternating two slots over several turns reads each turn's own max."""
    vocab = _vocab(device)
    rng = np.random.default_rng(5)
    n, V = 1000, vocab.raw_len.numel()
    slots = torch.zeros(2, dtype=torch.int32, device=device)
    for turn in range(5):
        R = int(rng.integers(1, 120))
        resp = torch.from_numpy(rng.integers(-3, V + 3, (n, R))).to(device)
        _, _, want = _want(resp, torch.arange(n, device=device), n, vocab)
        cur, nxt = slots[turn % 2:turn % 2 + 1], slots[1 - turn % 2:2 - turn % 2]
        nxt.fill_(12345)  # stale: the call zeroes it
        ops.gen_rows(resp, None, n, vocab.packed, None, None, cur, raw_next=nxt)
        assert int(cur.item()) == want and int(nxt.item()) == 0
    src = torch.full((n,), -1, dtype=torch.int64, device=device)
    src[::3] = torch.arange(len(range(0, n, 3)), device=device)
    resp = torch.from_numpy(rng.integers(0, V, (len(range(0, n, 3)), 40))).to(device)
    ids = torch.empty(n, 40, dtype=torch.int64, device=device)
    n_ids = torch.empty(n, dtype=torch.int32, device=device)
    has = torch.empty(n, dtype=torch.uint8, device=device)
    cur = torch.full((1,), 7, dtype=torch.int32, device=device)  # not zeroed by the chained form
    nxt = torch.ones(1, dtype=torch.int32, device=device)
    ops.gen_rows(resp, src, n, vocab.packed, ids, n_ids, cur, has, raw_next=nxt)
    w_ids, w_n, want = _want(resp, torch.arange(0, n, 3, device=device), n, vocab)
    assert torch.equal(ids, w_ids) and torch.equal(n_ids, w_n) and int(nxt.item()) == 0
    assert int(cur.item()) == max(7, want)
    with pytest.raises(ValueError):
        ops.gen_rows(resp, src, n, vocab.packed, ids, n_ids, cur, has, raw_next=cur)
