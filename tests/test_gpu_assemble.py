"""§8(f) rank 1: the training batch assembled on the device in one pass (rmi_assemble_batch):
left padding, attention_mask, position_ids = cumsum(attention_mask), and get_masks_and_scores
(ctx_manager.py:35-70, :278-306) — against the reference-run golden masks/scores (rows
recovered from its left-padded ids) and, at 8192 x 1024, against the host-padded batch
(torch) + the oracle's masks/scores."""
import numpy as np
import pytest
import torch

import oracle
from fake_tok import FakeQwenTok
from ragen_amd import ops
from ragen_amd.llm_agent.ctx_manager import assemble_batch
from trace_util import load

pytestmark = pytest.mark.gpu
PAD, SP, RT = 151643, 151644, 151645


def _rows_of(padded):
    rows = []
    for r in padded:
        k = 0
        while k < len(r) and r[k] == PAD:
            k += 1
        rows.append(r[k:])
    return rows


def test_assemble_golden(device):
    d = load("masks_scores")
    ids = d["input_ids"]
    rows = _rows_of(ids)
    lens, flat = d["scores_len"], d["scores_flat"]
    scores, o = [], 0
    for n in lens:
        scores.append(list(flat[o:o + n]))
        o += n
    tok = FakeQwenTok()
    for uts in (False, True):
        for erm in (False, True):
            i, am, pos, sc, lm, rm = assemble_batch(rows, tok, scores, uts, erm, device, S=ids.shape[1])
            key = f"uts{int(uts)}_erm{int(erm)}"
            np.testing.assert_array_equal(i.cpu().numpy(), ids)
            ref_am = (np.arange(ids.shape[1])[None, :] >= (ids.shape[1] - np.array([len(r) for r in rows]))[:, None])
            np.testing.assert_array_equal(am.cpu().numpy(), ref_am.astype(np.int64))
            np.testing.assert_array_equal(pos.cpu().numpy(), np.cumsum(ref_am, axis=1))
            np.testing.assert_array_equal(sc.cpu().numpy(), d[key + "_score"])
            np.testing.assert_array_equal(lm.cpu().numpy().astype(np.uint8), d[key + "_loss_mask"])
            np.testing.assert_array_equal(rm.cpu().numpy().astype(np.uint8), d[key + "_response_mask"])


def test_assemble_llama3_golden(device):
    """assemble_batch with a Llama-3 tokenizer (ids 128006 / 128009, no roll) on the rows of the
    reference-run Llama fixture: the same ids and the reference's masks / scores."""
    from fake_tok import FakeLlama3Tok
    d = load("masks_scores_llama")
    ids = d["input_ids"]
    rows = [r[np.argmax(r != 128001):] if (r != 128001).any() else r[:0] for r in ids]
    lens, flat = d["scores_len"], d["scores_flat"]
    scores, o = [], 0
    for n in lens:
        scores.append(list(flat[o:o + n]))
        o += n
    tok = FakeLlama3Tok()
    for uts in (False, True):
        for erm in (False, True):
            i, am, pos, sc, lm, rm = assemble_batch(rows, tok, scores, uts, erm, device, S=ids.shape[1])
            key = f"uts{int(uts)}_erm{int(erm)}"
            np.testing.assert_array_equal(i.cpu().numpy(), ids)
            np.testing.assert_array_equal(sc.cpu().numpy(), d[key + "_score"])
            np.testing.assert_array_equal(lm.cpu().numpy().astype(np.uint8), d[key + "_loss_mask"])
            np.testing.assert_array_equal(rm.cpu().numpy().astype(np.uint8), d[key + "_response_mask"])


def test_assemble_full_size(device):
    """8192 rows up to 1024 tokens of chat-shaped ids: == torch left padding + cumsum and the
    oracle's get_masks_and_scores on the padded ids, both score placements."""
    rng = np.random.default_rng(5)
    B = 8192
    rows, scores = [], []
    for b in range(B):
        r = [SP] + list(rng.integers(100, 1000, size=int(rng.integers(4, 60)))) + [RT, 198]
        sc = []
        while len(r) < int(rng.integers(200, 1000)):
            r += [SP] + list(rng.integers(100, 1000, size=int(rng.integers(8, 90)))) + [RT, 198]
            r += [SP] + list(rng.integers(100, 1000, size=int(rng.integers(4, 60)))) + [RT]
            sc.append(float(rng.choice([0.0, -0.1, 1.0, 10.9])))
        rows.append(np.array(r, np.int64))
        scores.append(sc)
    S = max(len(r) for r in rows)
    padded = np.full((B, S), PAD, np.int64)
    for b, r in enumerate(rows):
        padded[b, S - len(r):] = r
    am_ref = (padded != PAD) | (np.arange(S)[None, :] >= (S - np.array([len(r) for r in rows]))[:, None])
    T = max(len(x) for x in scores)
    tab = np.zeros((T, B))
    for b, x in enumerate(scores):
        tab[:len(x), b] = x
    n = np.array([len(x) for x in scores], np.int32)
    for uts in (False, True):
        i, am, pos, sc, lm, rm = assemble_batch(rows, FakeQwenTok(), scores, uts, True, device)
        np.testing.assert_array_equal(i.cpu().numpy(), padded)
        np.testing.assert_array_equal(am.cpu().numpy(), am_ref.astype(np.int64))
        np.testing.assert_array_equal(pos.cpu().numpy(), torch.from_numpy(am_ref.astype(np.int64)).cumsum(-1).numpy())
        osc, olm, orm, oerr = oracle.masks_and_scores(padded, SP, RT, tab, n, T, uts, True, True)
        np.testing.assert_array_equal(sc.cpu().numpy(), osc)
        np.testing.assert_array_equal(lm.cpu().numpy().astype(np.uint8), olm)
        np.testing.assert_array_equal(rm.cpu().numpy().astype(np.uint8), orm)


def test_assemble_edge_rows(device):
    """Empty rows, a one-token row, and S == 1."""
    tok = FakeQwenTok()
    i, am, pos, sc, lm, rm = assemble_batch([[], [SP], [SP, 5, RT]], tok, [[], [1.0], [2.0]], False, False, device)
    assert i.shape == (3, 3) and sc.shape == (3, 2)
    assert am.cpu().tolist() == [[0, 0, 0], [0, 0, 1], [1, 1, 1]]
    assert pos.cpu().tolist() == [[0, 0, 0], [0, 0, 1], [1, 2, 3]]
    i, am, pos, sc, lm, rm = assemble_batch([[7], [SP]], tok, [[], []], False, False, device)
    assert i.cpu().tolist() == [[7], [SP]] and sc.shape == (2, 0)


@pytest.mark.parametrize("S", [1, 2, 3, 5, 7, 64, 257, 1029])
def test_assemble_ragged_shapes_vs_host(device, S):
    """ops.assemble_batch over ragged rows of 0..S+5 tokens at widths S that are not multiples
    of the kernel's 4-id groups: the 32-B group loads and stores, the element-wise pad edge and
    row end, and rows longer than S (flagged RMI_ERR_UNSUP, their last S tokens kept) against
    host left padding + cumsum and the oracle's masks / scores on the assembled ids."""
    rng = np.random.default_rng(S)
    B, T = 300, 4
    rows = []
    for b in range(B):
        n = int(rng.integers(0, S + 6))
        r = rng.integers(100, 1000, size=n).astype(np.int64)
        r[rng.random(n) < 0.1] = SP
        r[rng.random(n) < 0.05] = RT
        rows.append(r)
    lens = np.array([len(r) for r in rows], np.int64)
    off = np.zeros(B + 1, np.int64)
    off[1:] = np.cumsum(lens)
    toks = np.concatenate(rows) if lens.sum() else np.zeros(1, np.int64)
    sc = rng.choice([0.0, -0.1, 1.0, 10.9], size=(T, B))
    n_sc = rng.integers(0, T + 1, size=B).astype(np.int32)
    padded = np.full((B, S), PAD, np.int64)
    am_ref = np.zeros((B, S), np.int64)
    for b, r in enumerate(rows):
        k = min(len(r), S)
        if k:
            padded[b, S - k:] = r[len(r) - k:]
            am_ref[b, S - k:] = 1
    for uts in (False, True):
        ids, am, pos, score, lm, rm, err = ops.assemble_batch(
            torch.from_numpy(toks).to(device), torch.from_numpy(off).to(device), S, PAD, SP, RT,
            torch.from_numpy(sc).to(device), torch.from_numpy(n_sc).to(device), T, uts, True, True)
        np.testing.assert_array_equal(ids.cpu().numpy(), padded)
        np.testing.assert_array_equal(am.cpu().numpy(), am_ref)
        np.testing.assert_array_equal(pos.cpu().numpy(), np.cumsum(am_ref, axis=1))
        exp_err = np.where(lens > S, 8, 0)  # RMI_ERR_UNSUP: an overlong row
        if S > 1:
            osc, olm, orm, oerr = oracle.masks_and_scores(padded, SP, RT, sc, n_sc, T, uts, True, True)
            ok = np.asarray(oerr) == 0  # rows where the reference raises (a turn with two reward tokens) are flagged only
            assert ok.sum() > B // 4
            np.testing.assert_array_equal(score.cpu().numpy()[ok], osc[ok])
            np.testing.assert_array_equal(lm.cpu().numpy().astype(np.uint8), olm)
            np.testing.assert_array_equal(rm.cpu().numpy().astype(np.uint8), orm)
            exp_err |= np.where(np.asarray(oerr) != 0, 4, 0)  # RMI_ERR_STATE: the reference raises
        np.testing.assert_array_equal(err.cpu().numpy(), exp_err.astype(np.uint8))


@pytest.mark.parametrize("S", [1, 3, 4, 64, 257, 1100])
def test_row_counts_equal_torch(device, S):
    """rmi_row_counts (formulate_rollouts' response_length row sums) == response_mask.sum(-1)."""
    g = torch.Generator(device="cpu").manual_seed(S)
    for B, dt in ((1003, torch.bool), (8, torch.uint8), (0, torch.bool)):
        m = (torch.rand(B, S, generator=g) < 0.3)
        m = (m if dt == torch.bool else (m.to(torch.uint8) * torch.randint(1, 256, (B, S), generator=g,
                                                                           dtype=torch.int32).to(torch.uint8))).to(device)
        got = ops.row_counts(m)
        assert torch.equal(got.cpu(), (m != 0).sum(-1).to(torch.int32).cpu())
