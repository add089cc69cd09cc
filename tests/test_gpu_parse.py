"""GPU parity of the response -> action boundary (rmi_detokenize, rmi_parse_actions) against
the oracle (oracle/parse.py, itself pinned to vectors recorded from the reference)."""
import json
import os
import random

import numpy as np
import pytest
import torch

from oracle import parse as P
from ragen_amd import ops, synthetic
from ragen_amd import _lib

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "parse_response.json")
SOKOBAN = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}


def _golden():
    d = json.load(open(GOLD))
    lk = {k: (None if v is None else {int(a): b for a, b in v.items()}) for k, v in d["lookups"].items()}
    return lk, d["cases"]


def _run(texts, device, think, K, sep, lookup, swapped=None, sel=None, Lact=0, prepend=True):
    buf, lens = synthetic.encode_rows(texts)
    cfg = ops.parse_config(think, K, sep, lookup, swapped, prepend=prepend)
    out = ops.parse_actions(cfg, torch.from_numpy(buf).to(device), torch.from_numpy(lens).to(device),
                            None if sel is None else torch.from_numpy(sel).to(device), True, Lact)
    torch.cuda.synchronize()
    return {k: (None if v is None else v.cpu().numpy()) for k, v in out.items()}


def _check_rows(texts, out, think, K, sep, lookup, prepend=True):
    for b, t in enumerate(texts):
        resp = P.prefixed(t, think) if prepend else t
        _, acts = P.parse_response(resp, think, K, sep)
        n = int(out["n_actions"][b])
        assert n == len(acts), (b, t, acts)
        ids = P.action_ids(acts, lookup)
        assert list(out["actions"][b, :n]) == ids, (b, t, acts)
        assert not out["actions"][b, n:].any()
        assert tuple(out["spans"][b]) == P.match_spans(resp, think), (b, t)
        if out["action_text"] is not None:
            for k in range(n):
                got = out["action_text"][b, k, :out["action_len"][b, k]].tobytes().decode("utf-8")
                assert got == acts[k], (b, t, k)
        assert out["err"][b] == 0


@pytest.fixture(params=["seg", "wave"])
def kernel(request, monkeypatch):
    """The four-responses-per-wave kernels (default for rows that fit) or, with
    RAGEN_AMD_PARSE1=1, the one-response-per-wave kernels."""
    if request.param == "wave":
        monkeypatch.setenv("RAGEN_AMD_PARSE1", "1")
    else:
        monkeypatch.delenv("RAGEN_AMD_PARSE1", raising=False)
    return request.param


@pytest.mark.parametrize("lookup_name", ["sokoban", "frozen_lake", "bandit", "kelvin", "none"])
def test_parse_matches_reference_vectors(device, lookup_name, kernel):
    lookups, cases = _golden()
    lk = lookups[lookup_name]
    groups = {}
    for c in cases:
        groups.setdefault((c["enable_think"], c["K"], c["sep"]), []).append(c)
    for (think, K, sep), cs in groups.items():
        texts = [c["text"] for c in cs]
        out = _run(texts, device, think, K, sep, lk, Lact=256 if lk is None else 0)
        for b, c in enumerate(cs):
            n = int(out["n_actions"][b])
            assert n == len(c["actions"]), c["text"]
            ids = [int(i) for i in out["actions"][b, :n]]
            if lk is None:
                got = [out["action_text"][b, k, :out["action_len"][b, k]].tobytes().decode("utf-8") for k in range(n)]
                assert got == c["mapped"]["none"], c["text"]
            else:
                assert [i for i in ids if i] == c["mapped"][lookup_name], c["text"]
        _check_rows(texts, out, think, K, sep, lk)


def test_parse_bandit_per_env_lookup(device, kernel):
    """Bandit's action_lookup is per env (bandit/env.py:25-39): sel picks the id column."""
    lo, hi = {1: "Phoenix", 2: "Dragon"}, {1: "Dragon", 2: "Phoenix"}
    texts = ["x</think><answer>Dragon</answer>", "x</think><answer> phoenix </answer>",
             "x</think><answer>DRAGON</answer>", "x</think><answer>tiger</answer>"] * 4
    sel = np.array([0, 0, 0, 0, 1, 1, 1, 1] * 2, np.uint8)
    out = _run(texts, device, True, 1, "||", lo, hi, sel=sel)
    for b, t in enumerate(texts):
        _, acts = P.parse_response(P.prefixed(t, True), True, 1)
        assert list(out["actions"][b, :out["n_actions"][b]]) == P.action_ids(acts, hi if sel[b] else lo)


def test_parse_full_batch_vs_oracle(device, kernel):
    """8192 SK-shaped responses (synthetic actions of the bench), with no-think prefix too."""
    ids, n = synthetic.rollout_actions(8192, 1, 5, 1, 4)
    for think in (True, False):
        texts = synthetic.responses_for_actions(ids[0], n[0], SOKOBAN, enable_think=think)
        out = _run(texts, device, think, 5, "||", SOKOBAN)
        _check_rows(texts, out, think, 5, "||", SOKOBAN)
        assert np.array_equal(out["n_actions"], n[0])
        assert np.array_equal(out["actions"], ids[0])


def test_parse_fuzz_and_edges(device, kernel):
    rng = random.Random(3)
    frags = ["<think>", "</think>", "<answer>", "</answer>", "<|im_end|>", "<|im_start|>", "|", "||", " ", "\n",
             "　", " ", "\xa0", "K", "Up", "down", "LEFT", "x", "é", "\U0001f600", "<", ">"]
    texts = ["".join(rng.choice(frags) for _ in range(rng.randint(0, 40))) for _ in range(3001)]
    # short rows (both kernels), then rows up to the parse limit (the one-response-per-wave kernel)
    for batch in (texts + [""], texts + ["", "</think><answer>" + "Up || " * 1300 + "</answer>", "a" * 8000]):
        for think in (True, False):
            for prepend in (True, False):
                out = _run(batch, device, think, 5, "||", SOKOBAN, prepend=prepend)
                _check_rows(batch, out, think, 5, "||", SOKOBAN, prepend=prepend)


def test_parse_seg_equals_wave(device, monkeypatch):
    """The four-responses-per-wave kernel == the one-response-per-wave kernel on every output
    (fuzz rows with every tag / separator / whitespace form, batch sizes not a multiple of 4,
    the pass-through lookup with action text, Bandit's per-row column)."""
    rng = random.Random(9)
    frags2 = ["<think>", "</think>", "<answer>", "</answer>", "<|im_end|>", "<|im_start|>", "|", "||", " ", "\n",
             "　", " ", "\xa0", "K", "Up", "down", "LEFT", "x", "é", "\U0001f600", "<", ">"]
    frags2 += ["\t", "phoenix", "DRAGON", "|| Up ||"]
    for B in (1, 3, 6, 1027):
        texts = ["".join(rng.choice(frags2) for _ in range(rng.randint(0, 60))) for _ in range(B)]
        buf, lens = synthetic.encode_rows(texts)
        tb, tl = torch.from_numpy(buf).to(device), torch.from_numpy(lens).to(device)
        sel = torch.from_numpy(np.array([rng.random() < 0.5 for _ in range(B)], np.uint8)).to(device)
        for think in (True, False):
            for cfg, lact, sl in ((ops.parse_config(think, 5, "||", SOKOBAN), 0, None),
                                  (ops.parse_config(think, 3, "||", None), 24, None),
                                  (ops.parse_config(think, 2, "||", {1: "Phoenix", 2: "Dragon"},
                                                    {1: "Dragon", 2: "Phoenix"}), 0, sel)):
                outs = []
                for mode in ("seg", "wave"):
                    if mode == "wave":
                        monkeypatch.setenv("RAGEN_AMD_PARSE1", "1")
                    else:
                        monkeypatch.delenv("RAGEN_AMD_PARSE1", raising=False)
                    outs.append(ops.parse_actions(cfg, tb, tl, sl, True, lact))
                torch.cuda.synchronize()
                a, w = outs
                n = a["n_actions"].cpu().numpy()
                assert torch.equal(a["n_actions"], w["n_actions"]) and torch.equal(a["spans"], w["spans"])
                assert torch.equal(a["err"], w["err"])
                aa, wa = a["actions"].cpu().numpy(), w["actions"].cpu().numpy()
                for b in range(B):
                    assert list(aa[b, :n[b]]) == list(wa[b, :n[b]]), (B, b, texts[b])
                if lact:
                    assert torch.equal(a["action_len"], w["action_len"])
                    at, wt, al = a["action_text"].cpu().numpy(), w["action_text"].cpu().numpy(), \
                        a["action_len"].cpu().numpy()
                    for b in range(B):
                        for k in range(n[b]):
                            assert at[b, k, :al[b, k]].tobytes() == wt[b, k, :al[b, k]].tobytes()


def test_parse_stride_envelope(device):
    buf = torch.zeros(2, 8196, dtype=torch.uint8, device=device)
    lens = torch.zeros(2, dtype=torch.int32, device=device)
    with pytest.raises(NotImplementedError):  # rows longer than 8192 bytes: RMI_EUNSUP
        ops.parse_actions(ops.parse_config(True, 5, "||", SOKOBAN), buf, lens)


def test_parse_bad_lengths_and_overlong_actions(device):
    buf, lens = synthetic.encode_rows(["x</think><answer>Up</answer>", "x</think><answer>abcdefghij</answer>"])
    lens_t = torch.from_numpy(np.array([-1, lens[1]], np.int32)).to(device)
    cfg = ops.parse_config(True, 5, "||", None)
    out = ops.parse_actions(cfg, torch.from_numpy(buf).to(device), lens_t, None, True, 4)
    torch.cuda.synchronize()
    err = out["err"].cpu().numpy()
    assert err[0] & _lib.ERR_STATE and out["n_actions"][0].item() == 0
    assert err[1] & _lib.ERR_UNSUP and out["action_len"][1, 0].item() == 4
    with pytest.raises(ValueError):
        ops.parse_actions(ops.parse_config(True, 0, "||", None), torch.from_numpy(buf).to(device), lens_t)


# ------------------------------------------------------------------ detokenize
def _random_table(V, seed):
    rng = np.random.default_rng(seed)
    table = []
    for i in range(V):
        k = int(rng.integers(0, 9)) if i % 11 else int(rng.integers(9, 41))  # some past the 12 inline bytes
        if i % 7 == 0:  # ASCII-only tokens
            table.append(bytes(rng.integers(32, 127, size=k).astype(np.uint8)))
        else:
            table.append(bytes(rng.integers(0, 256, size=k).astype(np.uint8)))
    skip = (rng.random(V) < 0.05).astype(np.uint8)
    return table, skip


def test_detokenize_vs_oracle(device):
    V = 5000
    table, skip = _random_table(V, 1)
    vt = ops.VocabTable.from_bytes(table, skip, device)
    rng = np.random.default_rng(2)
    B, R = 2048, 96
    ids = rng.integers(0, V, size=(B, R)).astype(np.int64)
    n_ids = rng.integers(0, R + 1, size=B).astype(np.int32)
    ids[5, 3] = V + 3   # out of range
    ids[6, 0] = -2
    n_ids[5] = max(n_ids[5], 4)
    n_ids[6] = max(n_ids[6], 1)
    out, n, err = ops.detokenize(torch.from_numpy(ids).to(device), vt, 4096, torch.from_numpy(n_ids).to(device))
    torch.cuda.synchronize()
    out, n, err = out.cpu().numpy(), n.cpu().numpy(), err.cpu().numpy()
    for b in range(B):
        row = [int(i) for i in ids[b, :n_ids[b]]]
        if b in (5, 6):
            assert err[b] & _lib.ERR_INDEX
            row = [i for i in row if 0 <= i < V]
        else:
            assert err[b] == 0
        want = P.detokenize(row, table, skip.astype(bool)).encode("utf-8")
        assert out[b, :n[b]].tobytes() == want, b


def test_detokenize_ascii_and_overflow(device):
    table = [b"ab", b"<think>", b" Up", b" ||", b"\xe2\x80", b"\xa8"] + [b"x" * 8]
    skip = np.zeros(len(table), np.uint8)
    vt = ops.VocabTable.from_bytes(table, skip, device)
    ids = np.array([[1, 2, 3, 2, 0, 4, 5, 6], [6] * 8], np.int64)
    out, n, err = ops.detokenize(torch.from_numpy(ids).to(device), vt, 32)
    torch.cuda.synchronize()
    assert out[0, :n[0]].cpu().numpy().tobytes() == b"<think> Up || Upab\xe2\x80\xa8" + b"x" * 8
    assert n[1].item() == 32 and err[1].item() & _lib.ERR_UNSUP and err[0].item() == 0


def test_detokenize_parse_step_pipeline(device):
    """token ids -> text -> action ids -> Sokoban turn, equal to the host-side path."""
    from ragen_amd.env import SokobanBatch
    from ragen_amd.env.configs import SokobanEnvConfig
    import oracle
    B, K = 1024, 5
    ids, n = synthetic.rollout_actions(B, 1, K, 1, 4)
    texts = synthetic.responses_for_actions(ids[0], n[0], SOKOBAN)
    # a byte vocabulary: one token per byte + a few words, greedy tokenisation
    words = [b"</think>", b"<answer>", b"</answer>", b" || ", b"Up", b"Down", b"Left", b"Right"]
    table = [bytes([i]) for i in range(256)] + words + [b"<|endoftext|>"]
    skip = np.zeros(len(table), np.uint8)
    skip[-1] = 1
    R = 0
    rows = []
    for t in texts:
        bts, row, i = t.encode("utf-8"), [], 0
        while i < len(bts):
            for w, wb in enumerate(words):
                if bts.startswith(wb, i):
                    row.append(256 + w)
                    i += len(wb)
                    break
            else:
                row.append(bts[i])
                i += 1
        rows.append(row)
        R = max(R, len(row))
    tok = np.full((B, R + 3), len(table) - 1, np.int64)  # right padded with the (special) pad id
    for b, r in enumerate(rows):
        tok[b, :len(r)] = r
    vt = ops.VocabTable.from_bytes(table, skip, device)
    text, tlen, err = ops.detokenize(torch.from_numpy(tok).to(device), vt, 2048)
    parsed = ops.parse_actions(ops.parse_config(True, K, "||", SOKOBAN), text, tlen)
    env = SokobanBatch(SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100), B, 1, K, device)
    env.reset(synthetic.env_seeds(B))
    fixed, state, player = env.room_fixed.cpu().numpy(), env.room_state.cpu().numpy(), env.player.cpu().numpy()
    env.step_turn(0, parsed["actions"], parsed["n_actions"], None, 10, -0.1)
    nes, bot = np.zeros(B, np.int32), np.zeros(B, np.int32)
    oep = oracle.Episode(B, 1)
    oracle.sokoban_turn(6, 6, 1, 100, fixed, state, player, nes, bot, oep, 0, ids[0], n[0])
    torch.cuda.synchronize()
    assert not err.any()
    assert np.array_equal(env.room_state.cpu().numpy(), state)
    assert np.array_equal(env.ep.turn_reward.cpu().numpy(), oep.turn_reward)
    assert np.array_equal(env.ep.penalty.cpu().numpy(), oep.penalty)


@pytest.mark.parametrize("name", ["sokoban_es", "frozenlake_es", "bandit_es", "countdown_es"])
def test_step_text_equals_dict_step(device, name, monkeypatch):
    """EnvStateManager.step_text (device parse + turn, nothing on the host) == step() fed with
    the host-parsed dicts, on the reference's recorded action traces."""
    from test_gpu_facade import _config, _hashseed0_reseed
    from trace_util import load, strings
    from ragen_amd.env import SokobanBatch
    from ragen_amd.llm_agent import EnvStateManager
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    d, S = load(name), strings()[name]
    es_host = EnvStateManager(_config(name), mode="train", device=device)
    es_dev = EnvStateManager(_config(name), mode="train", device=device)
    es_host.reset(seed=int(d["seed"]))
    es_dev.reset(seed=int(d["seed"]))
    B, T = int(d["B"]), int(d["T"])
    K = es_host.K
    active = list(range(B))
    for t in range(T):
        texts = []
        for i in range(B):
            if name == "countdown_es":
                a = S["answers"][t][i]
                acts = [] if a is None else [a]
            else:
                acts = [S["vocab"][c] for c in d["codes"][t, i] if c >= 0]
            texts.append("plan</think> <answer>" + " || ".join(acts) + "</answer>")
        inputs = []
        for i in active:
            llm_response, acts = P.parse_response(P.prefixed(texts[i], True), True, K)
            inputs.append({"env_id": i, "llm_response": llm_response, "llm_raw_response": texts[i], "actions": acts})
        has = np.zeros(B, np.uint8)
        has[active] = 1
        buf, lens = synthetic.encode_rows(texts)
        es_dev.step_text(torch.from_numpy(buf).to(device), torch.from_numpy(lens).to(device),
                         torch.from_numpy(has).to(device))
        active = [o["env_id"] for o in es_host.step(inputs)]
        torch.cuda.synchronize()
        for th, td in zip(es_host.tags, es_dev.tags):
            for f in ("num_actions", "flags", "n_turns", "penalty", "turn_reward", "turn_info", "turn_exec"):
                assert torch.equal(getattr(th.batch.ep, f), getattr(td.batch.ep, f)), (t, f)
        if not active:
            break


def test_detokenize_utf8_validity_edges(device):
    """Token byte strings that split multi-byte characters (valid once concatenated) and the
    invalid forms (overlong, surrogate, > U+10FFFF, lone / extra continuation bytes, truncated
    sequences at the row end, C0/C1/F5..FF): the device decode == bytes.decode("utf-8", "replace")."""
    rng = np.random.default_rng(17)
    valid_text = "Up — → 12 + 3 ✓ 😀 é ü 中文   x".encode("utf-8")
    invalid = [b"\xc0\xaf", b"\xe0\x80\xaf", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\x80", b"\xbf\xbf",
               b"\xc2", b"\xe2\x82", b"\xf0\x9f\x98", b"\xc2\x80\x80", b"\xf5", b"\xff", b"a\xe2\x28\xa1b"]
    rows = []
    for i in range(600):
        if i % 3 == 0:  # valid text cut at random byte boundaries into tokens
            src = valid_text * int(rng.integers(1, 4))
        else:
            src = valid_text[: int(rng.integers(0, len(valid_text)))] + invalid[i % len(invalid)] + \
                valid_text[: int(rng.integers(0, 8))]
        cuts = sorted(set(int(x) for x in rng.integers(0, len(src) + 1, size=int(rng.integers(0, 12)))))
        pieces = [src[a:b] for a, b in zip([0] + cuts, cuts + [len(src)]) if b > a]
        rows.append(pieces)
    table = sorted({p for r in rows for p in r})
    index = {p: i for i, p in enumerate(table)}
    R = max(len(r) for r in rows)
    ids = np.zeros((len(rows), R), np.int64)
    n_ids = np.array([len(r) for r in rows], np.int32)
    for i, r in enumerate(rows):
        ids[i, :len(r)] = [index[p] for p in r]
    vt = ops.VocabTable.from_bytes(table, np.zeros(len(table), np.uint8), device)
    out, n, err = ops.detokenize(torch.from_numpy(ids).to(device), vt, 512, torch.from_numpy(n_ids).to(device))
    torch.cuda.synchronize()
    out, n = out.cpu().numpy(), n.cpu().numpy()
    for i, r in enumerate(rows):
        want = b"".join(r).decode("utf-8", "replace").encode("utf-8")
        assert out[i, :n[i]].tobytes() == want, (i, b"".join(r))
    assert not err.any()


# ------------------------------------------------------- fused decode + parse (rmi_detok_parse)
def _byte_word_tokens(texts, words):
    """Greedy tokenisation over one token per byte + the given words (ids 256..)."""
    rows = []
    for t in texts:
        bts, row, i = t.encode("utf-8"), [], 0
        while i < len(bts):
            for w, wb in enumerate(words):
                if bts.startswith(wb, i):
                    row.append(256 + w)
                    i += len(wb)
                    break
            else:
                row.append(bts[i])
                i += 1
        rows.append(row)
    return rows


def _fused_vs_separate(device, ids, n_ids, vt, stride, cfg, sel=None, Lact=0):
    """rmi_detok_parse == rmi_detokenize then rmi_parse_actions, every output."""
    tid = torch.from_numpy(ids).to(device)
    tn = None if n_ids is None else torch.from_numpy(n_ids).to(device)
    ts = None if sel is None else torch.from_numpy(sel).to(device)
    text, tlen, derr = ops.detokenize(tid, vt, stride, tn)
    sep = ops.parse_actions(cfg, text, tlen, ts, True, Lact)
    fu = ops.detok_parse(tid, vt, stride, cfg, tn, ts, True, Lact)
    torch.cuda.synchronize()
    tl = tlen.cpu().numpy()
    ft = fu["text"].cpu().numpy()
    st = text.cpu().numpy()
    assert np.array_equal(fu["text_len"].cpu().numpy(), tl)
    for b in range(len(tl)):  # the row bytes (a row's dwords past its length are not written)
        assert ft[b, :tl[b]].tobytes() == st[b, :tl[b]].tobytes(), b
    assert torch.equal(fu["decode_err"], derr)
    for k in ("actions", "n_actions", "spans", "err", "action_text", "action_len"):
        if sep[k] is None:
            assert fu[k] is None
            continue
        if k == "action_text":  # the bytes past each action's length are not written
            al = sep["action_len"].cpu().numpy()
            a, f = sep[k].cpu().numpy(), fu[k].cpu().numpy()
            n = sep["n_actions"].cpu().numpy()
            for b in range(a.shape[0]):
                for j in range(n[b]):
                    assert a[b, j, :al[b, j]].tobytes() == f[b, j, :al[b, j]].tobytes(), (b, j)
            continue
        assert torch.equal(fu[k], sep[k]), k
    return fu


def test_detok_parse_fused_on_reference_vectors(device, kernel):
    """The 1530 recorded _parse_response vectors, tokenized over bytes + tag / name words,
    through the fused kernel == the separate kernels (themselves checked against the oracle
    above), every lookup, with action text for the pass-through lookup."""
    lookups, cases = _golden()
    words = [b"<think>", b"</think>", b"<answer>", b"</answer>", b"<|im_end|>", b" || ", b"Up", b"Down", b"Left",
             b"Right", b"  ", b"\xe2\x80\x83"]
    table = [bytes([i]) for i in range(256)] + words + [b"<|endoftext|>"]
    skip = np.zeros(len(table), np.uint8)
    skip[-1] = 1
    vt = ops.VocabTable.from_bytes(table, skip, device)
    groups = {}
    for c in cases:
        groups.setdefault((c["enable_think"], c["K"], c["sep"]), []).append(c)
    for lk_name in ("sokoban", "bandit", "kelvin", "none"):
        lk = lookups[lk_name]
        for (think, K, sep), cs in groups.items():
            rows = _byte_word_tokens([c["text"] for c in cs], words)
            R = max(len(r) for r in rows) + 2
            ids = np.full((len(rows), R), len(table) - 1, np.int64)  # right-padded with the skipped pad id
            for b, r in enumerate(rows):
                ids[b, :len(r)] = r
            stride = max(64, (max(len(c["text"].encode()) for c in cs) + 8) // 4 * 4)
            fu = _fused_vs_separate(device, ids, None, vt, stride, ops.parse_config(think, K, sep, lk),
                                    Lact=256 if lk is None else 0)
            # and against the recorded reference outputs
            n = fu["n_actions"].cpu().numpy()
            for b, c in enumerate(cs):
                assert n[b] == len(c["actions"]), c["text"]


def test_detok_parse_fused_edges(device, kernel):
    """Random vocabularies (long tokens past the inline 12 bytes, invalid UTF-8, skipped ids),
    out-of-range ids, ragged n_ids, rows truncated at the stride, Bandit's per-row id column,
    and rows at the parse row limit."""
    V = 3000
    table, skip = _random_table(V, 4)
    # answer-shaped tokens so that some rows parse to actions
    table += [b"x</think><answer>", b"Phoenix", b" || ", b"dragon", b"</answer>"]
    skip = np.concatenate([skip, np.zeros(5, np.uint8)])
    vt = ops.VocabTable.from_bytes(table, skip, device)
    rng = np.random.default_rng(8)
    B, R = 1500, 64
    ids = rng.integers(0, V, size=(B, R)).astype(np.int64)
    for b in range(0, B, 3):  # answer rows: head, names, separators, tail
        k = int(rng.integers(1, 6))
        body = [V] + [int(rng.choice([V + 1, V + 3, int(rng.integers(0, V))])) if j % 2 == 0 else V + 2
                      for j in range(2 * k - 1)] + [V + 4]
        ids[b, :len(body)] = body
    n_ids = rng.integers(0, R + 1, size=B).astype(np.int32)
    n_ids[::3] = R
    ids[7, 2], ids[8, 0] = V + 10, -5  # outside the vocabulary
    n_ids[7], n_ids[8] = R, R
    sel = (rng.random(B) < 0.5).astype(np.uint8)
    lo, hi = {1: "Phoenix", 2: "Dragon"}, {1: "Dragon", 2: "Phoenix"}
    for stride in (64, 1024, 8192):  # 64: most rows truncated (decode_err UNSUP)
        for think in (True, False):
            fu = _fused_vs_separate(device, ids, n_ids, vt, stride, ops.parse_config(think, 3, "||", lo, hi), sel)
            derr = fu["decode_err"].cpu().numpy()
            assert derr[7] & _lib.ERR_INDEX and derr[8] & _lib.ERR_INDEX
            if stride == 64:
                assert (derr & _lib.ERR_UNSUP).any()
            if stride == 1024 and think:
                assert (fu["n_actions"].cpu().numpy() > 0).sum() > B // 10
    with pytest.raises(NotImplementedError):  # the parse's row limit
        ops.detok_parse(torch.from_numpy(ids).to(device), vt, 8196, ops.parse_config(True, 3, "||", lo))
