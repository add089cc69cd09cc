"""CPU: the response -> action oracle (oracle/parse.py) pinned against vectors recorded from
the reference's own _parse_response / _extract_map_valid_actions, and its detokenize against
the installed `tokenizers` ByteLevel decoder.  No GPU."""
import json
import os
import random

import numpy as np
import pytest

from oracle import parse as P

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "parse_response.json")


def golden():
    d = json.load(open(GOLD))
    lk = {k: (None if v is None else {int(a): b for a, b in v.items()}) for k, v in d["lookups"].items()}
    return lk, d["cases"]


def test_oracle_matches_reference_parse_vectors():
    lookups, cases = golden()
    assert len(cases) >= 1500
    n_match = n_cascade = 0
    for c in cases:
        resp = P.prefixed(c["text"], c["enable_think"])
        llm_response, actions = P.parse_response(resp, c["enable_think"], c["K"], c["sep"])
        assert (llm_response, actions) == (c["llm_response"], c["actions"]), c["text"]
        for name, lk in lookups.items():
            assert P.map_actions(actions, lk) == c["mapped"][name], (name, c["text"])
            ids = P.action_ids(actions, lk)
            if lk is not None:
                assert [i for i in ids if i] == c["mapped"][name]
        s = P.match_spans(resp, c["enable_think"])
        if s[2] >= 0:
            n_match += 1
            content = resp.encode("utf-8")[s[2]:s[3]].decode("utf-8")
            n_cascade += any(t in content for t in P.SPECIAL_TOKENS)
    # the vectors exercise both the plain and the replace-cascade path
    assert n_match > 500 and n_cascade > 100


def _tiny_bytelevel_tokenizer():
    tokenizers = pytest.importorskip("tokenizers")
    from tokenizers import AddedToken, Tokenizer, decoders, models
    b2u = P.bytes_to_unicode()
    vocab = {c: i for i, c in enumerate(b2u.values())}
    for e in ["Ġhello", "Ġworld", "Up", "Ġ||", "ĠDown", "âĪ", "</", "think", ">", "<answer>", "Ġâ"]:
        vocab.setdefault(e, len(vocab))
    tok = Tokenizer(models.BPE(vocab=vocab, merges=[]))
    tok.decoder = decoders.ByteLevel()
    tok.add_special_tokens([AddedToken("<|im_end|>", special=True), AddedToken("<|endoftext|>", special=True)])
    tok.add_tokens([AddedToken("<think>", special=False), AddedToken(" spaced tok ", special=False),
                    AddedToken("é_x", special=False)])
    return tok, tokenizers


def test_detokenize_oracle_matches_tokenizers_bytelevel():
    tok, _ = _tiny_bytelevel_tokenizer()
    c2b = {c: b for b, c in P.bytes_to_unicode().items()}
    V = max(tok.get_vocab(with_added_tokens=True).values()) + 1
    table = [P.token_bytes(tok.id_to_token(i), c2b) if tok.id_to_token(i) is not None else b"" for i in range(V)]
    special = {tok.token_to_id("<|im_end|>"), tok.token_to_id("<|endoftext|>")}
    skip = [i in special for i in range(V)]
    rng = random.Random(5)
    for _ in range(2000):
        ids = [rng.randrange(V) for _ in range(rng.randint(0, 40))]
        assert P.detokenize(ids, table, skip) == tok.decode(ids, skip_special_tokens=True), ids


def test_vocab_table_from_hf_tokenizer_matches_oracle():
    """ops.VocabTable.from_tokenizer (host-side table builder) == the oracle's per-token rule,
    through transformers' fast-tokenizer wrapper (batch_decode as ctx_manager.py:334-337)."""
    import torch
    transformers = pytest.importorskip("transformers")
    tok, _ = _tiny_bytelevel_tokenizer()
    hf = transformers.PreTrainedTokenizerFast(tokenizer_object=tok, eos_token="<|im_end|>",
                                              pad_token="<|endoftext|>")
    hf.clean_up_tokenization_spaces = False
    from ragen_amd.ops import VocabTable
    vt = VocabTable.from_tokenizer(hf, torch.device("cpu"))
    off, data, skip = vt.off.numpy(), vt.data.numpy(), vt.skip.numpy()
    table = [data[off[i]:off[i + 1]].tobytes() for i in range(len(off) - 1)]
    rng = random.Random(9)
    rows = [[rng.randrange(len(table)) for _ in range(rng.randint(0, 30))] for _ in range(500)]
    want = hf.batch_decode(rows, skip_special_tokens=True)
    got = [P.detokenize(r, table, skip.astype(bool)) for r in rows]
    assert got == want


def test_vocab_pack_layout():
    """rmi_vocab_pack (host C, the table rmi_detokenize gathers from): every entry decodes back
    to its token's bytes / skip bit — inline for tokens of <= 12 bytes, by blob offset beyond —
    on random vocabularies with empty, 12-, 13- and long tokens."""
    import numpy as np
    import torch
    from ragen_amd.ops import VocabTable
    rng = random.Random(3)
    for trial in range(20):
        V = rng.randint(1, 400)
        table = [bytes(rng.randrange(256) for _ in range(rng.choice([0, 1, 3, 7, 11, 12, 13, 20, 300])))
                 for _ in range(V)]
        skip = [rng.random() < 0.1 for _ in range(V)]
        vt = VocabTable.from_bytes(table, skip, torch.device("cpu"))
        pk = vt.packed.numpy().view(np.uint32)
        blob = vt.data.numpy().tobytes()
        for t, (tb, sk) in enumerate(zip(table, skip)):
            meta = int(pk[t, 3])
            assert meta >> 31 == int(sk) and meta & 0xFFFFFF == len(tb)
            if len(tb) <= 12:
                got = b"".join(int(pk[t, k]).to_bytes(4, "little") for k in range(3))[:len(tb)]
                assert got == tb and b"".join(int(pk[t, k]).to_bytes(4, "little") for k in range(3))[len(tb):] == \
                    bytes(12 - len(tb))
            else:
                o = int(pk[t, 0])
                assert blob[o:o + len(tb)] == tb
            assert int(vt.raw_len[t]) == (0 if sk else len(tb))


def test_synthetic_responses_parse_to_their_actions():
    from ragen_amd import synthetic as S
    lk = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}
    ids, n = S.rollout_actions(256, 1, 5, 1, 4)
    texts = S.responses_for_actions(ids[0], n[0], lk)
    for b, t in enumerate(texts):
        _, acts = P.parse_response(P.prefixed(t, True), True, 5)
        assert len(acts) == n[0][b]
        got = P.action_ids(acts, lk)
        assert got == [int(x) for x in ids[0][b, :n[0][b]]]


def test_parse_response_from_spans_matches_regex():
    """EnvStateManager._materialize builds the history strings from the device parse's match
    spans (ctx_manager.parse_response_spans) instead of re-running the regex: equal to
    parse_response and to the reference's outputs on every vector, with the spans of the
    reference's match."""
    from ragen_amd.llm_agent.ctx_manager import parse_response, parse_response_spans
    for c in golden()[1]:
        resp = P.prefixed(c["text"], c["enable_think"])
        sp = P.match_spans(resp, c["enable_think"])
        got = parse_response_spans(resp, sp, c["enable_think"], c["sep"], c["K"])
        assert got == parse_response(resp, c["enable_think"], c["sep"], c["K"])
        assert got == (c["llm_response"], c["actions"])
