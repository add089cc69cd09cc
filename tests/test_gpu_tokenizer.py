"""rmi_bpe_encode (csrc/bpe.hip) against the `tokenizers` library — the tokenizer call of
ContextManager.get_lm_inputs (ctx_manager.py:265-278) — on the synthetic Qwen2-pipeline BPE
and the character-level FakeQwenTok: every case of tests/tok_cases.py (regex corners, added
tokens, Unicode classes, runs past the kernel's 64-byte view), fuzz at full batch size,
appending into an arena (out_len), the mark position, and the rows the kernel flags
(NFC-unsafe code points, rows past out_stride)."""
import numpy as np
import pytest
import torch

from fake_tok import FakeQwenTok
from ragen_amd import _lib, synthetic
from ragen_amd.tokenizer import DeviceTokenizer
from tok_cases import EDGE, fuzz, nfc_unsafe

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def qwen_tok():
    return synthetic.qwen_like_tokenizer()


def _cases(which):
    cases = EDGE + fuzz(3000, seed=5)
    if which == "fake":
        cases = [s for s in cases if all(ord(c) < 0x10000 for c in s)]
    return cases


@pytest.mark.parametrize("which", ["qwen", "fake"])
def test_encode_matches_tokenizers(device, qwen_tok, which):
    tok = qwen_tok if which == "qwen" else FakeQwenTok()
    dt = DeviceTokenizer.from_hf(tok, device)
    cases = _cases(which)
    got = dt.encode(cases)
    back = tok.backend_tokenizer
    for s, g in zip(cases, got):
        assert g == back.encode(s, add_special_tokens=False).ids, repr(s)


def test_encode_prompts_and_flags(device, qwen_tok):
    dt = DeviceTokenizer.from_hf(qwen_tok, device)
    msgs = [{"role": "system", "content": "You're a helpful assistant. "},
            {"role": "user", "content": "You are solving the Sokoban puzzle.\nTurn 1:\nState:\n######\n#_P_O#\n"
                                        "#__X_#\n######\nYou have 10 actions left. Always output: <think> [Your "
                                        "thoughts] </think> <answer> [your answer] </answer> with no extra text."},
            {"role": "assistant", "content": "<think>push it right</think><answer>Right || Up</answer>"},
            {"role": "user", "content": "Reward:\n-0.30000000000000004\n\nTurn 2:\nState:\n#__√_#\n"}]
    text = qwen_tok.apply_chat_template(msgs, add_generation_prompt=True, tokenize=False) + "<think>"
    assert dt.encode([text])[0] == qwen_tok(text).input_ids
    flagged = dt.encode(nfc_unsafe() + ["plain"])
    assert all(g is None for g in flagged[:-1]) and flagged[-1] == qwen_tok("plain").input_ids


def test_encode_append_mark_and_overflow(device, qwen_tok):
    """Rows appended at out_len (an arena), mark_byte -> mark_tok, a row past out_stride flagged
    and left unwritten."""
    dt = DeviceTokenizer.from_hf(qwen_tok, device)
    a = ["<|im_start|>user\nhello there<|im_end|>\n", "x", "<|im_start|>assistant\n<think>ok</think>"]
    b = ["<|im_start|>user\nReward:\n1.0\n<|im_end|>\n<|im_start|>assistant\n", "yy zz", "q" * 600]
    B, cap = len(a), 256
    out = torch.full((B, cap), -7, dtype=torch.int64, device=device)
    out_len = torch.zeros(B, dtype=torch.int32, device=device)

    def rows(texts):
        bs = [t.encode() for t in texts]
        st = (max(len(x) for x in bs) + 3) // 4 * 4
        buf = np.zeros((len(bs), st), np.uint8)
        for i, x in enumerate(bs):
            buf[i, :len(x)] = np.frombuffer(x, np.uint8)
        return torch.from_numpy(buf).to(device), torch.tensor([len(x) for x in bs], dtype=torch.int32, device=device)
    t1, l1 = rows(a)
    dt.encode_rows(t1, l1, out, out_len)
    t2, l2 = rows(b)
    mark = torch.tensor([b[0].index("<|im_start|>assistant"), 2, 0], dtype=torch.int32, device=device)
    n_tok, mark_tok, err = dt.encode_rows(t2, l2, out, out_len, mark)
    ol, o, e = out_len.cpu().tolist(), out.cpu().numpy(), err.cpu().tolist()
    enc = lambda s: qwen_tok(s).input_ids  # noqa: E731
    for i in range(2):
        exp = enc(a[i]) + enc(b[i])
        assert ol[i] == len(exp) and o[i, :ol[i]].tolist() == exp and e[i] == 0
    assert mark_tok.cpu().tolist()[0] == len(enc(a[0])) + len(enc(b[0][:mark[0].item()]))
    assert e[2] == _lib.ERR_UNSUP and ol[2] == len(enc(a[2]))  # 600 q's do not fit after row 2's first tokens
    assert (o[2, ol[2]:] == -7).all()


def test_word_cache_warm_cold_and_torn(device, qwen_tok):
    """The word cache (rmi_bpe_t.word_cache): the same rows encoded cold (cache empty, words
    inserted by many waves at once), warm (every word found) and with the cache off give the
    tokenizers library's ids.  Entries are written once and read exactly: an entry in the state
    a reader can see of a half-written one -- its first id or its first key word still zero --
    is a miss, not used, and no claimed slot is written again."""
    back = qwen_tok.backend_tokenizer
    cases = EDGE + fuzz(1500, seed=9)
    text = ("<|im_start|>user\nYou are solving the Sokoban puzzle.\nTurn 1:\nState:\n######\n#_P_O#\n#__X_#\n"
            "######\nYou have 10 actions left. Always output: <think> [Your thoughts] </think> <answer> [your "
            "answer] </answer> with no extra text.<|im_end|>\n")
    rows = cases + [text] * 4096  # the same words in thousands of rows of one launch
    want = [back.encode(s, add_special_tokens=False).ids for s in cases + [text]]
    want += want[-1:] * 4095
    dt = DeviceTokenizer.from_hf(qwen_tok, device)
    assert dt.word_cache is not None
    for run in ("cold", "warm"):
        got = dt.encode(rows)
        assert got == want, run
    wc = dt.word_cache.view(-1, 16)
    ready = torch.nonzero(wc[:, 4] < 0).flatten()  # the ready bit (bit 31)
    assert ready.numel() > 100
    wc[ready[0::2], 5] = 0  # the first id not visible yet
    wc[ready[1::2], 0] = 0  # the first key word not visible yet
    altered = wc.clone()
    assert dt.encode(rows) == want
    assert torch.equal(wc[ready], altered[ready]), "a claimed slot was written again"
    off = DeviceTokenizer.from_hf(qwen_tok, device)
    off.word_cache = None
    assert off.encode(rows) == want
