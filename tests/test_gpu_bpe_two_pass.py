"""The two-pass form of rmi_bpe_encode (the pre-tokenizer pass, the word pass, the one-kernel
pass over the rows the word pass flags; csrc/bpe.hip) against the one-kernel form and the
`tokenizers` library: every tests/tok_cases.py case and fuzz, with the word cache cold (every
word a miss: trips whose misses outgrow the word pass's scratch go to the retry pass), warm
(every word a hit), and off (every word merged in the word pass's scratch or retried)."""
import pytest
import torch

from ragen_amd import synthetic
from ragen_amd.tokenizer import DeviceTokenizer
from tok_cases import EDGE, fuzz

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def qwen_tok():
    return synthetic.qwen_like_tokenizer()


def test_two_pass_equals_one_kernel_and_tokenizers(device, qwen_tok):
    back = qwen_tok.backend_tokenizer
    prompt = ("<|im_start|>user\nYou are solving the Sokoban puzzle.\nTurn 1:\nState:\n######\n#_P_O#\n#__√_#\n"
              "######\nYou have 10 actions left. Reward:\n-0.30000000000000004\n<|im_end|>\n<|im_start|>assistant\n"
              "<think>push the box right, then up; supercalifragilisticexpialidocious words</think>"
              "<answer>Right || Up</answer><|im_end|>\n")
    # rows of 64+ distinct long words: a cold trip's misses outgrow the word pass's scratch
    import random
    rnd = random.Random(3)
    long_rows = [" ".join("".join(rnd.choice("abcdefghijklmnopqrstuvwxyz") for _ in range(rnd.randint(6, 14)))
                          for _ in range(90)) for _ in range(64)]
    cases = EDGE + fuzz(2000, seed=21) + [prompt] * 1024 + long_rows
    want = [back.encode(s, add_special_tokens=False).ids for s in cases]
    dt = DeviceTokenizer.from_hf(qwen_tok, device)
    for run in ("cold", "warm"):
        got = dt.encode(cases, two_pass=True)
        assert got == want, run
        if run == "cold":
            # the cold launch sent rows to the retry pass (trips of 64 misses outgrow 256 bytes)
            assert int(dt.pre[3][:len(cases)].sum()) > 0
    # warm: every row but the random-word ones (words of more ids than a cache entry holds, so
    # never cached) finished in the word pass
    assert int(dt.pre[3][:len(cases) - len(long_rows)].sum()) == 0
    assert dt.encode(cases) == want  # the one-kernel form on the same tables
    off = DeviceTokenizer.from_hf(qwen_tok, device)
    off.word_cache = None
    assert off.encode(cases, two_pass=True) == want


def test_two_pass_flags_like_one_kernel(device, qwen_tok):
    """Rows the pre-tokenizer pass fails (invalid UTF-8 is not text here: NFC-unsafe code points)
    and rows past the row bound are flagged the same way by both forms."""
    from tok_cases import nfc_unsafe
    dt = DeviceTokenizer.from_hf(qwen_tok, device)
    rows = nfc_unsafe() + ["plain text", "x" * 50]
    assert dt.encode(rows, two_pass=True) == dt.encode(rows)


def test_turn_chain_with_the_two_pass_bpe(device, qwen_tok, monkeypatch):
    """The turn chain with its BPE launch in the two-pass form == the step-by-step rollout (the
    one-kernel form) on a golden-trace config: every generation batch and the formulated batch."""
    from ragen_amd.env import SokobanBatch
    from ragen_amd.llm_agent.turn_chain import TurnChain
    from test_gpu_device_prompts import _ids, _responses
    from test_gpu_facade import TRACES, _config, _hashseed0_reseed
    from test_gpu_turn_chain import _run, _same
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    monkeypatch.setattr(TurnChain, "two_pass_bpe", True)
    name = "sokoban_es"
    cfg = _config(name)
    _, ng, gs, T, _ = TRACES[name]
    turn_tokens = [_ids(qwen_tok, _responses(name, t, ng * gs), device) for t in range(T)]
    chained, runs, proxy = _run(cfg, qwen_tok, turn_tokens, device, True, reps=2)
    plain, _, _ = _run(cfg, qwen_tok, turn_tokens, device, False, reps=2)
    assert runs == sum(len(o[1]) for o in chained)
    assert proxy.train_ctx_manager.prompts().dt.pre is not None  # the chain took the two-pass form
    for a, b in zip(chained, plain):
        _same(a, b)
