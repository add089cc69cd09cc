"""The host analysis behind the prompt encoder's expansions (llm_agent/prompts.py
ExpansionSplitter): for the constant stretches of the real prompt programs, the chosen middle
must tokenize the same whatever text surrounds the stretch --
ids(L + X + R) == ids(L + X[:q1]) + ids_mid + ids(X[q2:] + R) -- checked here on random
contexts far beyond the analysis' own probes (random mixes of letters, digits, punctuation,
whitespace, newlines, non-ASCII), with the Qwen2-pipeline byte-level BPE and the character
tokenizer of the tests."""
import random

import pytest

from fake_tok import FakeQwenTok
from ragen_amd import synthetic
from ragen_amd.config import default_config
from ragen_amd.llm_agent.prompts import ChatTemplate, ExpansionSplitter, format_prompt

ALPHABET = list("abcXYZ019 _.,<>'\"-#|\t\n\r") + [" ", "　", "é", "中", "😀", "½", "'s", "'re", "</answer>",
                                                 "<|im_end|>", "  ", "\n\n"]


def _rand(rng, n):
    return "".join(rng.choice(ALPHABET) for _ in range(n))


def _stretches(tok):
    cfg = default_config()
    tpl = ChatTemplate(tok)
    instr = cfg.custom_envs.SimpleSokoban.env_instruction
    c_mid = f" actions left. Always output: {format_prompt(True)} with no extra text. Strictly follow this format. "
    length = "Max response length: 100 words (tokens)."
    return [(tpl.head + instr + "\nTurn 1:\nState:\n", False),
            (c_mid + length + "\n" + tpl.u_suf, True),
            (tpl.a_pre, False),
            (tpl.u_pre + "Reward:\n", False),
            ("\n\nTurn 3:\nState:\n", False)]


@pytest.fixture(scope="module", params=["qwen", "fake"])
def tok(request):
    return synthetic.qwen_like_tokenizer() if request.param == "qwen" else FakeQwenTok()


def test_expansion_middles_are_context_free(tok):
    sp = ExpansionSplitter.for_tokenizer(tok)
    bt = tok.backend_tokenizer
    ids = lambda t: bt.encode(t, add_special_tokens=False).ids  # noqa: E731
    rng = random.Random(11)
    found = 0
    for x, right_free in _stretches(tok):
        r = sp.split(x, right_free)
        if r is None:
            continue
        found += 1
        q1, mid, q2 = r
        assert 0 <= q1 < q2 <= len(x) and mid == ids(x)[len(ids(x[:q1])):len(ids(x)) - len(ids(x[q2:]))]
        for _ in range(300):
            L = _rand(rng, rng.randint(0, 6))
            R = "" if right_free else _rand(rng, rng.randint(0, 6))
            assert ids(L + x + R) == ids(L + x[:q1]) + mid + ids(x[q2:] + R), (x, L, R)
    assert found >= 3  # the long stretches (instruction prefix, format / length lines) split


def test_expansion_long_stretch_mostly_skipped(tok):
    sp = ExpansionSplitter.for_tokenizer(tok)
    x, right_free = _stretches(tok)[0]
    q1, mid, q2 = sp.split(x, right_free)
    assert (q2 - q1) >= 0.9 * len(x)
