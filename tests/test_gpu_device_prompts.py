"""The device prompt path (§8(f) ranks 1-2, llm_agent/prompts.py) against the reference's host
path (ctx_manager.py:228-330: chat template + tokenizer over the whole history each turn) on
the configs and actions of all five golden traces, with the character tokenizer FakeQwenTok
and the Qwen2-pipeline byte-level BPE: every turn's generation batch (input_ids,
attention_mask, position_ids) read by an actor, the formulated batch, its metrics, env ids,
messages and the rollout cache must be identical.  A second test drives responses through
every branch of the response rebuild (no match, the special-token cascade, more than K actions,
whitespace and non-ASCII text, NFC-changing text and overlong rows built on the host)."""
import random

import numpy as np
import pytest
import torch

from fake_tok import FakeQwenTok
from ragen_amd import ops, synthetic
from ragen_amd.llm_agent import LLMAgentProxy, TokenActor
from ragen_amd.protocol import DataProto
from test_gpu_facade import TRACES, _config, _hashseed0_reseed
from trace_util import load, strings

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def qwen_tok():
    return synthetic.qwen_like_tokenizer()


def _responses(name, t, B):
    d = load(name)
    S = strings()[name]
    out = []
    for i in range(B):
        if name == "countdown_es":
            a = S["answers"][t][i]
            acts = [] if a is None else [a]
        else:
            acts = [S["vocab"][c] for c in d["codes"][t, i] if c >= 0]
        out.append(f"thinking about turn {t}</think> <answer>{' || '.join(acts)}</answer>")
    return out


def _ids(tok, texts, device):
    rows = [tok._ids(x) if isinstance(tok, FakeQwenTok) else tok(x).input_ids for x in texts]
    R = max(len(x) for x in rows)
    pad = tok.pad_token_id
    a = np.full((len(rows), R), pad, np.int64)
    for i, x in enumerate(rows):
        a[i, :len(x)] = x
    return torch.from_numpy(a).to(device)


def _vocab(tok, device):
    if isinstance(tok, FakeQwenTok):
        return ops.VocabTable.from_bytes(*tok.byte_table(), device)
    return ops.VocabTable.from_tokenizer(tok, device)


def _rollout(cfg, tok, turn_tokens, device, device_path):
    actor = TokenActor(turn_tokens, read_prompts=True)
    proxy = LLMAgentProxy(cfg, actor, tok, device=device)
    if device_path:
        proxy.train_ctx_manager.set_device_vocab(_vocab(tok, device))
    random.seed(7)
    out = proxy.rollout(DataProto(meta_info={}), val=False)
    prompts = [tuple(x.cpu() for x in p) for p in actor.prompts]
    return out, proxy, prompts


def _compare(ref, dev, ref_prompts, dev_prompts, ref_proxy, dev_proxy):
    assert len(ref_prompts) == len(dev_prompts)
    for t, (a, b) in enumerate(zip(ref_prompts, dev_prompts)):
        for k, x, y in zip(("input_ids", "attention_mask", "position_ids"), a, b):
            assert torch.equal(x, y), (t, k)
    assert set(ref.batch.keys()) == set(dev.batch.keys())
    for k in ref.batch.keys():
        assert torch.equal(ref.batch[k].cpu(), dev.batch[k].cpu()), k
    assert ref.meta_info == dev.meta_info
    for k in ("env_ids", "group_ids", "messages_list"):
        assert np.asarray(ref.non_tensor_batch[k]).tolist() == np.asarray(dev.non_tensor_batch[k]).tolist(), k
    assert ref_proxy.train_es_manager.rollout_cache == dev_proxy.train_es_manager.rollout_cache


@pytest.mark.parametrize("which", ["fake", "qwen"])
@pytest.mark.parametrize("name", list(TRACES))
def test_device_prompts_equal_host_prompts(device, name, which, qwen_tok, monkeypatch):
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    tok = FakeQwenTok() if which == "fake" else qwen_tok
    cfg = _config(name)
    _, ng, gs, T, _ = TRACES[name]
    B = ng * gs
    turn_tokens = [_ids(tok, _responses(name, t, B), device) for t in range(T)]
    ref, ref_proxy, ref_prompts = _rollout(cfg, tok, turn_tokens, device, False)
    dev, dev_proxy, dev_prompts = _rollout(cfg, tok, turn_tokens, device, True)
    pr = dev_proxy.train_ctx_manager.prompts()
    assert pr is not None and pr.host_rows_used == 0
    assert dev.batch["input_ids"].is_cuda  # the device path's batch stays on the GPU
    _compare(ref, dev, ref_prompts, dev_prompts, ref_proxy, dev_proxy)


EDGE_RESPONSES = [
    "no tags at all here",                                               # no match: the raw response
    "a</think><answer>Up || Down</answer>",                              # plain
    "  spaced thoughts \t</think>\n  <answer>  Left  ||  Right  </answer>",  # strips
    "x</think><answer>Up || Down || Left || Right || Up || Down || Left</answer>",  # > K: re-joined
    "t</think><answer>Up||||Down|| ||Left</answer>",                      # empty pieces
    "<think>nested</think></think><answer>Up <|im_end|> || Down</answer>",  # special-token cascade
    "a</think><answer><answer>Right</answer></answer>",                  # cascade in the answer
    "café — naïve 中文 😀</think><answer>Up</answer>",                    # non-ASCII
    "u v　</think><answer> Down </answer>",            # Unicode whitespace strips
    "e\u0301 combining</think><answer>Up</answer>",               # NFC-changing: host row
    "long " * 700 + "</think><answer>Up</answer>",                        # past the row buffer: host row
    "a</think><answer></answer>",                                         # empty answer
    "only answer <answer>Left</answer>",                                  # missing </think>
]


@pytest.mark.parametrize("think", [True, False])
def test_device_prompts_response_branches(device, qwen_tok, think, monkeypatch):
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    cfg = _config("sokoban_es")
    cfg.agent_proxy.enable_think = think
    _, ng, gs, T, _ = TRACES["sokoban_es"]
    B = ng * gs
    rng = np.random.default_rng(3)
    turn_tokens = []
    for t in range(T):
        texts = [EDGE_RESPONSES[int(rng.integers(len(EDGE_RESPONSES)))] for _ in range(B)]
        if not think:  # the generation continues after "<answer>": the thoughts become answer text
            texts = [(x.split("</think>")[0] + " " + x.split("</think>")[1].replace("<answer>", "", 1))
                     if "</think>" in x else x for x in texts]
        turn_tokens.append(_ids(qwen_tok, texts, device))
    ref, ref_proxy, ref_prompts = _rollout(cfg, qwen_tok, turn_tokens, device, False)
    with pytest.warns(RuntimeWarning, match="prompt rows built on the host"):
        dev, dev_proxy, dev_prompts = _rollout(cfg, qwen_tok, turn_tokens, device, True)
    assert dev_proxy.train_ctx_manager.prompts().host_rows_used > 0
    _compare(ref, dev, ref_prompts, dev_prompts, ref_proxy, dev_proxy)


@pytest.mark.parametrize("grouping", ["inductive", "batch"])
def test_device_formulate_groupings_repeated_tag(device, grouping, monkeypatch):
    """formulate_rollouts' reward normalisation on the device path (ContextManager.
    _normalize_device) == the host path (segments_for over the per-env tags,
    ctx_manager.py:184-191) with mean_std on a config that lists a tag twice: the reference
    groups "inductive" by tag NAME, so SimpleSokoban's two entries are one group."""
    from ragen_amd.config import AttrDict
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    cfg = _config("sokoban_es")
    ec = cfg.es_manager.train.env_configs
    ec.tags, ec.n_groups = ["SimpleSokoban", "LargerSokoban", "SimpleSokoban"], [3, 2, 3]
    cfg.agent_proxy.reward_normalization = AttrDict(grouping=grouping, method="mean_std")
    tok = FakeQwenTok()
    _, ng, gs, T, _ = TRACES["sokoban_es"]
    B = ng * gs
    turn_tokens = [_ids(tok, _responses("sokoban_es", t, B), device) for t in range(T)]
    ref, ref_proxy, ref_prompts = _rollout(cfg, tok, turn_tokens, device, False)
    dev, dev_proxy, dev_prompts = _rollout(cfg, tok, turn_tokens, device, True)
    assert dev_proxy.train_ctx_manager.prompts() is not None
    sc = ref.batch["rm_scores"][:, -1].cpu()
    if grouping == "inductive":  # the two SimpleSokoban entries normalised together: mean 0 over both
        sok = torch.cat([torch.arange(0, 48), torch.arange(80, 128)])
        assert abs(float(sc[sok].double().mean())) < 1e-5
    _compare(ref, dev, ref_prompts, dev_prompts, ref_proxy, dev_proxy)


@pytest.mark.parametrize("k", [1, 2])
@pytest.mark.parametrize("name", list(TRACES))
def test_device_prompts_context_window(device, name, k, monkeypatch):
    """agent_proxy.max_context_window = k (ctx_manager.py:244-246: the last k history entries,
    renumbered Turn 1..k) on the device path: every turn's generation batch, the formulated
    batch, its metrics and messages == the host path, on all five golden traces; the device
    rows are rebuilt on the device (no host rows)."""
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    tok = FakeQwenTok()
    cfg = _config(name)
    cfg.agent_proxy.max_context_window = k
    _, ng, gs, T, _ = TRACES[name]
    B = ng * gs
    turn_tokens = [_ids(tok, _responses(name, t, B), device) for t in range(T)]
    ref, ref_proxy, ref_prompts = _rollout(cfg, tok, turn_tokens, device, False)
    dev, dev_proxy, dev_prompts = _rollout(cfg, tok, turn_tokens, device, True)
    pr = dev_proxy.train_ctx_manager.prompts()
    assert pr is not None and pr.window == k and pr.host_rows_used == 0
    _compare(ref, dev, ref_prompts, dev_prompts, ref_proxy, dev_proxy)
    # the window holds at most k turns (test_context_window.py:60-84's assertion, per env)
    for msgs in dev.non_tensor_batch["messages_list"]:
        text = " ".join(m["content"] for m in msgs)
        assert text.count("\nTurn ") <= k and f"\nTurn {k + 1}:" not in text


def test_device_prompts_context_window_qwen_bpe(device, qwen_tok, monkeypatch):
    """The window rebuild with the Qwen2-pipeline byte-level BPE (rmi_bpe_encode) on the longest
    trace, k = 2."""
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    cfg = _config("frozenlake_es")
    cfg.agent_proxy.max_context_window = 2
    _, ng, gs, T, _ = TRACES["frozenlake_es"]
    B = ng * gs
    turn_tokens = [_ids(qwen_tok, _responses("frozenlake_es", t, B), device) for t in range(T)]
    ref, ref_proxy, ref_prompts = _rollout(cfg, qwen_tok, turn_tokens, device, False)
    dev, dev_proxy, dev_prompts = _rollout(cfg, qwen_tok, turn_tokens, device, True)
    assert dev_proxy.train_ctx_manager.prompts().host_rows_used == 0
    _compare(ref, dev, ref_prompts, dev_prompts, ref_proxy, dev_proxy)


@pytest.mark.parametrize("which", ["fake", "qwen"])
def test_device_turn_decode_overflow_second_pass(device, which, qwen_tok, monkeypatch):
    """The device turn's one readback: the decode's row comes from a hint (the longest generation
    seen), and generations longer than it overflow the first pass, are masked out of it and are
    stepped by a second pass over those envs (EnvStateManager._step_device).  With the hint
    pinned far below every generation each turn takes both passes; the rollout must still equal
    the host path exactly.  Without the pin, the readbacks are one per turn (+ the first turn's
    decode size and the first generation batch's row stats)."""
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    tok = FakeQwenTok() if which == "fake" else qwen_tok
    name = "sokoban_es"
    cfg = _config(name)
    _, ng, gs, T, _ = TRACES[name]
    B = ng * gs
    rng = np.random.default_rng(11)
    texts = [[r + " pad" * int(rng.integers(0, 40)) for r in _responses(name, t, B)] for t in range(T)]
    turn_tokens = [_ids(tok, texts[t], device) for t in range(T)]
    ref, ref_proxy, ref_prompts = _rollout(cfg, tok, turn_tokens, device, False)
    # pinned hint: every turn overflows
    actor = TokenActor(turn_tokens, read_prompts=True)
    proxy = LLMAgentProxy(cfg, actor, tok, device=device)
    proxy.train_ctx_manager.set_device_vocab(_vocab(tok, device))
    proxy.train_ctx_manager._raw_hint_pin = 24
    random.seed(7)
    dev = proxy.rollout(DataProto(meta_info={}), val=False)
    _compare(ref, dev, ref_prompts, [tuple(x.cpu() for x in p) for p in actor.prompts], ref_proxy, proxy)
    assert proxy.last_timing["readbacks"]["turns"] >= 2 * len(actor.prompts)
    # free hint: one readback per turn from the second rollout on
    proxy.train_ctx_manager._raw_hint_pin = None
    for _ in range(2):
        actor.turn, actor.prompts, actor.prompt_shapes = 0, [], []
        random.seed(7)
        dev = proxy.rollout(DataProto(meta_info={}), val=False)
    _compare(ref, dev, ref_prompts, [tuple(x.cpu() for x in p) for p in actor.prompts], ref_proxy, proxy)
    n_turns = len(actor.prompts)
    assert proxy.last_timing["readbacks"]["turns"] == n_turns + 1, proxy.last_timing


def test_gen_batch_takes_eager_stats_only_for_the_counted_ids(device, qwen_tok, monkeypatch):
    """The next batch's row stats come back with the turn (advance_eager) for exactly the env-id
    array the turn handed out; gen_batch given any other array (even an equal copy) reads the
    stats back itself -- and builds the same batch."""
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    name = "sokoban_es"
    cfg = _config(name)
    _, ng, gs, T, _ = TRACES[name]
    B = ng * gs
    turn_tokens = [_ids(qwen_tok, _responses(name, t, B), device) for t in range(T)]
    batches, counts = [], []
    for copy_ids in (False, True):
        proxy = LLMAgentProxy(cfg, TokenActor(turn_tokens), qwen_tok, device=device)
        ctx, es = proxy.train_ctx_manager, proxy.train_es_manager
        ctx.set_device_vocab(_vocab(qwen_tok, device))
        env_outputs = es.reset(seed=11)
        out = []
        for t in range(2):
            lm = ctx.get_lm_inputs(env_outputs, prepare_for_update=False)
            out.append(lm.batch["input_ids"].cpu())
            env_outputs = es.step(ctx.get_env_inputs(proxy.generate_sequences(lm)))
        ids = env_outputs.env_ids.copy() if copy_ids else env_outputs.env_ids
        c0 = ops.D2H_COUNT[0]
        out.append(ctx.prompts().gen_batch(ids)["input_ids"].cpu())
        counts.append(ops.D2H_COUNT[0] - c0)
        batches.append(out)
    assert counts == [0, 1]
    for a, b in zip(*batches):
        assert torch.equal(a, b)
