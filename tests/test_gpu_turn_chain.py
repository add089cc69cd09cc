"""The turn chain (rmi_turn_chain, llm_agent/turn_chain.py: one call per device turn) and the
formulate chain (rmi_formulate_stats + rmi_formulate_chain) against the step-by-step forms
(EnvStateManager._device_pass, ContextManager.formulate_device: the same kernels launched one by
one from Python, the normalisation and reductions as torch ops): LLMAgentProxy.rollout both ways on the golden traces' configs (Sokoban 6x6,
Sokoban 8x8 with 2 boxes, FrozenLake), with the character tokenizer and the Qwen2-pipeline BPE,
and on the bench's 8192-env workload -- every turn's generation batch, the formulated batch,
its metrics and the rollout cache identical, the chain taken on every turn, its per-turn buffers
reused by a second rollout."""
import random

import numpy as np
import pytest
import torch

from fake_tok import FakeQwenTok
from ragen_amd import ops, synthetic
from ragen_amd.llm_agent import EnvStateManager, LLMAgentProxy, TokenActor
from ragen_amd.llm_agent.ctx_manager import ContextManager
from ragen_amd.protocol import DataProto
from test_gpu_device_prompts import _ids, _responses, _vocab
from test_gpu_facade import TRACES, _config, _hashseed0_reseed

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def qwen_tok():
    return synthetic.qwen_like_tokenizer()


def _run(cfg, tok, turn_tokens, device, chain, reps=1, seed=7):
    EnvStateManager.use_turn_chain = chain
    ContextManager.use_formulate_chain = chain
    try:
        actor = TokenActor(turn_tokens, read_prompts=True)
        proxy = LLMAgentProxy(cfg, actor, tok, device=device)
        proxy.train_ctx_manager.set_device_vocab(_vocab(tok, device))
        random.seed(seed)
        outs = []
        for _ in range(reps):
            actor.prompts = []
            out = proxy.rollout(DataProto(meta_info={}), val=False)
            prompts = [tuple(x.cpu() for x in p) for p in actor.prompts]
            outs.append((out, prompts, proxy.train_es_manager.rollout_cache, dict(out.meta_info)))
        ch = proxy.train_es_manager.__dict__.get("_chain")
        fc = proxy.train_ctx_manager.__dict__.get("_fchain")
        assert (fc.runs if fc is not None else 0) == (reps if chain else 0)  # every formulate chained (or none)
        return outs, (ch.runs if ch is not None else 0), proxy
    finally:
        EnvStateManager.use_turn_chain = True
        ContextManager.use_formulate_chain = True


def _same(a, b):
    out_a, pr_a, rc_a, meta_a = a
    out_b, pr_b, rc_b, meta_b = b
    assert len(pr_a) == len(pr_b)
    for t, (x, y) in enumerate(zip(pr_a, pr_b)):
        for k, u, v in zip(("input_ids", "attention_mask", "position_ids"), x, y):
            assert torch.equal(u, v), (t, k)
    assert set(out_a.batch.keys()) == set(out_b.batch.keys())
    for k in out_a.batch.keys():
        assert torch.equal(out_a.batch[k].cpu(), out_b.batch[k].cpu()), k
    assert meta_a == meta_b
    assert rc_a == rc_b


@pytest.mark.parametrize("which", ["fake", "qwen"])
@pytest.mark.parametrize("name", ["sokoban_es", "sokoban8_es", "frozenlake_es"])
def test_turn_chain_equals_step_by_step(device, name, which, qwen_tok, monkeypatch):
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    tok = FakeQwenTok() if which == "fake" else qwen_tok
    cfg = _config(name)
    _, ng, gs, T, _ = TRACES[name]
    B = ng * gs
    turn_tokens = [_ids(tok, _responses(name, t, B), device) for t in range(T)]
    chained, runs, proxy = _run(cfg, tok, turn_tokens, device, True, reps=2)
    plain, runs0, _ = _run(cfg, tok, turn_tokens, device, False, reps=2)
    assert runs0 == 0
    n_turns = sum(len(o[1]) for o in chained)
    assert runs == n_turns, (runs, n_turns)  # every turn of both rollouts went through the chain
    for a, b in zip(chained, plain):
        _same(a, b)
    # generation batches of the second rollout were padded by the chain (the first's blocks free)
    assert proxy.train_es_manager._chain.padded > 0
    assert proxy.train_ctx_manager.prompts().host_rows_used == 0


def test_turn_chain_bench_workload(device):
    """The API leg's workload (8192 Sokoban envs x 5 turns, 10 % unknown action names, the
    Qwen2-pipeline BPE): two rollouts chained == step by step."""
    from ragen_amd.config import env_task
    B, T, K = 8192, 5, 5
    cfg = env_task("SimpleSokoban", B // 16, 16, max_turn=T, max_actions_per_turn=K)
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4)
    lk = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}
    tok = synthetic.qwen_like_tokenizer()
    tokens = []
    for t in range(T):
        enc = tok(synthetic.responses_for_actions(ids[t], n[t], lk, seed=100 + t), padding=False).input_ids
        R = max(len(x) for x in enc)
        a = np.full((B, R), tok.pad_token_id, np.int64)
        for i, x in enumerate(enc):
            a[i, :len(x)] = x
        tokens.append(torch.from_numpy(a).to(device))
    chained, runs, proxy = _run(cfg, tok, tokens, device, True, reps=2, seed=0)
    plain, _, _ = _run(cfg, tok, tokens, device, False, reps=2, seed=0)
    assert runs == sum(len(o[1]) for o in chained)
    # the second rollout's batches after the first turn were padded by the chain and taken
    assert proxy.train_es_manager._chain.padded == len(chained[1][1]) - 1
    assert proxy.train_ctx_manager.prompts().chain_padded == len(chained[1][1]) - 1
    for a, b in zip(chained, plain):
        _same(a, b)


def test_reward_text_cache_refuses_torn_entries(device, qwen_tok, monkeypatch):
    """The chained prompt launches' reward text cache (rmi_prompt_t.num_cache) is write-once and
    exact: after the first rollout, half of the cached entries lose a text word (as a reader would
    see an entry whose text is not yet visible: a zero byte below the length) and the other half
    their key (another value's slot); the second rollout prints the same prompts as the
    step-by-step path (every such entry is a miss and the row computes its text), and no claimed
    slot is written again (the altered entries are still as altered)."""
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    name = "sokoban_es"
    cfg = _config(name)
    _, ng, gs, T, _ = TRACES[name]
    turn_tokens = [_ids(qwen_tok, _responses(name, t, ng * gs), device) for t in range(T)]
    plain, _, _ = _run(cfg, qwen_tok, turn_tokens, device, False, reps=2)
    actor = TokenActor(turn_tokens, read_prompts=True)
    proxy = LLMAgentProxy(cfg, actor, qwen_tok, device=device)
    proxy.train_ctx_manager.set_device_vocab(_vocab(qwen_tok, device))
    random.seed(7)
    outs = []
    altered = None
    for rep in range(2):
        if rep == 1:
            nc = proxy.train_ctx_manager.prompts().num_cache.view(-1, 16)
            ready = torch.nonzero(nc[:, 2] < 0).flatten()  # the ready bit
            assert ready.numel() > 1  # the first rollout cached its rewards' text
            torn, foreign = ready[0::2], ready[1::2]
            nc[torn, 3] = 0                  # the text's first word not visible
            nc[foreign, 0] ^= 0x00010000     # another value's key
            altered = nc.clone()
        actor.prompts = []
        out = proxy.rollout(DataProto(meta_info={}), val=False)
        outs.append((out, [tuple(x.cpu() for x in p) for p in actor.prompts], proxy.train_es_manager.rollout_cache,
                     dict(out.meta_info)))
    nc = proxy.train_ctx_manager.prompts().num_cache.view(-1, 16)
    assert torch.equal(nc[ready], altered[ready]), "a claimed slot was written again"
    for a, b in zip(outs, plain):
        _same(a, b)


def test_turn_chain_decode_overflow_second_pass(device, monkeypatch):
    """A later turn's generations longer than the decode's row hint (the longest generation seen
    so far, with a margin): after the chained turn has run its whole chain for every env, the
    overflowed envs are masked out of that pass and stepped by a second pass
    (EnvStateManager._step_device).  Chained == step by step -- every generation batch, the
    formulated batch, its metrics and the rollout cache -- and the second pass ran in both."""
    from ragen_amd.env import SokobanBatch
    from ragen_amd.llm_agent import es_manager as esm
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    tok = FakeQwenTok()
    name = "sokoban_es"
    cfg = _config(name)
    _, ng, gs, T, _ = TRACES[name]
    B = ng * gs
    turn_tokens = []
    for t in range(T):
        texts = _responses(name, t, B)
        if t == 2:  # every third env thinks at length: ~5x the longest generation of turns 0-1
            texts = [("let me think " * 30 + x) if i % 3 == 0 else x for i, x in enumerate(texts)]
        turn_tokens.append(_ids(tok, texts, device))
    seconds = []
    real = esm.EnvStateManager._device_pass

    def counting(self, inp, t, first, *a, **kw):
        if first is not None:
            seconds.append(t)
        return real(self, inp, t, first, *a, **kw)

    monkeypatch.setattr(esm.EnvStateManager, "_device_pass", counting)
    chained, runs, _ = _run(cfg, tok, turn_tokens, device, True, reps=1)
    n_chain = len(seconds)
    plain, runs0, _ = _run(cfg, tok, turn_tokens, device, False, reps=1)
    assert runs == len(chained[0][1]) and runs0 == 0
    assert n_chain == 1 and seconds == [2, 2], seconds  # turn 2 took the second pass, both ways
    _same(chained[0], plain[0])
