"""LLMAgentProxy.rollout on the device path (generations as token ids on the GPU -> device
detokenize -> device parse + turn -> device render, history materialised lazily) against the
dict path (host batch_decode -> regex -> EnvStateManager.step dicts) on the configs and
actions of all five golden traces: the formulated batch, the metrics and every history dict
must be identical."""
import random

import numpy as np
import pytest
import torch

from fake_tok import FakeQwenTok
from ragen_amd import ops
from ragen_amd.llm_agent import LLMAgentProxy, TokenActor
from ragen_amd.protocol import DataProto
from test_gpu_facade import TRACES, _config, _hashseed0_reseed
from trace_util import load, strings

pytestmark = pytest.mark.gpu


def _turn_tokens(name, tok, device):
    d = load(name)
    S = strings()[name]
    B, T = int(d["B"]), int(d["T"])
    rows = []
    for t in range(T):
        texts = []
        for i in range(B):
            if name == "countdown_es":
                a = S["answers"][t][i]
                acts = [] if a is None else [a]
            else:
                acts = [S["vocab"][c] for c in d["codes"][t, i] if c >= 0]
            texts.append(f"thinking about turn {t}</think> <answer>{' || '.join(acts)}</answer>")
        ids = [tok._ids(x) for x in texts]
        R = max(len(x) for x in ids)
        a = np.full((B, R), tok.PAD, np.int64)
        for i, x in enumerate(ids):
            a[i, :len(x)] = x
        rows.append(torch.from_numpy(a).to(device))
    return rows


def _rollout(name, device, vocab):
    tok = FakeQwenTok()
    proxy = LLMAgentProxy(_config(name), TokenActor(_turn_tokens(name, tok, device)), tok, device=device)
    if vocab is not None:
        proxy.train_ctx_manager.set_device_vocab(vocab)
    random.seed(7)
    out = proxy.rollout(DataProto(meta_info={}), val=False)
    return out, proxy.train_es_manager.rollout_cache


@pytest.mark.parametrize("name", list(TRACES))
def test_device_rollout_equals_dict_rollout(device, name, monkeypatch):
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    tok = FakeQwenTok()
    vocab = ops.VocabTable.from_bytes(*tok.byte_table(), device)
    ref, ref_cache = _rollout(name, device, None)
    dev, dev_cache = _rollout(name, device, vocab)
    assert set(ref.batch.keys()) == set(dev.batch.keys())
    for k in ref.batch.keys():
        assert torch.equal(ref.batch[k].cpu(), dev.batch[k].cpu()), k
    assert ref.meta_info == dev.meta_info
    assert list(ref.non_tensor_batch["env_ids"]) == list(dev.non_tensor_batch["env_ids"])
    assert np.asarray(ref.non_tensor_batch["messages_list"]).tolist() == \
        np.asarray(dev.non_tensor_batch["messages_list"]).tolist()
    assert ref_cache == dev_cache


def test_device_step_undecodable_generation_raises_unstepped(device, monkeypatch):
    """A generation the device decode cannot take (an id outside the vocabulary) is masked out
    of the turn on the device and raised from the turn's one readback: ValueError, and that
    env's record is untouched while the others stepped (no host sync before the turn)."""
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    tok = FakeQwenTok()
    rows = _turn_tokens("sokoban_es", tok, device)
    rows[0] = rows[0].clone()
    rows[0][5, 0] = 10 ** 9  # env 5: an id past the vocabulary
    proxy = LLMAgentProxy(_config("sokoban_es"), TokenActor(rows), tok, device=device)
    proxy.train_ctx_manager.set_device_vocab(ops.VocabTable.from_bytes(*tok.byte_table(), device))
    es, ctx = proxy.train_es_manager, proxy.train_ctx_manager
    random.seed(7)
    outs = es.reset()
    lm = ctx.get_lm_inputs(outs, prepare_for_update=False)
    env_inputs = ctx.get_env_inputs(proxy.generate_sequences(lm))
    with pytest.raises(ValueError, match="env 5"):
        es.step(env_inputs)
    n_turns = es.tags[0].batch.ep.n_turns.cpu().numpy()
    assert n_turns[5] == 0 and (np.delete(n_turns, 5) == 1).all()


@pytest.mark.parametrize("draw_between", [False, True])
def test_reset_prefetch_gives_the_same_rooms(device, monkeypatch, draw_between):
    """EnvStateManager.prefetch_next after a reset with a drawn train seed starts the next reset's
    room generation in the background (for the seed random will draw next, peeked without drawing it).  Two resets
    give the same rooms with and without the prefetch, also when random is drawn from in between
    (then the prefetch is for another seed and not taken)."""
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    tok = FakeQwenTok()
    got = {}
    for pf in (False, True):
        proxy = LLMAgentProxy(_config("sokoban_es"), TokenActor(_turn_tokens("sokoban_es", tok, device)), tok,
                              device=device)
        es = proxy.train_es_manager
        es.prefetch_resets = pf
        random.seed(11)
        rooms = []
        for k in range(3):
            es.reset()
            b = es.tags[0].batch
            assert b.reset_prefetched == (pf and k > 0 and not draw_between)
            rooms.append([x.cpu().numpy().copy() for x in (b.room_fixed, b.init_state, b.init_player)])
            es.prefetch_next()  # (LLMAgentProxy.rollout calls it when a rollout is done)
            assert (getattr(b, "_prefetched", None) is not None) == pf
            if draw_between:
                random.random()
        got[pf] = (rooms, random.random())
    for a, b in zip(got[False][0], got[True][0]):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    assert got[False][1] == got[True][1]  # the peek leaves random's sequence alone


def test_load_rooms_equals_load_state(device):
    """rmi_sokoban_load_rooms (the distinct rooms expanded on the device, fused with the reset)
    leaves every env as load_state with the expanded host rooms does; an out-of-range row index
    loads an empty room and flags RMI_ERR_INDEX."""
    from ragen_amd import _lib
    from ragen_amd.env import SokobanBatch
    from ragen_amd.env.configs import SokobanEnvConfig
    B = 1000
    seeds = np.repeat(np.arange(125, dtype=np.int64) + 900, 8)
    cfg = SokobanEnvConfig(num_boxes=1, search_depth=100)
    a = SokobanBatch(cfg, B, 4, 3, device)
    b = SokobanBatch(cfg, B, 4, 3, device)
    for x in (a, b):  # dirty state the reset must overwrite
        x.room_state.fill_(7)
        x.ep.turn_exec.fill_(1)
        x.ep.penalty.fill_(-1)
    a.reset(seeds)
    assert len(SokobanBatch.generate_unique(seeds, 6, 6, 1, 100)[0]) == 125
    b.load_state(*SokobanBatch.generate(seeds, 6, 6, 1, 100))
    for k in ("room_fixed", "room_state", "player", "num_env_steps", "boxes_on_target", "init_state", "init_player"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    for k in ("num_actions", "flags", "n_turns", "penalty", "turn_reward", "turn_info", "turn_exec"):
        assert torch.equal(getattr(a.ep, k), getattr(b.ep, k)), k
    rows, inv = SokobanBatch.generate_unique(seeds, 6, 6, 1, 100)
    room_of = torch.from_numpy(inv.astype(np.int32)).to(device)
    room_of[3] = 125
    err = torch.empty(B, dtype=torch.uint8, device=device)
    ops.sokoban_load_rooms(a.struct(), a.ep, torch.from_numpy(rows).to(device), room_of, a.init_state,
                           a.init_player, err)
    e = err.cpu().numpy()
    assert e[3] == _lib.ERR_INDEX and not np.delete(e, 3).any()
    assert not a.room_state[3].any() and torch.equal(a.room_state[4], b.room_state[4])


@pytest.mark.parametrize("uts", [False, True])
def test_device_formulate_llama3_against_oracle(device, uts, monkeypatch):
    """formulate_rollouts on the device path with a Llama-3 tokenizer (get_special_tokens'
    second branch, ctx_manager.py:27-29: ids 128006 / 128009 and no Qwen roll at :60-62), both
    score placements: the batch's masks and scores == the oracle's get_masks_and_scores (roll
    off) on the batch's own ids with the history scores (ctx_manager.py:282), and without turn
    scores the last column == the oracle's group normalisation of sum + penalty
    (ctx_manager.py:213-223); the device rollout == the dict rollout as for Qwen."""
    import oracle
    from fake_tok import FakeLlama3Tok
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    name = "sokoban_es"
    tok = FakeLlama3Tok()
    vocab = ops.VocabTable.from_bytes(*tok.byte_table(), device)
    outs = []
    for v in (None, vocab):
        cfg = _config(name)
        cfg.agent_proxy.use_turn_scores = uts
        proxy = LLMAgentProxy(cfg, TokenActor(_turn_tokens(name, tok, device)), tok, device=device)
        if v is not None:
            proxy.train_ctx_manager.set_device_vocab(v)
        random.seed(7)
        outs.append((proxy.rollout(DataProto(meta_info={}), val=False), proxy.train_es_manager.rollout_cache))
    (ref, ref_cache), (out, cache) = outs
    for k in ref.batch.keys():
        assert torch.equal(ref.batch[k].cpu(), out.batch[k].cpu()), k
    assert ref.meta_info == out.meta_info and ref_cache == cache
    ids = out.batch["input_ids"].cpu().numpy()
    assert (ids == 128006).any() and (ids == 128009).any() and not (ids == 151644).any()
    scores = [[h.get("reward", 0.0) for h in e["history"]] for e in cache]
    B, T = len(scores), max(len(x) for x in scores)
    tab = np.zeros((T, B))
    for b, x in enumerate(scores):
        tab[:len(x), b] = x
    n = np.array([len(x) for x in scores], np.int32)
    sc, lm, rm, err = oracle.masks_and_scores(ids, 128006, 128009, tab, n, T, uts, True, False)
    assert not err.any()
    np.testing.assert_array_equal(out.batch["loss_mask"].cpu().numpy().astype(np.uint8), lm)
    got = out.batch["rm_scores"].cpu().numpy()
    if uts:
        np.testing.assert_array_equal(got, sc)
        assert (got != 0).any()
    else:
        np.testing.assert_array_equal(got[:, :-1], sc[:, :-1])
        pen = np.array([e.get("penalty", 0) for e in cache], np.float32)
        gid = np.array([e["group_id"] for e in cache])
        seg = np.concatenate([[0], np.nonzero(np.diff(gid))[0] + 1, [B]]).astype(np.int32)
        np.testing.assert_array_equal(got[:, -1], oracle.group_normalize(sc[:, -1], pen, seg, "identity"))
