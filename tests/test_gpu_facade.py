"""The drop-in Python surface (EnvStateManager / ContextManager / LLMAgentProxy /
compute_advantage) driven exactly as the reference drives its own, on the GPU engine,
compared with the golden traces recorded from the reference."""
import numpy as np
import pytest
import torch

from ragen_amd.config import default_config, env_task
from ragen_amd.llm_agent import ContextManager, EnvStateManager, LLMAgentProxy, ScriptedActor, get_masks_and_scores
from ragen_amd.protocol import DataProto
from ragen_amd.trainer import compute_advantage, filter_rollout
from fake_tok import FakeQwenTok
from trace_util import load, strings

pytestmark = pytest.mark.gpu

TRACES = {"sokoban_es": ("SimpleSokoban", 8, 16, 5, 5), "sokoban8_es": ("LargerSokoban", 2, 16, 5, 5),
          "frozenlake_es": ("FrozenLake", 8, 16, 8, 5), "bandit_es": ("Bandit", 4, 16, 1, 1),
          "countdown_es": ("Countdown", 4, 16, 4, 1)}


def _config(name):
    tag, ng, gs, T, K = TRACES[name]
    cfg = env_task(tag, ng, gs, max_turn=T, max_actions_per_turn=K)
    if tag == "Countdown":
        cfg.custom_envs.Countdown.env_config = {"data": strings()["countdown_data"]}
    return cfg


def _hashseed0_reseed(s):
    """abs(hash(str(s))) % 2**32 as the golden-generating process computed it (PYTHONHASHSEED=0)."""
    import os
    import subprocess
    import sys
    out = subprocess.run([sys.executable, "-c", f"print(abs(hash(str({int(s)}))) % (2 ** 32))"],
                         env=dict(os.environ, PYTHONHASHSEED="0"), capture_output=True, text=True, check=True)
    return int(out.stdout)


@pytest.mark.parametrize("name", list(TRACES))
def test_es_manager_replays_reference_trace(device, name, monkeypatch):
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    d = load(name)
    S = strings()[name]
    es = EnvStateManager(_config(name), mode="train", device=device)
    outs = es.reset(seed=int(d["seed"]))
    assert [o["history"][0]["state"] for o in outs] == S["init_obs"]
    B, T = int(d["B"]), int(d["T"])
    active = list(range(B))
    for t in range(T):
        inputs = []
        for i in active:
            if name == "countdown_es":
                a = S["answers"][t][i]
                acts = [] if a is None else [a]
            else:
                acts = [S["vocab"][c] for c in d["codes"][t, i] if c >= 0]
            inputs.append({"env_id": i, "llm_response": "r", "llm_raw_response": "r", "actions": acts})
        outs = es.step(inputs)
        active = [o["env_id"] for o in outs]
        assert sorted(active) == list(np.nonzero(d["active_after"][t])[0]), t
        for i in range(B):
            if d["act_in"][t, i]:
                h = es.rollout_cache[i]["history"][-2]
                assert float(h["reward"]) == d["turn_reward"][t, i]
                assert len(h["actions"]) == d["n_exec"][t, i]
                inf = int(d["info"][t, i])
                assert bool(h["info"]) == bool(inf & 1)
                if inf & 1:
                    assert h["info"]["action_is_effective"] == bool(inf & 2)
                    assert h["info"]["success"] == bool(inf & 8)
            st = es.envs[i]["status"]
            assert st.num_actions == d["num_actions"][t, i]
            assert st.terminated == bool(d["term"][t, i]) and st.truncated == bool(d["trunc"][t, i])
            assert float(es.rollout_cache[i]["penalty"]) == d["penalty"][t, i]
        if not active:
            break
    final = es.get_rollout_states()
    tag = TRACES[name][0]
    for i, f in enumerate(final):
        for k in ("success", "num_actions", "action_is_effective", "action_is_valid"):
            ref = d["metric_" + k][i]
            got = f["metrics"].get(f"{tag}/{k}", np.nan)
            assert (np.isnan(ref) and np.isnan(got)) or ref == got, (i, k, ref, got)
    assert [f["history"][-1]["state"] for f in final] == S["final_obs"]


def test_normalize_score_tensor_golden(device):
    d = load("normalize")
    B = len(d["scores"])
    tags = ["A"] * 48 + ["B"] * 48
    for grouping in ("state", "inductive", "batch"):
        for method in ("mean_std", "mean", "asym_clip", "identity"):
            cfg = default_config(agent_proxy={"reward_normalization": {"grouping": grouping, "method": method}},
                                 es_manager={"train": {"env_configs": {"tags": ["SimpleSokoban"], "n_groups": [6]},
                                                       "env_groups": 6}})
            cm = ContextManager(cfg, tokenizer=None, device=device)
            st = torch.zeros(B, 4)
            st[:, -1] = torch.from_numpy(d["scores"])
            outs = [{"group_id": int(g), "tag": t, "penalty": float(p)}
                    for g, t, p in zip(d["group_id"], tags, d["penalty"])]
            res = cm._normalize_score_tensor(st, outs)
            np.testing.assert_allclose(res[:, -1].numpy(), d[f"norm_{grouping}_{method}"], atol=1e-5, rtol=0)


def test_get_masks_and_scores_golden(device):
    d = load("masks_scores")
    tok = FakeQwenTok()
    ids = torch.from_numpy(d["input_ids"]).to(device)
    lens = d["scores_len"]
    flat = d["scores_flat"]
    scores, o = [], 0
    for n in lens:
        scores.append(list(flat[o:o + n]))
        o += n
    for uts in (False, True):
        for erm in (False, True):
            st, lm, rm = get_masks_and_scores(ids, tok, scores, use_turn_scores=uts, enable_response_mask=erm)
            key = f"uts{int(uts)}_erm{int(erm)}"
            np.testing.assert_array_equal(st.cpu().numpy(), d[key + "_score"])
            np.testing.assert_array_equal(lm.cpu().numpy().astype(np.uint8), d[key + "_loss_mask"])
            np.testing.assert_array_equal(rm.cpu().numpy().astype(np.uint8), d[key + "_response_mask"])


def test_get_masks_and_scores_llama3_golden(device):
    """The Llama-3 branch (ctx_manager.py:27-29, no roll at :60-62) on the device kernel == the
    reference-run fixture (tests/golden/make_golden_llama.py), all four mode pairs."""
    from fake_tok import FakeLlama3Tok
    d = load("masks_scores_llama")
    tok = FakeLlama3Tok()
    ids = torch.from_numpy(d["input_ids"]).to(device)
    lens, flat = d["scores_len"], d["scores_flat"]
    scores, o = [], 0
    for n in lens:
        scores.append(list(flat[o:o + n]))
        o += n
    for uts in (False, True):
        for erm in (False, True):
            st, lm, rm = get_masks_and_scores(ids, tok, scores, use_turn_scores=uts, enable_response_mask=erm)
            key = f"uts{int(uts)}_erm{int(erm)}"
            np.testing.assert_array_equal(st.cpu().numpy(), d[key + "_score"])
            np.testing.assert_array_equal(lm.cpu().numpy().astype(np.uint8), d[key + "_loss_mask"])
            np.testing.assert_array_equal(rm.cpu().numpy().astype(np.uint8), d[key + "_response_mask"])


def test_parse_response_golden(device):
    for case in strings()["parse_response"]:
        cfg = default_config(agent_proxy={"enable_think": case["enable_think"]})
        cm = ContextManager(cfg, tokenizer=None, device=device)
        llm_response, actions = cm._parse_response(case["response"])
        assert llm_response == case["llm_response"] and actions == case["actions"], case


def test_context_window_truncation(device):
    """The reference's only unit test (tests/llm_agent/test_context_window.py:60-84), ported:
    max_context_window=2 drops turn 1 from the prompt."""
    class DummyTok(FakeQwenTok):
        def apply_chat_template(self, messages, add_generation_prompt, tokenize):
            return " ".join(m["content"] for m in messages)

    cfg = default_config(agent_proxy={"max_context_window": 2, "enable_think": False, "action_sep": "|",
                                      "reward_normalization": {"grouping": "batch", "method": "identity"}},
                         es_manager={"train": {"env_groups": 1, "group_size": 1,
                                               "env_configs": {"n_groups": [1], "tags": ["SimpleSokoban"]}}})
    cm = ContextManager(cfg, DummyTok(), device=device)
    env_outputs = [{"env_id": 0, "group_id": 0, "tag": "SimpleSokoban", "penalty": 0, "metrics": {},
                    "history": [{"state": "S1", "llm_response": "R1", "reward": 1, "actions_left": 3},
                                {"state": "S2", "llm_response": "R2", "reward": 2, "actions_left": 2},
                                {"state": "S3", "actions_left": 1}]}]
    out = cm.get_lm_inputs(env_outputs, prepare_for_update=False)
    msgs = out.non_tensor_batch["messages_list"][0]
    text = " ".join(m["content"] for m in msgs)
    assert "S1" not in text and "S2" in text and "S3" in text and "R1" not in text


def test_compute_advantage_golden(device):
    d = load("gae")
    B = d["mask"].shape[0]
    for est, bl in (("grpo", False), ("gae", False), ("gae", True)):
        m = torch.from_numpy(d["mask"]).bool()
        dp = DataProto({"token_level_rewards": torch.from_numpy(d["rew_turn"]), "values": torch.from_numpy(d["values"]),
                        "response_mask": m, "loss_mask": m}, {"uid": np.array([str(i) for i in range(B)], object)})
        dp = compute_advantage(dp, est, gamma=1.0, lam=0.95, multi_turn=True, bi_level_gae=bl, high_level_gamma=0.95)
        np.testing.assert_allclose(dp.batch["advantages"].numpy(), d[f"ca_{est}_{int(bl)}_adv"], atol=1e-5, rtol=1e-6)
        if est == "gae":
            np.testing.assert_array_equal(dp.batch["returns"].numpy(), d[f"ca_{est}_{int(bl)}_ret"])


def test_filter_rollout_golden(device):
    d = load("filter")
    sc = torch.from_numpy(d["r0.25_std_scores"])
    dp = DataProto({"original_rm_scores": sc, "x": torch.arange(sc.shape[0])}, {"env_ids": np.arange(sc.shape[0])})
    out, met = filter_rollout(dp, 64, 16, 0.25, "std")
    np.testing.assert_array_equal(out.non_tensor_batch["env_ids"], d["r0.25_std_kept_env_ids"])
    assert abs(met["rollout/in_group_std"] - float(d["r0.25_std_rollout__in_group_std"])) < 1e-6


def test_agent_proxy_rollout_end_to_end(device):
    """LLMAgentProxy.rollout with a scripted policy: reset -> (ctx -> actor -> ctx -> es) x T -> formulate."""
    cfg = env_task("SimpleSokoban", 4, 16, max_turn=5, max_actions_per_turn=5)
    cfg.agent_proxy.reward_normalization.method = "mean_std"
    rng = np.random.default_rng(0)
    names = ["Up", "Down", "Left", "Right", "Jump"]

    def policy(env_id, turn):
        acts = " || ".join(names[int(x)] for x in rng.integers(0, 5, size=int(rng.integers(1, 4))))
        return f"go</think><answer>{acts}</answer>"
    proxy = LLMAgentProxy(cfg, ScriptedActor(policy), FakeQwenTok(), device=device)
    out = proxy.rollout(DataProto(meta_info={}), val=False)
    B = 64
    assert out.batch["input_ids"].shape[0] == B
    assert out.batch["rm_scores"].shape == out.batch["loss_mask"].shape
    m = out.meta_info["metrics"]
    assert 0.0 <= m["SimpleSokoban/success"] <= 1.0 and m["SimpleSokoban/num_actions"] > 0
    # each row's score sits in the last column, normalised per group of 16 (mean_std)
    last = out.batch["rm_scores"][:, -1].view(4, 16)
    assert torch.all(last.mean(-1).abs() < 1e-4)


def test_es_manager_mixed_tags_equal_single_tag_runs(device):
    """Two tags in one EnvStateManager (es_manager.py:44-73: env ids laid out tag after tag,
    seeds seed + i // group_size across the whole list) == each tag run alone with the seed its
    first group gets, turn by turn: the per-tag grouping of the inputs, the batched name
    mapping and the one-launch-per-tag step."""
    gs, T, K = 4, 3, 5
    ov = {"es_manager": {"train": {"env_groups": 4, "group_size": gs,
                                   "env_configs": {"tags": ["SimpleSokoban", "FrozenLake"], "n_groups": [2, 2]}}},
          "agent_proxy": {"max_turn": T, "max_actions_per_turn": K}}
    mixed = EnvStateManager(default_config(**ov), mode="train", device=device)
    alone = [EnvStateManager(env_task(tag, 2, gs, max_turn=T, max_actions_per_turn=K), mode="train", device=device)
             for tag in ("SimpleSokoban", "FrozenLake")]
    seed = 77
    mixed.reset(seed=seed)
    alone[0].reset(seed=seed)
    alone[1].reset(seed=seed + 2)  # FrozenLake's first group is group 2 of the mixed list
    names = ["Up", "down", "LEFT", "Right", "jump"]
    rng = np.random.default_rng(3)
    active = list(range(16))
    for t in range(T):
        acts = {i: [names[int(a)] for a in rng.integers(0, 5, int(rng.integers(0, K + 1)))] for i in active}
        # inputs in a shuffled env order: the grouping must not depend on it
        order = [int(i) for i in rng.permutation(active)]
        outs = mixed.step([{"env_id": i, "llm_response": "x", "llm_raw_response": "y", "actions": acts[i]}
                           for i in order])
        ref = []
        for j, es in enumerate(alone):
            mine = [i for i in order if (i >= 8) == (j == 1)]
            if mine:
                ref += es.step([{"env_id": i - 8 * j, "llm_response": "x", "llm_raw_response": "y",
                                 "actions": acts[i]} for i in mine])
        got = {o["env_id"]: o for o in outs}
        want = {r["env_id"] + (8 if r["tag"] == "FrozenLake" else 0): r for r in ref}
        assert sorted(got) == sorted(want)
        assert [o["env_id"] for o in outs] == [i for i in order if i in want]  # input order kept
        for i in got:
            assert got[i]["history"] == want[i]["history"], (t, i)
            assert got[i]["penalty"] == want[i]["penalty"]
        active = [o["env_id"] for o in outs]
        if not active:
            break
