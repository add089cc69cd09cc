"""The validation rollout's golden record (tests/golden/val_rollout.json, made by
make_golden_val.py from the reference's own EnvStateManager / ContextManager in mode "val":
seed 123, group_size 1, 256 SimpleSokoban + 32 FrozenLake groups) against this package's host
pieces, on the CPU:

* the response parse (ctx_manager.py:148-173) of every turn's generation gives the history's
  llm_response / llm_raw_response and the executed actions' count bound;
* the message builder + the tokenizer (ctx_manager.py:228-306) over the reference's rollout
  cache give the formulated batch's exact input_ids / attention_mask / position_ids;
* the fixture itself: val seeds, one env per group, the tag boundary.

The GPU test (tests/test_gpu_val_rollout.py) runs LLMAgentProxy.rollout(val=True) on the
device and dict paths against the same record."""
import hashlib
import json
import os

import numpy as np
import torch

from fake_tok import FakeQwenTok
from ragen_amd.config import default_config
from ragen_amd.llm_agent.ctx_manager import ContextManager, parse_response

HERE = os.path.dirname(os.path.abspath(__file__))


def load_val():
    with open(os.path.join(HERE, "golden", "val_rollout.json")) as f:
        return json.load(f)


def digest(t):
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()


def test_val_fixture_shape():
    d = load_val()
    ov = d["overrides"]["es_manager"]["val"]
    assert ov["group_size"] == 1 and ov["env_configs"]["n_groups"] == [256, 32] and d["seed"] == 123
    rc = d["rollout_cache"]
    assert len(rc) == 288 and [c["env_id"] for c in rc] == list(range(288))
    assert [c["group_id"] for c in rc] == list(range(288))          # group_size 1: a group per env
    assert {c["tag"] for c in rc[:256]} == {"SimpleSokoban"} and {c["tag"] for c in rc[256:]} == {"FrozenLake"}
    assert d["turns"][0]["env_ids"] == list(range(288))


def test_val_responses_parse_like_the_reference():
    d = load_val()
    cfg = default_config(**d["overrides"])
    ap = cfg.agent_proxy
    rc = d["rollout_cache"]
    n = 0
    for t, turn in enumerate(d["turns"]):
        for e, text in zip(turn["env_ids"], turn["responses"]):
            raw = "<think>" + text
            llm_response, actions = parse_response(raw, ap.enable_think, ap.action_sep, ap.max_actions_per_turn)
            h = rc[e]["history"][t]
            assert h["llm_raw_response"] == raw and h["llm_response"] == llm_response, (t, e)
            assert len(h["actions"]) <= len(actions)  # executed: the known names, up to actions left
            n += 1
    assert n == sum(len(t["env_ids"]) for t in d["turns"])


def test_val_formulated_batch_from_host_messages():
    d = load_val()
    cfg = default_config(**d["overrides"])
    tok = FakeQwenTok()
    ctx = ContextManager(cfg, tok, mode="val", device="cpu")
    # the rollout states as formulate_rollouts received them: the trimmed cache + the last entry
    states = [dict(c, history=c["history"] + [dict(last)]) for c, last in zip(d["rollout_cache"], d["last_entries"])]
    texts, _ = ctx._build_messages(states, True)
    enc = tok(texts, return_tensors="pt", padding=True, padding_side="left", truncation=False)
    f = d["formulated"]
    assert list(enc.input_ids.shape) == f["shape"]
    assert digest(enc.input_ids) == f["sha256"]["input_ids"]
    assert digest(enc.attention_mask) == f["sha256"]["attention_mask"]
    assert digest(enc.attention_mask.cumsum(dim=-1)) == f["sha256"]["position_ids"]
    assert digest(enc.input_ids[:, 1:]) == f["sha256"]["responses"]
    # the trajectory scores: the turn rewards' sum in f32 plus the format penalty, identity
    # normalisation (base.yaml:96-97, ctx_manager.py:175-226)
    sums = np.array([sum(float(h.get("reward", 0.0)) for h in c["history"]) for c in d["rollout_cache"]], np.float32)
    pen = np.array([c["penalty"] for c in d["rollout_cache"]], np.float32)
    assert np.array_equal(sums + pen, np.array(f["rm_scores_last"], np.float32))
    assert f["env_ids"] == list(range(288)) and f["group_ids"] == list(range(288))


def test_val_generation_batches_from_host_messages():
    """Turn 0's generation batch: the reset prompts (every env, seed 123's rooms)."""
    d = load_val()
    cfg = default_config(**d["overrides"])
    tok = FakeQwenTok()
    ctx = ContextManager(cfg, tok, mode="val", device="cpu")
    states = [{"env_id": e, "group_id": e, "tag": c["tag"], "penalty": 0,
               "history": [{"state": s, "actions_left": c["history"][0]["actions_left"]}]}
              for e, (c, s) in enumerate(zip(d["rollout_cache"], d["init_obs"]))]
    out = ctx.get_lm_inputs_eager(states, False)
    t0 = d["turns"][0]
    assert list(out.batch["input_ids"].shape) == t0["shape"]
    for k in ("input_ids", "attention_mask", "position_ids"):
        assert digest(out.batch[k]) == t0["sha256"][k], k
    assert torch.equal(out.batch["responses"], out.batch["input_ids"][:, 1:])
