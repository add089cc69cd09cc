"""agent_proxy.max_context_window on the host message builder (ContextManager._build_messages,
ctx_manager.py:240-246) against the messages the REFERENCE's get_lm_inputs built for the same
histories (tests/golden/context_window.json, recorded by tests/golden/make_golden_window.py):
k in {None, 1, 2, 3}, both prepare_for_update settings, with and without think, on the
reference unit test's own history (tests/llm_agent/test_context_window.py:60-84), a rollout-
shaped history and a first turn.  The device path rebuilds the same windows
(tests/test_gpu_device_prompts.py::test_device_prompts_context_window).

Note on the reference's unit test: it calls get_lm_inputs(prepare_for_update=True) on a history
whose every entry has a 'state', so the reference's code first drops the last entry
(ctx_manager.py:240-241) and then keeps [S1, S2]; its assertion '"S1" not in messages' does not
hold for the reference's own code there (the recorded messages contain S1).  It holds for
prepare_for_update=False, which keeps [S2, S3]; both outcomes are pinned below."""
import copy
import json
import os

from ragen_amd.config import env_task
from ragen_amd.llm_agent.ctx_manager import ContextManager

HERE = os.path.dirname(os.path.abspath(__file__))


class DummyTokenizer:
    name_or_path = "qwen"

    def apply_chat_template(self, messages, add_generation_prompt, tokenize):
        return " ".join(m["content"] for m in messages)


def _ctx(k, think):
    cfg = env_task("SimpleSokoban", 1, 1)
    cfg.agent_proxy.max_context_window = k
    cfg.agent_proxy.enable_think = think
    ctx = ContextManager(cfg, tokenizer=DummyTokenizer(), device="cpu")
    ctx.prefix_lookup = {0: "Initial prompt"}
    ctx.env_config_lookup = {0: {"max_tokens": 128}}
    return ctx


def _golden():
    with open(os.path.join(HERE, "golden", "context_window.json")) as f:
        return json.load(f)


def test_context_window_matches_reference_messages():
    g = _golden()
    assert len(g["cases"]) == 48
    for c in g["cases"]:
        ctx = _ctx(c["k"], c["think"])
        outs = [{"env_id": 0, "group_id": 0, "history": copy.deepcopy(g["histories"][c["history"]])}]
        _, msgs = ctx._build_messages(outs, c["update"])
        assert msgs[0] == c["messages"], c


def test_reference_unit_test_assertion():
    """test_context_window.py:60-84's history with k = 2."""
    g = _golden()
    by = {(c["history"], c["k"], c["update"], c["think"]): c["messages"] for c in g["cases"]}
    for update, kept in ((False, ("S2", "S3")), (True, ("S1", "S2"))):
        ctx = _ctx(2, False)
        outs = [{"env_id": 0, "group_id": 0, "history": copy.deepcopy(g["histories"]["reference_test"])}]
        _, msgs = ctx._build_messages(outs, update)
        m = str(msgs[0])
        assert all(s in m for s in kept) and sum(s in m for s in ("S1", "S2", "S3")) == 2
        assert "Turn 1:" in m and "Turn 2:" in m and "Turn 3:" not in m  # renumbered
        assert msgs[0] == by[("reference_test", 2, update, False)]
