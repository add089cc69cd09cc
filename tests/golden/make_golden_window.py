"""Golden vectors for agent_proxy.max_context_window (ctx_manager.py:240-246), recorded by RUNNING
THE READ-ONLY REFERENCE's ContextManager.get_lm_inputs on the inputs of its own unit test
(tests/llm_agent/test_context_window.py:60-84) and on longer histories, for k in {None, 1, 2, 3}
and both prepare_for_update settings: the messages_list it builds.

TEST INFRASTRUCTURE.  Run in the build container only:

    python tests/golden/make_golden_window.py   -> tests/golden/context_window.json

Only data (inputs + the reference's messages) is written; no reference source is stored.
"""
import copy
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refshim  # noqa: E402

refshim.install()

from ragen.llm_agent import ctx_manager as ctxm  # noqa: E402


class AD(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    @staticmethod
    def wrap(x):
        if isinstance(x, dict):
            return AD({k: AD.wrap(v) for k, v in x.items()})
        if isinstance(x, list):
            return [AD.wrap(v) for v in x]
        return x


class DummyTokenizer:
    """The reference test's tokenizer: the template joins the contents."""
    name_or_path = "qwen"

    def apply_chat_template(self, messages, add_generation_prompt, tokenize):
        return " ".join(m["content"] for m in messages)

    def __call__(self, texts, return_tensors=None, padding=None, padding_side=None, truncation=None):
        n = len(texts)

        class Out:
            input_ids = torch.tensor([[1, 2, 3]] * n)
            attention_mask = torch.tensor([[1, 1, 1]] * n)
        return Out()

    def encode(self, text):
        return [42, 43]


HISTORIES = {
    # the reference test's history (every entry complete)
    "reference_test": [{"state": "S1", "llm_response": "R1", "reward": 0.1, "actions_left": 5},
                       {"state": "S2", "llm_response": "R2", "reward": 0.2, "actions_left": 4},
                       {"state": "S3", "llm_response": "R3", "reward": 0.3, "actions_left": 3}],
    # as EnvStateManager leaves it: the last entry holds the next state only
    "rollout": [{"state": "S1", "llm_response": "R1", "reward": 0.1, "actions_left": 5},
                {"state": "S2", "llm_response": "R2", "reward": -0.1, "actions_left": 4},
                {"state": "S3", "llm_response": "R3", "reward": 1.0, "actions_left": 3},
                {"state": "S4", "actions_left": 2}],
    "first_turn": [{"state": "S1", "actions_left": 5}],
}


def run(history, k, update, think):
    cfg = AD.wrap({"agent_proxy": {"max_context_window": k, "enable_think": think, "use_turn_scores": False,
                                   "action_sep": "|", "reward_normalization": {"grouping": "batch",
                                                                               "method": "identity"}},
                   "enable_response_mask": False,
                   "es_manager": {"train": {"env_configs": {"n_groups": [1], "tags": ["sokoban"]}, "group_size": 1}},
                   "custom_envs": {"sokoban": {"env_type": "sokoban", "max_actions_per_traj": 10}},
                   "actor_rollout_ref": {"rollout": {"response_length": 128}}})
    ctx = ctxm.ContextManager.__new__(ctxm.ContextManager)
    ctx.config = cfg
    ctx.tokenizer = DummyTokenizer()
    ctx.prefix_lookup = {0: "Initial prompt"}
    ctx.env_config_lookup = {0: {"max_tokens": 128}}
    ctx.env_nums = {"": 1}
    outs = [{"env_id": 0, "group_id": 0, "history": copy.deepcopy(history), "metrics": {}, "penalty": 0.0}]
    if update:  # the reference's update path runs the masks / scores code on the dummy ids
        ctx.special_token_list = []
    dp = ctx.get_lm_inputs(outs, prepare_for_update=update)
    return [list(m) for m in dp.non_tensor_batch["messages_list"]][0]


def main():
    cases = []
    for name, h in HISTORIES.items():
        for k in (None, 1, 2, 3):
            for update in (True, False):
                for think in (False, True):
                    try:
                        msgs = run(h, k, update, think)
                    except Exception as e:  # recorded: the reference raises there
                        msgs = {"raises": type(e).__name__}
                    cases.append({"history": name, "k": k, "update": update, "think": think, "messages": msgs})
    with open(os.path.join(HERE, "context_window.json"), "w") as f:
        json.dump({"histories": HISTORIES, "cases": cases}, f, indent=0)
    print(len(cases), "cases written")


if __name__ == "__main__":
    main()
