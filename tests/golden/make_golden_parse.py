"""Golden vectors for the response -> action path, made by RUNNING THE READ-ONLY REFERENCE.

TEST INFRASTRUCTURE (build container only; /root/reference is absent on the GPU box):

    PYTHONHASHSEED=0 python tests/golden/make_golden_parse.py

Executes the reference's ContextManager._parse_response (ctx_manager.py:148-173) on
"<think>"/"<answer>" + response exactly as get_env_inputs builds it (:338-339), and
EnvStateManager._extract_map_valid_actions (es_manager.py:230-240) with the Sokoban,
FrozenLake and Bandit lookups.  Writes tests/golden/parse_response.json (data only).
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refshim  # noqa: E402

refshim.install()

from ragen.llm_agent import ctx_manager as ctxm  # noqa: E402
from ragen.llm_agent.es_manager import EnvStateManager  # noqa: E402
from make_golden import AD  # noqa: E402

LOOKUPS = {
    "sokoban": {1: "Up", 2: "Down", 3: "Left", 4: "Right"},
    "frozen_lake": {1: "Left", 2: "Down", 3: "Right", 4: "Up"},
    "bandit": {1: "Phoenix", 2: "Dragon"},
    "bandit_swapped": {1: "Dragon", 2: "Phoenix"},
    "kelvin": {1: "Kick", 2: "Back"},
    "none": None,
}

HAND = [
    "go</think><answer>Up || Down</answer>",
    "x</think>  <answer> Left||right ||  UP || down || left || Right </answer>",
    "a</think><answer></answer>",
    "no closing tags at all",
    "a</think><answer>Up</answer><think>b</think><answer>Down</answer>",
    "<think></answer> 123. </think><answer> <answer> say || hi </answer></answer>",
    "multi\nline</think>\n<answer>Right || <|im_end|>Left</answer>",
    "t</think>  <answer>　Up ||\x85Down\x1c</answer>",
    "t</think>x<answer>Up</answer></think> <answer>Left</answer>",
    "t</think><answer>Up|||Down||||Left</answer>",
    "t</think><answer>Kick || KICK || kKICK || İp</answer>",
    "t</think><answer>Up<|im_start|>|Down || Le<think>ft</answer>",
    "t</think><answer></ans<think>wer>Up</answer>",
    "t</think><answer><think> Up || Down </think></answer>",
    "t</think><answer>  ||  || Up ||   </answer>",
    "t</think><answer>Up || Down || Left || Right || Up || Down || Left</answer>",
    "t</th ink><answer>Up</answer>",
    "t</think> \t\r\n <answer>Up</answer",
    "t</think><answer>Phoenix || dragon || PHOENIX</answer>",
    "éè</think><answer>Up · Down || � || Right</answer>",
    "",
    "</think>",
    "</think><answer>",
    "</think><answer></answer>",
    "t</think><answer>Up</answer></answer>",
    "t</think><answer>Up || 12 + 3 * (4 - 1) || 5</answer>",
    "t</think><answer><|im_end|></answer>",
    "t</think><answer>Up​ || Down</answer>",
    "t</think><answer>Up᠎|| Down⁠</answer>",
    "<answer>Up</answer>",
]

FRAGS = ["<think>", "</think>", "<answer>", "</answer>", "<|im_start|>", "<|im_end|>", "<", ">", "</", "/",
         "<answer", "</answer", "think>", "|", "||", "|||", " ", "  ", "\n", "\t", "\r", "\x0b", "\x0c",
         "\x1c", "\x1f", "\x85", "\xa0", " ", " ", " ", " ", " ", " ", " ",
         "　", "​", "é", "K", "İ", "�", "\U0001f600", "Up", "up", "UP", "Down",
         "Left", "LEFT", "Right", "right", "Phoenix", "DRAGON", "kick", "KICK", "back", "x", "go", "1", "23",
         "+", "*", "(", ")", "=", ",", ";"]


def fuzz_case(rng):
    n = rng.randint(0, 24)
    parts = [rng.choice(FRAGS) for _ in range(n)]
    if rng.random() < 0.7:  # mostly well-formed envelopes with noisy insides
        think = "".join(rng.choice(FRAGS) for _ in range(rng.randint(0, 6)))
        gap = rng.choice(["", " ", "\n", "   ", "x", "　"])
        body = rng.choice([" || ", "||", " | ", "|||"]).join(
            "".join(rng.choice(FRAGS[40:] if rng.random() < 0.8 else FRAGS) for _ in range(rng.randint(0, 3)))
            for _ in range(rng.randint(0, 8)))
        tail = "".join(rng.choice(FRAGS) for _ in range(rng.randint(0, 3)))
        return think + "</think>" + gap + "<answer>" + body + rng.choice(["</answer>", "</answer>", ""]) + tail
    return "".join(parts)


def main():
    rng = random.Random(20250704)
    texts = HAND + [fuzz_case(rng) for _ in range(1500)]
    cases = []
    for i, text in enumerate(texts):
        think = (i % 5) != 4
        K = [5, 1, 3, 8][i % 4]
        sep = "||" if i % 7 else ","
        cm = ctxm.ContextManager.__new__(ctxm.ContextManager)
        cm.config = AD.wrap({"agent_proxy": {"enable_think": think, "max_actions_per_turn": K}})
        cm.action_sep = sep
        cm.special_token_list = ["<think>", "</think>", "<answer>", "</answer>", "<|im_start|>", "<|im_end|>"]
        response = ("<think>" if think else "<answer>") + text  # get_env_inputs :338-339
        llm_response, actions = cm._parse_response(response)
        mapped = {}
        for name, lk in LOOKUPS.items():
            entry = {"env": AD({"config": AD({"action_lookup": lk})})}
            mapped[name] = EnvStateManager._extract_map_valid_actions(None, entry, actions)
        cases.append({"text": text, "enable_think": think, "K": K, "sep": sep, "llm_response": llm_response,
                      "actions": actions, "mapped": mapped})
    out = {"lookups": {k: (None if v is None else {str(a): b for a, b in v.items()}) for k, v in LOOKUPS.items()},
           "cases": cases}
    with open(os.path.join(HERE, "parse_response.json"), "w") as f:
        json.dump(out, f, ensure_ascii=True, indent=0)
    print(len(cases), "parse cases written")


if __name__ == "__main__":
    main()
