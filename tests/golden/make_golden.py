"""Generate the golden vectors under tests/golden/ by RUNNING THE READ-ONLY REFERENCE.

TEST INFRASTRUCTURE.  Run in the build container only (the reference at
/root/reference does not exist on the GPU box):

    PYTHONHASHSEED=0 python tests/golden/make_golden.py

Third-party code the reference calls but does not vendor is supplied by
``refshim`` (restatements, see its docstring).  Everything else executed here is
the reference's own Python: ragen/llm_agent/es_manager.py (EnvStateManager),
ragen/env/*/env.py, ragen/env/sokoban/utils.py (generate_room),
ragen/env/frozen_lake/utils.py (generate_random_map), ragen/llm_agent/ctx_manager.py
(_normalize_score_tensor, get_masks_and_scores, _parse_response),
ragen/trainer/core_algos.py (compute_bi_level_gae_advantage_return) and the
``_filter_rollout`` / ``compute_advantage`` functions of
ragen/trainer/agent_trainer.py (extracted with ``ast`` and executed).

Only data (inputs + expected outputs) is written; no reference source is stored.
"""
import ast
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refshim  # noqa: E402

refshim.install()

from ragen.env import REGISTERED_ENVS, REGISTERED_ENV_CONFIGS  # noqa: E402
from ragen.env.countdown import env as cd_env_mod  # noqa: E402
from ragen.env.sokoban.env import SokobanEnv  # noqa: E402
from ragen.env.sokoban.config import SokobanEnvConfig  # noqa: E402
from ragen.llm_agent.es_manager import EnvStateManager  # noqa: E402
from ragen.llm_agent import ctx_manager as ctxm  # noqa: E402
from ragen.trainer import core_algos  # noqa: E402

assert os.environ.get("PYTHONHASHSEED") == "0", "run with PYTHONHASHSEED=0 (Sokoban reseed uses hash())"


class AD(dict):
    """Attribute dict standing in for an OmegaConf DictConfig."""

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


CUSTOM_ENVS = {
    "SimpleSokoban": {"env_type": "sokoban", "max_actions_per_traj": 10,
                      "env_config": {"dim_x": 6, "dim_y": 6, "num_boxes": 1, "max_steps": 100}},
    "LargerSokoban": {"env_type": "sokoban", "max_actions_per_traj": 10,
                      "env_config": {"dim_x": 8, "dim_y": 8, "num_boxes": 2, "max_steps": 100,
                                     "search_depth": 10}},
    "FrozenLake": {"env_type": "frozen_lake", "max_actions_per_traj": 10, "env_config": None},
    "Bandit": {"env_type": "bandit", "max_actions_per_traj": 1,
               "env_config": {"lo_arm_name": "Phoenix", "hi_arm_name": "Dragon"}},
    "Countdown": {"env_type": "countdown", "max_actions_per_traj": 1, "env_config": None},
}


def make_cfg(tag, n_groups, group_size):
    return AD.wrap({
        "es_manager": {"format_penalty": -0.1,
                       "train": {"env_groups": n_groups, "group_size": group_size,
                                 "env_configs": {"tags": [tag], "n_groups": [n_groups]}}},
        "custom_envs": CUSTOM_ENVS,
    })


# ----------------------------------------------------------------- countdown data
def synthetic_countdown_data(n, seed):
    """Synthetic Countdown instances (the parquet is an HF download, absent offline):
    3-4 numbers in [1, 99], target = signed sum under a random sign pattern, kept only
    if the reference's own ``has_solution`` accepts it (countdown/env.py:23-33)."""
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        k = int(rng.integers(3, 5))
        nums = [int(x) for x in rng.integers(1, 100, size=k)]
        signs = rng.choice([-1, 1], size=k)
        target = int(sum(int(s) * v for s, v in zip(signs, nums)))
        if cd_env_mod.has_solution(list(nums), target):
            out.append({"nums": nums, "target": target})
    return out


CD_DATA = synthetic_countdown_data(257, 7)
cd_env_mod.CountdownEnv._get_data_from_parquet = lambda self, path: CD_DATA


# ------------------------------------------------------------------ action synth
VOCAB = {
    "sokoban": ["jump", "Up", "Down", "Left", "Right", "up", "DOWN", "left", "RIGHT", "push", ""],
    "frozen_lake": ["jump", "Left", "Down", "Right", "Up", "left", "DOWN", "right", "UP", "stay"],
    "bandit": ["pull", "Phoenix", "Dragon", "phoenix", "DRAGON", "dragon", "PHOENIX", "arm"],
}
UNKNOWN = {"sokoban": [0, 9, 10], "frozen_lake": [0, 9], "bandit": [0, 7]}


def synth_actions(rng, env_type, k_max):
    """n ~ U{0..K}; each action a known name (random case) w.p. 0.9 else an unknown one."""
    vocab = VOCAB[env_type]
    unk = UNKNOWN[env_type]
    known = [i for i in range(len(vocab)) if i not in unk]
    n = int(rng.integers(0, k_max + 1))
    codes = []
    for _ in range(n):
        if rng.random() < 0.1:
            codes.append(int(rng.choice(unk)))
        else:
            codes.append(int(rng.choice(known)))
    return codes


def countdown_answer(rng, inst):
    """Grammar-generated answers: correct / format-only / wrong numbers / empty."""
    nums = list(inst["nums"])
    u = rng.random()
    if u < 0.25:
        return None  # no parsable action this turn
    perm = list(rng.permutation(len(nums)))
    ops = ["+", "-", "*", "/"]
    if u < 0.5:  # a correct signed-sum answer
        target = inst["target"]
        # find a sign pattern (has_solution guarantees one)
        import itertools
        for signs in itertools.product([1, -1], repeat=len(nums)):
            if sum(s * v for s, v in zip(signs, nums)) == target:
                break
        expr = ""
        for i, (s, v) in enumerate(zip(signs, nums)):
            if i == 0:
                expr += ("-" if s < 0 else "") + str(v)
            else:
                expr += (" - " if s < 0 else " + ") + str(v)
        if rng.random() < 0.3:
            expr = "(" + expr + ")"
        return expr
    if u < 0.75:  # format-only: right numbers, random operators/parens
        toks = [str(nums[p]) for p in perm]
        expr = toks[0]
        for t in toks[1:]:
            expr += " " + ops[int(rng.integers(0, 4))] + " " + t
        if rng.random() < 0.3:
            expr = "(" + expr + ") * 1" if False else "(" + expr + ")"
        return expr
    # wrong numbers or odd syntax
    choices = [
        " + ".join(str(v + 1) for v in nums),
        " + ".join(str(v) for v in nums[:-1]),
        "".join(str(v) for v in nums),
        " ".join(str(v) for v in nums),
        " ** ".join(str(v) for v in nums[:2]) + "".join(" - " + str(v) for v in nums[2:]),
        " // ".join(str(v) for v in nums),
        "x + " + " + ".join(str(v) for v in nums),
    ]
    return choices[int(rng.integers(0, len(choices)))]


# ----------------------------------------------------------------- es trace runner
def run_es_trace(tag, n_groups, group_size, n_turns, k_max, seed, action_seed):
    cfg = make_cfg(tag, n_groups, group_size)
    es = EnvStateManager(cfg, mode="train")
    env_type = CUSTOM_ENVS[tag]["env_type"]
    B = n_groups * group_size
    rng = np.random.default_rng(action_seed)
    outs = es.reset(seed=seed)
    init_obs = [o["history"][0]["state"] for o in outs]
    rec = {"B": B, "T": n_turns, "K": k_max, "seed": seed, "group_size": group_size}

    def snap_state():
        d = {}
        if env_type == "sokoban":
            d["room_state"] = np.stack([e["env"].room_state.astype(np.int8).ravel() for e in es.envs])
            d["player"] = np.stack([np.asarray(e["env"].player_position, dtype=np.int64) for e in es.envs])
            d["num_env_steps"] = np.array([e["env"].num_env_steps for e in es.envs], np.int32)
            d["boxes_on_target"] = np.array([e["env"].boxes_on_target for e in es.envs], np.int32)
        elif env_type == "frozen_lake":
            d["s"] = np.array([int(e["env"].s) for e in es.envs], np.int32)
            st = [e["env"].np_random.bit_generator.state["state"] for e in es.envs]
            d["rng_state"] = np.array([[s["state"] >> 64, s["state"] & (2**64 - 1),
                                        s["inc"] >> 64, s["inc"] & (2**64 - 1)] for s in st], np.uint64)
        elif env_type == "bandit":
            st = [e["env"].np_random.bit_generator.state["state"] for e in es.envs]
            d["rng_state"] = np.array([[s["state"] >> 64, s["state"] & (2**64 - 1),
                                        s["inc"] >> 64, s["inc"] & (2**64 - 1)] for s in st], np.uint64)
        return d

    init = snap_state()
    if env_type == "sokoban":
        init["room_fixed"] = np.stack([e["env"].room_fixed.astype(np.int8).ravel() for e in es.envs])
    if env_type == "frozen_lake":
        init["desc"] = np.stack([np.frombuffer(e["env"].desc.tobytes(), np.uint8) for e in es.envs])
    if env_type == "bandit":
        init["hi_is_first"] = np.array([e["env"].ACTION_LOOKUP[1] == e["config"].hi_arm_name
                                        for e in es.envs], np.uint8)
    if env_type == "countdown":
        nums = np.zeros((B, 4), np.int32)
        nn = np.zeros(B, np.int32)
        tg = np.zeros(B, np.int32)
        for i, e in enumerate(es.envs):
            inst = e["env"].data[e["env"].index]
            nums[i, :len(inst["nums"])] = inst["nums"]
            nn[i] = len(inst["nums"])
            tg[i] = inst["target"]
        init.update(nums=nums, n_nums=nn, target=tg)
    for k, v in init.items():
        rec["init_" + k] = v

    T = n_turns
    act_in = np.zeros((T, B), np.uint8)          # env received an input this turn
    n_act = np.zeros((T, B), np.int32)
    codes = np.full((T, B, k_max), -1, np.int32)
    answers = [[None] * B for _ in range(T)]
    turn_reward = np.zeros((T, B), np.float64)
    n_exec = np.zeros((T, B), np.int32)
    info = np.zeros((T, B), np.uint8)   # bit0 has_info, bit1 effective, bit2 valid, bit3 success
    penalty = np.zeros((T, B), np.float64)
    num_actions = np.zeros((T, B), np.int32)
    term = np.zeros((T, B), np.uint8)
    trunc = np.zeros((T, B), np.uint8)
    active_after = np.zeros((T, B), np.uint8)
    states = {}
    active = list(range(B))
    for t in range(T):
        inputs = []
        for i in active:
            a_codes = []
            if env_type == "countdown":
                inst = es.envs[i]["env"].data[es.envs[i]["env"].index]
                ans = countdown_answer(rng, inst)
                acts = [] if ans is None else [ans]
                answers[t][i] = ans
            else:
                a_codes = synth_actions(rng, env_type, k_max)
                acts = [VOCAB[env_type][c] for c in a_codes]
                acts = [a for a in acts if a.strip()]  # ctx_manager drops empty action strings
                a_codes = [c for c in a_codes if VOCAB[env_type][c].strip()]
            act_in[t, i] = 1
            n_act[t, i] = len(acts)
            codes[t, i, :len(a_codes)] = a_codes
            inputs.append({"env_id": i, "llm_response": "r", "llm_raw_response": "r", "actions": acts})
        outs = es.step(inputs)
        active = [o["env_id"] for o in outs]
        for i in range(B):
            hist = es.rollout_cache[i]["history"]
            if act_in[t, i]:
                h = hist[-2]
                turn_reward[t, i] = float(h["reward"])
                n_exec[t, i] = len(h["actions"])
                inf = h["info"]
                if inf:
                    info[t, i] = (1 | (2 * bool(inf["action_is_effective"])) | (4 * bool(inf["action_is_valid"]))
                                  | (8 * bool(inf["success"])))
            st = es.envs[i]["status"]
            penalty[t, i] = es.rollout_cache[i]["penalty"]
            num_actions[t, i] = st.num_actions
            term[t, i] = st.terminated
            trunc[t, i] = st.truncated
        for i in active:
            active_after[t, i] = 1
        for k, v in snap_state().items():
            states.setdefault(k, []).append(v)
    rec.update(act_in=act_in, n_act=n_act, codes=codes, turn_reward=turn_reward, n_exec=n_exec,
               info=info, penalty=penalty, num_actions=num_actions, term=term, trunc=trunc,
               active_after=active_after)
    for k, v in states.items():
        rec["turn_" + k] = np.stack(v)
    final = es.get_rollout_states()
    keys = ["success", "num_actions", "action_is_effective", "action_is_valid"]
    for k in keys:
        rec["metric_" + k] = np.array([f["metrics"].get(f"{tag}/{k}", np.nan) for f in final], np.float64)
    # trajectory scores exactly as ctx_manager builds them (get_lm_inputs:282, get_masks_and_scores:64-65)
    scores = [[h.get("reward", 0.0) for h in f["history"][:-1]] for f in final]
    rec["score_f32"] = torch.tensor([sum(s) for s in scores], dtype=torch.float32).numpy()
    rec["penalty_f32"] = torch.tensor([f.get("penalty", 0) for f in final], dtype=torch.float32).numpy()
    rec["group_id"] = np.array([f["group_id"] for f in final], np.int32)
    strings = {"vocab": VOCAB.get(env_type, []), "init_obs": init_obs,
               "final_obs": [f["history"][-1]["state"] for f in final],
               "answers": answers if env_type == "countdown" else None}
    return rec, strings


# ------------------------------------------------------------------- sokoban rooms
def sokoban_rooms():
    out = {}
    for tag, seeds in (("SimpleSokoban", list(range(0, 512)) + [3248, 3701]),
                       ("LargerSokoban", list(range(0, 64)))):
        cfg = SokobanEnvConfig(**CUSTOM_ENVS[tag]["env_config"])
        env = SokobanEnv(cfg)
        fixed, state, player = [], [], []
        for s in seeds:
            env.reset(seed=s)
            fixed.append(env.room_fixed.astype(np.int8).ravel())
            state.append(env.room_state.astype(np.int8).ravel())
            player.append(np.asarray(env.player_position, np.int64))
        out[tag + "_seeds"] = np.array(seeds, np.int64)
        # value the reference reseeds with when generation fails (sokoban/env.py:41)
        out[tag + "_reseed"] = np.array([abs(hash(str(s))) % (2 ** 32) for s in seeds], np.int64)
        out[tag + "_fixed"] = np.stack(fixed)
        out[tag + "_state"] = np.stack(state)
        out[tag + "_player"] = np.stack(player)
    # the reseed fallback value for the failing seeds (sokoban/env.py:41)
    out["reseed_of_3248"] = np.array([abs(hash(str(3248))) % (2 ** 32)], np.int64)
    out["reseed_of_3701"] = np.array([abs(hash(str(3701))) % (2 ** 32)], np.int64)
    return out


# ----------------------------------------------------------- ctx_manager functions
def make_ctx(grouping, method):
    cm = ctxm.ContextManager.__new__(ctxm.ContextManager)
    cm.config = AD.wrap({"agent_proxy": {"use_turn_scores": False,
                                          "reward_normalization": {"grouping": grouping, "method": method}}})
    return cm


def normalize_cases():
    rng = np.random.default_rng(11)
    out = {}
    B, gs = 96, 16
    # scores: sums of -0.1 steps, +1/+10, ties, constant groups
    base = rng.choice([-1.0, -0.5, -0.3, 0.0, 0.9, 10.4, 10.8, -1.1], size=B).astype(np.float32)
    base[0:16] = np.float32(-0.5)          # constant group -> zero std branch
    base[16:32] = np.float32(0.3)
    pen = rng.choice([0.0, -0.1, -0.2, -0.30000000000000004], size=B)
    tags = np.array(["A"] * 48 + ["B"] * 48)
    out["scores"] = base
    out["penalty"] = pen
    out["group_id"] = np.arange(B) // gs
    out["tag_id"] = (tags == "B").astype(np.int32)
    for grouping in ("state", "inductive", "batch"):
        for method in ("mean_std", "mean", "asym_clip", "identity"):
            cm = make_ctx(grouping, method)
            st = torch.zeros(B, 4, dtype=torch.float32)
            st[:, -1] = torch.from_numpy(base)
            env_outputs = [{"group_id": int(g), "tag": str(t), "penalty": float(p)}
                           for g, t, p in zip(out["group_id"], tags, pen)]
            res = cm._normalize_score_tensor(st, env_outputs)
            out[f"norm_{grouping}_{method}"] = res[:, -1].numpy().copy()
    return out


class FakeQwenTok:
    name_or_path = "Qwen/Qwen2.5-0.5B-Instruct"
    IM_START, IM_END = 151644, 151645

    def encode(self, text):
        return {"<|im_start|>": [self.IM_START], "<|im_end|>": [self.IM_END]}[text]


def masks_scores_cases():
    """Token rows shaped like Qwen chat transcripts: pad, system, (user, assistant)*turns."""
    rng = np.random.default_rng(5)
    tok = FakeQwenTok()
    B = 24
    rows, all_scores = [], []
    for b in range(B):
        n_turns = int(rng.integers(1, 5))
        ids = [tok.IM_START] + list(rng.integers(100, 1000, size=int(rng.integers(3, 8)))) + [tok.IM_END, 198]
        sc = []
        for t in range(n_turns):
            ids += [tok.IM_START] + list(rng.integers(100, 1000, size=int(rng.integers(2, 9)))) + [tok.IM_END, 198]
            ids += [tok.IM_START] + list(rng.integers(100, 1000, size=int(rng.integers(2, 9)))) + [tok.IM_END]
            if t < n_turns - 1 or rng.random() < 0.5:
                ids += [198]
            sc.append(float(rng.choice([-0.1, 0.9, 0.0, 10.9, -1.1])))
        rows.append(ids)
        all_scores.append(sc)
    S = max(len(r) for r in rows) + 2
    pad = 151643
    input_ids = np.full((B, S), pad, np.int64)
    for b, r in enumerate(rows):
        input_ids[b, S - len(r):] = r                      # left padding
    out = {"input_ids": input_ids,
           "scores_flat": np.array([s for sc in all_scores for s in sc], np.float64),
           "scores_len": np.array([len(sc) for sc in all_scores], np.int32)}
    for uts in (False, True):
        for erm in (False, True):
            st, lm, rm = ctxm.get_masks_and_scores(torch.from_numpy(input_ids), tok, all_scores,
                                                   use_turn_scores=uts, enable_response_mask=erm)
            key = f"uts{int(uts)}_erm{int(erm)}"
            out[key + "_score"] = st.numpy()
            out[key + "_loss_mask"] = lm.numpy().astype(np.uint8)
            out[key + "_response_mask"] = rm.numpy().astype(np.uint8)
    return out


def parse_response_cases():
    cases = [
        "<think>go</think><answer>Up || Down</answer>",
        "<think>x</think>  <answer> Left||right ||  UP || down || left || Right </answer>",
        "<think>a</think><answer></answer>",
        "no tags at all",
        "<think>a</think><answer>Up</answer><think>b</think><answer>Down</answer>",
        "<think><think></answer> 123. </think><answer> <answer> say || hi </answer></answer>",
        "<answer>Up</answer>",
        "<think>multi\nline</think>\n<answer>Right || <|im_end|>Left</answer>",
    ]
    res = []
    for think in (True, False):
        cm = ctxm.ContextManager.__new__(ctxm.ContextManager)
        cm.config = AD.wrap({"agent_proxy": {"enable_think": think, "max_actions_per_turn": 5}})
        cm.action_sep = "||"
        cm.special_token_list = ["<think>", "</think>", "<answer>", "</answer>", "<|im_start|>", "<|im_end|>"]
        for c in cases:
            llm_response, actions = cm._parse_response(c)
            res.append({"enable_think": think, "response": c, "llm_response": llm_response, "actions": actions})
    return res


# ------------------------------------------------------- agent_trainer functions
def _extract(fn_name, path="/root/reference/ragen/trainer/agent_trainer.py"):
    src = open(path).read()
    tree = ast.parse(src)
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name == fn_name:
            return ast.get_source_segment(src, node)
    raise KeyError(fn_name)


def filter_cases():
    import textwrap
    src = textwrap.dedent(_extract("_filter_rollout"))

    class _Batch:
        pass
    out = {}
    rng = np.random.default_rng(3)
    G, gs, L = 64, 16, 6
    for ratio, ftype in ((0.25, "std"), (0.25, "std_rev"), (1.0, "std"), (0.5, "std")):
        # 1/4 of groups non-constant, the rest zero-std (tie hazard)
        sc = np.zeros((G * gs, L), np.float32)
        last = rng.choice([-0.5, -1.0, 10.4, 0.9], size=G * gs).astype(np.float32)
        for g in range(G):
            if g % 4:
                last[g * gs:(g + 1) * gs] = last[g * gs]
        sc[:, -1] = last
        cfg = AD.wrap({"actor_rollout_ref": {"rollout": {"rollout_filter_ratio": ratio, "rollout_filter_type": ftype}},
                       "es_manager": {"train": {"env_groups": G, "group_size": gs}}})

        class _Self:
            config = cfg
        ns = {"torch": torch, "np": np, "self": _Self()}
        exec(src, ns)
        b = _Batch()
        b.batch = {"original_rm_scores": torch.from_numpy(sc)}

        class _TD(dict):
            def __getitem__(self, k):
                if isinstance(k, str):
                    return dict.__getitem__(self, k)
                return _TD({kk: v[k] for kk, v in self.items()})
        b.batch = _TD(b.batch)
        b.non_tensor_batch = {"env_ids": np.arange(G * gs)}
        nb, metrics = ns["_filter_rollout"](b)
        key = f"r{ratio}_{ftype}"
        out[key + "_scores"] = sc
        out[key + "_kept_env_ids"] = np.asarray(nb.non_tensor_batch["env_ids"])
        for mk, mv in metrics.items():
            out[key + "_" + mk.replace("/", "__")] = np.array(float(mv), np.float64)
    return out


def gae_cases():
    rng = np.random.default_rng(9)
    out = {}
    B, L = 48, 160
    mask = np.zeros((B, L), bool)
    rew = np.zeros((B, L), np.float32)
    rew_turn = np.zeros((B, L), np.float32)
    for b in range(B):
        pos = int(rng.integers(0, 30))
        last = None
        while True:
            pos += int(rng.integers(3, 20))       # state block (mask 0)
            n = int(rng.integers(2, 25))          # response block (mask 1)
            if pos + n >= L:
                break
            mask[b, pos:pos + n] = True
            last = pos + n - 1
            rew_turn[b, last] = np.float32(rng.choice([-0.1, 0.9, 10.9, -1.1, 0.5]))
            pos += n
        if last is None:
            mask[b, L - 3:L - 1] = True
            last = L - 2
            rew_turn[b, last] = 0.5
        rew[b, last] = np.float32(rng.choice([-0.5, 1.0, 10.4, -1.2]))
        if rew_turn[b, last] == 0:
            rew_turn[b, last] = 1.0
    values = (rng.standard_normal((B, L)).astype(np.float32) * mask).astype(np.float32)
    out.update(mask=mask.astype(np.uint8), rew=rew, rew_turn=rew_turn, values=values)
    tmask = torch.from_numpy(mask)
    for gamma, lam in ((1.0, 1.0), (1.0, 0.95), (0.99, 0.95)):
        k = f"g{gamma}_l{lam}"
        for rname, r in (("last", rew), ("turn", rew_turn)):
            a, ret = refshim.compute_gae_advantage_return(torch.from_numpy(r), torch.from_numpy(values), tmask,
                                                         gamma, lam)
            out[f"gae_{rname}_{k}_adv"] = a.numpy()
            out[f"gae_{rname}_{k}_ret"] = ret.numpy()
            a, ret = refshim.compute_gae_advantage_return_masked(torch.from_numpy(r), torch.from_numpy(values),
                                                                tmask, gamma, lam)
            out[f"gaem_{rname}_{k}_adv"] = a.numpy()
            out[f"gaem_{rname}_{k}_ret"] = ret.numpy()
            a, ret = core_algos.compute_bi_level_gae_advantage_return(torch.from_numpy(r), torch.from_numpy(values),
                                                                     tmask, gamma, lam, 0.95)
            out[f"bilevel_{rname}_{k}_adv"] = a.numpy()
            out[f"bilevel_{rname}_{k}_ret"] = ret.numpy()
    # raw (pre-whitening) legacy advantages to pin the exact scan
    a, ret = refshim.compute_gae_advantage_return(torch.from_numpy(rew_turn), torch.from_numpy(values), tmask, 1.0, 0.95)
    out["raw_ret_turn_g1_l0.95"] = ret.numpy()
    # the reference's own __main__ example (core_algos.py:96-102)
    a, ret = core_algos.compute_bi_level_gae_advantage_return(
        torch.tensor([[0, 0, 0, 0, 1, 0, 0, 0, 0, 1]]), torch.tensor([[0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9, 1.0]]),
        torch.ones(1, 10), 1, 1, 0.95)
    out["main_example_adv"] = a.numpy()
    out["main_example_ret"] = ret.numpy()
    # bi-level IndexError case: last valid position has zero reward
    try:
        core_algos.compute_bi_level_gae_advantage_return(torch.tensor([[0.0, 1.0, 0.0, 0.0]]), torch.zeros(1, 4),
                                                         torch.tensor([[1, 1, 1, 1]]), 1.0, 1.0, 0.95)
        out["bilevel_zero_last_raises"] = np.array(0)
    except IndexError:
        out["bilevel_zero_last_raises"] = np.array(1)
    # compute_advantage (agent_trainer.py:60-137) on GRPO with unique uids and on GAE
    src = _extract("compute_advantage")

    class AdvantageEstimator:
        GAE, GRPO = "gae", "grpo"
        REINFORCE_PLUS_PLUS_BASELINE, REINFORCE_PLUS_PLUS, REMAX, RLOO = "rpb", "rpp", "remax", "rloo"

    class _DP:
        def __init__(self, batch, ntb):
            self.batch, self.non_tensor_batch = batch, ntb
    ns = {"AdvantageEstimator": AdvantageEstimator, "core_algos": core_algos, "torch": torch, "DataProto": object,
          "compute_response_mask": None}
    exec(src, ns)
    for est, bl in (("grpo", False), ("gae", False), ("gae", True)):
        dp = _DP({"token_level_rewards": torch.from_numpy(rew_turn), "values": torch.from_numpy(values),
                  "response_mask": tmask, "loss_mask": tmask}, {"uid": np.array([str(i) for i in range(B)], object)})
        dp = ns["compute_advantage"](dp, est, gamma=1.0, lam=0.95, multi_turn=True, bi_level_gae=bl,
                                     high_level_gamma=0.95)
        out[f"ca_{est}_{int(bl)}_adv"] = dp.batch["advantages"].numpy()
        out[f"ca_{est}_{int(bl)}_ret"] = dp.batch["returns"].numpy()
    # GRPO with real groups of 4 (index = group) for the segmented kernel
    idx = np.array([str(i // 4) for i in range(B)], object)
    a, _ = refshim.compute_grpo_outcome_advantage(torch.from_numpy(rew_turn), tmask.float(), idx)
    out["grpo_g4_adv"] = a.numpy()
    return out


def bandit_kat():
    """bandit/env.py:87-104 __main__: seeds 500..1499, action 1."""
    env = REGISTERED_ENVS["bandit"](REGISTERED_ENV_CONFIGS["bandit"]())
    rewards, swaps = [], []
    for s in range(500, 1500):
        env.reset(seed=s)
        swaps.append(int(env.ACTION_LOOKUP[1] == env.hi_arm_name))
        rewards.append(env.step(1)[1])
    return {"seeds": [500, 1500], "rewards": rewards, "hi_is_first": swaps,
            "mean": float(np.mean(rewards)), "std": float(np.std(rewards))}


def countdown_kat():
    nums, target = [3, 5, 2, 7], 3
    exprs = ["3 + 5 - 2 - 7 + 4", "5 + 7 - 3 - 2 + 0", "7 - 5 + 3 - 2", "(7 - 5) * 3 / 2", "7 - 5 + 3 - 2.0",
             "3 * 5 - 7 - 2", "", "x", "7 5 3 2", "2 ** 3 - 5 - 7", "7 // 2 + 3 - 5", "(7 - 5 + 3 - 2)",
             "-(-7) - 5 + 3 - 2", "7 - 5 + 3 - 2 = 3", "7 - 05 + 3 - 2", "7 -5 +3 -2", "7/0 + 5 - 3 - 2",
             "((7 - 5) + (3 - 2))", "7 % 5 + 3 - 2", "+7 - 5 + 3 - 2", "7 - 5 + 3 - 2 ", " 7 - 5 + 3 - 2",
             "7 * 5 / 3 / 2", "7 - 5 + 3 -- 2", "7 - 5 + 3 - (2", "1e1 - 5 - 2", "7 - 5 + 3 - 2 + 0*1",
             "7 * (5 - 3) - 2 * 5", "7 - 5 + 3 - 2\n", "7 - (5 - 3) * 2", "2 + 3 + 5 + 7", "7 - 5 + 3 - 2 - 1 + 1"]
    env = cd_env_mod.CountdownEnv.__new__(cd_env_mod.CountdownEnv)
    env.config = cd_env_mod.CountdownEnvConfig()
    gt = {"nums": nums, "target": target}
    res = []
    for e in exprs:
        res.append({"expr": e, "reward": float(env.compute_reward(e, gt)),
                    "format": bool(cd_env_mod.check_format(e, nums)),
                    "correct": bool(cd_env_mod.check_correctness(e, target))})
    return {"nums": nums, "target": target, "cases": res}


def main():
    np.savez_compressed(os.path.join(HERE, "sokoban_rooms.npz"), **sokoban_rooms())
    strings_all = {}
    for name, args in {"sokoban_es": ("SimpleSokoban", 8, 16, 5, 5, 1000, 20250704),
                       "sokoban8_es": ("LargerSokoban", 2, 16, 5, 5, 77, 4),
                       "frozenlake_es": ("FrozenLake", 8, 16, 8, 5, 1000, 20250705),
                       "bandit_es": ("Bandit", 4, 16, 1, 1, 1000, 20250706),
                       "countdown_es": ("Countdown", 4, 16, 4, 1, 1000, 20250707)}.items():
        rec, strings = run_es_trace(*args)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **rec)
        strings_all[name] = strings
    strings_all["countdown_data"] = CD_DATA
    strings_all["parse_response"] = parse_response_cases()
    strings_all["bandit_kat"] = bandit_kat()
    strings_all["countdown_kat"] = countdown_kat()
    with open(os.path.join(HERE, "strings.json"), "w") as f:
        json.dump(strings_all, f, indent=0)
    np.savez_compressed(os.path.join(HERE, "normalize.npz"), **normalize_cases())
    np.savez_compressed(os.path.join(HERE, "masks_scores.npz"), **masks_scores_cases())
    np.savez_compressed(os.path.join(HERE, "filter.npz"), **filter_cases())
    np.savez_compressed(os.path.join(HERE, "gae.npz"), **gae_cases())
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()
