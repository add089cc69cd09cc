"""Config objects with OmegaConf-like attribute access (hydra/omegaconf are absent offline).

``default_config()`` holds the hot-path keys of config/base.yaml and config/envs.yaml
(base.yaml:75-124, envs.yaml:1-148) with the same names and default values; task
overrides (``_2_sokoban`` etc.) are plain nested dict updates.  YAML files with the same
structure load through ``load_config``.
"""
import copy

import yaml


class AttrDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    @staticmethod
    def wrap(x):
        if isinstance(x, AttrDict):
            return x
        if isinstance(x, dict):
            return AttrDict({k: AttrDict.wrap(v) for k, v in x.items()})
        if isinstance(x, list):
            return [AttrDict.wrap(v) for v in x]
        return x


_SOKOBAN_INSTR = ("You are solving the Sokoban puzzle. You are the player and you need to push all boxes to targets. "
                  "When you are right next to a box, you can push it by moving in the same direction. You cannot push "
                  "a box through a wall, and you cannot pull a box. The answer should be a sequence of actions, like "
                  "<answer>Right || Right || Up</answer>")

DEFAULTS = {
    "model_path": "Qwen/Qwen2.5-0.5B-Instruct",
    "enable_response_mask": True,
    "actor_rollout_ref": {"rollout": {"response_length": 400, "rollout_filter_ratio": 0.25,
                                      "rollout_filter_type": "std", "n": 1}},
    "algorithm": {"gamma": 1.0, "lam": 1.0, "high_level_gamma": 0.95, "adv_estimator": "gae",
                  "bi_level_gae": False, "norm_adv_by_std_in_grpo": True},
    "agent_proxy": {"max_context_window": -1, "max_turn": 5, "action_sep": "||", "max_actions_per_turn": 5,
                    "use_turn_scores": False, "enable_think": True,
                    "reward_normalization": {"grouping": "state", "method": "identity"}},
    "es_manager": {"format_penalty": -0.1,
                   "train": {"env_groups": 8, "group_size": 16,
                             "env_configs": {"tags": ["SimpleSokoban"], "n_groups": [8]}},
                   "val": {"env_groups": 256, "group_size": 1,
                           "env_configs": {"tags": ["SimpleSokoban"], "n_groups": [256]}}},
    "custom_envs": {
        "SimpleSokoban": {"env_type": "sokoban", "max_actions_per_traj": 10, "env_instruction": _SOKOBAN_INSTR,
                          "max_tokens": 100,
                          "env_config": {"dim_x": 6, "dim_y": 6, "num_boxes": 1, "max_steps": 100}},
        "LargerSokoban": {"env_type": "sokoban", "max_actions_per_traj": 10, "env_instruction": _SOKOBAN_INSTR,
                          "max_tokens": 100,
                          "env_config": {"dim_x": 8, "dim_y": 8, "num_boxes": 2, "max_steps": 100,
                                         "search_depth": 10}},
        "Countdown": {"env_type": "countdown", "max_actions_per_traj": 1,
                      "env_instruction": ("You are solving the Countdown puzzle. You should use the num list to create "
                                          "an equation that equals the target. Example answer format: <think> To find "
                                          "an equation using [3, 5, 2] to get 4. Let's check 2 + 5 = 7, 7 - 3 = 4. So "
                                          "the answer is 2 + 5 - 3 = 4. </think><answer>2 + 5 - 3</answer>"),
                      "max_tokens": 100, "env_config": None},
        "Bandit": {"env_type": "bandit", "max_actions_per_traj": 1, "env_instruction": "", "max_tokens": 100,
                   "env_config": {"lo_arm_name": "Phoenix", "hi_arm_name": "Dragon"}},
        "BanditTest": {"env_type": "bandit", "max_actions_per_traj": 1, "env_instruction": "", "max_tokens": 100,
                       "env_config": {"lo_arm_name": "Trader", "hi_arm_name": "Librarian"}},
        "FrozenLake": {"env_type": "frozen_lake", "max_actions_per_traj": 10,
                       "env_instruction": ("You are solving the FrozenLake puzzle. Forbid the whole and go to the "
                                           "target. You may move to the unintended direction due to the slippery ice. "
                                           "Example answer format: <think>To forbid the hole and go to the target, I "
                                           "should go left then go up.</think><answer>Left || Up</answer>"),
                       "max_tokens": 100, "env_config": None},
    },
}


def _merge(a, b):
    for k, v in b.items():
        if isinstance(v, dict) and isinstance(a.get(k), dict):
            _merge(a[k], v)
        else:
            a[k] = copy.deepcopy(v)
    return a


def default_config(**overrides) -> AttrDict:
    cfg = copy.deepcopy(DEFAULTS)
    _merge(cfg, overrides)
    return AttrDict.wrap(cfg)


def env_task(tag: str, env_groups: int, group_size: int = 16, max_turn=None, max_actions_per_turn=None,
             **extra) -> AttrDict:
    """Config for a single-tag training run (the shape of config/_1_bandit.yaml .. _4_countdown.yaml)."""
    ov = {"es_manager": {"train": {"env_groups": env_groups, "group_size": group_size,
                                   "env_configs": {"tags": [tag], "n_groups": [env_groups]}}}}
    ap = {}
    if max_turn is not None:
        ap["max_turn"] = max_turn
    if max_actions_per_turn is not None:
        ap["max_actions_per_turn"] = max_actions_per_turn
    if ap:
        ov["agent_proxy"] = ap
    _merge(ov, extra)
    return default_config(**ov)


def load_config(path_or_dict) -> AttrDict:
    if isinstance(path_or_dict, dict):
        return default_config(**path_or_dict)
    with open(path_or_dict) as f:
        return default_config(**(yaml.safe_load(f) or {}))
