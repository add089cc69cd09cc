"""Batched Countdown (replaces ragen/env/countdown/env.py:36-81; reward rule on device)."""
import itertools
from typing import List, Optional

import numpy as np
import torch

from .. import _lib, ops
from ..torch_ops import ep_args
from .base import BatchEnv
from .configs import CountdownEnvConfig


def has_solution(nums, target):
    """countdown/env.py:23-33: +-n1 +-n2 +-n3 +-n4 == target for some sign pattern."""
    nums = list(nums) + [0] * (4 - len(nums))
    return any(sum(c[i] * nums[i] for i in range(4)) == target for c in itertools.product([1, -1], repeat=4))


def synthetic_instances(n: int, seed: int):
    """Synthetic stand-in for the HF parquet (absent offline): 3-4 numbers in [1, 99] and a
    signed-sum target; only instances accepted by has_solution are kept."""
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        k = int(rng.integers(3, 5))
        nums = [int(x) for x in rng.integers(1, 100, size=k)]
        signs = rng.choice([-1, 1], size=k)
        target = int(sum(int(s) * v for s, v in zip(signs, nums)))
        if has_solution(nums, target):
            out.append({"nums": nums, "target": target})
    return out


def load_instances(config: CountdownEnvConfig):
    """CountdownEnv._get_data_from_parquet (countdown/env.py:45-49)."""
    if config.data is not None:
        return list(config.data)
    import datasets  # local parquet only; the HF download is not available offline
    df = datasets.load_dataset("parquet", data_files=config.train_path)["train"].select(range(config.max_instances))
    df = df.filter(lambda x: has_solution(x["nums"], x["target"]))
    return [{"nums": list(r["nums"]), "target": int(r["target"])} for r in df]


class CountdownBatch(BatchEnv):
    env_type = "countdown"
    MAX_NUMS = 4  # the reference's instances (has_solution pads to 4, countdown/env.py:25-27)

    def __init__(self, config: CountdownEnvConfig, n_envs, max_turns, max_actions_per_turn, device=None,
                 max_answer_bytes: int = 128, max_nums: int = MAX_NUMS):
        super().__init__(config or CountdownEnvConfig(), n_envs, max_turns, max_actions_per_turn, device)
        if not 1 <= max_nums <= 8:
            raise ValueError("max_nums: the kernel holds 1..8 numbers per instance")
        self.MAX_NUMS = int(max_nums)
        self.data = load_instances(self.config)
        self.Lmax = int(max_answer_bytes)
        d = self.device
        self.nums = torch.zeros(self.B, self.MAX_NUMS, dtype=torch.int32, device=d)
        self.n_nums = torch.zeros(self.B, dtype=torch.int32, device=d)
        self.target = torch.zeros(self.B, dtype=torch.int32, device=d)
        self.index = np.zeros(self.B, np.int64)
        self._last_obs = [None] * self.B

    def struct(self):
        c = self.config
        return _lib.Countdown(self.MAX_NUMS, float(c.score), float(c.format_score), self.nums.data_ptr(),
                              self.n_nums.data_ptr(), self.target.data_ptr())

    def action_lookup(self, i):
        return None  # language actions: every parsed answer is executed as is

    def map_actions(self, i, actions: List[str]) -> List[int]:
        return [k + 1 for k in range(len(actions))]

    def map_actions_many(self, rows, actions):
        return [list(range(1, len(a) + 1)) for a in actions]

    def reset(self, seeds):
        self.seeds = np.asarray(seeds, np.int64).copy()
        self.index = self.seeds % len(self.data)  # countdown/env.py:53
        nums = np.zeros((self.B, self.MAX_NUMS), np.int32)
        nn = np.zeros(self.B, np.int32)
        tg = np.zeros(self.B, np.int32)
        for i, ix in enumerate(self.index):
            inst = self.data[int(ix)]
            if len(inst["nums"]) > self.MAX_NUMS:
                raise NotImplementedError(f"{len(inst['nums'])} numbers > max_nums={self.MAX_NUMS} for this batch")
            nums[i, :len(inst["nums"])] = inst["nums"]
            nn[i] = len(inst["nums"])
            tg[i] = inst["target"]
        self.nums.copy_(torch.from_numpy(nums))
        self.n_nums.copy_(torch.from_numpy(nn))
        self.target.copy_(torch.from_numpy(tg))
        self.ep.reset_()
        self._last_obs = [None] * self.B
        self._invalidate()

    def parse_setup(self, enable_think: bool, action_sep: str, prepend: bool = True):
        """No action_lookup: the answers pass through as text (es_manager.py:235-236)."""
        return ops.parse_config(enable_think, self.K, action_sep, None, prepend=prepend), None, self.Lmax

    def encode_answers(self, answers: List[List[str]]):
        """[B][<=K] answer strings -> (u8[B,K,Lmax], i32[B,K]) host arrays (UTF-8)."""
        buf = np.zeros((self.B, self.K, self.Lmax), np.uint8)
        lens = np.zeros((self.B, self.K), np.int32)
        for i, lst in enumerate(answers):
            for k, a in enumerate((lst or [])[:self.K]):
                b = a.encode("utf-8")
                if len(b) > self.Lmax:
                    raise ValueError(f"answer longer than max_answer_bytes={self.Lmax}")
                buf[i, k, :len(b)] = np.frombuffer(b, np.uint8)
                lens[i, k] = len(b)
        return buf, lens

    def step_turn(self, turn, actions, n_actions, has_input, max_actions_per_traj, format_penalty, err=None,
                  answers: Optional[torch.Tensor] = None, answer_len: Optional[torch.Tensor] = None, **kw):
        c = self.config
        torch.ops.ragen_amd.countdown_step_turn(self.nums, self.n_nums, self.target, *ep_args(self.ep), actions,
                                                n_actions, has_input, err, answers, answer_len, int(turn),
                                                int(max_actions_per_traj), float(format_penalty), float(c.score),
                                                float(c.format_score))
        self._invalidate()

    def note_executed(self, turn, env_id, executed_ids):
        if executed_ids:
            self._last_obs[env_id] = turn

    def render(self, i: int) -> str:
        if self._last_obs[i] is None:  # countdown/env.py:55
            inst = self.data[int(self.index[i])]
            return f"Target: {inst['target']}, nums: {inst['nums']}"
        if self._host is None:
            self._host = self.ep.turn_reward.cpu().numpy()
        r = float(self._host[self._last_obs[i], i])
        # compute_reward returns int 0, format_score (0.1) or int score (1)
        rs = str(int(r)) if r in (0.0, float(self.config.score)) and float(r).is_integer() else str(r)
        return f"Your answer get {rs} points."
