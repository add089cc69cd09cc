"""Batched Bandit (replaces ragen/env/bandit/env.py:14-86)."""
import numpy as np
import torch

from .. import _lib, ops
from ..torch_ops import ep_args
from .base import BatchEnv
from .configs import BanditEnvConfig

# bandit/env.py:6-12 (exact text, trailing spaces included: it is part of the observation)
INIT_PROMPT = ("You are playing a bandit game. Goal: Maximize your total reward by choosing which arm to pull. \n"
               "Game Rules: \n"
               "1. There are 2 arms, named {name_a} and {name_b}\n"
               "2. Each arm has its own reward distribution, related to their names. \n"
               "3. Analyze the symbolic meaning of each arm's name to guess how their reward distribution might "
               "behave.\n"
               "4. Based on the symbolic meaning of their names, which arm do you think is more likely to give higher "
               "rewards on average? Choose between {name_a} and {name_b}, and output like <answer> {name_a} "
               "</answer> or <answer> {name_b} </answer>.\n")


class BanditBatch(BatchEnv):
    env_type = "bandit"

    def __init__(self, config: BanditEnvConfig, n_envs, max_turns, max_actions_per_turn, device=None):
        super().__init__(config or BanditEnvConfig(), n_envs, max_turns, max_actions_per_turn, device)
        d = self.device
        self.hi_is_first = torch.zeros(self.B, dtype=torch.uint8, device=d)
        self.rng = torch.zeros(4, self.B, dtype=torch.int64, device=d)
        self._hi_first_host = np.zeros(self.B, np.uint8)
        self._last_obs = [None] * self.B

    def struct(self):
        c = self.config
        return _lib.Bandit(int(c.action_space_start), float(c.lo_arm_score), float(c.hi_arm_loscore),
                           float(c.hi_arm_hiscore), float(c.hi_arm_hiscore_prob), self.hi_is_first.data_ptr(),
                           self.rng.data_ptr())

    # BanditEnv.reset + _randomize_arms (bandit/env.py:25-39, :52-60): the env's Generator
    # reseeded (gymnasium seeding.np_random) and one draw < 0.5 -> lo arm first; seeded on the
    # device for every env at once (rmi_pcg64_seed)
    def reset(self, seeds):
        self.seeds = np.asarray(seeds, np.int64).copy()
        rng, last = torch.ops.ragen_amd.pcg64_seed(torch.from_numpy(self.seeds).to(self.device), 1)
        self.rng.copy_(rng)
        self.hi_is_first.copy_((last >= 0.5).to(torch.uint8))
        self._hi_first_host = self.hi_is_first.cpu().numpy()
        self.ep.reset_()
        self._last_obs = [None] * self.B
        self._invalidate()

    def load_state(self, hi_first, rng):
        self._hi_first_host = np.asarray(hi_first, np.uint8).copy()
        self.hi_is_first.copy_(torch.from_numpy(self._hi_first_host))
        self.rng.copy_(torch.from_numpy(np.ascontiguousarray(rng).view(np.int64)))
        self.ep.reset_()
        self._last_obs = [None] * self.B
        self._invalidate()

    def parse_setup(self, enable_think: bool, action_sep: str, prepend: bool = True):
        """Per-env lookup (bandit/env.py:25-39): column 1 = hi arm first, selected by hi_is_first."""
        c, s = self.config, int(self.config.action_space_start)
        lo_first = {s: c.lo_arm_name, s + 1: c.hi_arm_name}
        hi_first = {s: c.hi_arm_name, s + 1: c.lo_arm_name}
        return ops.parse_config(enable_think, self.K, action_sep, lo_first, hi_first, prepend=prepend), \
            self.hi_is_first, 0

    def parse_sel(self):
        return self.hi_is_first

    def map_actions_many(self, rows, actions):
        c, s0 = self.config, int(self.config.action_space_start)
        hi, lo = c.hi_arm_name.lower(), c.lo_arm_name.lower()
        revs = ({lo: s0, hi: s0 + 1}, {hi: s0, lo: s0 + 1})  # by hi_is_first (action_lookup below)
        hf = self._hi_first_host
        return [[revs[1 if hf[i] else 0].get(a.lower(), 0) for a in acts] for i, acts in zip(rows, actions)]

    def action_lookup(self, i):
        c, s = self.config, int(self.config.action_space_start)
        if self._hi_first_host[i]:
            return {s: c.hi_arm_name, s + 1: c.lo_arm_name}
        return {s: c.lo_arm_name, s + 1: c.hi_arm_name}

    def step_turn(self, turn, actions, n_actions, has_input, max_actions_per_traj, format_penalty, err=None, **kw):
        c = self.config
        torch.ops.ragen_amd.bandit_step_turn(self.hi_is_first, self.rng, *ep_args(self.ep), actions, n_actions,
                                             has_input, err, int(turn), int(max_actions_per_traj),
                                             float(format_penalty), int(c.action_space_start), float(c.lo_arm_score),
                                             float(c.hi_arm_loscore), float(c.hi_arm_hiscore),
                                             float(c.hi_arm_hiscore_prob))
        self._invalidate()

    def render(self, i: int) -> str:
        # render_cache (bandit/env.py:49-50): the init prompt after reset,
        # f"{arm_name}: {reward} points" after a step (bandit/env.py:66-67)
        if self._last_obs[i] is None:
            lk, s = self.action_lookup(i), int(self.config.action_space_start)
            return INIT_PROMPT.format(name_a=lk[s], name_b=lk[s + 1])
        if self._host is None:
            self._host = self.ep.turn_reward.cpu().numpy()
        turn, arm = self._last_obs[i]
        return f"{arm}: {float(self._host[turn, i])} points"

    def note_executed(self, turn, env_id, executed_ids):
        """Called by the facade after a turn with the ids the kernel executed."""
        if executed_ids:
            self._last_obs[env_id] = (turn, self.action_lookup(env_id)[executed_ids[-1]])
