"""Import shims used ONLY by ``make_golden.py`` to run the read-only RAGEN reference
(``/root/reference``) inside this container and record golden vectors.

TEST INFRASTRUCTURE — never imported by the product package, never shipped as
product code, never run on the GPU box (the reference does not exist there).

The reference imports several third-party packages that are absent offline
(``gym``, ``gymnasium``, ``gym_sokoban``, ``verl``, ``hydra``, ``omegaconf``,
``tensordict``).  This module installs minimal stand-ins into ``sys.modules``.
Where the reference *calls* third-party arithmetic (gym_sokoban's step/reward,
gymnasium's FrozenLake transition table + ``categorical_sample``, verl's GAE /
masked_whiten / GRPO) the stand-in is a restatement of that package's published
algorithm.  Everything else that runs is
the reference's own code.

Pinned third-party semantics (versions unpinned in reference requirements.txt):
  * gym_sokoban 0.0.6 ``SokobanEnv.step/_push/_move/_calc_reward``      (App. A.1)
  * gymnasium >= 1.1 ``FrozenLakeEnv`` P-table with success_rate = 1/3   (App. A.2)
  * gymnasium ``utils.seeding.np_random`` = Generator(PCG64(SeedSequence(seed)))
  * verl (mid-2025) ``compute_gae_advantage_return`` legacy form, ``masked_whiten``,
    ``compute_grpo_outcome_advantage``                                    (App. A.4)
"""
import sys
import types
from collections import defaultdict

import numpy as np
import torch

REFERENCE = "/root/reference"


# --------------------------------------------------------------------------- gym
def _discrete_cls():
    class Discrete:
        def __init__(self, n, start=0, seed=None):
            self.n = int(n)
            self.start = int(start)

        def contains(self, x):
            return self.start <= int(x) < self.start + self.n
    return Discrete


def _np_random(seed=None):
    if seed is not None and not (isinstance(seed, (int, np.integer)) and seed >= 0):
        raise ValueError(f"Seed must be a python integer >= 0, actual type: {type(seed)}")
    seed_seq = np.random.SeedSequence(seed)
    return np.random.Generator(np.random.PCG64(seed_seq)), seed_seq.entropy


class _GymnasiumEnv:
    """gymnasium.Env: only the seeding behaviour the reference relies on."""
    _np_random = None
    metadata = {"render_modes": []}

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self._np_random, _ = _np_random(seed)

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random, _ = _np_random(None)
        return self._np_random

    @np_random.setter
    def np_random(self, value):
        self._np_random = value

    def close(self):
        pass


def _categorical_sample(prob_n, np_random):
    prob_n = np.asarray(prob_n)
    csprob_n = np.cumsum(prob_n)
    return np.argmax(csprob_n > np_random.random())


class _GymFrozenLake(_GymnasiumEnv):
    """Restatement of gymnasium.envs.toy_text.frozen_lake.FrozenLakeEnv (>= 1.1)."""

    def __init__(self, render_mode=None, desc=None, map_name="4x4", is_slippery=True,
                 success_rate=1.0 / 3.0):
        self.desc = desc = np.asarray(desc, dtype="c")
        self.nrow, self.ncol = nrow, ncol = desc.shape
        self.reward_range = (0, 1)
        nA, nS = 4, nrow * ncol
        self.initial_state_distrib = np.array(desc == b"S").astype("float64").ravel()
        self.initial_state_distrib /= self.initial_state_distrib.sum()
        self.P = {s: {a: [] for a in range(nA)} for s in range(nS)}

        def to_s(row, col):
            return row * ncol + col

        def inc(row, col, a):
            if a == 0:
                col = max(col - 1, 0)
            elif a == 1:
                row = min(row + 1, nrow - 1)
            elif a == 2:
                col = min(col + 1, ncol - 1)
            elif a == 3:
                row = max(row - 1, 0)
            return (row, col)

        def update_probability_matrix(row, col, action):
            new_row, new_col = inc(row, col, action)
            new_state = to_s(new_row, new_col)
            new_letter = desc[new_row, new_col]
            terminated = bytes(new_letter) in b"GH"
            reward = float(new_letter == b"G")
            return new_state, reward, terminated

        for row in range(nrow):
            for col in range(ncol):
                s = to_s(row, col)
                for a in range(4):
                    li = self.P[s][a]
                    letter = desc[row, col]
                    if letter in b"GH":
                        li.append((1.0, s, 0, True))
                    elif is_slippery:
                        for b in [(a - 1) % 4, a, (a + 1) % 4]:
                            p = success_rate if b == a else (1.0 - success_rate) / 2.0
                            li.append((p, *update_probability_matrix(row, col, b)))
                    else:
                        li.append((1.0, *update_probability_matrix(row, col, a)))
        self.render_mode = render_mode
        self.s = 0
        self.lastaction = None

    def reset(self, *, seed=None, options=None):
        super().reset(seed=seed)
        self.s = _categorical_sample(self.initial_state_distrib, self.np_random)
        self.lastaction = None
        return int(self.s), {"prob": 1}

    def step(self, a):
        transitions = self.P[self.s][a]
        i = _categorical_sample([t[0] for t in transitions], self.np_random)
        p, s, r, t = transitions[i]
        self.s = s
        self.lastaction = a
        return int(s), r, t, False, {"prob": p}


# ------------------------------------------------------------------ gym_sokoban
CHANGE_COORDINATES = {0: (-1, 0), 1: (1, 0), 2: (0, -1), 3: (0, 1)}


class _GymSokoban:
    """Restatement of gym_sokoban.envs.sokoban_env.SokobanEnv (0.0.6) step logic.

    The per-step RGB render that upstream returns from ``step`` is skipped (its
    result is discarded by RAGEN, sokoban/env.py:46)."""

    def __init__(self, dim_room=(10, 10), max_steps=120, num_boxes=4, num_gen_steps=None,
                 reset=True):
        self.dim_room = dim_room
        self.num_gen_steps = int(1.7 * (dim_room[0] + dim_room[1])) if num_gen_steps is None else num_gen_steps
        self.num_boxes = num_boxes
        self.boxes_on_target = 0
        self.penalty_for_step = -0.1
        self.penalty_box_off_target = -1
        self.reward_box_on_target = 1
        self.reward_finished = 10
        self.reward_last = 0
        self.max_steps = max_steps
        # upstream ctor calls reset() (RAGEN override, unseeded); not needed for goldens

    def step(self, action, observation_mode="rgb_array"):
        assert action in range(9)
        self.num_env_steps += 1
        moved_box = False
        if action == 0:
            moved_player = False
        elif action < 5:
            moved_player, moved_box = self._push(action)
        else:
            moved_player = self._move(action)
        self._calc_reward()
        done = self._check_if_done()
        info = {"action.moved_player": moved_player, "action.moved_box": moved_box}
        return None, self.reward_last, done, info

    def _push(self, action):
        change = CHANGE_COORDINATES[(action - 1) % 4]
        new_position = self.player_position + change
        current_position = self.player_position.copy()
        new_box_position = new_position + change
        if new_box_position[0] >= self.room_state.shape[0] or new_box_position[1] >= self.room_state.shape[1]:
            return False, False
        can_push_box = self.room_state[new_position[0], new_position[1]] in [3, 4]
        can_push_box &= self.room_state[new_box_position[0], new_box_position[1]] in [1, 2]
        if can_push_box:
            self.player_position = new_position
            self.room_state[(new_position[0], new_position[1])] = 5
            self.room_state[current_position[0], current_position[1]] = self.room_fixed[current_position[0], current_position[1]]
            box_type = 4
            if self.room_fixed[new_box_position[0], new_box_position[1]] == 2:
                box_type = 3
            self.room_state[new_box_position[0], new_box_position[1]] = box_type
            return True, True
        return self._move(action), False

    def _move(self, action):
        change = CHANGE_COORDINATES[(action - 1) % 4]
        new_position = self.player_position + change
        current_position = self.player_position.copy()
        if self.room_state[new_position[0], new_position[1]] in [1, 2]:
            self.player_position = new_position
            self.room_state[(new_position[0], new_position[1])] = 5
            self.room_state[current_position[0], current_position[1]] = self.room_fixed[current_position[0], current_position[1]]
            return True
        return False

    def _calc_reward(self):
        self.reward_last = self.penalty_for_step
        empty_targets = self.room_state == 2
        player_on_target = (self.room_fixed == 2) & (self.room_state == 5)
        total_targets = empty_targets | player_on_target
        current_boxes_on_target = self.num_boxes - np.where(total_targets)[0].shape[0]
        if current_boxes_on_target > self.boxes_on_target:
            self.reward_last += self.reward_box_on_target
        elif current_boxes_on_target < self.boxes_on_target:
            self.reward_last += self.penalty_box_off_target
        if self._check_if_all_boxes_on_target():
            self.reward_last += self.reward_finished
        self.boxes_on_target = current_boxes_on_target

    def _check_if_done(self):
        return self._check_if_all_boxes_on_target() or self._check_if_maxsteps()

    def _check_if_maxsteps(self):
        return self.max_steps == self.num_env_steps

    def _check_if_all_boxes_on_target(self):
        empty_targets = self.room_state == 2
        player_hiding_target = (self.room_fixed == 2) & (self.room_state == 5)
        return np.where(empty_targets | player_hiding_target)[0].shape[0] == 0

    def close(self):
        pass


# ------------------------------------------------------------------------- verl
def masked_mean(values, mask, axis=None):
    return (values * mask).sum(axis=axis) / mask.sum(axis=axis)


def masked_var(values, mask, unbiased=True):
    mean = masked_mean(values, mask)
    centered_values = values - mean
    variance = masked_mean(centered_values ** 2, mask)
    if unbiased:
        mask_sum = mask.sum()
        if mask_sum == 0:
            raise ValueError("At least one element in the mask has to be 1.")
        if mask_sum == 1:
            raise ValueError("The sum of the mask is one, which can cause a division by zero.")
        bessel_correction = mask_sum / (mask_sum - 1)
        variance = variance * bessel_correction
    return variance


def masked_whiten(values, mask, shift_mean=True):
    mean, var = masked_mean(values, mask), masked_var(values, mask)
    whitened = (values - mean) * torch.rsqrt(var + 1e-8)
    if not shift_mean:
        whitened += mean
    return whitened


def compute_gae_advantage_return(token_level_rewards, values, response_mask, gamma, lam):
    """verl legacy form (App. A.4)."""
    with torch.no_grad():
        lastgaelam = 0
        advantages_reversed = []
        gen_len = token_level_rewards.shape[-1]
        for t in reversed(range(gen_len)):
            nextvalues = values[:, t + 1] if t < gen_len - 1 else 0.0
            delta = token_level_rewards[:, t] + gamma * nextvalues - values[:, t]
            lastgaelam = delta + gamma * lam * lastgaelam
            advantages_reversed.append(lastgaelam)
        advantages = torch.stack(advantages_reversed[::-1], dim=1)
        returns = advantages + values
        advantages = masked_whiten(advantages, response_mask)
    return advantages, returns


def compute_gae_advantage_return_masked(token_level_rewards, values, response_mask, gamma, lam):
    """verl newer form (App. A.4), mask given as float."""
    with torch.no_grad():
        nextvalues = 0
        lastgaelam = 0
        advantages_reversed = []
        gen_len = token_level_rewards.shape[-1]
        m = response_mask.float()
        for t in reversed(range(gen_len)):
            delta = token_level_rewards[:, t] + gamma * nextvalues - values[:, t]
            lastgaelam_ = delta + gamma * lam * lastgaelam
            nextvalues = values[:, t] * m[:, t] + (1 - m[:, t]) * nextvalues
            lastgaelam = lastgaelam_ * m[:, t] + (1 - m[:, t]) * lastgaelam
            advantages_reversed.append(lastgaelam)
        advantages = torch.stack(advantages_reversed[::-1], dim=1)
        returns = advantages + values
        advantages = masked_whiten(advantages, response_mask)
    return advantages, returns


def compute_grpo_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6,
                                   norm_adv_by_std_in_grpo=True):
    scores = token_level_rewards.sum(dim=-1)
    id2score = defaultdict(list)
    id2mean, id2std = {}, {}
    with torch.no_grad():
        bsz = scores.shape[0]
        for i in range(bsz):
            id2score[index[i]].append(scores[i])
        for idx in id2score:
            if len(id2score[idx]) == 1:
                id2mean[idx] = torch.tensor(0.0)
                id2std[idx] = torch.tensor(1.0)
            elif len(id2score[idx]) > 1:
                id2mean[idx] = torch.mean(torch.tensor(id2score[idx]))
                id2std[idx] = torch.std(torch.tensor([id2score[idx]]))
            else:
                raise ValueError(f"no score in prompt index: {idx}")
        for i in range(bsz):
            if norm_adv_by_std_in_grpo:
                scores[i] = (scores[i] - id2mean[index[i]]) / (id2std[index[i]] + epsilon)
            else:
                scores[i] = scores[i] - id2mean[index[i]]
        scores = scores.unsqueeze(-1) * response_mask
    return scores, scores


# ------------------------------------------------------------------ installation
def _mod(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def install():
    """Install the stand-ins and put the reference on sys.path."""
    if REFERENCE not in sys.path:
        sys.path.insert(0, REFERENCE)
    Discrete = _discrete_cls()

    # gym (used by sokoban/env.py only for spaces.discrete.Discrete)
    gym = _mod("gym", Env=object)
    spaces = _mod("gym.spaces")
    spaces.discrete = _mod("gym.spaces.discrete", Discrete=Discrete)
    gym.spaces = spaces

    # gymnasium
    gn = _mod("gymnasium", Env=_GymnasiumEnv)
    gsp = _mod("gymnasium.spaces")
    gsp.discrete = _mod("gymnasium.spaces.discrete", Discrete=Discrete)
    gn.spaces = gsp
    gut = _mod("gymnasium.utils")
    gut.seeding = _mod("gymnasium.utils.seeding", np_random=_np_random)
    gn.utils = gut
    genvs = _mod("gymnasium.envs")
    gtt = _mod("gymnasium.envs.toy_text")
    gtt.frozen_lake = _mod("gymnasium.envs.toy_text.frozen_lake", FrozenLakeEnv=_GymFrozenLake)
    genvs.toy_text = gtt
    gn.envs = genvs

    # gym_sokoban
    gs = _mod("gym_sokoban")
    ge = _mod("gym_sokoban.envs")
    ge.sokoban_env = _mod("gym_sokoban.envs.sokoban_env", SokobanEnv=_GymSokoban)
    gs.envs = ge

    # hydra / omegaconf / tensordict
    def _main(*a, **k):
        return lambda f: f
    _mod("hydra", main=_main)

    class _OC:
        @staticmethod
        def register_new_resolver(*a, **k):
            pass
    _mod("omegaconf", OmegaConf=_OC, DictConfig=dict)

    class TensorDict(dict):
        def __init__(self, d, batch_size=None):
            super().__init__(d)
            self.batch_size = batch_size
    _mod("tensordict", TensorDict=TensorDict)

    # verl
    class DataProto:
        def __init__(self, batch=None, non_tensor_batch=None, meta_info=None):
            self.batch = batch
            self.non_tensor_batch = non_tensor_batch or {}
            self.meta_info = meta_info or {}
    verl = _mod("verl", DataProto=DataProto)
    vu = _mod("verl.utils")
    vu.torch_functional = _mod("verl.utils.torch_functional", masked_whiten=masked_whiten,
                                masked_mean=masked_mean, masked_var=masked_var)
    vd = _mod("verl.utils.dataset")
    vd.rl_dataset = _mod("verl.utils.dataset.rl_dataset", collate_fn=lambda x: x)
    vu.dataset = vd
    verl.utils = vu
    vt = _mod("verl.trainer")
    vp = _mod("verl.trainer.ppo")
    vp.core_algos = _mod(
        "verl.trainer.ppo.core_algos", torch=torch, verl_F=vu.torch_functional,
        compute_gae_advantage_return=compute_gae_advantage_return,
        compute_grpo_outcome_advantage=compute_grpo_outcome_advantage,
        __all__=["torch", "verl_F", "compute_gae_advantage_return", "compute_grpo_outcome_advantage"])
    vt.ppo = vp
    verl.trainer = vt
