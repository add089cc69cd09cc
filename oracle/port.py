"""Reference-shaped CPU port of the Sokoban rollout — TEST INFRASTRUCTURE / cpu_baseline.

Per-env Python objects exactly as the reference runs them on the Ray driver:
EnvStateManager.step's per-env loop (es_manager.py:105-171) with its name->id map
(:230-240), history/rollout-cache dict bookkeeping and a text render per step and per turn,
over SokobanEnv.step (sokoban/env.py:44-51) on gym_sokoban's numpy step logic
(App. A.1; the upstream per-step RGB render is omitted, so this baseline is FASTER than
the true reference path).  Timed by bench.py's cpu_baseline leg; its outputs are checked
against the C oracle in tests/test_oracle_port.py.
"""
import numpy as np

GRID_LOOKUP = {0: "#", 1: "_", 2: "O", 3: "√", 4: "X", 5: "P", 6: "S"}
ACTION_LOOKUP = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}
NAMES = {0: "jump", 1: "Up", 2: "down", 3: "LEFT", 4: "Right"}  # synthetic id -> LLM action text
CHANGE = {0: (-1, 0), 1: (1, 0), 2: (0, -1), 3: (0, 1)}


class SokobanPort:
    def __init__(self, fixed, state, player, num_boxes=1, max_steps=100):
        self.room_fixed = fixed.astype(np.int64)
        self.room_state = state.astype(np.int64)
        self.player_position = np.array(player, dtype=np.int64)
        self.num_boxes, self.max_steps = num_boxes, max_steps
        self.num_env_steps = self.boxes_on_target = 0
        self.reward_last = 0
        self.config_action_lookup = ACTION_LOOKUP

    # gym_sokoban
    def _push(self, action):
        change = CHANGE[(action - 1) % 4]
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
            self.room_state[current_position[0], current_position[1]] = \
                self.room_fixed[current_position[0], current_position[1]]
            box_type = 3 if self.room_fixed[new_box_position[0], new_box_position[1]] == 2 else 4
            self.room_state[new_box_position[0], new_box_position[1]] = box_type
            return True, True
        return self._move(action), False

    def _move(self, action):
        change = CHANGE[(action - 1) % 4]
        new_position = self.player_position + change
        current_position = self.player_position.copy()
        if self.room_state[new_position[0], new_position[1]] in [1, 2]:
            self.player_position = new_position
            self.room_state[(new_position[0], new_position[1])] = 5
            self.room_state[current_position[0], current_position[1]] = \
                self.room_fixed[current_position[0], current_position[1]]
            return True
        return False

    def _calc_reward(self):
        self.reward_last = -0.1
        empty_targets = self.room_state == 2
        player_on_target = (self.room_fixed == 2) & (self.room_state == 5)
        total_targets = empty_targets | player_on_target
        cur = self.num_boxes - np.where(total_targets)[0].shape[0]
        if cur > self.boxes_on_target:
            self.reward_last += 1
        elif cur < self.boxes_on_target:
            self.reward_last += -1
        if self._all_on_target():
            self.reward_last += 10
        self.boxes_on_target = cur

    def _all_on_target(self):
        empty_targets = self.room_state == 2
        player_hiding_target = (self.room_fixed == 2) & (self.room_state == 5)
        return np.where(empty_targets | player_hiding_target)[0].shape[0] == 0

    def gym_step(self, action):
        self.num_env_steps += 1
        if action < 5:
            self._push(action)
        else:
            self._move(action)
        self._calc_reward()
        done = self._all_on_target() or (self.max_steps == self.num_env_steps)
        return None, self.reward_last, done, {}

    # RAGEN SokobanEnv
    def step(self, action):
        previous_pos = self.player_position
        _, reward, done, _ = self.gym_step(action)
        next_obs = self.render()
        action_effective = not np.array_equal(previous_pos, self.player_position)
        info = {"action_is_effective": action_effective, "action_is_valid": True,
                "success": self.boxes_on_target == self.num_boxes}
        return next_obs, reward, done, info

    def render(self):
        room = np.where((self.room_state == 5) & (self.room_fixed == 2), 6, self.room_state)
        return "\n".join("".join(GRID_LOOKUP.get(cell, "?") for cell in row) for row in room.tolist())


def make_sokoban_envs(fixed, state, player, H=6, W=6):
    envs = []
    for i in range(fixed.shape[0]):
        env = SokobanPort(fixed[i].reshape(H, W), state[i].reshape(H, W), player[i])
        status = {"truncated": False, "terminated": False, "num_actions": 0, "rewards": []}
        cache = {"env_id": i, "history": [{"state": env.render(), "actions_left": 10}], "penalty": 0}
        envs.append({"env": env, "status": status, "cache": cache, "max_actions_per_traj": 10})
    return envs


def es_step(envs, all_env_inputs, format_penalty=-0.1):
    """EnvStateManager.step (es_manager.py:105-171) over the port envs."""
    outputs = []
    for env_input in all_env_inputs:
        entry = envs[env_input["env_id"]]
        env, status, cache = entry["env"], entry["status"], entry["cache"]
        actions_left_before = entry["max_actions_per_traj"] - status["num_actions"]
        rev = {v.lower(): k for k, v in env.config_action_lookup.items()}
        acts = [a.lower() for a in env_input["actions"]]
        valid = [rev[a] for a in acts if a in rev]
        acc_reward, turn_info, turn_done, executed = 0, {}, False, []
        for a in valid[:actions_left_before]:
            _, reward, done, info = env.step(a)
            acc_reward += reward
            turn_info.update(info)
            executed.append(a)
            if done:
                turn_done = True
                break
        if len(valid) != len(env_input["actions"]) or not valid:
            cache["penalty"] += format_penalty
        obs = env.render()
        status["num_actions"] += len(executed)
        status["rewards"].append(acc_reward)
        if turn_done:
            status["terminated"] = True
            status["truncated"] = not turn_info.get("success", False)
        cache["history"][-1].update({"actions": executed, "reward": acc_reward, "info": turn_info,
                                     "llm_response": env_input["llm_response"],
                                     "llm_raw_response": env_input["llm_raw_response"]})
        cache["history"].append({"state": obs, "actions_left": entry["max_actions_per_traj"] - status["num_actions"]})
        if status["num_actions"] >= entry["max_actions_per_traj"] and not turn_done:
            status["truncated"] = status["terminated"] = True
            turn_done = True
        if not turn_done:
            outputs.append(cache)
    return outputs


def sokoban_rollout(envs, ids, n, max_actions=10):
    """Turn loop (agent_proxy.py:143-159 without the LLM): returns env.step calls made."""
    T = ids.shape[0]
    active = list(range(len(envs)))
    steps0 = sum(e["env"].num_env_steps for e in envs)
    for t in range(T):
        inputs = [{"env_id": i, "llm_response": "", "llm_raw_response": "",
                   "actions": [NAMES[int(a)] for a in ids[t, i, :int(n[t, i])]]} for i in active]
        outs = es_step(envs, inputs)
        active = [o["env_id"] for o in outs]
        if not active:
            break
    return sum(e["env"].num_env_steps for e in envs) - steps0


def timed_rollouts(fixed, state0, player0, ids, n, max_actions, reps):
    """``reps`` fresh rollouts of these envs (reset excluded from timing) -> (env steps, seconds).
    The unit of work of bench.py's multi-process CPU baseline (one call per worker process)."""
    import time
    steps, dt = 0, 0.0
    for _ in range(reps):
        envs = make_sokoban_envs(fixed, state0, player0)
        t0 = time.perf_counter()
        steps += sokoban_rollout(envs, ids, n, max_actions)
        dt += time.perf_counter() - t0
    return steps, dt


def verl_gae_whiten(r, v, mask, gamma=1.0, lam=1.0):
    """verl compute_gae_advantage_return (legacy; SURVEY App. A.4, called from
    agent_trainer.py:77-83) + masked_whiten (core_algos.py:90) as the reference runs them:
    torch on the host, one Python iteration per token column.  CPU baseline of the advantage
    step; checked against the C oracle in tests/test_oracle_port.py.  torch tensors in/out."""
    import torch
    with torch.no_grad():
        L = r.shape[1]
        last = torch.zeros_like(r[:, 0])
        rev = []
        for t in reversed(range(L)):
            nxt = v[:, t + 1] if t < L - 1 else 0.0
            delta = r[:, t] + gamma * nxt - v[:, t]
            last = delta + gamma * lam * last
            rev.append(last)
        adv = torch.stack(rev[::-1], dim=1)
        ret = adv + v
        m = mask.to(adv.dtype)
        n = m.sum()
        mean = (adv * m).sum() / n
        var = (((adv - mean) ** 2) * m).sum() / n * (n / (n - 1))  # unbiased, as verl masked_var
        adv = (adv - mean) * torch.rsqrt(var + 1e-8)
        return adv, ret
