"""Parity oracle — TEST INFRASTRUCTURE.

CPU restatement of RAGEN's rollout/advantage hot path, used only by tests/,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` — as the checker,
never as the product path (``ragen_amd`` has no CPU fallback and never imports this).

  * ``oracle/ragen_oracle.c``  plain-C restatement (built by ``oracle/Makefile`` into
    ``oracle/_build/libragen_oracle.so``), bound here with ctypes over numpy arrays;
  * ``countdown_reward``        the reference's own three-line rule (countdown/env.py:9-21)
    evaluated with Python's ``re`` and ``eval`` — i.e. the exact reference semantics;
  * ``oracle/port.py``          per-env Python objects mirroring EnvStateManager + the env
    classes (the timed CPU baseline).

Pinned against tests/golden/*.npz (recorded by running the reference itself) in
tests/test_oracle.py.
"""
import ctypes
import os
import re
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libragen_oracle.so")

FLAG_TERM, FLAG_TRUNC, FLAG_DONE = 1, 2, 4
INFO_PRESENT, INFO_EFF, INFO_VALID, INFO_SUCC = 1, 2, 4, 8


def build():
    r = subprocess.run(["make", "-s", "-C", HERE], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + r.stdout + r.stderr)
    return LIB_PATH


class _Ep(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int32), ("T", ctypes.c_int32)] + [
        (n, ctypes.c_void_p) for n in ("num_actions", "flags", "n_turns", "penalty", "turn_reward", "turn_info",
                                       "turn_exec")]


class _Turn(ctypes.Structure):
    _fields_ = [("turn", ctypes.c_int32), ("K", ctypes.c_int32), ("actions", ctypes.c_void_p),
                ("n_actions", ctypes.c_void_p), ("has_input", ctypes.c_void_p),
                ("max_actions_per_traj", ctypes.c_int32), ("format_penalty", ctypes.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.orc_pcg64_random.restype = ctypes.c_double
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class Episode:
    """Host mirror of the episode SoA (same layout as ragen_amd.ops.EpisodeState)."""

    def __init__(self, B, T):
        self.num_actions = np.zeros(B, np.int32)
        self.flags = np.zeros(B, np.uint8)
        self.n_turns = np.zeros(B, np.int32)
        self.penalty = np.zeros(B, np.float64)
        self.turn_reward = np.zeros((T, B), np.float64)
        self.turn_info = np.zeros((T, B), np.uint8)
        self.turn_exec = np.zeros((T, B), np.uint8)
        self.B, self.T = B, T

    def struct(self):
        return _Ep(self.B, self.T, _p(self.num_actions), _p(self.flags), _p(self.n_turns), _p(self.penalty),
                   _p(self.turn_reward), _p(self.turn_info), _p(self.turn_exec))


def _turn(turn, actions, n_actions, has_input, max_actions, fpen):
    actions = np.ascontiguousarray(actions, np.int8)
    n_actions = np.ascontiguousarray(n_actions, np.uint8)
    hi = None if has_input is None else np.ascontiguousarray(has_input, np.uint8)
    t = _Turn(turn, actions.shape[1], _p(actions), _p(n_actions), _p(hi), max_actions, fpen)
    return t, (actions, n_actions, hi)


def sokoban_turn(H, W, num_boxes, max_steps, fixed, state, player, nes, bot, ep, turn, actions, n_actions,
                 has_input=None, max_actions=10, fpen=-0.1):
    t, keep = _turn(turn, actions, n_actions, has_input, max_actions, fpen)
    err = np.zeros(ep.B, np.uint8)
    lib().orc_sokoban_turn(H, W, num_boxes, max_steps, _p(fixed), _p(state), _p(player), _p(nes), _p(bot),
                           ctypes.byref(ep.struct()), ctypes.byref(t), _p(err))
    return err


def frozenlake_turn(nrow, ncol, slippery, cs, desc, s, rng, ep, turn, actions, n_actions, has_input=None,
                    max_actions=10, fpen=-0.1):
    t, keep = _turn(turn, actions, n_actions, has_input, max_actions, fpen)
    err = np.zeros(ep.B, np.uint8)
    lib().orc_frozenlake_turn(nrow, ncol, int(slippery), ctypes.c_double(cs[0]), ctypes.c_double(cs[1]),
                              ctypes.c_double(cs[2]), _p(desc), _p(s), _p(rng), ctypes.byref(ep.struct()),
                              ctypes.byref(t), _p(err))
    return err


def bandit_turn(start, lo, hl, hh, hp, hi_first, rng, ep, turn, actions, n_actions, has_input=None, max_actions=1,
                fpen=-0.1):
    t, keep = _turn(turn, actions, n_actions, has_input, max_actions, fpen)
    err = np.zeros(ep.B, np.uint8)
    lib().orc_bandit_turn(start, ctypes.c_double(lo), ctypes.c_double(hl), ctypes.c_double(hh), ctypes.c_double(hp),
                          _p(hi_first), _p(rng), ctypes.byref(ep.struct()), ctypes.byref(t), _p(err))
    return err


def pcg64_random(st):
    st = np.ascontiguousarray(st, np.uint64)
    u = lib().orc_pcg64_random(_p(st))
    return u, st


def rollout_metrics(ep):
    out = np.zeros((ep.B, 4), np.float64)
    lib().orc_rollout_metrics(ctypes.byref(ep.struct()), _p(out))
    return out


def trajectory_scores(ep):
    s = np.zeros(ep.B, np.float32)
    p = np.zeros(ep.B, np.float32)
    lib().orc_trajectory_scores(ctypes.byref(ep.struct()), _p(s), _p(p))
    return s, p


NORM = {"identity": 0, "mean": 1, "mean_std": 2, "asym_clip": 3}


def group_normalize(score, pen, seg, method):
    score = np.ascontiguousarray(score, np.float32)
    pen = None if pen is None else np.ascontiguousarray(pen, np.float32)
    seg = np.ascontiguousarray(seg, np.int32)
    out = np.zeros_like(score)
    lib().orc_group_normalize(_p(score), _p(pen), _p(seg), len(seg) - 1, len(score), NORM[method], _p(out))
    return out


def gae(r, v, mask, gamma, lam, variant="legacy"):
    r = np.ascontiguousarray(r, np.float32)
    v = np.ascontiguousarray(v, np.float32)
    m = np.ascontiguousarray(mask, np.uint8)
    adv = np.zeros_like(r)
    ret = np.zeros_like(r)
    lib().orc_gae(_p(r), _p(v), _p(m), ctypes.c_int64(r.shape[0]), ctypes.c_int64(r.shape[1]),
                  ctypes.c_double(gamma), ctypes.c_double(lam), 0 if variant == "legacy" else 1, _p(adv), _p(ret))
    return adv, ret


def bilevel_gae(r, v, mask, gamma, lam, hlg):
    r = np.ascontiguousarray(r, np.float32)
    v = np.ascontiguousarray(v, np.float32)
    m = np.ascontiguousarray(mask, np.uint8)
    adv = np.zeros_like(r)
    ret = np.zeros_like(r)
    err = np.zeros(r.shape[0], np.uint8)
    lib().orc_bilevel_gae(_p(r), _p(v), _p(m), ctypes.c_int64(r.shape[0]), ctypes.c_int64(r.shape[1]),
                          ctypes.c_double(gamma), ctypes.c_double(lam), ctypes.c_double(hlg), _p(adv), _p(ret),
                          _p(err))
    return adv, ret, err


def masked_whiten(x, mask):
    x = np.array(x, np.float32, copy=True)
    m = np.ascontiguousarray(mask, np.uint8)
    rc = lib().orc_masked_whiten(_p(x), _p(m), ctypes.c_int64(x.shape[0]), ctypes.c_int64(x.shape[1]))
    if rc:
        raise ValueError("masked_whiten: mask sum must be >= 2")
    return x


def grpo(r, mask, seg, eps=1e-6, norm_by_std=True):
    r = np.ascontiguousarray(r, np.float32)
    m = np.ascontiguousarray(mask, np.uint8)
    seg = np.ascontiguousarray(seg, np.int32)
    adv = np.zeros_like(r)
    ret = np.zeros_like(r)
    lib().orc_grpo(_p(r), _p(m), ctypes.c_int64(r.shape[0]), ctypes.c_int64(r.shape[1]), _p(seg), len(seg) - 1,
                   ctypes.c_double(eps), int(norm_by_std), _p(adv), _p(ret))
    return adv, ret


def reinforce_pp(r, mask, gamma, whiten=True):
    """verl REINFORCE++ (ragen_oracle.c: orc_reinforce_pp): -> (adv, ret); adv = the whitened
    returns times the mask (whitening in double, as orc_masked_whiten)."""
    r = np.ascontiguousarray(r, np.float32)
    m = np.ascontiguousarray(mask, np.uint8)
    ret = np.zeros_like(r)
    lib().orc_reinforce_pp(_p(r), _p(m), ctypes.c_int64(r.shape[0]), ctypes.c_int64(r.shape[1]),
                           ctypes.c_double(gamma), _p(ret))
    adv = masked_whiten(ret, m) * (m != 0) if whiten else ret.copy()
    return adv.astype(np.float32), ret


def remax(r, mask, base):
    r = np.ascontiguousarray(r, np.float32)
    m = np.ascontiguousarray(mask, np.uint8)
    base = np.ascontiguousarray(base, np.float32)
    adv = np.zeros_like(r)
    ret = np.zeros_like(r)
    lib().orc_remax(_p(r), _p(m), _p(base), ctypes.c_int64(r.shape[0]), ctypes.c_int64(r.shape[1]), _p(adv), _p(ret))
    return adv, ret


def rloo(r, mask, seg):
    r = np.ascontiguousarray(r, np.float32)
    m = np.ascontiguousarray(mask, np.uint8)
    seg = np.ascontiguousarray(seg, np.int32)
    adv = np.zeros_like(r)
    lib().orc_rloo(_p(r), _p(m), ctypes.c_int64(r.shape[0]), ctypes.c_int64(r.shape[1]), _p(seg), len(seg) - 1,
                   _p(adv))
    return adv, adv


def reinforce_pp_baseline(r, mask, seg):
    """verl REINFORCE++-baseline: the group-centred score tiled over the mask (GRPO without
    std), whitened, times the mask."""
    adv, _ = grpo(r, mask, seg, norm_by_std=False)
    m = np.ascontiguousarray(mask, np.uint8)
    adv = masked_whiten(adv, m) * (m != 0)
    return adv.astype(np.float32), adv.astype(np.float32)


def filter_groups(scores, G, gs, ratio, ftype):
    scores = np.ascontiguousarray(scores, np.float32)
    sd = np.zeros(G, np.float32)
    mx = np.zeros(G, np.float32)
    mn = np.zeros(G, np.float32)
    keep = np.zeros(G, np.uint8)
    met = np.zeros(6, np.float64)
    lib().orc_filter(_p(scores), G, gs, ctypes.c_double(ratio), 0 if ftype == "std" else 1, _p(sd), _p(mx), _p(mn),
                     _p(keep), _p(met))
    return keep, met, (sd, mx, mn)


# --------------------------------------------------------- Countdown rule (exact reference)
def masks_and_scores(ids, sp, rt, scores_tb, n_scores, n_slots, use_turn_scores, enable_response_mask, roll):
    """get_masks_and_scores (ctx_manager.py:35-70) -> (score f32[B,S-1], loss u8, resp u8, err u8[B])."""
    ids = np.ascontiguousarray(ids, np.int64)
    B, S = ids.shape
    sc = np.ascontiguousarray(scores_tb, np.float64).reshape(-1, B) if B else np.zeros((0, 0))
    n = np.ascontiguousarray(n_scores, np.int32)
    So = max(S - 1, 0)
    score = np.zeros((B, So), np.float32)
    lm = np.zeros((B, So), np.uint8)
    rm = np.zeros((B, So), np.uint8)
    err = np.zeros(B, np.uint8)
    flags = (1 if use_turn_scores else 0) | (2 if enable_response_mask else 0) | (4 if roll else 0)
    lib().orc_masks_and_scores(_p(ids), ctypes.c_int64(B), ctypes.c_int64(S), ctypes.c_int64(int(sp)),
                               ctypes.c_int64(int(rt)), _p(sc), _p(n), sc.shape[0], int(n_slots), flags, _p(score),
                               _p(lm), _p(rm), _p(err))
    return score, lm, rm, err


def sokoban_render(state, fixed, H, W, lookup):
    """SokobanEnv.render text (sokoban/env.py:53-61) of one env: player on target -> 6."""
    room = np.where((state == 5) & (fixed == 2), 6, state).reshape(H, W)
    return "\n".join("".join(lookup.get(int(c), "?") for c in row) for row in room.tolist())


def frozenlake_render(desc, s, n, lookup):
    """FrozenLakeEnv.render text (frozen_lake/env.py:47-61) of one env (desc: bytes of the map)."""
    d = np.asarray(desc).reshape(n, n)
    ml = {ord("P"): 0, ord("F"): 1, ord("H"): 2, ord("G"): 3, ord("S"): 1}
    codes = np.vectorize(lambda x: ml.get(int(x), 1))(d)
    if 0 <= s < n * n:
        letter = d[s // n, s % n]
        codes[s // n, s % n] = 4 if letter == ord("H") else 5 if letter == ord("G") else 0
    return "\n".join("".join(lookup.get(int(c), "?") for c in row) for row in codes)


def check_format(equation, nums):  # countdown/env.py:9-14
    try:
        nums_in_eq = [int(n) for n in re.findall(r"\d+", equation)]
        return sorted(nums_in_eq) == sorted(nums)
    except Exception:
        return False


def check_correctness(equation_str, target):  # countdown/env.py:16-21
    try:
        result = eval(equation_str, {"__builtins__": None}, {})
        return abs(result - target) < 1e-5
    except Exception:
        return False


def countdown_reward(answer, nums, target, score=1, format_score=0.1):  # countdown/env.py:69-78
    if not check_format(answer, nums):
        return 0
    if not check_correctness(answer, target):
        return format_score
    return score


def countdown_turn(answers, nums, targets, ep, turn, has_input=None, max_actions=1, fpen=-0.1, score=1,
                   format_score=0.1):
    """One EnvStateManager.step (es_manager.py:149-169) over CountdownEnv.step
    (countdown/env.py:58-62) for every env, written into the Episode record ``ep``.

    answers[b]: the parsed answer strings of env b (list, maybe empty).  Countdown has no
    action_lookup, so every string is a valid action (es_manager.py:235-236) and the format
    penalty is charged only for an empty list (:158-159).  A step is always done, so at most
    one answer executes per turn (_execute_actions :116-128); a turn without an answer
    costs the penalty and leaves the env active unless the cap of :163-166 is reached.
    ``left <= 0`` executes nothing (DESIGN deviation 5: Python's ``valid[:left]`` would slice
    from the end, a state the reference never reaches by itself).
    has_input[b] (optional): env b receives an input this turn; default = not done."""
    for b in range(ep.B):
        active = bool(has_input[b]) if has_input is not None else not (int(ep.flags[b]) & FLAG_DONE)
        if not active:
            continue
        valid = list(answers[b])
        left = max_actions - int(ep.num_actions[b])
        acc, info, turn_done, executed = 0, None, False, 0
        for a in (valid[:left] if left > 0 else []):
            reward = countdown_reward(a, list(nums[b]), int(targets[b]), score, format_score)
            acc += reward
            info = (reward > 0, reward == score)
            executed += 1
            turn_done = True  # countdown/env.py:60: done is always True
            break
        if not valid:
            ep.penalty[b] += fpen
        ep.num_actions[b] += executed
        ep.n_turns[b] += 1
        ep.turn_reward[turn, b] = acc
        ep.turn_exec[turn, b] = executed
        ep.turn_info[turn, b] = 0 if info is None else (INFO_PRESENT | (INFO_EFF if info[0] else 0) | INFO_VALID
                                                        | (INFO_SUCC if info[1] else 0))
        f = int(ep.flags[b]) & ~FLAG_DONE
        if turn_done:
            f |= FLAG_TERM
            f = (f & ~FLAG_TRUNC) if info[1] else (f | FLAG_TRUNC)
        if ep.num_actions[b] >= max_actions and not turn_done:
            f |= FLAG_TERM | FLAG_TRUNC
            turn_done = True
        if turn_done:
            f |= FLAG_DONE
        ep.flags[b] = f
