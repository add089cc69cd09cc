"""The hot path as PyTorch custom operators: ``torch.ops.ragen_amd.*``.

Every entry point of the C ABI (include/ragen_amd.h) is registered with the dispatcher through
``torch.library`` (``Library.define`` + ``impl``, see ``_Op``) — a schema inferred from the
implementation's annotations (argument types, which tensors an op mutates in place),
a CUDA (= HIP on ROCm) implementation that enqueues the HIP kernel on the current stream of
the tensors' device, and a fake (meta) implementation so shape propagation, FakeTensor
tracing and ``torch.compile`` see the ops as opaque nodes.  The trainer-facing facades
(``ragen_amd.llm_agent``, ``ragen_amd.trainer``, ``ragen_amd.env``) call these operators, so
the reference's callers (agent_trainer.py:514-515, 623-633; agent_proxy.py:146-157) drive the
kernels through ordinary torch ops, as north_star asks.

The ops are registered for the CUDA dispatch key only: a CPU tensor raises
``NotImplementedError`` from the dispatcher (the engine has no CPU path).

Episode record arguments are the seven tensors of ``ops.EpisodeState`` in its field order
(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec), each listed among
the mutated arguments of the ops that write the record.
"""
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import _lib, ops

NS = "ragen_amd"
EP = ("num_actions", "flags", "n_turns", "penalty", "turn_reward", "turn_info", "turn_exec")
NORM = {"identity": 0, "mean": 1, "mean_std": 2, "asym_clip": 3}
FILTER = {"std": 0, "std_rev": 1}
VARIANT = {"legacy": 0, "masked": 1}


_LIB = torch.library.Library(NS, "DEF")
_NAMES = []


class _Op:
    """One operator: the schema inferred from the implementation's annotations (mutated
    arguments marked ``Tensor(a!)``), the implementation registered for the CUDA dispatch key,
    a fake kernel added with ``.register_fake``.  Registered through ``torch.library.Library``
    rather than ``custom_op``: the same dispatcher op, without custom_op's Python autograd and
    alias-check layers around every call (≈12 µs a call on the host, and the turn loop makes
    a dozen calls per turn)."""

    def __init__(self, name, fn, mutates):
        self.name = name
        _LIB.define(name + torch.library.infer_schema(fn, mutates_args=tuple(mutates)))
        _LIB.impl(name, fn, "CUDA")
        _NAMES.append(name)
        self.__wrapped__ = fn
        self.__doc__, self.__name__ = fn.__doc__, fn.__name__

    def register_fake(self, fake):
        torch.library.register_fake(f"{NS}::{self.name}", fake, lib=_LIB)
        return fake

    def __call__(self, *args, **kwargs):
        return getattr(torch.ops.ragen_amd, self.name)(*args, **kwargs)


def _op(name, mutates=()):
    return lambda fn: _Op(name, fn, mutates)


class _Direct:
    """``direct.<op>``: an op's implementation called straight from Python — the same code the
    dispatcher runs for the CUDA key, without the dispatcher's argument boxing (≈6-8 µs a call
    on the host).  The engine's own device turn loop calls its ops this way; callers outside
    it use ``torch.ops.ragen_amd.<op>``."""

    def __getattr__(self, name):
        fn = globals()[name].__wrapped__
        setattr(self, name, fn)
        return fn


direct = _Direct()


def _ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec) -> ops.EpisodeState:
    return ops.EpisodeState(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec)


def ep_args(ep: ops.EpisodeState):
    """The seven record tensors of an EpisodeState, in the ops' argument order."""
    return tuple(getattr(ep, k) for k in EP)


def _ptr(t):
    return None if t is None else t.data_ptr()


# ====================================================================== Sokoban (A4)
def _sokoban(room_fixed, room_state, player, num_env_steps, boxes_on_target, H, W, num_boxes, max_steps):
    ops._dev(room_fixed, room_state, player, num_env_steps, boxes_on_target)
    for t, dt, nm in ((room_fixed, torch.uint8, "room_fixed"), (room_state, torch.uint8, "room_state"),
                      (player, torch.int8, "player"), (num_env_steps, torch.uint8, "num_env_steps"),
                      (boxes_on_target, torch.int8, "boxes_on_target")):
        ops._dt(t, dt, nm)
    return _lib.Sokoban(int(H), int(W), int(num_boxes), int(max_steps), _ptr(room_fixed), _ptr(room_state),
                        _ptr(player), _ptr(num_env_steps), _ptr(boxes_on_target))


_SOK_MUT = ("room_state", "player", "num_env_steps", "boxes_on_target") + EP


@_op("sokoban_step_turn", _SOK_MUT + ("err",))
def sokoban_step_turn(room_fixed: Tensor, room_state: Tensor, player: Tensor, num_env_steps: Tensor,
                      boxes_on_target: Tensor, num_actions: Tensor, flags: Tensor, n_turns: Tensor, penalty: Tensor,
                      turn_reward: Tensor, turn_info: Tensor, turn_exec: Tensor, actions: Tensor, n_actions: Tensor,
                      has_input: Optional[Tensor], err: Optional[Tensor], turn: int, max_actions_per_traj: int,
                      format_penalty: float, H: int, W: int, num_boxes: int, max_steps: int) -> None:
    """EnvStateManager.step (es_manager.py:105-171) over SokobanEnv.step (sokoban/env.py:44-51)."""
    env = _sokoban(room_fixed, room_state, player, num_env_steps, boxes_on_target, H, W, num_boxes, max_steps)
    ep = _ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec)
    ops._dev(room_state, flags, actions, n_actions, has_input, err)
    ops.sokoban_step_turn(env, ep, ops.turn_struct(turn, actions, n_actions, has_input, max_actions_per_traj,
                                                   format_penalty), err)


@_op("sokoban_step_turn_first", _SOK_MUT + ("err",))
def sokoban_step_turn_first(room_fixed: Tensor, room_state: Tensor, player: Tensor, num_env_steps: Tensor,
                            boxes_on_target: Tensor, num_actions: Tensor, flags: Tensor, n_turns: Tensor,
                            penalty: Tensor, turn_reward: Tensor, turn_info: Tensor, turn_exec: Tensor,
                            actions: Tensor, n_actions: Tensor, has_input: Optional[Tensor], err: Optional[Tensor],
                            init_state: Tensor, init_player: Tensor, turn: int, max_actions_per_traj: int,
                            format_penalty: float, H: int, W: int, num_boxes: int, max_steps: int) -> None:
    """SokobanEnv.reset's device part (sokoban/env.py:37-38, es_manager.py:95) + the first turn."""
    env = _sokoban(room_fixed, room_state, player, num_env_steps, boxes_on_target, H, W, num_boxes, max_steps)
    ep = _ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec)
    ops._dev(room_state, flags, actions, n_actions, has_input, err, init_state, init_player)
    ops.sokoban_step_turn_first(env, ep, ops.turn_struct(turn, actions, n_actions, has_input, max_actions_per_traj,
                                                         format_penalty), init_state, init_player, err)


@_op("sokoban_step_turn_finalize", _SOK_MUT + ("err", "metrics", "score", "pen", "norm"))
def sokoban_step_turn_finalize(room_fixed: Tensor, room_state: Tensor, player: Tensor, num_env_steps: Tensor,
                               boxes_on_target: Tensor, num_actions: Tensor, flags: Tensor, n_turns: Tensor,
                               penalty: Tensor, turn_reward: Tensor, turn_info: Tensor, turn_exec: Tensor,
                               actions: Tensor, n_actions: Tensor, has_input: Optional[Tensor], err: Optional[Tensor],
                               metrics: Optional[Tensor], score: Optional[Tensor], pen: Optional[Tensor],
                               norm: Optional[Tensor], turn: int, max_actions_per_traj: int, format_penalty: float,
                               H: int, W: int, num_boxes: int, max_steps: int, group_size: int, method: int) -> None:
    """The rollout's last turn + get_rollout_states / scores / _normalize_score_tensor
    (es_manager.py:173-207, ctx_manager.py:175-226) over groups of group_size envs."""
    env = _sokoban(room_fixed, room_state, player, num_env_steps, boxes_on_target, H, W, num_boxes, max_steps)
    ep = _ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec)
    ops._dev(room_state, flags, actions, n_actions, has_input, err, metrics, score, pen, norm)
    fin = ops.finalize_struct(group_size, _method_name(method), norm, metrics, score, pen)
    ops.sokoban_step_turn_finalize(env, ep, ops.turn_struct(turn, actions, n_actions, has_input, max_actions_per_traj,
                                                            format_penalty), fin, err)


@_op("sokoban_reset", _SOK_MUT)
def sokoban_reset(room_fixed: Tensor, room_state: Tensor, player: Tensor, num_env_steps: Tensor,
                  boxes_on_target: Tensor, num_actions: Tensor, flags: Tensor, n_turns: Tensor, penalty: Tensor,
                  turn_reward: Tensor, turn_info: Tensor, turn_exec: Tensor, init_state: Tensor, init_player: Tensor,
                  H: int, W: int, num_boxes: int, max_steps: int) -> None:
    """SokobanEnv.reset's device part (sokoban/env.py:37-38) + EnvStatus() (es_manager.py:95)."""
    env = _sokoban(room_fixed, room_state, player, num_env_steps, boxes_on_target, H, W, num_boxes, max_steps)
    ops._dev(room_state, flags, init_state, init_player)
    ops.sokoban_reset(env, _ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec), init_state,
                      init_player)


def _method_name(method: int) -> str:
    for k, v in NORM.items():
        if v == method:
            return k
    raise ValueError(f"Invalid normalization method: {method}")


# =================================================================== FrozenLake (A7)
def _frozenlake(desc, s, rng, nrow, ncol, is_slippery, cs0, cs1, cs2):
    ops._dev(desc, s, rng)
    ops._dt(desc, torch.uint8, "desc")
    ops._dt(s, torch.int32, "s")
    ops._dt(rng, torch.int64, "rng")
    return _lib.FrozenLake(int(nrow), int(ncol), int(is_slippery), float(cs0), float(cs1), float(cs2), _ptr(desc),
                           _ptr(s), _ptr(rng))


_FL_MUT = ("s", "rng") + EP


@_op("frozenlake_step_turn", _FL_MUT + ("err",))
def frozenlake_step_turn(desc: Tensor, s: Tensor, rng: Tensor, num_actions: Tensor, flags: Tensor, n_turns: Tensor,
                         penalty: Tensor, turn_reward: Tensor, turn_info: Tensor, turn_exec: Tensor, actions: Tensor,
                         n_actions: Tensor, has_input: Optional[Tensor], err: Optional[Tensor], turn: int,
                         max_actions_per_traj: int, format_penalty: float, nrow: int, ncol: int, is_slippery: bool,
                         cs0: float, cs1: float, cs2: float) -> None:
    """EnvStateManager.step over FrozenLakeEnv.step (frozen_lake/env.py:39-45, gymnasium App. A.2)."""
    env = _frozenlake(desc, s, rng, nrow, ncol, is_slippery, cs0, cs1, cs2)
    ops._dev(s, flags, actions, n_actions, has_input, err)
    ops.frozenlake_step_turn(env, _ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec),
                             ops.turn_struct(turn, actions, n_actions, has_input, max_actions_per_traj,
                                             format_penalty), err)


@_op("frozenlake_step_turn_first", ("desc",) + _FL_MUT + ("err",))
def frozenlake_step_turn_first(desc: Tensor, s: Tensor, rng: Tensor, num_actions: Tensor, flags: Tensor,
                               n_turns: Tensor, penalty: Tensor, turn_reward: Tensor, turn_info: Tensor,
                               turn_exec: Tensor, actions: Tensor, n_actions: Tensor, has_input: Optional[Tensor],
                               err: Optional[Tensor], init_desc: Tensor, init_s: Tensor, init_rng: Tensor, turn: int,
                               max_actions_per_traj: int, format_penalty: float, nrow: int, ncol: int,
                               is_slippery: bool, cs0: float, cs1: float, cs2: float) -> None:
    """FrozenLakeEnv.reset's device part (frozen_lake/env.py:28-37) + the first turn."""
    env = _frozenlake(desc, s, rng, nrow, ncol, is_slippery, cs0, cs1, cs2)
    ops._dev(s, flags, actions, n_actions, has_input, err, init_desc, init_s, init_rng)
    ops.frozenlake_step_turn_first(env, _ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec),
                                   ops.turn_struct(turn, actions, n_actions, has_input, max_actions_per_traj,
                                                   format_penalty), init_desc, init_s, init_rng, err)


@_op("frozenlake_step_turn_finalize", _FL_MUT + ("err", "metrics", "score", "pen", "norm"))
def frozenlake_step_turn_finalize(desc: Tensor, s: Tensor, rng: Tensor, num_actions: Tensor, flags: Tensor,
                                  n_turns: Tensor, penalty: Tensor, turn_reward: Tensor, turn_info: Tensor,
                                  turn_exec: Tensor, actions: Tensor, n_actions: Tensor, has_input: Optional[Tensor],
                                  err: Optional[Tensor], metrics: Optional[Tensor], score: Optional[Tensor],
                                  pen: Optional[Tensor], norm: Optional[Tensor], turn: int, max_actions_per_traj: int,
                                  format_penalty: float, nrow: int, ncol: int, is_slippery: bool, cs0: float,
                                  cs1: float, cs2: float, group_size: int, method: int) -> None:
    """The rollout's last FrozenLake turn + the fused finalize (as sokoban_step_turn_finalize)."""
    env = _frozenlake(desc, s, rng, nrow, ncol, is_slippery, cs0, cs1, cs2)
    ops._dev(s, flags, actions, n_actions, has_input, err, metrics, score, pen, norm)
    fin = ops.finalize_struct(group_size, _method_name(method), norm, metrics, score, pen)
    ops.frozenlake_step_turn_finalize(env, _ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info,
                                               turn_exec),
                                      ops.turn_struct(turn, actions, n_actions, has_input, max_actions_per_traj,
                                                      format_penalty), fin, err)


@_op("frozenlake_reset", ("desc",) + _FL_MUT)
def frozenlake_reset(desc: Tensor, s: Tensor, rng: Tensor, num_actions: Tensor, flags: Tensor, n_turns: Tensor,
                     penalty: Tensor, turn_reward: Tensor, turn_info: Tensor, turn_exec: Tensor, init_desc: Tensor,
                     init_s: Tensor, init_rng: Tensor, nrow: int, ncol: int, is_slippery: bool, cs0: float, cs1: float,
                     cs2: float) -> None:
    """FrozenLakeEnv.reset's device part (frozen_lake/env.py:28-37) + EnvStatus()."""
    env = _frozenlake(desc, s, rng, nrow, ncol, is_slippery, cs0, cs1, cs2)
    ops._dev(s, flags, init_desc, init_s, init_rng)
    ops.frozenlake_reset(env, _ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec), init_desc,
                         init_s, init_rng)


# ======================================================================= Bandit (A8)
@_op("bandit_step_turn", ("rng",) + EP + ("err",))
def bandit_step_turn(hi_is_first: Tensor, rng: Tensor, num_actions: Tensor, flags: Tensor, n_turns: Tensor,
                     penalty: Tensor, turn_reward: Tensor, turn_info: Tensor, turn_exec: Tensor, actions: Tensor,
                     n_actions: Tensor, has_input: Optional[Tensor], err: Optional[Tensor], turn: int,
                     max_actions_per_traj: int, format_penalty: float, action_space_start: int, lo_arm_score: float,
                     hi_arm_loscore: float, hi_arm_hiscore: float, hi_arm_hiscore_prob: float) -> None:
    """EnvStateManager.step over BanditEnv.step (bandit/env.py:62-76)."""
    ops._dev(hi_is_first, rng, flags, actions, n_actions, has_input, err)
    env = _lib.Bandit(int(action_space_start), float(lo_arm_score), float(hi_arm_loscore), float(hi_arm_hiscore),
                      float(hi_arm_hiscore_prob), _ptr(hi_is_first), _ptr(rng))
    ops.bandit_step_turn(env, _ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec),
                         ops.turn_struct(turn, actions, n_actions, has_input, max_actions_per_traj, format_penalty),
                         err)


# ==================================================================== Countdown (A9)
def _countdown(nums, n_nums, target, score, format_score):
    ops._dev(nums, n_nums, target)
    for t, nm in ((nums, "nums"), (n_nums, "n_nums"), (target, "target")):
        ops._dt(t, torch.int32, nm)
    return _lib.Countdown(int(nums.shape[1]), float(score), float(format_score), _ptr(nums), _ptr(n_nums),
                          _ptr(target))


@_op("countdown_step_turn", EP + ("err",))
def countdown_step_turn(nums: Tensor, n_nums: Tensor, target: Tensor, num_actions: Tensor, flags: Tensor,
                        n_turns: Tensor, penalty: Tensor, turn_reward: Tensor, turn_info: Tensor, turn_exec: Tensor,
                        actions: Tensor, n_actions: Tensor, has_input: Optional[Tensor], err: Optional[Tensor],
                        answers: Tensor, answer_len: Tensor, turn: int, max_actions_per_traj: int,
                        format_penalty: float, score: float, format_score: float) -> None:
    """EnvStateManager.step over CountdownEnv.step (countdown/env.py:58-78)."""
    env = _countdown(nums, n_nums, target, score, format_score)
    ops._dev(nums, flags, actions, n_actions, has_input, err, answers, answer_len)
    ops.countdown_step_turn(env, _ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec),
                            ops.turn_struct(turn, actions, n_actions, has_input, max_actions_per_traj,
                                            format_penalty), answers, answer_len, err)


@_op("countdown_reward")
def countdown_reward(nums: Tensor, n_nums: Tensor, target: Tensor, answers: Tensor, answer_len: Tensor, score: float,
                     format_score: float) -> Tuple[Tensor, Tensor, Tensor]:
    """compute_reward (countdown/env.py:69-78) per answer -> (reward f64, flags u8, err u8)."""
    env = _countdown(nums, n_nums, target, score, format_score)
    ops._dev(nums, answers, answer_len)
    return ops.countdown_reward(env, answers, answer_len)


@countdown_reward.register_fake
def _(nums, n_nums, target, answers, answer_len, score, format_score):
    n = answers.shape[0]
    return (answers.new_empty(n, dtype=torch.float64), answers.new_empty(n, dtype=torch.uint8),
            answers.new_empty(n, dtype=torch.uint8))


# ============================================================ seeding (A7 / A8 reset)
@_op("pcg64_seed")
def pcg64_seed(seeds: Tensor, draws: int) -> Tuple[Tensor, Tensor]:
    """Generator(PCG64(SeedSequence(seed))) per seed + `draws` random() calls -> (rng i64[4,n], last f64[n])."""
    rng, last = ops.pcg64_seed(seeds, draws)
    return rng, last


@pcg64_seed.register_fake
def _(seeds, draws):
    n = seeds.shape[0]
    return seeds.new_empty(4, n, dtype=torch.int64), seeds.new_empty(n, dtype=torch.float64)


# ============================================================== episode (A10, A16)
@_op("rollout_metrics")
def rollout_metrics(num_actions: Tensor, flags: Tensor, n_turns: Tensor, penalty: Tensor, turn_reward: Tensor,
                    turn_info: Tensor, turn_exec: Tensor) -> Tensor:
    """get_rollout_states (es_manager.py:173-207) -> f64[B, 4]."""
    return ops.rollout_metrics(_ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec))


@rollout_metrics.register_fake
def _(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec):
    return flags.new_empty(flags.shape[0], 4, dtype=torch.float64)


@_op("trajectory_scores")
def trajectory_scores(num_actions: Tensor, flags: Tensor, n_turns: Tensor, penalty: Tensor, turn_reward: Tensor,
                      turn_info: Tensor, turn_exec: Tensor) -> Tuple[Tensor, Tensor]:
    """Trajectory score sum(turn rewards) and penalty as f32 (ctx_manager.py:282, :217)."""
    return ops.trajectory_scores(_ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec))


@trajectory_scores.register_fake
def _(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec):
    B = flags.shape[0]
    return flags.new_empty(B, dtype=torch.float32), flags.new_empty(B, dtype=torch.float32)


@_op("rollout_finalize", ("metrics", "score", "pen", "norm"))
def rollout_finalize(num_actions: Tensor, flags: Tensor, n_turns: Tensor, penalty: Tensor, turn_reward: Tensor,
                     turn_info: Tensor, turn_exec: Tensor, seg: Tensor, method: int, metrics: Optional[Tensor],
                     score: Optional[Tensor], pen: Optional[Tensor], norm: Tensor) -> None:
    """Metrics + trajectory scores + _normalize_score_tensor in one launch (contiguous segments)."""
    ops.rollout_finalize(_ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec), seg,
                         _method_name(method), norm, metrics, score, pen)


@_op("group_normalize")
def group_normalize(score: Tensor, pen: Optional[Tensor], seg: Tensor, method: int) -> Tensor:
    """_normalize_score_tensor (ctx_manager.py:175-226) over contiguous segments seg i32[G+1]."""
    return ops.group_normalize(score, pen, seg, _method_name(method))


@group_normalize.register_fake
def _(score, pen, seg, method):
    return torch.empty_like(score)


# ======================================================================= filter (A12)
@_op("row_sum")
def row_sum(x: Tensor) -> Tensor:
    """rm_scores.sum(-1) in fp64 then f32 (agent_trainer.py:467)."""
    return ops.row_sum(x)


@row_sum.register_fake
def _(x):
    return x.new_empty(x.shape[0], dtype=torch.float32)


@_op("filter_groups")
def filter_groups(scores: Tensor, num_groups: int, group_size: int, ratio: float,
                  ftype: int) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """_filter_rollout (agent_trainer.py:461-500) -> (keep u8[G], metrics f64[6], std, max, mean f32[G])."""
    keep, met, (sd, mx, mn) = ops.filter_groups(scores, num_groups, group_size, ratio,
                                                "std" if ftype == 0 else "std_rev")
    return keep, met, sd, mx, mn


@filter_groups.register_fake
def _(scores, num_groups, group_size, ratio, ftype):
    G = num_groups
    return (scores.new_empty(G, dtype=torch.uint8), scores.new_empty(6, dtype=torch.float64),
            scores.new_empty(G, dtype=torch.float32), scores.new_empty(G, dtype=torch.float32),
            scores.new_empty(G, dtype=torch.float32))


# ================================================================ token masks (A11)
@_op("masks_and_scores")
def masks_and_scores(ids: Tensor, special_token: int, reward_token: int, scores: Tensor, n_scores: Tensor,
                     n_slots: int, use_turn_scores: bool, enable_response_mask: bool,
                     roll: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """get_masks_and_scores (ctx_manager.py:35-70) -> (score f32, loss_mask, response_mask bool [B,S-1], err u8[B])."""
    return ops.masks_and_scores(ids, special_token, reward_token, scores, n_scores, n_slots, use_turn_scores,
                                enable_response_mask, roll)


@masks_and_scores.register_fake
def _(ids, special_token, reward_token, scores, n_scores, n_slots, use_turn_scores, enable_response_mask, roll):
    B, S = ids.shape
    So = max(S - 1, 0)
    return (ids.new_empty(B, So, dtype=torch.float32), ids.new_empty(B, So, dtype=torch.bool),
            ids.new_empty(B, So, dtype=torch.bool), ids.new_empty(B, dtype=torch.uint8))


@_op("assemble_batch")
def assemble_batch(tokens: Tensor, row_off: Tensor, S: int, pad_id: int, special_token: int, reward_token: int,
                   scores: Tensor, n_scores: Tensor, n_slots: int, use_turn_scores: bool, enable_response_mask: bool,
                   roll: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """formulate_rollouts' batch (ctx_manager.py:278-306) from ragged token rows, one pass ->
    (input_ids, attention_mask, position_ids, score, loss_mask, response_mask, err)."""
    return ops.assemble_batch(tokens, row_off, S, pad_id, special_token, reward_token, scores, n_scores, n_slots,
                              use_turn_scores, enable_response_mask, roll)


@assemble_batch.register_fake
def _(tokens, row_off, S, pad_id, special_token, reward_token, scores, n_scores, n_slots, use_turn_scores,
      enable_response_mask, roll):
    B = row_off.shape[0] - 1
    So = max(S - 1, 0)
    i = tokens.new_empty(B, S, dtype=torch.int64)
    return (i, torch.empty_like(i), torch.empty_like(i), tokens.new_empty(B, So, dtype=torch.float32),
            tokens.new_empty(B, So, dtype=torch.bool), tokens.new_empty(B, So, dtype=torch.bool),
            tokens.new_empty(B, dtype=torch.uint8))


@_op("assemble_rows")
def assemble_rows(tokens: Tensor, row_start: Tensor, row_len: Tensor, S: int, pad_id: int, special_token: int,
                  reward_token: int, scores: Tensor, n_scores: Tensor, n_slots: int, use_turn_scores: bool,
                  enable_response_mask: bool, roll: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """assemble_batch over rows given by (start, length), e.g. the device prompt arena."""
    return ops.assemble_rows(tokens, row_start, row_len, S, pad_id, special_token, reward_token, scores, n_scores,
                             n_slots, use_turn_scores, enable_response_mask, roll)


@assemble_rows.register_fake
def _(tokens, row_start, row_len, S, pad_id, special_token, reward_token, scores, n_scores, n_slots, use_turn_scores,
      enable_response_mask, roll):
    B = row_start.shape[0]
    So = max(S - 1, 0)
    i = tokens.new_empty(B, S, dtype=torch.int64)
    return (i, torch.empty_like(i), torch.empty_like(i), tokens.new_empty(B, So, dtype=torch.float32),
            tokens.new_empty(B, So, dtype=torch.bool), tokens.new_empty(B, So, dtype=torch.bool),
            tokens.new_empty(B, dtype=torch.uint8))


@_op("gen_rows", ("ids", "n_ids", "raw_max", "has", "raw_next"))
def gen_rows(resp: Tensor, src: Optional[Tensor], n_envs: int, vocab_packed: Tensor, ids: Optional[Tensor],
             n_ids: Optional[Tensor], raw_max: Tensor, has: Optional[Tensor] = None,
             raw_next: Optional[Tensor] = None) -> None:
    """The input side of get_env_inputs (ctx_manager.py:332-337): the turn's generations onto
    the env batch and the longest row's raw bytes (rmi_gen_rows; with raw_next the chained form,
    raw_max zero on entry and raw_next zeroed for the next turn)."""
    ops.gen_rows(resp, src, n_envs, vocab_packed, ids, n_ids, raw_max, has, raw_next)


@_op("pad_rows")
def pad_rows(arena: Tensor, arena_len: Tensor, rows: Tensor, tail: Tensor, S: int,
             pad_id: int) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """The generation batch of get_lm_inputs (ctx_manager.py:265-278) from the prompt arena."""
    return ops.pad_rows(arena, arena_len, rows, tail, S, pad_id)


@pad_rows.register_fake
def _(arena, arena_len, rows, tail, S, pad_id):
    n = rows.shape[0]
    i = arena.new_empty(n, S)
    return i, torch.empty_like(i), torch.empty_like(i), arena.new_empty(n, dtype=torch.uint8)


# ================================================================== advantages (A13)
@_op("gae", ("row_stats",))
def gae(r: Tensor, v: Tensor, mask: Tensor, gamma: float, lam: float, variant: int,
        row_stats: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
    """verl compute_gae_advantage_return before whitening (App. A.4); variant 0 legacy, 1 masked."""
    return ops.gae(r, v, mask, gamma, lam, "legacy" if variant == 0 else "masked", row_stats)


@gae.register_fake
def _(r, v, mask, gamma, lam, variant, row_stats):
    return torch.empty_like(r), torch.empty_like(r)


@_op("bilevel_gae", ("row_stats", "err"))
def bilevel_gae(r: Tensor, v: Tensor, mask: Tensor, gamma: float, lam: float, high_level_gamma: float,
                row_stats: Optional[Tensor], err: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
    """compute_bi_level_gae_advantage_return before whitening (core_algos.py:4-88); err u8[B]
    flags the rows where the reference raises IndexError (core_algos.py:79)."""
    return ops.bilevel_gae(r, v, mask, gamma, lam, high_level_gamma, row_stats, check_errors=False, err=err)


@bilevel_gae.register_fake
def _(r, v, mask, gamma, lam, high_level_gamma, row_stats, err):
    return torch.empty_like(r), torch.empty_like(r)


@_op("masked_whiten_", ("x",))
def masked_whiten_(x: Tensor, mask: Tensor, row_stats: Optional[Tensor]) -> Tensor:
    """verl masked_whiten in place (core_algos.py:90) -> i32[1] status (0 ok, 1/2: verl's ValueError)."""
    _, scratch = ops.masked_whiten_(x, mask, row_stats)
    return ops.whiten_status(scratch).clone()


@masked_whiten_.register_fake
def _(x, mask, row_stats):
    return x.new_empty(1, dtype=torch.int32)


@_op("masked_whiten_stats_", ("x",))
def masked_whiten_stats_(x: Tensor, stats: Tensor) -> Tensor:
    """masked_whiten of this shard's rows with all shards' per-row partials -> i32[1] status."""
    _, scratch = ops.masked_whiten_stats_(x, stats)
    return ops.whiten_status(scratch).clone()


@masked_whiten_stats_.register_fake
def _(x, stats):
    return x.new_empty(1, dtype=torch.int32)


@_op("whiten_row_stats")
def whiten_row_stats(x: Tensor, mask: Tensor) -> Tensor:
    """Per-row fp64 (sum, sum_sq, count) over the mask -> f64[B, 3]."""
    return ops.whiten_row_stats(x, mask)


@whiten_row_stats.register_fake
def _(x, mask):
    return x.new_empty(x.shape[0], 3, dtype=torch.float64)


@_op("grpo_outcome")
def grpo_outcome(r: Tensor, mask: Tensor, seg: Tensor, eps: float, norm_by_std: bool) -> Tuple[Tensor, Tensor]:
    """verl compute_grpo_outcome_advantage over contiguous row groups seg i32[G+1] (device)."""
    return ops.grpo_outcome(r, mask, seg, eps, norm_by_std)


@grpo_outcome.register_fake
def _(r, mask, seg, eps, norm_by_std):
    return torch.empty_like(r), torch.empty_like(r)


@_op("reinforce_pp_returns", ("row_stats",))
def reinforce_pp_returns(r: Tensor, mask: Tensor, gamma: float, row_stats: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
    """verl compute_reinforce_plus_plus_outcome_advantage before its whitening (adv = ret)."""
    return ops.reinforce_pp_returns(r, mask, gamma, row_stats)


@reinforce_pp_returns.register_fake
def _(r, mask, gamma, row_stats):
    return torch.empty_like(r), torch.empty_like(r)


@_op("remax")
def remax(r: Tensor, mask: Tensor, baseline: Tensor) -> Tuple[Tensor, Tensor]:
    """verl compute_remax_outcome_advantage."""
    return ops.remax(r, mask, baseline)


@remax.register_fake
def _(r, mask, baseline):
    return torch.empty_like(r), torch.empty_like(r)


@_op("rloo_outcome")
def rloo_outcome(r: Tensor, mask: Tensor, seg: Tensor) -> Tuple[Tensor, Tensor]:
    """verl compute_rloo_outcome_advantage over contiguous row groups seg i32[G+1] (device)."""
    return ops.rloo_outcome(r, mask, seg)


@rloo_outcome.register_fake
def _(r, mask, seg):
    return torch.empty_like(r), torch.empty_like(r)


@_op("mask_mul_", ("x",))
def mask_mul_(x: Tensor, mask: Tensor) -> None:
    """x *= (mask != 0) in place."""
    ops.mask_mul_(x, mask)


@mask_mul_.register_fake
def _(x, mask):
    return None


# ============================================================= text boundary (§8(f) 2)
def _glyphs(glyph_bytes: List[int], glyph_len: List[int]):
    import numpy as np
    if len(glyph_bytes) != 16 or len(glyph_len) != 16:
        raise ValueError("glyph tables hold 16 entries")
    return np.asarray(glyph_bytes, np.uint32), np.asarray(glyph_len, np.uint8)


def render_stride(cells: int, rows: int) -> int:
    return (cells * 4 + rows - 1 + 3) // 4 * 4


@_op("sokoban_render")
def sokoban_render(room_fixed: Tensor, room_state: Tensor, H: int, W: int, glyph_bytes: List[int],
                   glyph_len: List[int]) -> Tuple[Tensor, Tensor]:
    """SokobanEnv.render text of every env (sokoban/env.py:53-61) -> (UTF-8 rows u8[B, stride], len i32[B])."""
    ops._dev(room_fixed, room_state)
    B = room_state.shape[0]
    env = _lib.Sokoban(int(H), int(W), 0, 0, _ptr(room_fixed), _ptr(room_state), None, None, None)
    gb, gl = _glyphs(glyph_bytes, glyph_len)
    stride = render_stride(H * W, H)
    out = torch.empty(B, stride, dtype=torch.uint8, device=room_state.device)
    n = torch.empty(B, dtype=torch.int32, device=room_state.device)
    ops.check(ops.lib().rmi_sokoban_render(env, B, gb.ctypes.data, gl.ctypes.data, out.data_ptr(), stride,
                                           n.data_ptr(), ops._stream(room_state.device)), "rmi_sokoban_render")
    return out, n


_RENDER_TEMPLATES = {}  # glyph table -> its rmi_render_t (pointers unset)


def _render_struct(glyph_bytes: List[int], glyph_len: List[int], obs: Tensor, obs_len: Tensor) -> _lib.Render:
    key = (tuple(glyph_bytes), tuple(glyph_len))
    R = _RENDER_TEMPLATES.get(key)
    if R is None:
        gb, gl = _glyphs(glyph_bytes, glyph_len)
        if (gl > 4).any():
            raise ValueError("glyphs are at most 4 UTF-8 bytes")
        R = _lib.Render()
        for k in range(16):
            R.glyph_bytes[k], R.glyph_len[k] = int(gb[k]), int(gl[k])
        if len(_RENDER_TEMPLATES) > 64:
            _RENDER_TEMPLATES.clear()
        _RENDER_TEMPLATES[key] = R
    r = _lib.Render.from_buffer_copy(R)
    r.out, r.stride, r.len = obs.data_ptr(), int(obs.shape[1]), obs_len.data_ptr()
    return r


@_op("sokoban_step_turn_render", _SOK_MUT + ("err", "obs", "obs_len"))
def sokoban_step_turn_render(room_fixed: Tensor, room_state: Tensor, player: Tensor, num_env_steps: Tensor,
                             boxes_on_target: Tensor, num_actions: Tensor, flags: Tensor, n_turns: Tensor,
                             penalty: Tensor, turn_reward: Tensor, turn_info: Tensor, turn_exec: Tensor,
                             actions: Tensor, n_actions: Tensor, has_input: Optional[Tensor], err: Optional[Tensor],
                             obs: Tensor, obs_len: Tensor, glyph_bytes: List[int], glyph_len: List[int], turn: int,
                             max_actions_per_traj: int, format_penalty: float, H: int, W: int, num_boxes: int,
                             max_steps: int) -> None:
    """EnvStateManager.step (es_manager.py:105-171) and SokobanEnv.render of the next state
    (sokoban/env.py:53-61) in one launch: obs u8[B, stride] / obs_len i32[B] as sokoban_render's."""
    env = _sokoban(room_fixed, room_state, player, num_env_steps, boxes_on_target, H, W, num_boxes, max_steps)
    ep = _ep(num_actions, flags, n_turns, penalty, turn_reward, turn_info, turn_exec)
    ops._dev(room_state, flags, actions, n_actions, has_input, err, obs, obs_len)
    ops._dt(obs, torch.uint8, "obs")
    ops._dt(obs_len, torch.int32, "obs_len")
    if obs.dim() != 2 or obs.shape[0] != room_state.shape[0] or obs_len.numel() != room_state.shape[0]:
        raise ValueError("obs / obs_len must have one row per env")
    ops.sokoban_step_turn_render(env, ep, ops.turn_struct(turn, actions, n_actions, has_input, max_actions_per_traj,
                                                          format_penalty),
                                 _render_struct(glyph_bytes, glyph_len, obs, obs_len), err)


@sokoban_render.register_fake
def _(room_fixed, room_state, H, W, glyph_bytes, glyph_len):
    B = room_state.shape[0]
    return room_state.new_empty(B, render_stride(H * W, H)), room_state.new_empty(B, dtype=torch.int32)


@_op("frozenlake_render")
def frozenlake_render(desc: Tensor, s: Tensor, nrow: int, ncol: int, glyph_bytes: List[int],
                      glyph_len: List[int]) -> Tuple[Tensor, Tensor]:
    """FrozenLakeEnv.render text of every env (frozen_lake/env.py:47-61) -> (u8[B, stride], i32[B])."""
    ops._dev(desc, s)
    B = s.shape[0]
    env = _lib.FrozenLake(int(nrow), int(ncol), 0, 0.0, 0.0, 0.0, _ptr(desc), _ptr(s), None)
    gb, gl = _glyphs(glyph_bytes, glyph_len)
    stride = render_stride(nrow * ncol, nrow)
    out = torch.empty(B, stride, dtype=torch.uint8, device=s.device)
    n = torch.empty(B, dtype=torch.int32, device=s.device)
    ops.check(ops.lib().rmi_frozenlake_render(env, B, gb.ctypes.data, gl.ctypes.data, out.data_ptr(), stride,
                                              n.data_ptr(), ops._stream(s.device)), "rmi_frozenlake_render")
    return out, n


@frozenlake_render.register_fake
def _(desc, s, nrow, ncol, glyph_bytes, glyph_len):
    B = s.shape[0]
    return s.new_empty(B, render_stride(nrow * ncol, nrow), dtype=torch.uint8), s.new_empty(B, dtype=torch.int32)


@_op("detokenize")
def detokenize(ids: Tensor, n_ids: Optional[Tensor], vocab_packed: Tensor, vocab_bytes: Tensor,
               stride: int) -> Tuple[Tensor, Tensor, Tensor]:
    """tokenizer.batch_decode(responses, skip_special_tokens=True) (ctx_manager.py:334-337) over
    the packed vocabulary (ops.VocabTable.packed) -> (UTF-8 rows u8[B, stride], len i32[B], err u8[B])."""
    B = ids.shape[0]
    st = (int(stride) + 3) // 4 * 4
    out = (torch.empty(B, st, dtype=torch.uint8, device=ids.device), torch.empty(B, dtype=torch.int32, device=ids.device),
           torch.empty(B, dtype=torch.uint8, device=ids.device))  # every row's error byte is written
    return ops.detokenize_packed(ids, vocab_packed, vocab_bytes, st, n_ids, out)


@detokenize.register_fake
def _(ids, n_ids, vocab_packed, vocab_bytes, stride):
    B = ids.shape[0]
    st = (int(stride) + 3) // 4 * 4
    return (ids.new_empty(B, st, dtype=torch.uint8), ids.new_empty(B, dtype=torch.int32),
            ids.new_empty(B, dtype=torch.uint8))


def parse_cfg_words(cfg: _lib.ParseCfg) -> List[int]:
    """An rmi_parse_cfg_t as little-endian signed 64-bit words (the form the parse ops take: a
    192-byte struct is 24 list items, not 192 — each list item costs the dispatcher a conversion)."""
    import ctypes
    import struct
    b = ctypes.string_at(ctypes.addressof(cfg), ctypes.sizeof(cfg))
    b += b"\0" * (-len(b) % 8)
    return list(struct.unpack(f"<{len(b) // 8}q", b))


def _parse_cfg(cfg_words: List[int]) -> _lib.ParseCfg:
    import ctypes
    import struct
    n = ctypes.sizeof(_lib.ParseCfg)
    if len(cfg_words) != (n + 7) // 8:
        raise ValueError("cfg must be the words of an rmi_parse_cfg_t (torch_ops.parse_cfg_words)")
    return _lib.ParseCfg.from_buffer_copy(struct.pack(f"<{len(cfg_words)}q", *cfg_words)[:n])


@_op("parse_actions")
def parse_actions(cfg: List[int], text: Tensor, text_len: Tensor, sel: Optional[Tensor], with_spans: bool,
                  action_text_len: int) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """_parse_response + _extract_map_valid_actions (ctx_manager.py:148-173, es_manager.py:230-240)
    -> (actions i8[B,K], n_actions u8[B], spans i32[B,4] (0 rows without spans),
        action_text u8[B,K,Lact], action_len i32[B,K], err u8[B])."""
    c = _parse_cfg(cfg)
    o = ops.parse_actions(c, text, text_len, sel, with_spans, action_text_len)
    B, K = text.shape[0], int(c.K)
    dev = text.device
    spans = o["spans"] if o["spans"] is not None else torch.empty(0, 4, dtype=torch.int32, device=dev)
    at = o["action_text"] if o["action_text"] is not None else torch.empty(B, K, 0, dtype=torch.uint8, device=dev)
    al = o["action_len"] if o["action_len"] is not None else _zeros_i32(B, K, dev)
    return o["actions"], o["n_actions"], spans, at, al, o["err"]


@parse_actions.register_fake
def _(cfg, text, text_len, sel, with_spans, action_text_len):
    B, K = text.shape[0], int(_parse_cfg(cfg).K)
    return (text.new_empty(B, K, dtype=torch.int8), text.new_empty(B, dtype=torch.uint8),
            text.new_empty(B if with_spans else 0, 4, dtype=torch.int32),
            text.new_empty(B, K, action_text_len, dtype=torch.uint8), text.new_empty(B, K, dtype=torch.int32),
            text.new_empty(B, dtype=torch.uint8))


_ZEROS = {}  # (B, K, device) -> a zero i32[B, K] (the unused action_len output; read only)


def _zeros_i32(B, K, dev):
    z = _ZEROS.get((B, K, dev))
    if z is None:
        if len(_ZEROS) > 64:
            _ZEROS.clear()
        z = _ZEROS[(B, K, dev)] = torch.zeros(B, K, dtype=torch.int32, device=dev)
    return z


@_op("detok_parse")
def detok_parse(ids: Tensor, n_ids: Optional[Tensor], vocab_packed: Tensor, vocab_bytes: Tensor, stride: int,
                cfg: List[int], sel: Optional[Tensor], with_spans: bool,
                action_text_len: int) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """batch_decode + _parse_response + the name map in one launch (ctx_manager.py:332-352,
    :148-173, es_manager.py:230-240) -> (text u8[B, stride], text_len i32[B], decode_err u8[B],
    actions i8[B,K], n_actions u8[B], spans i32[B,4] (0 rows without spans), action_text
    u8[B,K,Lact], action_len i32[B,K], parse_err u8[B])."""
    c = _parse_cfg(cfg)
    vt = ops.VocabTable.__new__(ops.VocabTable)
    vt.packed, vt.data = vocab_packed, vocab_bytes
    o = ops.detok_parse(ids, vt, stride, c, n_ids, sel, with_spans, action_text_len)
    B, K = ids.shape[0], int(c.K)
    dev = ids.device
    spans = o["spans"] if o["spans"] is not None else torch.empty(0, 4, dtype=torch.int32, device=dev)
    at = o["action_text"] if o["action_text"] is not None else torch.empty(B, K, 0, dtype=torch.uint8, device=dev)
    al = o["action_len"] if o["action_len"] is not None else _zeros_i32(B, K, dev)
    return o["text"], o["text_len"], o["decode_err"], o["actions"], o["n_actions"], spans, at, al, o["err"]


@detok_parse.register_fake
def _(ids, n_ids, vocab_packed, vocab_bytes, stride, cfg, sel, with_spans, action_text_len):
    B, K = ids.shape[0], int(_parse_cfg(cfg).K)
    st = (int(stride) + 3) // 4 * 4
    return (ids.new_empty(B, st, dtype=torch.uint8), ids.new_empty(B, dtype=torch.int32),
            ids.new_empty(B, dtype=torch.uint8), ids.new_empty(B, K, dtype=torch.int8),
            ids.new_empty(B, dtype=torch.uint8), ids.new_empty(B if with_spans else 0, 4, dtype=torch.int32),
            ids.new_empty(B, K, action_text_len, dtype=torch.uint8), ids.new_empty(B, K, dtype=torch.int32),
            ids.new_empty(B, dtype=torch.uint8))


_BPE_STRUCTS = {}  # the tables' tensors (held) + params -> their validated rmi_bpe_t


def _bpe_struct(*args):
    """rmi_bpe_t of a tokenizer's device tables, validated and built once per set of tables (the
    tables are constant across calls; the cache holds the tensors, so a key's objects stay the
    same objects, and their data pointers are part of the key)."""
    key = tuple((id(a), a.data_ptr()) if isinstance(a, Tensor) else
                (tuple(a) if isinstance(a, (list, tuple)) else a) for a in args)
    hit = _BPE_STRUCTS.get(key)
    if hit is not None:
        return hit[0]
    s = _bpe_struct_build(*args)
    if len(_BPE_STRUCTS) >= 16:
        _BPE_STRUCTS.clear()
    _BPE_STRUCTS[key] = (s, args)
    return s


def _bpe_struct_build(cp_block, cp_class, byte_id, merges, added_bytes, added_off, added_id, params, word_cache=None,
                      exp_off=None, exp_ids=None, added_words=None, ascii_class=None, pre=None):
    from .tokenizer import Bpe
    ops._dev(cp_block, cp_class, byte_id, merges, added_bytes, added_off, added_id)
    if len(params) != 13:
        raise ValueError("params: merge_mask, merge_shift, pretok, nfc, n_added, added_first[8]")
    s = Bpe(cp_block.data_ptr(), cp_class.data_ptr(), byte_id.data_ptr(), merges.data_ptr(), params[0], params[1],
            params[2], params[3], params[4], added_bytes.data_ptr(), added_off.data_ptr(), added_id.data_ptr())
    for i in range(8):
        s.added_first[i] = params[5 + i] & 0xFFFFFFFF
    if word_cache is not None:
        ops._dev(word_cache)
        ops._dt(word_cache, torch.int32, "word_cache")
        n = word_cache.numel() // 16
        if n < 1 or n & (n - 1) or word_cache.numel() != 16 * n:
            raise ValueError("word_cache: 16 int32 per entry, a power-of-two number of entries")
        s.word_cache, s.word_cache_mask = word_cache.data_ptr(), n - 1
    if exp_off is not None:  # expansions: placeholder added tokens standing for id sequences
        ops._dev(exp_off, exp_ids)
        ops._dt(exp_off, torch.int32, "exp_off")
        ops._dt(exp_ids, torch.int32, "exp_ids")
        s.n_exp, s.exp_off, s.exp_ids = exp_off.numel() - 1, exp_off.data_ptr(), exp_ids.data_ptr()
        s.n_exp_ids = int(exp_ids.numel())
    if added_words is not None:  # staging tables (rmi_bpe_t.added_words / ascii_class)
        ops._dev(added_words)
        ops._dt(added_words, torch.int64, "added_words")
        if added_words.numel() != 4 * params[4] or params[4] > 64:
            raise ValueError("added_words: 4 words per added token, at most 64 tokens")
        s.added_words = added_words.data_ptr()
    if ascii_class is not None:
        ops._dev(ascii_class)
        ops._dt(ascii_class, torch.uint8, "ascii_class")
        if ascii_class.numel() != 128:
            raise ValueError("ascii_class: 128 classes")
        s.ascii_class = ascii_class.data_ptr()
    if pre is not None:  # the two-pass scratch: (pre, pre_gid, pre_np, pre_retry)
        p_, g_, n_, r_ = pre
        ops._dev(p_, g_, n_, r_)
        if p_.numel() != g_.numel() or n_.numel() != r_.numel() or n_.numel() < p_.numel() // 4:
            raise ValueError("pre / pre_gid: pre_cap entries each, pre_np / pre_retry: pre_cap / 4")
        s.pre, s.pre_gid, s.pre_np, s.pre_retry = p_.data_ptr(), g_.data_ptr(), n_.data_ptr(), r_.data_ptr()
        s.pre_cap = p_.numel() if n_.numel() else 0
    return s


@_op("bpe_encode", ("out", "out_len", "word_cache"))
def bpe_encode(cp_block: Tensor, cp_class: Tensor, byte_id: Tensor, merges: Tensor, added_bytes: Tensor,
               added_off: Tensor, added_id: Tensor, params: List[int], text: Tensor, text_len: Tensor, out: Tensor,
               out_len: Optional[Tensor], mark_byte: Optional[Tensor], max_len: int = 0,
               word_cache: Optional[Tensor] = None, exp_off: Optional[Tensor] = None,
               exp_ids: Optional[Tensor] = None, added_words: Optional[Tensor] = None,
               ascii_class: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Tensor]:
    """The tokenizer call of get_lm_inputs (ctx_manager.py:265-278) for a byte-level BPE:
    every text row's ids appended to ``out`` (rmi_bpe_encode; tables: ragen_amd.tokenizer).
    max_len (0: the row pitch) bounds the rows' length and sizes the kernel's LDS.
    -> (n_tok i32[B], mark_tok i32[B], err u8[B])."""
    import ctypes
    tok = _bpe_struct(cp_block, cp_class, byte_id, merges, added_bytes, added_off, added_id, params, word_cache,
                      exp_off, exp_ids, added_words, ascii_class)
    ops._dev(text, text_len, out, out_len, mark_byte)
    ops._dt(text, torch.uint8, "text")
    ops._dt(text_len, torch.int32, "text_len")
    ops._dt(out, torch.int64, "out")
    ops._dt(out_len, torch.int32, "out_len")
    ops._dt(mark_byte, torch.int32, "mark_byte")
    B = text.shape[0]
    if text_len.shape[0] != B or out.shape[0] != B or out.dim() != 2:
        raise ValueError("text, text_len and out must have one row per text")
    dev = text.device
    n_tok = torch.empty(B, dtype=torch.int32, device=dev)
    # (the kernel writes every row's mark when given a mark_byte; otherwise the result is zeros)
    mark_tok = torch.empty(B, dtype=torch.int32, device=dev) if mark_byte is not None else \
        torch.zeros(B, dtype=torch.int32, device=dev)
    err = torch.empty(B, dtype=torch.uint8, device=dev)
    pitch = int(text.shape[1])
    cap = (int(max_len) + 3) // 4 * 4 if max_len else pitch
    ops.check(ops.lib().rmi_bpe_encode(ctypes.addressof(tok), text.data_ptr(), pitch, max(min(cap, pitch), 4),
                                       text_len.data_ptr(), B, out.data_ptr(), int(out.shape[1]), _ptr(out_len),
                                       n_tok.data_ptr(),
                                       _ptr(mark_byte), mark_tok.data_ptr() if mark_byte is not None else None,
                                       err.data_ptr(), ops._stream(dev)), "rmi_bpe_encode")
    return n_tok, mark_tok, err


@bpe_encode.register_fake
def _(cp_block, cp_class, byte_id, merges, added_bytes, added_off, added_id, params, text, text_len, out, out_len,
      mark_byte, max_len=0, word_cache=None, exp_off=None, exp_ids=None, added_words=None, ascii_class=None):
    B = text.shape[0]
    return (text.new_empty(B, dtype=torch.int32), text.new_empty(B, dtype=torch.int32),
            text.new_empty(B, dtype=torch.uint8))


_PROMPT_TEMPLATES = {}  # (program, sep) -> the rmi_prompt_t of its pieces and scalars (pointers unset)


def _prompt_template(program, sep) -> _lib.Prompt:
    key = (tuple(program), tuple(sep))
    P = _PROMPT_TEMPLATES.get(key)
    if P is None:
        n = program[0]
        if n > _lib.PROMPT_MAX_PIECES or len(program) != 1 + 3 * n + 5 or len(sep) > 16:
            raise ValueError("bad prompt program")
        P = _lib.Prompt()
        P.n_pieces = n
        for i in range(n):
            P.pieces[i] = _lib.Piece(*program[1 + 3 * i:4 + 3 * i])
        P.n_tags, P.obs_stride, P.resp_stride, P.enable_think, P.K = program[1 + 3 * n:]
        P.sep_len = len(sep)
        for i, x in enumerate(sep):
            P.sep[i] = x
        if len(_PROMPT_TEMPLATES) >= 256:  # one program per turn number and stride in practice
            _PROMPT_TEMPLATES.clear()
        _PROMPT_TEMPLATES[key] = P
    return _lib.Prompt.from_buffer_copy(P)


def prompt_struct(program: List[int], sep: List[int], tensors, turn=None) -> _lib.Prompt:
    """program = [n_pieces, (kind, a, b) * n_pieces, n_tags, obs_stride, resp_stride, enable_think, K];
    tensors = (pool, tag_const, tag, obs, obs_len, ints, reward, reward_int, resp, resp_len, spans, cond, active);
    turn = (turn_exec, flags, int_reward_tags, last_turn): the turn form (rmi_prompt_t).  The pieces
    and scalars of a program are built once (_prompt_template); each call sets the pointers."""
    pool, tag_const, tag, obs, obs_len, ints, reward, reward_int, resp, resp_len, spans, cond, active = tensors
    P = _prompt_template(program, sep)
    P.pool, P.tag_const, P.tag = _ptr(pool), _ptr(tag_const), _ptr(tag)
    P.obs, P.obs_len, P.ints = _ptr(obs), _ptr(obs_len), _ptr(ints)
    P.reward, P.reward_int, P.resp = _ptr(reward), _ptr(reward_int), _ptr(resp)
    P.resp_len, P.spans = _ptr(resp_len), _ptr(spans)
    P.cond, P.active = _ptr(cond), _ptr(active)
    P.pool_len = pool.numel() if pool is not None else 0
    if turn is not None and turn[0] is not None:
        P.turn_exec, P.flags = _ptr(turn[0]), _ptr(turn[1])
        P.int_reward_tags, P.last_turn = int(turn[2]) & 0xFFFFFFFF, int(turn[3])
    return P


@_op("prompt_text")
def prompt_text(program: List[int], sep: List[int], B: int, stride: int, pool: Optional[Tensor],
                tag_const: Optional[Tensor], tag: Optional[Tensor], obs: Optional[Tensor], obs_len: Optional[Tensor],
                ints: Optional[Tensor], reward: Optional[Tensor], reward_int: Optional[Tensor], resp: Optional[Tensor],
                resp_len: Optional[Tensor], spans: Optional[Tensor], cond: Optional[Tensor],
                active: Optional[Tensor], turn_exec: Optional[Tensor] = None, flags: Optional[Tensor] = None,
                int_reward_tags: int = 0, last_turn: int = 0) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """The prompt text one turn appends (ctx_manager.py:248-263, rmi_prompt_text)
    -> (text u8[B, stride], text_len i32[B], mark i32[B], err u8[B]).  With turn_exec (and
    flags) the turn form: reward_int / cond derived on the device (rmi_prompt_t)."""
    ts = (pool, tag_const, tag, obs, obs_len, ints, reward, reward_int, resp, resp_len, spans, cond, active)
    dev = ops._dev(*ts, turn_exec, flags)
    if turn_exec is not None:
        if flags is None:
            raise ValueError("the turn form needs flags with turn_exec")
        ops._dt(turn_exec, torch.uint8, "turn_exec")
        ops._dt(flags, torch.uint8, "flags")
    for t, dt, nm in ((pool, torch.uint8, "pool"), (tag_const, torch.int32, "tag_const"), (tag, torch.uint8, "tag"),
                      (obs, torch.uint8, "obs"), (obs_len, torch.int32, "obs_len"), (ints, torch.int32, "ints"),
                      (reward, torch.float64, "reward"), (reward_int, torch.uint8, "reward_int"),
                      (resp, torch.uint8, "resp"), (resp_len, torch.int32, "resp_len"), (spans, torch.int32, "spans"),
                      (cond, torch.uint8, "cond"), (active, torch.uint8, "active")):
        ops._dt(t, dt, nm)
    import ctypes
    P = prompt_struct(program, sep, ts, (turn_exec, flags, int_reward_tags, last_turn))
    out = torch.empty(B, stride, dtype=torch.uint8, device=dev)
    n = torch.empty(B, dtype=torch.int32, device=dev)
    mark = torch.empty(B, dtype=torch.int32, device=dev)
    err = torch.empty(B, dtype=torch.uint8, device=dev)
    ops.check(ops.lib().rmi_prompt_text(ctypes.byref(P), B, out.data_ptr(), stride, n.data_ptr(), mark.data_ptr(),
                                        err.data_ptr(), ops._stream(dev)), "rmi_prompt_text")
    return out, n, mark, err


@prompt_text.register_fake
def _(program, sep, B, stride, pool, tag_const, tag, obs, obs_len, ints, reward, reward_int, resp, resp_len, spans,
      cond, active, turn_exec=None, flags=None, int_reward_tags=0, last_turn=0):
    t = next(x for x in (pool, obs, resp, reward) if x is not None)
    return (t.new_empty(B, stride, dtype=torch.uint8), t.new_empty(B, dtype=torch.int32),
            t.new_empty(B, dtype=torch.int32), t.new_empty(B, dtype=torch.uint8))


# the mutating ops return nothing: their fake kernels only have to exist
for _name in ("gen_rows", "sokoban_step_turn", "sokoban_step_turn_first", "sokoban_step_turn_finalize",
              "sokoban_step_turn_render",
              "sokoban_reset", "frozenlake_step_turn", "frozenlake_step_turn_first", "frozenlake_step_turn_finalize",
              "frozenlake_reset", "bandit_step_turn", "countdown_step_turn", "rollout_finalize"):
    torch.library.register_fake(f"{NS}::{_name}", lambda *a, **k: None, lib=_LIB)

OPS = tuple(sorted(_NAMES))
