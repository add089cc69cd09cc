"""Tensor-level entry points: thin, validated wrappers over the C ABI (include/ragen_amd.h).

Every function takes torch tensors that already live on the GPU, enqueues the HIP kernel
on torch's current stream and returns without synchronising.  Validation mirrors the
reference's error behaviour (ValueError for bad arguments; IndexError for the bi-level
GAE case the reference raises on, core_algos.py:79, when ``check=True``).
"""
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import _lib
from ._lib import check, lib


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _stream(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def _dev(*ts):
    for t in ts:
        if t is not None:
            if not t.is_cuda:
                raise ValueError("ragen_amd ops take GPU tensors (the engine has no CPU path)")
            if not t.is_contiguous():
                raise ValueError("ragen_amd ops take contiguous tensors")


def _dt(t, dtype, name):
    if t is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")


# ----------------------------------------------------------------- episode state (A1)
@dataclass
class EpisodeState:
    """Device SoA of EnvStatus + rollout-cache bookkeeping (es_manager.py:17-24, :85)."""
    num_actions: torch.Tensor   # i32[B]
    flags: torch.Tensor         # u8[B]   FLAG_* bits
    n_turns: torch.Tensor       # i32[B]
    penalty: torch.Tensor       # f64[B]
    turn_reward: torch.Tensor   # f64[T,B]
    turn_info: torch.Tensor     # u8[T,B]
    turn_exec: torch.Tensor     # u8[T,B]
    arena: Optional[torch.Tensor] = None  # u8[nbytes]: every field above is a view into it

    # field order inside the arena (each field 256-B aligned)
    FIELDS = (("num_actions", torch.int32, False), ("flags", torch.uint8, False), ("n_turns", torch.int32, False),
              ("penalty", torch.float64, False), ("turn_reward", torch.float64, True),
              ("turn_info", torch.uint8, True), ("turn_exec", torch.uint8, True))

    @staticmethod
    def layout(B: int, T: int):
        """-> ([(name, dtype, shape, byte offset)], total bytes) of the arena."""
        out, off = [], 0
        for name, dt, per_turn in EpisodeState.FIELDS:
            shape = (T, B) if per_turn else (B,)
            n = int(np.prod(shape)) * torch.empty((), dtype=dt).element_size()
            out.append((name, dt, shape, off))
            off += (n + 255) // 256 * 256
        return out, off

    @staticmethod
    def empty(B: int, T: int, device) -> "EpisodeState":
        """All fields live in one contiguous zeroed arena, so a rank's whole episode record is a
        single buffer: one collective moves it (ragen_amd.distributed.gather_episode)."""
        fields, total = EpisodeState.layout(B, T)
        arena = torch.zeros(max(total, 1), dtype=torch.uint8, device=device)
        views = {name: EpisodeState.view(arena, dt, shape, off) for name, dt, shape, off in fields}
        return EpisodeState(arena=arena, **views)

    @staticmethod
    def pool(n: int, B: int, T: int, device):
        """n arenas back to back in one zeroed buffer -> (u8[n, nbytes], [EpisodeState] * n), so
        several rollouts' records move in one collective."""
        fields, total = EpisodeState.layout(B, T)
        buf = torch.zeros(n, max(total, 1), dtype=torch.uint8, device=device)
        eps = [EpisodeState(arena=row, **{name: EpisodeState.view(row, dt, shape, off)
                                          for name, dt, shape, off in fields}) for row in buf]
        return buf, eps

    @staticmethod
    def view(buf: torch.Tensor, dt, shape, off: int) -> torch.Tensor:
        n = int(np.prod(shape)) * torch.empty((), dtype=dt).element_size()
        return buf[off:off + n].view(dt).view(*shape)

    def reset_(self):
        if self.arena is not None:
            self.arena.zero_()
            return self
        for t in (self.num_actions, self.flags, self.n_turns, self.penalty, self.turn_reward, self.turn_info,
                  self.turn_exec):
            t.zero_()
        return self

    @property
    def B(self):
        return self.flags.shape[0]

    @property
    def T(self):
        return self.turn_reward.shape[0]

    def struct(self) -> _lib.Episode:
        _dev(self.num_actions, self.flags, self.n_turns, self.penalty, self.turn_reward, self.turn_info,
             self.turn_exec)
        return _lib.Episode(self.B, self.T, _ptr(self.num_actions), _ptr(self.flags), _ptr(self.n_turns),
                            _ptr(self.penalty), _ptr(self.turn_reward), _ptr(self.turn_info), _ptr(self.turn_exec))


def turn_struct(turn: int, actions: torch.Tensor, n_actions: torch.Tensor, has_input: Optional[torch.Tensor],
                max_actions_per_traj: int, format_penalty: float) -> _lib.Turn:
    _dev(actions, n_actions, has_input)
    _dt(actions, torch.int8, "actions")
    _dt(n_actions, torch.uint8, "n_actions")
    _dt(has_input, torch.uint8, "has_input")
    K = actions.shape[1] if actions.dim() == 2 else 0
    return _lib.Turn(int(turn), int(K), _ptr(actions), _ptr(n_actions), _ptr(has_input), int(max_actions_per_traj),
                     float(format_penalty))


# ------------------------------------------------------------------------ env steps
def sokoban_step_turn(env: _lib.Sokoban, ep: EpisodeState, turn: _lib.Turn, err: Optional[torch.Tensor] = None):
    check(lib().rmi_sokoban_step_turn(env, ep.struct(), turn, _ptr(err), _stream()), "rmi_sokoban_step_turn")


def finalize_struct(group_size: int, method: str, norm: Optional[torch.Tensor],
                    metrics: Optional[torch.Tensor] = None, score: Optional[torch.Tensor] = None,
                    pen: Optional[torch.Tensor] = None) -> _lib.Finalize:
    """Outputs of the fused last turn (see sokoban_step_turn_finalize); the tensors must outlive
    every launch (or graph replay) that uses the struct."""
    if method not in _lib.NORM_METHODS:
        raise ValueError(f"Invalid normalization method: {method}")
    _dev(norm, metrics, score, pen)
    _dt(norm, torch.float32, "norm")
    _dt(score, torch.float32, "score")
    _dt(pen, torch.float32, "pen")
    _dt(metrics, torch.float64, "metrics")
    return _lib.Finalize(int(group_size), _lib.NORM_METHODS[method], _ptr(metrics), _ptr(score), _ptr(pen),
                         _ptr(norm))


def sokoban_step_turn_finalize(env: _lib.Sokoban, ep: EpisodeState, turn: _lib.Turn, fin: _lib.Finalize,
                               err: Optional[torch.Tensor] = None):
    """The rollout's last turn + rollout_finalize (uniform groups of fin.group_size) in one launch.
    Groups that would straddle a wave take the two launches instead (same results)."""
    rc = lib().rmi_sokoban_step_turn_finalize(env, ep.struct(), turn, _ptr(err), fin, _stream())
    if rc == _lib.RMI_EUNSUP and fin.group_size >= 1 and ep.B % fin.group_size == 0:
        sokoban_step_turn(env, ep, turn, err)
        seg = torch.arange(0, ep.B + 1, fin.group_size, dtype=torch.int32, device=ep.flags.device)
        check(lib().rmi_rollout_finalize(ep.struct(), _ptr(seg), seg.numel() - 1, fin.method, fin.metrics,
                                         fin.score, fin.pen, fin.norm, _stream()), "rmi_rollout_finalize")
        return
    check(rc, "rmi_sokoban_step_turn_finalize")


def sokoban_reset(env: _lib.Sokoban, ep: EpisodeState, init_state: torch.Tensor, init_player: torch.Tensor):
    """Fused device reset from the generated rooms (state, player, counters, episode record)."""
    _dev(init_state, init_player)
    check(lib().rmi_sokoban_reset(env, ep.struct(), _ptr(init_state), _ptr(init_player), _stream()),
          "rmi_sokoban_reset")


def frozenlake_reset(env: _lib.FrozenLake, ep: EpisodeState, init_desc: torch.Tensor, init_s: torch.Tensor,
                     init_rng: torch.Tensor):
    """Fused device reset from the generated maps (desc, start state, seeded PCG64, record)."""
    _dev(init_desc, init_s, init_rng)
    check(lib().rmi_frozenlake_reset(env, ep.struct(), _ptr(init_desc), _ptr(init_s), _ptr(init_rng), _stream()),
          "rmi_frozenlake_reset")


def frozenlake_step_turn(env: _lib.FrozenLake, ep: EpisodeState, turn: _lib.Turn,
                         err: Optional[torch.Tensor] = None):
    check(lib().rmi_frozenlake_step_turn(env, ep.struct(), turn, _ptr(err), _stream()), "rmi_frozenlake_step_turn")


def bandit_step_turn(env: _lib.Bandit, ep: EpisodeState, turn: _lib.Turn, err: Optional[torch.Tensor] = None):
    check(lib().rmi_bandit_step_turn(env, ep.struct(), turn, _ptr(err), _stream()), "rmi_bandit_step_turn")


def countdown_step_turn(env: _lib.Countdown, ep: EpisodeState, turn: _lib.Turn, answers: torch.Tensor,
                        answer_len: torch.Tensor, err: Optional[torch.Tensor] = None):
    _dev(answers, answer_len)
    _dt(answers, torch.uint8, "answers")
    _dt(answer_len, torch.int32, "answer_len")
    check(lib().rmi_countdown_step_turn(env, ep.struct(), turn, _ptr(answers), _ptr(answer_len), answers.shape[-1],
                                        _ptr(err), _stream()), "rmi_countdown_step_turn")


def countdown_reward(env: _lib.Countdown, answers: torch.Tensor, answer_len: torch.Tensor):
    """Batch of compute_reward() calls (countdown/env.py:69-78): returns (reward f64, flags u8, err u8)."""
    _dev(answers, answer_len)
    n = answers.shape[0]
    dev = answers.device
    reward = torch.empty(n, dtype=torch.float64, device=dev)
    flags = torch.empty(n, dtype=torch.uint8, device=dev)
    err = torch.empty(n, dtype=torch.uint8, device=dev)
    check(lib().rmi_countdown_reward(env, _ptr(answers), _ptr(answer_len), answers.shape[-1], n, _ptr(reward),
                                     _ptr(flags), _ptr(err), _stream()), "rmi_countdown_reward")
    return reward, flags, err


def generate_sokoban_rooms(seeds, H: int, W: int, num_boxes: int, search_depth: int, n_threads: int = 8):
    """Host-side level generation (sokoban/utils.py:221-278) -> numpy arrays (fixed, state, player, status)."""
    import numpy as np
    seeds = np.ascontiguousarray(np.asarray(seeds, dtype=np.int64))
    n = seeds.shape[0]
    fixed = np.zeros((n, H * W), np.uint8)
    state = np.zeros((n, H * W), np.uint8)
    player = np.zeros((n, 2), np.int8)
    status = np.zeros(n, np.uint8)
    rc = lib().rmi_sokoban_generate_rooms(seeds.ctypes.data, n, H, W, num_boxes, search_depth, fixed.ctypes.data,
                                          state.ctypes.data, player.ctypes.data, status.ctypes.data, n_threads)
    if rc != 0:
        raise ValueError("rmi_sokoban_generate_rooms: invalid arguments (seeds must be in [0, 2**32))")
    return fixed, state, player, status


# ------------------------------------------------------------------- episode reductions
def rollout_metrics(ep: EpisodeState) -> torch.Tensor:
    out = torch.empty(ep.B, 4, dtype=torch.float64, device=ep.flags.device)
    check(lib().rmi_rollout_metrics(ep.struct(), _ptr(out), _stream()), "rmi_rollout_metrics")
    return out


def trajectory_scores(ep: EpisodeState):
    dev = ep.flags.device
    score = torch.empty(ep.B, dtype=torch.float32, device=dev)
    pen = torch.empty(ep.B, dtype=torch.float32, device=dev)
    check(lib().rmi_trajectory_scores(ep.struct(), _ptr(score), _ptr(pen), _stream()), "rmi_trajectory_scores")
    return score, pen


def rollout_finalize(ep: EpisodeState, seg: torch.Tensor, method: str, norm: torch.Tensor,
                     metrics: Optional[torch.Tensor] = None, score: Optional[torch.Tensor] = None,
                     pen: Optional[torch.Tensor] = None):
    """Fused get_rollout_states metrics + trajectory scores + reward normalisation (one launch)."""
    if method not in _lib.NORM_METHODS:
        raise ValueError(f"Invalid normalization method: {method}")
    _dev(seg, norm, metrics, score, pen)
    check(lib().rmi_rollout_finalize(ep.struct(), _ptr(seg), seg.numel() - 1, _lib.NORM_METHODS[method],
                                     _ptr(metrics), _ptr(score), _ptr(pen), _ptr(norm), _stream()),
          "rmi_rollout_finalize")
    return norm


def group_normalize(score: torch.Tensor, pen: Optional[torch.Tensor], seg: torch.Tensor, method: str,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if method not in _lib.NORM_METHODS:
        raise ValueError(f"Invalid normalization method: {method}")
    _dev(score, pen, seg)
    _dt(score, torch.float32, "score")
    _dt(pen, torch.float32, "pen")
    _dt(seg, torch.int32, "seg")
    out = torch.empty_like(score) if out is None else out
    check(lib().rmi_group_normalize(_ptr(score), _ptr(pen), _ptr(seg), seg.numel() - 1, score.numel(),
                                    _lib.NORM_METHODS[method], _ptr(out), _stream()), "rmi_group_normalize")
    return out


def filter_groups(scores: torch.Tensor, num_groups: int, group_size: int, ratio: float, ftype: str):
    if ftype not in ("std", "std_rev"):
        raise ValueError(f"Invalid rollout filter type: {ftype}")
    _dev(scores)
    _dt(scores, torch.float32, "scores")
    dev = scores.device
    g_std = torch.empty(num_groups, dtype=torch.float32, device=dev)
    g_max = torch.empty_like(g_std)
    g_mean = torch.empty_like(g_std)
    keep = torch.empty(num_groups, dtype=torch.uint8, device=dev)
    metrics = torch.empty(6, dtype=torch.float64, device=dev)
    check(lib().rmi_filter_groups(_ptr(scores), num_groups, group_size, float(ratio), 0 if ftype == "std" else 1,
                                  _ptr(g_std), _ptr(g_max), _ptr(g_mean), _ptr(keep), _ptr(metrics), _stream()),
          "rmi_filter_groups")
    return keep, metrics, (g_std, g_max, g_mean)


def row_sum(x: torch.Tensor) -> torch.Tensor:
    _dev(x)
    _dt(x, torch.float32, "x")
    out = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
    check(lib().rmi_row_sum(_ptr(x), x.shape[0], x.shape[1], _ptr(out), _stream()), "rmi_row_sum")
    return out


# ------------------------------------------------------------- text observations (A6)
def glyph_table(lookup):
    """grid_lookup {code: str} -> (u32[16] packed UTF-8, u8[16] lengths) host arrays."""
    gb = np.zeros(16, np.uint32)
    gl = np.zeros(16, np.uint8)
    for code, ch in (lookup or {}).items():
        if 0 <= int(code) < 16:
            b = str(ch).encode("utf-8")
            if len(b) > 4:
                raise ValueError(f"glyph for {code} longer than 4 UTF-8 bytes")
            gb[int(code)] = int.from_bytes(b.ljust(4, b"\0"), "little")
            gl[int(code)] = len(b)
    return gb, gl


def _render(fn, env_struct, B: int, cells: int, rows: int, lookup, device):
    gb, gl = glyph_table(lookup)
    stride = (cells * 4 + rows - 1 + 3) // 4 * 4
    out = torch.empty(B, stride, dtype=torch.uint8, device=device)
    n = torch.empty(B, dtype=torch.int32, device=device)
    check(fn(env_struct, B, gb.ctypes.data, gl.ctypes.data, _ptr(out), stride, _ptr(n), _stream()), fn.__name__)
    return out, n


def decode_rows(out: torch.Tensor, n: torch.Tensor):
    """u8[B, stride] + i32[B] lengths -> list of str (one host copy, one decode per row)."""
    buf = out.cpu().numpy()
    lens = n.cpu().numpy()
    return [buf[i, :lens[i]].tobytes().decode("utf-8") for i in range(len(lens))]


def sokoban_render(env: _lib.Sokoban, B: int, lookup, device):
    """SokobanEnv.render text of every env (sokoban/env.py:53-61) -> (u8[B,stride], i32[B])."""
    return _render(lib().rmi_sokoban_render, env, B, env.H * env.W, env.H, lookup, device)


def frozenlake_render(env: _lib.FrozenLake, B: int, lookup, device):
    """FrozenLakeEnv.render text of every env (frozen_lake/env.py:47-61) -> (u8[B,stride], i32[B])."""
    return _render(lib().rmi_frozenlake_render, env, B, env.nrow * env.ncol, env.nrow, lookup, device)


# ------------------------------------------------------------------- token masks (A11)
def masks_and_scores(ids: torch.Tensor, special_token: int, reward_token: int, scores: torch.Tensor,
                     n_scores: torch.Tensor, n_slots: int, use_turn_scores: bool, enable_response_mask: bool,
                     roll: bool):
    """get_masks_and_scores (ctx_manager.py:35-70) on the device.  ids i64[B,S]; scores f64[T,B]
    turn-major (e.g. EpisodeState.turn_reward); n_scores i32[B]; n_slots = zip_longest length.
    -> (score f32[B,S-1], loss_mask bool[B,S-1], response_mask bool[B,S-1], err u8[B])."""
    _dev(ids, scores, n_scores)
    _dt(ids, torch.int64, "input_ids")
    _dt(scores, torch.float64, "scores")
    _dt(n_scores, torch.int32, "n_scores")
    ids = ids.contiguous()
    B, S = ids.shape
    T = scores.shape[0] if scores.dim() == 2 else 0
    if T and scores.shape[1] != B:
        raise ValueError(f"scores must be [T, B={B}], got {tuple(scores.shape)}")
    dev = ids.device
    So = max(S - 1, 0)
    score = torch.empty(B, So, dtype=torch.float32, device=dev)
    lm = torch.empty(B, So, dtype=torch.bool, device=dev)
    rm = torch.empty(B, So, dtype=torch.bool, device=dev)
    err = torch.zeros(B, dtype=torch.uint8, device=dev)
    flags = ((_lib.MS_TURN_SCORES if use_turn_scores else 0) | (_lib.MS_RESPONSE_MASK if enable_response_mask else 0)
             | (_lib.MS_ROLL if roll else 0))
    check(lib().rmi_masks_and_scores(_ptr(ids), B, S, int(special_token), int(reward_token), _ptr(scores.contiguous()),
                                     _ptr(n_scores), T, int(n_slots), flags, _ptr(score), _ptr(lm), _ptr(rm), _ptr(err),
                                     _stream()), "rmi_masks_and_scores")
    return score, lm, rm, err


# ------------------------------------------------------------------------ advantages
def _mask_u8(mask: torch.Tensor) -> torch.Tensor:
    if mask.dtype == torch.bool:
        return mask.view(torch.uint8)
    if mask.dtype == torch.uint8:
        return mask
    return (mask != 0).to(torch.uint8)


def gae(r, v, mask, gamma, lam, variant="legacy", row_stats=None):
    _dev(r, v, mask)
    _dt(r, torch.float32, "token_level_rewards")
    _dt(v, torch.float32, "values")
    m = _mask_u8(mask).contiguous()
    B, L = r.shape
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    check(lib().rmi_gae(_ptr(r), _ptr(v), _ptr(m), B, L, float(gamma), float(lam), 0 if variant == "legacy" else 1,
                        _ptr(adv), _ptr(ret), _ptr(row_stats), _stream()), "rmi_gae")
    return adv, ret


def bilevel_gae(r, v, mask, gamma, lam, high_level_gamma, row_stats=None, check_errors=True):
    _dev(r, v, mask)
    _dt(r, torch.float32, "token_level_rewards")
    _dt(v, torch.float32, "values")
    m = _mask_u8(mask).contiguous()
    B, L = r.shape
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    err = torch.empty(B, dtype=torch.uint8, device=r.device)
    check(lib().rmi_bilevel_gae(_ptr(r), _ptr(v), _ptr(m), B, L, float(gamma), float(lam), float(high_level_gamma),
                                _ptr(adv), _ptr(ret), _ptr(row_stats), _ptr(err), _stream()), "rmi_bilevel_gae")
    if check_errors and bool(err.any()):
        raise IndexError("index out of range: last loss-mask position of a row carries no reward "
                         "(reference core_algos.py:79)")
    return adv, ret


def masked_whiten_(x, mask, row_stats=None):
    _dev(x, mask, row_stats)
    m = _mask_u8(mask).contiguous()
    B, L = x.shape
    nbytes = int(lib().rmi_whiten_scratch_bytes(B))
    scratch = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
    check(lib().rmi_masked_whiten(_ptr(x), _ptr(m), B, L, _ptr(row_stats), _ptr(scratch), _stream()),
          "rmi_masked_whiten")
    return x, scratch


def grpo_outcome(r, mask, seg, eps=1e-6, norm_by_std=True):
    _dev(r, mask, seg)
    m = _mask_u8(mask).contiguous()
    B, L = r.shape
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    check(lib().rmi_grpo_outcome(_ptr(r), _ptr(m), B, L, _ptr(seg), seg.numel() - 1, float(eps), int(norm_by_std),
                                 _ptr(adv), _ptr(ret), _stream()), "rmi_grpo_outcome")
    return adv, ret
