"""Tensor-level entry points: thin, validated wrappers over the C ABI (include/ragen_amd.h).

Every function takes torch tensors that already live on the GPU, enqueues the HIP kernel
on torch's current stream and returns without synchronising.  Validation mirrors the
reference's error behaviour (ValueError for bad arguments; IndexError for the bi-level
GAE case the reference raises on, core_algos.py:79, when ``check=True``).
"""
import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import _lib
from ._lib import check, lib


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


_raw_stream = torch._C._cuda_getCurrentRawStream  # (device index) -> hipStream_t, no Stream object


def _stream(device):
    """torch's current stream ON THE TENSORS' DEVICE (not on the process's current device), as
    the raw hipStream_t (torch.cuda.current_stream builds a Stream object: several us a call,
    and the turn loop passes a stream to a dozen launches per turn)."""
    idx = device if isinstance(device, int) else device.index
    return _raw_stream(torch.cuda.current_device() if idx is None else idx)


_DEVICES = {}  # device index -> torch.device


def _dev(*ts):
    """Validate GPU tensors (contiguous, one device) -> that device (None if all are None)."""
    idx = None
    for t in ts:
        if t is not None:
            if not t.is_cuda:
                raise ValueError("ragen_amd ops take GPU tensors (the engine has no CPU path)")
            if not t.is_contiguous():
                raise ValueError("ragen_amd ops take contiguous tensors")
            i = t.get_device()
            if idx is None:
                idx = i
            elif i != idx:
                raise ValueError(f"ragen_amd ops take tensors on one device, got cuda:{idx} and cuda:{i}")
    if idx is None:
        return None
    d = _DEVICES.get(idx)
    if d is None:
        d = _DEVICES[idx] = torch.device("cuda", idx)
    return d


def _dt(t, dtype, name):
    if t is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")


# ----------------------------------------------------------------- episode state (A1)
@dataclass
class EpisodeState:
    """Device SoA of EnvStatus + rollout-cache bookkeeping (es_manager.py:17-24, :85)."""
    num_actions: torch.Tensor   # u8[B]
    flags: torch.Tensor         # u8[B]   FLAG_* bits
    n_turns: torch.Tensor       # u8[B]
    penalty: torch.Tensor       # f64[B]
    turn_reward: torch.Tensor   # f64[T,B]
    turn_info: torch.Tensor     # u8[T,B]
    turn_exec: torch.Tensor     # u8[T,B]
    arena: Optional[torch.Tensor] = None  # u8[nbytes]: every field above is a view into it

    # field order inside the arena (each field 256-B aligned)
    FIELDS = (("num_actions", torch.uint8, False), ("flags", torch.uint8, False), ("n_turns", torch.uint8, False),
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

    @property
    def device(self):
        return self.flags.device

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
    check(lib().rmi_sokoban_step_turn(env, ep.struct(), turn, _ptr(err), _stream(ep.device)), "rmi_sokoban_step_turn")


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
    rc = lib().rmi_sokoban_step_turn_finalize(env, ep.struct(), turn, _ptr(err), fin, _stream(ep.device))
    if rc == _lib.RMI_EUNSUP and fin.group_size >= 1 and ep.B % fin.group_size == 0:
        sokoban_step_turn(env, ep, turn, err)
        seg = torch.arange(0, ep.B + 1, fin.group_size, dtype=torch.int32, device=ep.flags.device)
        check(lib().rmi_rollout_finalize(ep.struct(), _ptr(seg), seg.numel() - 1, fin.method, fin.metrics,
                                         fin.score, fin.pen, fin.norm, _stream(ep.device)), "rmi_rollout_finalize")
        return
    check(rc, "rmi_sokoban_step_turn_finalize")


def sokoban_step_turn_first(env: _lib.Sokoban, ep: EpisodeState, turn: _lib.Turn, init_state: torch.Tensor,
                            init_player: torch.Tensor, err: Optional[torch.Tensor] = None):
    """sokoban_reset(init_state, init_player) + sokoban_step_turn(turn) in one launch: a fresh
    episode's first turn (the record is written, never read)."""
    _dev(init_state, init_player, err)
    _dt(init_state, torch.uint8, "init_state")
    _dt(init_player, torch.int8, "init_player")
    check(lib().rmi_sokoban_step_turn_first(env, ep.struct(), turn, _ptr(init_state), _ptr(init_player), _ptr(err),
                                            _stream(ep.device)), "rmi_sokoban_step_turn_first")


def sokoban_reset(env: _lib.Sokoban, ep: EpisodeState, init_state: torch.Tensor, init_player: torch.Tensor):
    """Fused device reset from the generated rooms (state, player, counters, episode record)."""
    _dev(init_state, init_player)
    check(lib().rmi_sokoban_reset(env, ep.struct(), _ptr(init_state), _ptr(init_player), _stream(ep.device)),
          "rmi_sokoban_reset")


def sokoban_load_rooms(env: _lib.Sokoban, ep: EpisodeState, rooms: torch.Tensor, room_of: Optional[torch.Tensor],
                       init_state: torch.Tensor, init_player: torch.Tensor, err: Optional[torch.Tensor] = None):
    """Fused device reset from the distinct generated rooms u8[U, 2HW+2] (env i takes row
    room_of[i], or row i): room_fixed, init_state / init_player, then the reset (rmi_sokoban_load_rooms)."""
    _dev(rooms, room_of, init_state, init_player, err)
    _dt(rooms, torch.uint8, "rooms")
    _dt(room_of, torch.int32, "room_of")
    _dt(init_state, torch.uint8, "init_state")
    _dt(init_player, torch.int8, "init_player")
    _dt(err, torch.uint8, "err")
    HW = env.H * env.W
    if rooms.dim() != 2 or rooms.shape[1] != 2 * HW + 2:
        raise ValueError(f"rooms: u8[U, {2 * HW + 2}] rows (fixed | state | player)")
    B = ep.B
    if init_state.numel() != B * HW or init_player.numel() != 2 * B or (room_of is not None and room_of.numel() != B) \
            or (err is not None and err.numel() != B) or (room_of is None and rooms.shape[0] < B):
        raise ValueError("init_state / init_player / room_of / err: one row per env")
    check(lib().rmi_sokoban_load_rooms(env, ep.struct(), _ptr(rooms), rooms.shape[0], _ptr(room_of), _ptr(init_state),
                                       _ptr(init_player), _ptr(err), _stream(ep.device)), "rmi_sokoban_load_rooms")


def frozenlake_reset(env: _lib.FrozenLake, ep: EpisodeState, init_desc: torch.Tensor, init_s: torch.Tensor,
                     init_rng: torch.Tensor):
    """Fused device reset from the generated maps (desc, start state, seeded PCG64, record)."""
    _dev(init_desc, init_s, init_rng)
    check(lib().rmi_frozenlake_reset(env, ep.struct(), _ptr(init_desc), _ptr(init_s), _ptr(init_rng), _stream(ep.device)),
          "rmi_frozenlake_reset")


def pcg64_seed(seeds: torch.Tensor, draws: int = 0, rng: Optional[torch.Tensor] = None):
    """Generator(PCG64(SeedSequence(seed))) seeded per element of seeds i64[n] on the device and
    advanced by `draws` random() calls (gymnasium seeding.np_random; bandit/env.py:25-39,
    frozen_lake/env.py:28-37).  -> (rng i64[4, n] (state hi, lo, inc hi, lo), last draw f64[n]).
    Raises ValueError for a negative seed, as SeedSequence does."""
    _dev(seeds, rng)
    _dt(seeds, torch.int64, "seeds")
    n = seeds.shape[0]
    if rng is None:
        rng = torch.empty(4, n, dtype=torch.int64, device=seeds.device)
    if rng.dim() != 2 or rng.shape[0] != 4 or rng.shape[1] != n or not rng.is_contiguous():
        raise ValueError("rng must be a contiguous i64[4, n]")
    last = torch.empty(n, dtype=torch.float64, device=seeds.device)
    err = torch.empty(n, dtype=torch.uint8, device=seeds.device)
    check(lib().rmi_pcg64_seed(_ptr(seeds), n, int(draws), _ptr(rng), n, _ptr(last), _ptr(err),
                               _stream(seeds.device)), "rmi_pcg64_seed")
    if n and bool(err.any()):
        raise ValueError("expected non-negative integer seeds")
    return rng, last


def frozenlake_step_turn_finalize(env: _lib.FrozenLake, ep: EpisodeState, turn: _lib.Turn, fin: _lib.Finalize,
                                  err: Optional[torch.Tensor] = None):
    """frozenlake_step_turn + rollout_finalize (uniform contiguous groups) in one launch.  Groups
    that would straddle the one-wave workgroup take the two launches instead (same results)."""
    _dev(err)
    rc = lib().rmi_frozenlake_step_turn_finalize(env, ep.struct(), turn, _ptr(err), fin, _stream(ep.device))
    if rc == _lib.RMI_EUNSUP and fin.group_size >= 1 and ep.B % fin.group_size == 0:
        frozenlake_step_turn(env, ep, turn, err)
        seg = torch.arange(0, ep.B + 1, fin.group_size, dtype=torch.int32, device=ep.flags.device)
        check(lib().rmi_rollout_finalize(ep.struct(), _ptr(seg), seg.numel() - 1, fin.method, fin.metrics,
                                         fin.score, fin.pen, fin.norm, _stream(ep.device)), "rmi_rollout_finalize")
        return
    check(rc, "rmi_frozenlake_step_turn_finalize")


def frozenlake_step_turn_first(env: _lib.FrozenLake, ep: EpisodeState, turn: _lib.Turn, init_desc: torch.Tensor,
                               init_s: torch.Tensor, init_rng: torch.Tensor, err: Optional[torch.Tensor] = None):
    """frozenlake_reset(init_*) + frozenlake_step_turn(turn) in one launch (a fresh episode's first turn)."""
    _dev(init_desc, init_s, init_rng, err)
    check(lib().rmi_frozenlake_step_turn_first(env, ep.struct(), turn, _ptr(init_desc), _ptr(init_s), _ptr(init_rng),
                                               _ptr(err), _stream(ep.device)), "rmi_frozenlake_step_turn_first")


def frozenlake_step_turn(env: _lib.FrozenLake, ep: EpisodeState, turn: _lib.Turn,
                         err: Optional[torch.Tensor] = None):
    check(lib().rmi_frozenlake_step_turn(env, ep.struct(), turn, _ptr(err), _stream(ep.device)), "rmi_frozenlake_step_turn")


def bandit_step_turn(env: _lib.Bandit, ep: EpisodeState, turn: _lib.Turn, err: Optional[torch.Tensor] = None):
    check(lib().rmi_bandit_step_turn(env, ep.struct(), turn, _ptr(err), _stream(ep.device)), "rmi_bandit_step_turn")


def countdown_step_turn(env: _lib.Countdown, ep: EpisodeState, turn: _lib.Turn, answers: torch.Tensor,
                        answer_len: torch.Tensor, err: Optional[torch.Tensor] = None):
    _dev(answers, answer_len)
    _dt(answers, torch.uint8, "answers")
    _dt(answer_len, torch.int32, "answer_len")
    check(lib().rmi_countdown_step_turn(env, ep.struct(), turn, _ptr(answers), _ptr(answer_len), answers.shape[-1],
                                        _ptr(err), _stream(ep.device)), "rmi_countdown_step_turn")


def countdown_reward(env: _lib.Countdown, answers: torch.Tensor, answer_len: torch.Tensor):
    """Batch of compute_reward() calls (countdown/env.py:69-78): returns (reward f64, flags u8, err u8)."""
    _dev(answers, answer_len)
    n = answers.shape[0]
    dev = answers.device
    reward = torch.empty(n, dtype=torch.float64, device=dev)
    flags = torch.empty(n, dtype=torch.uint8, device=dev)
    err = torch.empty(n, dtype=torch.uint8, device=dev)
    check(lib().rmi_countdown_reward(env, _ptr(answers), _ptr(answer_len), answers.shape[-1], n, _ptr(reward),
                                     _ptr(flags), _ptr(err), _stream(answers.device)), "rmi_countdown_reward")
    return reward, flags, err


def host_threads() -> int:
    """Worker threads for host-side work: OMP_NUM_THREADS when set (the GPU boxes set their CPU
    share there), else the CPUs this process may run on, capped at 16."""
    import os
    v = os.environ.get("OMP_NUM_THREADS", "")
    if v.isdigit() and int(v) > 0:
        return int(v)
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def generate_sokoban_rooms(seeds, H: int, W: int, num_boxes: int, search_depth: int, n_threads: int = 0):
    """Host-side level generation (sokoban/utils.py:221-278) -> numpy arrays (fixed, state, player, status).
    n_threads 0: host_threads(); each thread takes a contiguous range of the seeds."""
    import numpy as np
    n_threads = n_threads or host_threads()
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


class RoomsJob:
    """generate_sokoban_rooms on a native host thread (rmi_sokoban_generate_rooms_start): no
    Python thread and no GIL held while it runs.  wait() -> (fixed, state, player, status)."""

    def __init__(self, seeds, H: int, W: int, num_boxes: int, search_depth: int, n_threads: int = 0):
        import numpy as np
        self.seeds = np.ascontiguousarray(np.asarray(seeds, dtype=np.int64))
        n = self.seeds.shape[0]
        self.out = (np.zeros((n, H * W), np.uint8), np.zeros((n, H * W), np.uint8), np.zeros((n, 2), np.int8),
                    np.zeros(n, np.uint8))
        f, st, p, ok = self.out
        self._job = lib().rmi_sokoban_generate_rooms_start(self.seeds.ctypes.data, n, H, W, num_boxes, search_depth,
                                                           f.ctypes.data, st.ctypes.data, p.ctypes.data,
                                                           ok.ctypes.data, n_threads or host_threads())
        if not self._job:
            raise RuntimeError("rmi_sokoban_generate_rooms_start: could not start a host thread")

    def wait(self):
        job, self._job = self._job, None
        if job is None:
            raise RuntimeError("RoomsJob.wait: already waited on")
        if lib().rmi_sokoban_generate_rooms_wait(job) != 0:
            raise ValueError("rmi_sokoban_generate_rooms: invalid arguments (seeds must be in [0, 2**32))")
        return self.out

    def __del__(self):  # a job nobody took: joined before its buffers go
        if getattr(self, "_job", None):
            lib().rmi_sokoban_generate_rooms_wait(self._job)
            self._job = None


# ------------------------------------------------------------------- episode reductions
def rollout_metrics(ep: EpisodeState) -> torch.Tensor:
    out = torch.empty(ep.B, 4, dtype=torch.float64, device=ep.flags.device)
    check(lib().rmi_rollout_metrics(ep.struct(), _ptr(out), _stream(ep.device)), "rmi_rollout_metrics")
    return out


def trajectory_scores(ep: EpisodeState):
    dev = ep.flags.device
    score = torch.empty(ep.B, dtype=torch.float32, device=dev)
    pen = torch.empty(ep.B, dtype=torch.float32, device=dev)
    check(lib().rmi_trajectory_scores(ep.struct(), _ptr(score), _ptr(pen), _stream(ep.device)), "rmi_trajectory_scores")
    return score, pen


def rollout_finalize(ep: EpisodeState, seg: torch.Tensor, method: str, norm: torch.Tensor,
                     metrics: Optional[torch.Tensor] = None, score: Optional[torch.Tensor] = None,
                     pen: Optional[torch.Tensor] = None):
    """Fused get_rollout_states metrics + trajectory scores + reward normalisation (one launch)."""
    if method not in _lib.NORM_METHODS:
        raise ValueError(f"Invalid normalization method: {method}")
    _dev(seg, norm, metrics, score, pen)
    check(lib().rmi_rollout_finalize(ep.struct(), _ptr(seg), seg.numel() - 1, _lib.NORM_METHODS[method],
                                     _ptr(metrics), _ptr(score), _ptr(pen), _ptr(norm), _stream(ep.device)),
          "rmi_rollout_finalize")
    return norm


def group_normalize(score: torch.Tensor, pen: Optional[torch.Tensor], seg: torch.Tensor, method: str,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if method not in _lib.NORM_METHODS:
        raise ValueError(f"Invalid normalization method: {method}")
    _dev(score, pen)
    _dt(score, torch.float32, "score")
    _dt(pen, torch.float32, "pen")
    seg = segments(seg, score.numel(), score.device)
    out = torch.empty_like(score) if out is None else out
    check(lib().rmi_group_normalize(_ptr(score), _ptr(pen), _ptr(seg), seg.numel() - 1, score.numel(),
                                    _lib.NORM_METHODS[method], _ptr(out), _stream(score.device)), "rmi_group_normalize")
    return out


def filter_groups(scores: torch.Tensor, num_groups: int, group_size: int, ratio: float, ftype: str):
    if ftype not in ("std", "std_rev"):
        raise ValueError(f"Invalid rollout filter type: {ftype}")
    _dev(scores)
    _dt(scores, torch.float32, "scores")
    if scores.numel() != num_groups * group_size:
        raise RuntimeError(f"shape '[{num_groups}, {group_size}]' is invalid for input of size {scores.numel()}")
    dev = scores.device
    g_std = torch.empty(num_groups, dtype=torch.float32, device=dev)
    g_max = torch.empty_like(g_std)
    g_mean = torch.empty_like(g_std)
    keep = torch.empty(num_groups, dtype=torch.uint8, device=dev)
    metrics = torch.empty(6, dtype=torch.float64, device=dev)
    check(lib().rmi_filter_groups(_ptr(scores), scores.numel(), num_groups, group_size, float(ratio),
                                  0 if ftype == "std" else 1,
                                  _ptr(g_std), _ptr(g_max), _ptr(g_mean), _ptr(keep), _ptr(metrics), _stream(scores.device)),
          "rmi_filter_groups")
    return keep, metrics, (g_std, g_max, g_mean)


def row_sum(x: torch.Tensor) -> torch.Tensor:
    _dev(x)
    _dt(x, torch.float32, "x")
    out = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
    check(lib().rmi_row_sum(_ptr(x), x.shape[0], x.shape[1], _ptr(out), _stream(x.device)), "rmi_row_sum")
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


def _render(fn, env_struct, B: int, cells: int, rows: int, lookup, device, out=None):
    gb, gl = glyph_table(lookup)
    stride = (cells * 4 + rows - 1 + 3) // 4 * 4
    if out is not None:  # (rows, lengths) of a previous call: no allocation (graph-capturable)
        out, n = out
    else:
        out = torch.empty(B, stride, dtype=torch.uint8, device=device)
        n = torch.empty(B, dtype=torch.int32, device=device)
    check(fn(env_struct, B, gb.ctypes.data, gl.ctypes.data, _ptr(out), stride, _ptr(n), _stream(out.device)), fn.__name__)
    return out, n


def decode_rows(out: torch.Tensor, n: torch.Tensor):
    """u8[B, stride] + i32[B] lengths -> list of str (one host copy, one decode per row)."""
    st = out.shape[1] if out.dim() == 2 else 0
    b = out.cpu().numpy().tobytes()  # one bytes object, sliced per row (no numpy view per row)
    return [b[i * st:i * st + ln].decode("utf-8") for i, ln in enumerate(n.cpu().tolist())]


def sokoban_render(env: _lib.Sokoban, B: int, lookup, device, out=None):
    """SokobanEnv.render text of every env (sokoban/env.py:53-61) -> (u8[B,stride], i32[B])."""
    return _render(lib().rmi_sokoban_render, env, B, env.H * env.W, env.H, lookup, device, out)


def render_struct(lookup, H: int, W: int, out: torch.Tensor, n: torch.Tensor) -> _lib.Render:
    """rmi_render_t of a grid_lookup and the (rows u8[B, stride], lengths i32[B]) it fills; the
    tensors must outlive every launch (or graph replay) that uses the struct."""
    _dev(out, n)
    _dt(out, torch.uint8, "out")
    _dt(n, torch.int32, "len")
    gb, gl = glyph_table(lookup)
    r = _lib.Render()
    for k in range(16):
        r.glyph_bytes[k], r.glyph_len[k] = int(gb[k]), int(gl[k])
    r.out, r.stride, r.len = _ptr(out), int(out.shape[1]), _ptr(n)
    return r


def render_buffers(B: int, H: int, W: int, device):
    """(rows u8[B, stride], lengths i32[B]) for a Sokoban render of H x W rooms."""
    stride = (H * W * 4 + H - 1 + 3) // 4 * 4
    return (torch.empty(B, stride, dtype=torch.uint8, device=device),
            torch.empty(B, dtype=torch.int32, device=device))


def sokoban_step_turn_render(env: _lib.Sokoban, ep: EpisodeState, turn: _lib.Turn, obs: _lib.Render,
                             err: Optional[torch.Tensor] = None, fin: Optional[_lib.Finalize] = None,
                             init_state: Optional[torch.Tensor] = None, init_player: Optional[torch.Tensor] = None):
    """A turn (plain; with fin the rollout's last, fused with its end; with init_state /
    init_player a fresh episode's first, fused with its reset) and every env's observation after
    it, rendered by the same launch into obs (rmi_sokoban_step_turn_render)."""
    _dev(init_state, init_player, err)
    rc = lib().rmi_sokoban_step_turn_render(env, ep.struct(), turn, _ptr(err), fin, _ptr(init_state),
                                            _ptr(init_player), obs, _stream(ep.device))
    if rc == _lib.RMI_EUNSUP and fin is not None and fin.group_size >= 1 and ep.B % fin.group_size == 0:
        # groups that would straddle a wave: the turn with its render, then the finalize
        sokoban_step_turn_render(env, ep, turn, obs, err)
        seg = torch.arange(0, ep.B + 1, fin.group_size, dtype=torch.int32, device=ep.flags.device)
        check(lib().rmi_rollout_finalize(ep.struct(), _ptr(seg), seg.numel() - 1, fin.method, fin.metrics,
                                         fin.score, fin.pen, fin.norm, _stream(ep.device)), "rmi_rollout_finalize")
        return
    check(rc, "rmi_sokoban_step_turn_render")


def frozenlake_render(env: _lib.FrozenLake, B: int, lookup, device, out=None):
    """FrozenLakeEnv.render text of every env (frozen_lake/env.py:47-61) -> (u8[B,stride], i32[B])."""
    return _render(lib().rmi_frozenlake_render, env, B, env.nrow * env.ncol, env.nrow, lookup, device, out)


# ------------------------------------------------- response -> action ids (§8(f) rank 2)
def _pack16(b: bytes):
    if not 1 <= len(b) <= 16:
        raise ValueError(f"string of {len(b)} bytes: 1..16 supported")
    v = b.ljust(16, b"\0")
    return int.from_bytes(v[:8], "little"), int.from_bytes(v[8:], "little")


def parse_config(enable_think: bool, max_actions_per_turn: int, action_sep: str = "||", action_lookup=None,
                 swapped_lookup=None, prepend: bool = True) -> _lib.ParseCfg:
    """rmi_parse_cfg_t for agent_proxy.{enable_think, max_actions_per_turn, action_sep} and an env's
    action_lookup ({id: name}; None = actions pass through as text).  ``swapped_lookup`` is the
    second id column selected per env by ``sel`` (Bandit's per-env lookup, bandit/env.py:25-39);
    it must name the same strings.  Names are matched as ``name.lower()`` (es_manager.py:237-239);
    duplicate lowered names keep the last id, as the dict comprehension does."""
    c = _lib.ParseCfg()
    c.enable_think, c.prepend, c.K = int(bool(enable_think)), int(bool(prepend)), int(max_actions_per_turn)
    c.sep_len = len(action_sep.encode("utf-8"))
    c.sep_lo, c.sep_hi = _pack16(action_sep.encode("utf-8"))
    if action_lookup is None:
        c.n_names = 0
        return c
    cols = []
    for lk in (action_lookup, swapped_lookup if swapped_lookup is not None else action_lookup):
        rev = {}
        for k, v in lk.items():
            rev[str(v).lower()] = int(k)
        cols.append(rev)
    if set(cols[0]) != set(cols[1]):
        raise ValueError("swapped_lookup must name the same actions")
    names = list(cols[0])
    if len(names) > _lib.PARSE_MAX_NAMES:
        raise NotImplementedError(f"{len(names)} action names > {_lib.PARSE_MAX_NAMES}")
    c.n_names = len(names)
    for j, nm in enumerate(names):
        b = nm.encode("utf-8")
        if not nm.isascii():
            raise NotImplementedError(f"non-ASCII action name {nm!r}")
        c.name_len[j] = len(b)
        c.name_lo[j], c.name_hi[j] = _pack16(b)
        for col in range(2):
            i = cols[col][nm]
            if not 1 <= i <= 127:
                raise NotImplementedError(f"action id {i}: 1..127 supported (0 marks an unknown name)")
            c.name_id[col][j] = i
    return c


def parse_actions(cfg: _lib.ParseCfg, text: torch.Tensor, text_len: torch.Tensor, sel: Optional[torch.Tensor] = None,
                  with_spans: bool = True, action_text_len: int = 0, out: Optional[dict] = None):
    """_parse_response + _extract_map_valid_actions for every row (ctx_manager.py:148-173,
    es_manager.py:230-240).  text u8[B,stride] UTF-8 rows, text_len i32[B].
    -> dict(actions i8[B,K], n_actions u8[B], spans i32[B,4] | None, action_text u8[B,K,Lact] | None,
            action_len i32[B,K] | None, err u8[B]).  ``out``: a previous result to write into
    (no allocation: graph-capturable)."""
    _dev(text, text_len, sel)
    _dt(text, torch.uint8, "text")
    _dt(text_len, torch.int32, "text_len")
    _dt(sel, torch.uint8, "sel")
    B, stride = text.shape
    dev = text.device
    K = int(cfg.K)
    if out is not None:
        actions, n_actions, spans, at, al, err = (out[k] for k in ("actions", "n_actions", "spans", "action_text",
                                                                   "action_len", "err"))
        if actions.shape != (B, K) or (at is not None and at.shape != (B, K, int(action_text_len))):
            raise ValueError("out= buffers do not match this batch")
    else:
        actions = torch.empty(B, K, dtype=torch.int8, device=dev)
        n_actions = torch.empty(B, dtype=torch.uint8, device=dev)
        spans = torch.empty(B, 4, dtype=torch.int32, device=dev) if with_spans else None
        at = al = None
        if action_text_len:
            at = torch.empty(B, K, int(action_text_len), dtype=torch.uint8, device=dev)
            al = torch.empty(B, K, dtype=torch.int32, device=dev)
        err = torch.empty(B, dtype=torch.uint8, device=dev)
    check(lib().rmi_parse_actions(ctypes.byref(cfg), _ptr(text), _ptr(text_len), B, stride, _ptr(sel), _ptr(actions),
                                  _ptr(n_actions), _ptr(spans), _ptr(at), _ptr(al), int(action_text_len), _ptr(err),
                                  _stream(text.device)), "rmi_parse_actions")
    return {"actions": actions, "n_actions": n_actions, "spans": spans, "action_text": at, "action_len": al,
            "err": err}


@dataclass
class VocabTable:
    """Device byte table of a byte-level BPE vocabulary: token t decodes to
    bytes[off[t]:off[t+1]]; skip[t] = special token (dropped by skip_special_tokens=True).
    ``packed`` u32[V,4] is rmi_detokenize's form of it (rmi_vocab_pack: the bytes of a token of
    <= 12 bytes inline, its length and skip bit), built once on the host; ``raw_len`` i32[V]
    the bytes each id decodes to (0 when skipped), which sizes the decoded rows."""
    off: torch.Tensor    # i64[V+1]
    data: torch.Tensor   # u8[total]
    skip: torch.Tensor   # u8[V]
    max_token_bytes: int = 0  # longest token's bytes (0 = unknown): sizes the decoded rows
    packed: Optional[torch.Tensor] = None   # u32[V,4] (held as i32)
    raw_len: Optional[torch.Tensor] = None  # i32[V]

    def __post_init__(self):
        if self.packed is None:
            off = np.ascontiguousarray(self.off.cpu().numpy(), np.int64)
            data = np.ascontiguousarray(self.data.cpu().numpy(), np.uint8)
            skip = np.ascontiguousarray(self.skip.cpu().numpy(), np.uint8)
            V = skip.shape[0]
            if off.shape[0] != V + 1:
                raise ValueError(f"off must hold V + 1 = {V + 1} offsets, got {off.shape[0]}")
            pk = np.zeros((V, 4), np.uint32)
            rc = lib().rmi_vocab_pack(off.ctypes.data, data.ctypes.data if data.size else None, data.size, V,
                                      skip.ctypes.data, pk.ctypes.data)
            if rc == _lib.RMI_EUNSUP:
                raise NotImplementedError("a token longer than 2^24 - 1 bytes, or a vocabulary blob past 4 GiB")
            check(rc, "rmi_vocab_pack")
            self.packed = torch.from_numpy(pk.view(np.int32)).to(self.data.device)
            lens = (off[1:] - off[:-1]).astype(np.int32)
            lens[skip != 0] = 0
            self.raw_len = torch.from_numpy(lens).to(self.data.device)

    @staticmethod
    def from_bytes(table, skip, device) -> "VocabTable":
        lens = np.array([len(b) for b in table], np.int64)
        off = np.zeros(len(table) + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        blob = b"".join(table)
        data = np.frombuffer(blob + b"\0" * (4 + (-len(blob)) % 4), np.uint8).copy()  # whole dwords
        return VocabTable(torch.from_numpy(off).to(device), torch.from_numpy(data).to(device),
                          torch.from_numpy(np.asarray(skip, np.uint8)).to(device), int(lens.max()) if len(lens) else 0)

    @staticmethod
    def from_tokenizer(tokenizer, device, skip_special_tokens: bool = True) -> "VocabTable":
        """Per-id byte strings of a HF fast tokenizer whose decoder is ByteLevel (Qwen2,
        Llama-3): regular tokens through the byte<->char map; tokens with a char outside the
        map (added tokens) as their own UTF-8 bytes — the tokenizers ByteLevel decoder."""
        import json
        dec = json.loads(tokenizer.backend_tokenizer.to_str()).get("decoder") or {}
        kinds = {dec.get("type")} | {d.get("type") for d in dec.get("decoders", [])}
        if "ByteLevel" not in kinds:
            raise NotImplementedError("device detokenize supports byte-level BPE tokenizers only")
        if getattr(tokenizer, "clean_up_tokenization_spaces", False):
            raise NotImplementedError("clean_up_tokenization_spaces=True is not supported on the device")
        char_to_byte = {c: b for b, c in _bytes_to_unicode().items()}
        V = len(tokenizer)
        toks = tokenizer.convert_ids_to_tokens(list(range(V)))
        special = set(tokenizer.all_special_ids) if skip_special_tokens else set()
        if skip_special_tokens:
            for i, at in tokenizer.added_tokens_decoder.items():
                if at.special:
                    special.add(int(i))
        table, skip = [], []
        for i, t in enumerate(toks):
            if t is None:
                table.append(b"")
            else:
                try:
                    table.append(bytes(char_to_byte[ch] for ch in t))
                except KeyError:
                    table.append(t.encode("utf-8"))
            skip.append(1 if i in special else 0)
        return VocabTable.from_bytes(table, skip, device)


def _bytes_to_unicode():
    bs = list(range(33, 127)) + list(range(161, 173)) + list(range(174, 256))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, map(chr, cs)))


def detokenize(ids: torch.Tensor, vocab: VocabTable, stride: int, n_ids: Optional[torch.Tensor] = None,
               out=None):
    """tokenizer.batch_decode(ids, skip_special_tokens=True) (ctx_manager.py:334-337) on the
    device: ids i64[B,R] -> (text u8[B,stride] UTF-8 rows, text_len i32[B], err u8[B]).
    ``out``: a previous result to write into (no allocation: graph-capturable)."""
    _dev(ids, n_ids)
    _dt(ids, torch.int64, "ids")
    _dt(n_ids, torch.int32, "n_ids")
    B, R = ids.shape
    stride = (int(stride) + 3) // 4 * 4
    dev = ids.device
    if out is not None:
        out, n, err = out
        if out.shape != (B, stride):
            raise ValueError("out= buffers do not match this batch")
    else:
        out = torch.empty(B, stride, dtype=torch.uint8, device=dev)
        n = torch.empty(B, dtype=torch.int32, device=dev)
        err = torch.empty(B, dtype=torch.uint8, device=dev)
    return detokenize_packed(ids, vocab.packed, vocab.data, stride, n_ids, (out, n, err))


def detokenize_packed(ids: torch.Tensor, packed: torch.Tensor, data: torch.Tensor, stride: int,
                      n_ids: Optional[torch.Tensor], out):
    """rmi_detokenize over a packed vocabulary (VocabTable.packed) into out = (text, len, err)."""
    _dev(ids, n_ids, packed, data)
    _dt(packed, torch.int32, "vocab_packed")
    text, n, err = out
    B, R = ids.shape
    if packed.dim() != 2 or packed.shape[1] != 4 or not packed.is_contiguous():
        raise ValueError("vocab_packed must be a contiguous u32[V, 4]")
    check(lib().rmi_detokenize(_ptr(ids), B, R, _ptr(n_ids), _ptr(packed), _ptr(data), data.numel(), packed.shape[0],
                               _ptr(text), text.shape[1], _ptr(n), _ptr(err), _stream(ids.device)), "rmi_detokenize")
    return text, n, err


def detok_parse(ids: torch.Tensor, vocab: "VocabTable", stride: int, cfg: _lib.ParseCfg,
                n_ids: Optional[torch.Tensor] = None, sel: Optional[torch.Tensor] = None, with_spans: bool = True,
                action_text_len: int = 0, out: Optional[dict] = None):
    """detokenize + parse_actions in one launch (rmi_detok_parse): response ids i64[B,R] ->
    dict(text u8[B,stride], text_len i32[B], decode_err u8[B], and parse_actions' outputs).
    ``out``: a previous result to write into (graph-capturable)."""
    _dev(ids, n_ids, sel, vocab.packed, vocab.data)
    _dt(ids, torch.int64, "ids")
    _dt(n_ids, torch.int32, "n_ids")
    _dt(sel, torch.uint8, "sel")
    B, R = ids.shape
    stride = (int(stride) + 3) // 4 * 4
    dev = ids.device
    K = int(cfg.K)
    if out is not None:
        if out["text"].shape != (B, stride) or out["actions"].shape != (B, K):
            raise ValueError("out= buffers do not match this batch")
        o = out
    else:
        o = {"text": torch.empty(B, stride, dtype=torch.uint8, device=dev),
             "text_len": torch.empty(B, dtype=torch.int32, device=dev),
             "decode_err": torch.empty(B, dtype=torch.uint8, device=dev),
             "actions": torch.empty(B, K, dtype=torch.int8, device=dev),
             "n_actions": torch.empty(B, dtype=torch.uint8, device=dev),
             "spans": torch.empty(B, 4, dtype=torch.int32, device=dev) if with_spans else None,
             "action_text": None, "action_len": None,
             "err": torch.empty(B, dtype=torch.uint8, device=dev)}
        if action_text_len:
            o["action_text"] = torch.empty(B, K, int(action_text_len), dtype=torch.uint8, device=dev)
            o["action_len"] = torch.empty(B, K, dtype=torch.int32, device=dev)
    check(lib().rmi_detok_parse(_ptr(ids), B, R, _ptr(n_ids), _ptr(vocab.packed), _ptr(vocab.data), vocab.data.numel(),
                                vocab.packed.shape[0], _ptr(o["text"]), stride, _ptr(o["text_len"]),
                                _ptr(o["decode_err"]), ctypes.byref(cfg), _ptr(sel), _ptr(o["actions"]),
                                _ptr(o["n_actions"]), _ptr(o["spans"]), _ptr(o["action_text"]), _ptr(o["action_len"]),
                                int(action_text_len), _ptr(o["err"]), _stream(dev)), "rmi_detok_parse")
    return o



def token_rows_struct(ids: torch.Tensor, vocab: "VocabTable", cfg: _lib.ParseCfg, out: dict,
                      n_ids: Optional[torch.Tensor] = None, sel: Optional[torch.Tensor] = None) -> _lib.TokenRows:
    """rmi_token_rows_t of a token batch and a detok_parse result dict ``out`` (its text, lengths,
    spans and error bytes are written; its actions / n_actions are the turn's, see
    sokoban_token_turn).  The tensors (and cfg) must outlive every launch that uses the struct."""
    _dev(ids, n_ids, sel, vocab.packed, vocab.data)
    _dt(ids, torch.int64, "ids")
    _dt(n_ids, torch.int32, "n_ids")
    _dt(sel, torch.uint8, "sel")
    t = _lib.TokenRows()
    t.ids, t.R, t.n_ids = _ptr(ids), int(ids.shape[1]), _ptr(n_ids)
    t.vocab_packed, t.vocab_bytes = _ptr(vocab.packed), _ptr(vocab.data)
    t.n_bytes, t.V = vocab.data.numel(), vocab.packed.shape[0]
    t.text, t.stride, t.text_len = _ptr(out["text"]), int(out["text"].shape[1]), _ptr(out["text_len"])
    t.decode_err, t.cfg, t.sel = _ptr(out["decode_err"]), ctypes.pointer(cfg), _ptr(sel)
    t.spans, t.parse_err = _ptr(out["spans"]), _ptr(out["err"])
    t._keep = (cfg,)
    return t


def sokoban_token_turn(tok: _lib.TokenRows, env: _lib.Sokoban, ep: EpisodeState, turn: _lib.Turn, obs: _lib.Render,
                       err: Optional[torch.Tensor] = None, fin: Optional[_lib.Finalize] = None,
                       init_state: Optional[torch.Tensor] = None, init_player: Optional[torch.Tensor] = None):
    """One Sokoban turn from the generations' token ids in ONE launch (rmi_sokoban_token_turn):
    detok_parse into tok's buffers with the actions into turn.actions / turn.n_actions, then the
    turn (plain; fin: the rollout's last; init_state / init_player: the first) and the render
    into obs — the outputs of detok_parse followed by sokoban_step_turn_render."""
    _dev(init_state, init_player, err)
    rc = lib().rmi_sokoban_token_turn(ctypes.byref(tok), env, ep.struct(), turn, _ptr(err), fin, _ptr(init_state),
                                      _ptr(init_player), obs, _stream(ep.device))
    if rc == _lib.RMI_EUNSUP and fin is not None:
        # finalize groups that straddle a wave: the token turn, then the finalize
        sokoban_token_turn(tok, env, ep, turn, obs, err)
        seg = torch.arange(0, ep.B + 1, fin.group_size, dtype=torch.int32, device=ep.flags.device)
        check(lib().rmi_rollout_finalize(ep.struct(), _ptr(seg), seg.numel() - 1, fin.method, fin.metrics,
                                         fin.score, fin.pen, fin.norm, _stream(ep.device)), "rmi_rollout_finalize")
        return
    check(rc, "rmi_sokoban_token_turn")

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
    err = torch.empty(B, dtype=torch.uint8, device=dev)
    flags = ((_lib.MS_TURN_SCORES if use_turn_scores else 0) | (_lib.MS_RESPONSE_MASK if enable_response_mask else 0)
             | (_lib.MS_ROLL if roll else 0))
    check(lib().rmi_masks_and_scores(_ptr(ids), B, S, int(special_token), int(reward_token), _ptr(scores.contiguous()),
                                     _ptr(n_scores), T, int(n_slots), flags, _ptr(score), _ptr(lm), _ptr(rm), _ptr(err),
                                     _stream(ids.device)), "rmi_masks_and_scores")
    return score, lm, rm, err


def assemble_batch(tokens: torch.Tensor, row_off: torch.Tensor, S: int, pad_id: int, special_token: int,
                   reward_token: int, scores: torch.Tensor, n_scores: torch.Tensor, n_slots: int, use_turn_scores: bool,
                   enable_response_mask: bool, roll: bool):
    """The formulate_rollouts batch (ctx_manager.py:278-306) from ragged token rows in one pass:
    tokens i64[N] (rows back to back), row_off i64[B+1], S >= the longest row.
    -> (input_ids, attention_mask, position_ids i64[B,S], score f32[B,S-1], loss_mask,
        response_mask bool[B,S-1], err u8[B])."""
    _dev(tokens, row_off, scores, n_scores)
    _dt(tokens, torch.int64, "tokens")
    _dt(row_off, torch.int64, "row_off")
    _dt(scores, torch.float64, "scores")
    _dt(n_scores, torch.int32, "n_scores")
    B = row_off.numel() - 1
    T = scores.shape[0] if scores.dim() == 2 else 0
    if T and scores.shape[1] != B:
        raise ValueError(f"scores must be [T, B={B}], got {tuple(scores.shape)}")
    dev = tokens.device
    So = max(int(S) - 1, 0)
    ids = torch.empty(B, S, dtype=torch.int64, device=dev)
    am = torch.empty_like(ids)
    pos = torch.empty_like(ids)
    score = torch.empty(B, So, dtype=torch.float32, device=dev)
    lm = torch.empty(B, So, dtype=torch.bool, device=dev)
    rm = torch.empty(B, So, dtype=torch.bool, device=dev)
    err = torch.empty(B, dtype=torch.uint8, device=dev)
    flags = ((_lib.MS_TURN_SCORES if use_turn_scores else 0) | (_lib.MS_RESPONSE_MASK if enable_response_mask else 0)
             | (_lib.MS_ROLL if roll else 0))
    check(lib().rmi_assemble_batch(_ptr(tokens), _ptr(row_off), B, int(S), int(pad_id), int(special_token),
                                   int(reward_token), _ptr(scores), _ptr(n_scores), T, int(n_slots), flags, _ptr(ids),
                                   _ptr(am), _ptr(pos), _ptr(score), _ptr(lm), _ptr(rm), _ptr(err), _stream(dev)),
          "rmi_assemble_batch")
    return ids, am, pos, score, lm, rm, err


def assemble_rows(tokens: torch.Tensor, row_start: torch.Tensor, row_len: torch.Tensor, S: int, pad_id: int,
                  special_token: int, reward_token: int, scores: torch.Tensor, n_scores: torch.Tensor, n_slots: int,
                  use_turn_scores: bool, enable_response_mask: bool, roll: bool):
    """assemble_batch with rows tokens[row_start[b] .. + row_len[b]) (the prompt arena)."""
    _dev(tokens, row_start, row_len, scores, n_scores)
    _dt(tokens, torch.int64, "tokens")
    _dt(row_start, torch.int64, "row_start")
    _dt(row_len, torch.int32, "row_len")
    _dt(scores, torch.float64, "scores")
    _dt(n_scores, torch.int32, "n_scores")
    B = row_start.numel()
    T = scores.shape[0] if scores.dim() == 2 else 0
    if T and scores.shape[1] != B:
        raise ValueError(f"scores must be [T, B={B}], got {tuple(scores.shape)}")
    dev = tokens.device
    So = max(int(S) - 1, 0)
    ids = torch.empty(B, S, dtype=torch.int64, device=dev)
    am = torch.empty_like(ids)
    pos = torch.empty_like(ids)
    score = torch.empty(B, So, dtype=torch.float32, device=dev)
    lm = torch.empty(B, So, dtype=torch.bool, device=dev)
    rm = torch.empty(B, So, dtype=torch.bool, device=dev)
    err = torch.empty(B, dtype=torch.uint8, device=dev)
    flags = ((_lib.MS_TURN_SCORES if use_turn_scores else 0) | (_lib.MS_RESPONSE_MASK if enable_response_mask else 0)
             | (_lib.MS_ROLL if roll else 0))
    check(lib().rmi_assemble_rows(_ptr(tokens), _ptr(row_start), _ptr(row_len), B, int(S), int(pad_id),
                                  int(special_token), int(reward_token), _ptr(scores), _ptr(n_scores), T, int(n_slots),
                                  flags, _ptr(ids), _ptr(am), _ptr(pos), _ptr(score), _ptr(lm), _ptr(rm), _ptr(err),
                                  _stream(dev)), "rmi_assemble_rows")
    return ids, am, pos, score, lm, rm, err


def row_counts(mask: torch.Tensor) -> torch.Tensor:
    """i32[B]: the nonzero bytes of each row of a bool / u8 [B, S] mask (rmi_row_counts)."""
    _dev(mask)
    if mask.dtype not in (torch.bool, torch.uint8) or mask.dim() != 2:
        raise ValueError("mask: bool or u8 [B, S]")
    out = torch.empty(mask.shape[0], dtype=torch.int32, device=mask.device)
    check(lib().rmi_row_counts(_ptr(mask), mask.shape[0], mask.shape[1], _ptr(out), _stream(mask.device)),
          "rmi_row_counts")
    return out


def gen_rows(resp: torch.Tensor, src: Optional[torch.Tensor], n_envs: int, vocab_packed: torch.Tensor,
             ids: Optional[torch.Tensor], n_ids: Optional[torch.Tensor], raw_max: torch.Tensor,
             has: Optional[torch.Tensor] = None, raw_next: Optional[torch.Tensor] = None):
    """rmi_gen_rows: the turn's generations onto the env batch (ids / n_ids / has written when
    src is given) and the longest row's raw bytes into raw_max i32[1].  With raw_next
    (rmi_gen_rows_chained): raw_max is 0 already and raw_next is zeroed for the next call."""
    _dev(resp, src, vocab_packed, ids, n_ids, raw_max, has, raw_next)
    _dt(raw_next, torch.int32, "raw_next")
    _dt(has, torch.uint8, "has")
    _dt(resp, torch.int64, "resp")
    _dt(src, torch.int64, "src")
    _dt(ids, torch.int64, "ids")
    _dt(n_ids, torch.int32, "n_ids")
    _dt(raw_max, torch.int32, "raw_max")
    if resp.dim() != 2 or raw_max.numel() < 1:
        raise ValueError("resp must be [n, R] and raw_max hold one int32")
    R = resp.shape[1]
    if src is not None and (src.numel() != n_envs or ids is None or tuple(ids.shape) != (n_envs, R)
                            or (n_ids is not None and n_ids.numel() != n_envs)
                            or (has is not None and has.numel() != n_envs)):
        raise ValueError("src, ids and n_ids must have one row per env")
    if src is None and (resp.shape[0] != n_envs or ids is not None or has is not None):
        raise ValueError("without src resp holds every env's row (and ids is not written)")
    if raw_next is not None:
        if raw_next.numel() < 1 or raw_next.data_ptr() == raw_max.data_ptr():
            raise ValueError("raw_next: one int32 apart from raw_max")
        check(lib().rmi_gen_rows_chained(_ptr(resp), resp.shape[0], R, _ptr(src), int(n_envs), _ptr(vocab_packed),
                                         vocab_packed.shape[0], _ptr(ids), _ptr(n_ids), _ptr(has), _ptr(raw_max),
                                         _ptr(raw_next), _stream(resp.device)),
              "rmi_gen_rows_chained")
        return
    check(lib().rmi_gen_rows(_ptr(resp), resp.shape[0], R, _ptr(src), int(n_envs), _ptr(vocab_packed),
                             vocab_packed.shape[0], _ptr(ids), _ptr(n_ids), _ptr(has), _ptr(raw_max),
                             _stream(resp.device)),
          "rmi_gen_rows")


def pad_rows(arena: torch.Tensor, arena_len: torch.Tensor, rows: torch.Tensor, tail: torch.Tensor, S: int,
             pad_id: int):
    """The left-padded generation batch from arena rows + a common tail (rmi_pad_rows)
    -> (input_ids, attention_mask, position_ids i64[n, S], err u8[n])."""
    _dev(arena, arena_len, rows, tail)
    _dt(arena, torch.int64, "arena")
    _dt(arena_len, torch.int32, "arena_len")
    _dt(rows, torch.int64, "rows")
    _dt(tail, torch.int64, "tail")
    n = rows.numel()
    dev = arena.device
    P = (n * S + 1) & ~1  # one allocation, the outputs at k * P: 16-B aligned alike (column pairs)
    flat = torch.empty(3 * P, dtype=torch.int64, device=dev)
    ids, am, pos = (flat[k * P:k * P + n * S].view(n, S) for k in range(3))
    err = torch.empty(n, dtype=torch.uint8, device=dev)
    check(lib().rmi_pad_rows(_ptr(arena), arena.shape[1], _ptr(arena_len), _ptr(rows), n, _ptr(tail), tail.numel(),
                             int(S), int(pad_id), _ptr(ids), _ptr(am), _ptr(pos), _ptr(err), _stream(dev)),
          "rmi_pad_rows")
    return ids, am, pos, err


# ------------------------------------------------------------------- turn-loop glue
_TORCH_DTYPE = {np.dtype(np.uint8): torch.uint8, np.dtype(np.int8): torch.int8, np.dtype(np.int32): torch.int32,
                np.dtype(np.int64): torch.int64, np.dtype(np.float32): torch.float32,
                np.dtype(np.float64): torch.float64, np.dtype(np.bool_): torch.bool}


class _PinnedRing:
    """Pinned staging for the turn loop's small host -> device copies: consecutive slices of one
    pinned block, freed all at once by the next readback that waits on the (one) stream every
    copy since the last reset went to (d2h); a copy that does not fit goes through torch."""

    def __init__(self, nbytes=1 << 22):
        self.buf = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        self.np = self.buf.numpy()
        self.base = self.buf.data_ptr()
        self.off = 0
        self.stream = None  # the stream of every copy since the last reset (None: none yet)

    def reset_after_sync(self, stream):
        if self.stream is None or self.stream == stream:
            self.off, self.stream = 0, None


_RING = []


def h2d(a: np.ndarray, device) -> torch.Tensor:
    """A host array -> the device through pinned memory, without blocking the host: a slice of
    the pinned ring (_PinnedRing) and one async copy (rmi_upload), or torch's pin_memory path."""
    a = np.ascontiguousarray(a)
    dt = _TORCH_DTYPE.get(a.dtype)
    if not _RING:
        _RING.append(_PinnedRing())
    ring = _RING[0]
    s = _stream(device)
    n = a.nbytes
    if dt is None or n > ring.np.size - ring.off or (ring.stream is not None and ring.stream != s):
        return torch.from_numpy(a).pin_memory().to(device, non_blocking=True)
    o = ring.off
    ring.off = (o + n + 255) & ~255
    ring.stream = s
    ring.np[o:o + n] = a.reshape(-1).view(np.uint8)
    out = torch.empty(a.shape, dtype=dt, device=device)
    check(lib().rmi_upload(out.data_ptr(), ring.base + o, n, s), "rmi_upload")
    return out


D2H_COUNT = [0]  # readbacks through d2h so far (the bench reports them per rollout)
_NP_DTYPE = {torch.uint8: np.uint8, torch.int8: np.int8, torch.int32: np.int32, torch.int64: np.int64,
             torch.float32: np.float32, torch.float64: np.float64, torch.bool: np.bool_}


def d2h(t: torch.Tensor, owner) -> np.ndarray:
    """A small device tensor -> a host numpy copy, through a pinned buffer kept on ``owner``
    (an async copy, then the stream waited on): a pageable ``.cpu()`` stages through the
    runtime's bounce buffer at several times the cost."""
    nbytes = t.numel() * t.element_size()
    buf = getattr(owner, "_pin_buf", None)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8, pin_memory=True)
        owner._pin_buf = buf
    if not t.is_contiguous():
        t = t.contiguous()
    D2H_COUNT[0] += 1
    # one C call: the async copy into the pinned buffer, then the stream waited on
    s = _stream(t.device)
    check(lib().rmi_readback(buf.data_ptr(), t.data_ptr(), nbytes, s), "rmi_readback")
    if _RING:  # every upload enqueued on this stream has run
        _RING[0].reset_after_sync(s)
    return buf[:nbytes].numpy().view(_NP_DTYPE[t.dtype]).copy()


def turn_inputs(has_t: Optional[torch.Tensor], dec_err: torch.Tensor, has: torch.Tensor, err: torch.Tensor):
    """rmi_turn_inputs: has = (has_t or 1) and not dec_err, err = 0 (u8[B] each)."""
    dev = _dev(has_t, dec_err, has, err)
    for t, nm in ((has_t, "has_t"), (dec_err, "dec_err"), (has, "has"), (err, "err")):
        _dt(t, torch.uint8, nm)
    B = dec_err.numel()
    if has.numel() != B or err.numel() != B or (has_t is not None and has_t.numel() != B):
        raise ValueError("has_t, dec_err, has and err must have one entry per env")
    check(lib().rmi_turn_inputs(_ptr(has_t), _ptr(dec_err), B, _ptr(has), _ptr(err), _stream(dev)), "rmi_turn_inputs")


def readback_bytes(B: int) -> int:
    """The size of the turn's packed readback buffer for B envs: rmi_turn_readback's (flags |
    err | dec_err | max text_len, max obs_len), then room for rmi_next_rows_stats' three ints
    (readback_stats), the longest generation's raw bytes (readback_raw) and the count of the
    generation batch's rows rmi_pad_rows flagged (readback_pad), and rmi_turn_readback_pad's
    summary: the OR of the err / dec_err bytes and the count of done envs (readback_summary)."""
    return ((3 * B + 3) & ~3) + 8 + 28


def readback_stats(pack: torch.Tensor, B: int) -> torch.Tensor:
    """The i32[3] of the packed readback buffer that rmi_next_rows_stats writes."""
    o = ((3 * B + 3) & ~3) + 8
    return pack[o:o + 12].view(torch.int32)


def readback_raw(pack: torch.Tensor, B: int) -> torch.Tensor:
    """The i32[1] of the packed readback buffer that carries the turn's longest generation."""
    o = ((3 * B + 3) & ~3) + 20
    return pack[o:o + 4].view(torch.int32)


def readback_pad(pack: torch.Tensor, B: int) -> torch.Tensor:
    """The i32[1] of the packed readback buffer that counts the generation batch's flagged rows."""
    o = ((3 * B + 3) & ~3) + 24
    return pack[o:o + 4].view(torch.int32)


def readback_summary(tail) -> tuple:
    """(OR of the step error bytes, OR of the decode error bytes, count of envs with
    FLAG_DONE) from the host copy of the readback tail (i32 view from its offset on)
    rmi_turn_readback_pad wrote."""
    w = int(tail[7])
    return w & 0xFF, (w >> 8) & 0xFF, int(tail[8])


def count_nonzero_into(x: torch.Tensor, out: torch.Tensor):
    """out i32[1] = the nonzero bytes of the u8 vector x (rmi_row_counts over one row): no
    allocation, no readback of its own."""
    _dev(x, out)
    _dt(x, torch.uint8, "x")
    _dt(out, torch.int32, "out")
    check(lib().rmi_row_counts(_ptr(x), 1, x.numel(), _ptr(out), _stream(out.device)), "rmi_row_counts")


def turn_readback(flags, err, dec_err, num_actions, max_actions, text_len, obs_len, flags_copy, left, pack):
    """rmi_turn_readback: flags_copy = flags, left = max_actions - num_actions, and the packed
    readback (flags | err | dec_err | max text_len, max obs_len) -> pack."""
    dev = _dev(flags, err, dec_err, num_actions, max_actions, text_len, obs_len, flags_copy, left, pack)
    for t, dt, nm in ((flags, torch.uint8, "flags"), (err, torch.uint8, "err"), (dec_err, torch.uint8, "dec_err"),
                      (num_actions, torch.uint8, "num_actions"), (max_actions, torch.int32, "max_actions"),
                      (text_len, torch.int32, "text_len"), (obs_len, torch.int32, "obs_len"),
                      (flags_copy, torch.uint8, "flags_copy"), (left, torch.int32, "left"), (pack, torch.uint8, "pack")):
        _dt(t, dt, nm)
    B = flags.numel()
    for t in (err, dec_err, num_actions, max_actions, text_len, obs_len, flags_copy, left):
        if t is not None and t.numel() != B:
            raise ValueError("every per-env input must have one entry per env")
    if pack.numel() < readback_bytes(B):
        raise ValueError(f"pack needs {readback_bytes(B)} bytes")
    check(lib().rmi_turn_readback(_ptr(flags), _ptr(err), _ptr(dec_err), _ptr(num_actions), _ptr(max_actions),
                                  _ptr(text_len), _ptr(obs_len), B, _ptr(flags_copy), _ptr(left), _ptr(pack),
                                  _stream(dev)), "rmi_turn_readback")


def prompt_commit(bpe_err, text_err, active, mark_tok, len_upd, bad):
    """rmi_prompt_commit: bad = the taking-part rows with an encode or text error; with mark_tok
    len_upd = mark_tok on those rows."""
    dev = _dev(bpe_err, text_err, active, mark_tok, len_upd, bad)
    for t, dt, nm in ((bpe_err, torch.uint8, "bpe_err"), (text_err, torch.uint8, "text_err"),
                      (active, torch.uint8, "active"), (mark_tok, torch.int32, "mark_tok"),
                      (len_upd, torch.int32, "len_upd"), (bad, torch.uint8, "bad")):
        _dt(t, dt, nm)
    B = bad.numel()
    for t in (bpe_err, text_err, active, mark_tok, len_upd):
        if t is not None and t.numel() != B:
            raise ValueError("every input must have one entry per env")
    check(lib().rmi_prompt_commit(_ptr(bpe_err), _ptr(text_err), _ptr(active), _ptr(mark_tok), _ptr(len_upd), B,
                                  _ptr(bad), _stream(dev)), "rmi_prompt_commit")


def prompt_commit_stats(bpe_err, text_err, active, mark_tok, len_upd, bad, length, has, flags, stats):
    """rmi_prompt_commit_stats: prompt_commit, then next_rows_stats over the bad rows it wrote,
    in one launch."""
    dev = _dev(bpe_err, text_err, active, mark_tok, len_upd, bad, length, has, flags, stats)
    for t, dt, nm in ((bpe_err, torch.uint8, "bpe_err"), (text_err, torch.uint8, "text_err"),
                      (active, torch.uint8, "active"), (mark_tok, torch.int32, "mark_tok"),
                      (len_upd, torch.int32, "len_upd"), (bad, torch.uint8, "bad"), (length, torch.int32, "len"),
                      (has, torch.uint8, "has"), (flags, torch.uint8, "flags"), (stats, torch.int32, "stats")):
        _dt(t, dt, nm)
    B = bad.numel()
    for t in (bpe_err, text_err, active, mark_tok, len_upd, length, has, flags):
        if t is not None and t.numel() != B:
            raise ValueError("every input must have one entry per env")
    if stats.numel() < 3:
        raise ValueError("stats: three ints")
    check(lib().rmi_prompt_commit_stats(_ptr(bpe_err), _ptr(text_err), _ptr(active), _ptr(mark_tok), _ptr(len_upd), B,
                                        _ptr(bad), _ptr(length), _ptr(has), _ptr(flags), _ptr(stats), _stream(dev)),
          "rmi_prompt_commit_stats")


def next_rows_stats(length, has, flags, bad, stats):
    """rmi_next_rows_stats: stats i32[3] = (max length over the envs with has (None: every env)
    and flags without FLAG_DONE, any bad, their count)."""
    dev = _dev(length, has, flags, bad, stats)
    _dt(length, torch.int32, "len")
    _dt(has, torch.uint8, "has")
    _dt(flags, torch.uint8, "flags")
    _dt(bad, torch.uint8, "bad")
    _dt(stats, torch.int32, "stats")
    B = length.numel()
    if flags.numel() != B or (has is not None and has.numel() != B) or (bad is not None and bad.numel() != B) \
            or stats.numel() < 3:
        raise ValueError("next_rows_stats: len, has, flags and bad hold one entry per env, stats three ints")
    check(lib().rmi_next_rows_stats(_ptr(length), _ptr(has), _ptr(flags), _ptr(bad), B, _ptr(stats), _stream(dev)),
          "rmi_next_rows_stats")


def rows_stats(length, rows, n_rows: int, bad, stats):
    """rmi_rows_stats: stats i32[2] = (max length[rows], any bad)."""
    dev = _dev(length, rows, bad, stats)
    _dt(length, torch.int32, "len")
    _dt(rows, torch.int64, "rows")
    _dt(bad, torch.uint8, "bad")
    _dt(stats, torch.int32, "stats")
    B = length.numel()
    if (bad is not None and bad.numel() != B) or stats.numel() < 2 or (rows is not None and rows.numel() != n_rows) \
            or (rows is None and n_rows > B):
        raise ValueError("rows_stats: bad holds one entry per env, stats two ints, rows n_rows entries")
    check(lib().rmi_rows_stats(_ptr(length), _ptr(rows), int(n_rows), _ptr(bad), B, _ptr(stats), _stream(dev)),
          "rmi_rows_stats")


# ------------------------------------------------------------------------ advantages
def _mask_u8(mask: torch.Tensor) -> torch.Tensor:
    """A boolean mask as u8 bytes.  The kernels read any nonzero byte as 1 (RAGEN passes a bool
    loss_mask, ctx_manager.py:46-49); a float mask is binarised the same way (nonzero = in)."""
    if mask.dtype == torch.bool:
        return mask.view(torch.uint8)
    if mask.dtype == torch.uint8:
        return mask
    return (mask != 0).to(torch.uint8)


def _rows(r, *others, names=()):
    if r.dim() != 2:
        raise ValueError(f"expected a [B, L] tensor, got shape {tuple(r.shape)}")
    for t, nm in zip(others, names):
        if t is not None and tuple(t.shape) != tuple(r.shape):
            raise ValueError(f"{nm} must have shape {tuple(r.shape)}, got {tuple(t.shape)}")
    return r.shape


def _row_stats(row_stats, B):
    if row_stats is not None:
        _dt(row_stats, torch.float64, "row_stats")
        if tuple(row_stats.shape) != (B, 3):
            raise ValueError(f"row_stats must be f64[{B}, 3], got {tuple(row_stats.shape)}")


def gae(r, v, mask, gamma, lam, variant="legacy", row_stats=None):
    """verl compute_gae_advantage_return before whitening (App. A.4): -> (adv, ret) f32[B, L];
    row_stats f64[B, 3] (optional) receives the per-row whitening partials."""
    if variant not in ("legacy", "masked"):
        raise ValueError(f"GAE variant must be 'legacy' or 'masked', got {variant!r}")
    _dev(r, v, mask, row_stats)
    _dt(r, torch.float32, "token_level_rewards")
    _dt(v, torch.float32, "values")
    B, L = _rows(r, v, mask, names=("values", "response_mask"))
    _row_stats(row_stats, B)
    m = _mask_u8(mask).contiguous()
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    check(lib().rmi_gae(_ptr(r), _ptr(v), _ptr(m), B, L, float(gamma), float(lam), 0 if variant == "legacy" else 1,
                        _ptr(adv), _ptr(ret), _ptr(row_stats), _stream(r.device)), "rmi_gae")
    return adv, ret


def bilevel_gae(r, v, mask, gamma, lam, high_level_gamma, row_stats=None, check_errors=True, err=None):
    """compute_bi_level_gae_advantage_return before whitening (core_algos.py:4-88).  Rows where
    the reference raises IndexError (core_algos.py:79) are flagged in err u8[B]; with
    check_errors the flag is read back (one sync) and raised as IndexError."""
    _dev(r, v, mask, row_stats, err)
    _dt(r, torch.float32, "token_level_rewards")
    _dt(v, torch.float32, "values")
    B, L = _rows(r, v, mask, names=("values", "loss_mask"))
    _row_stats(row_stats, B)
    m = _mask_u8(mask).contiguous()
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    if err is None:
        err = torch.empty(B, dtype=torch.uint8, device=r.device)
    elif err.dtype != torch.uint8 or err.shape != (B,):
        raise ValueError(f"err must be u8[{B}]")
    check(lib().rmi_bilevel_gae(_ptr(r), _ptr(v), _ptr(m), B, L, float(gamma), float(lam), float(high_level_gamma),
                                _ptr(adv), _ptr(ret), _ptr(row_stats), _ptr(err), _stream(r.device)), "rmi_bilevel_gae")
    if check_errors and bool(err.any()):
        raise IndexError("index out of range: last loss-mask position of a row carries no reward "
                         "(reference core_algos.py:79)")
    return adv, ret


WHITEN_OK, WHITEN_EMPTY, WHITEN_ONE = 0, 1, 2


def whiten_status(scratch: torch.Tensor) -> torch.Tensor:
    """The i32 status a whitening launch left in its scratch (device scalar; no sync):
    0 ok, 1 mask sum 0, 2 mask sum 1 (verl's masked_var raises ValueError for 1 and 2)."""
    return scratch[8:12].view(torch.int32)


def raise_whiten_status(code: int):
    if code == WHITEN_EMPTY:
        raise ValueError("At least one element in the mask has to be 1.")
    if code == WHITEN_ONE:
        raise ValueError("The sum of the mask is one, which can cause a division by zero.")


def masked_whiten_(x, mask, row_stats=None):
    """verl masked_whiten in place on x f32[B, L] (mean / unbiased var over the masked elements,
    applied to every element).  row_stats f64[B, 3] from rmi_gae saves the stats pass.
    -> (x, scratch); whiten_status(scratch) holds verl's error cases (no sync here)."""
    _dev(x, mask, row_stats)
    _dt(x, torch.float32, "values")
    B, L = _rows(x, mask, names=("mask",))
    _row_stats(row_stats, B)
    m = _mask_u8(mask).contiguous()
    nbytes = int(lib().rmi_whiten_scratch_bytes(B))
    scratch = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
    check(lib().rmi_masked_whiten(_ptr(x), _ptr(m), B, L, _ptr(row_stats), _ptr(scratch), _stream(x.device)),
          "rmi_masked_whiten")
    return x, scratch


def whiten_row_stats(x, mask, out=None):
    """Per-row fp64 whitening partials (sum, sum_sq, count) of x f32[B, L] over the mask."""
    _dev(x, mask, out)
    _dt(x, torch.float32, "values")
    B, L = _rows(x, mask, names=("mask",))
    out = torch.empty(B, 3, dtype=torch.float64, device=x.device) if out is None else out
    _row_stats(out, B)
    m = _mask_u8(mask).contiguous()
    check(lib().rmi_whiten_row_stats(_ptr(x), _ptr(m), B, L, _ptr(out), _stream(x.device)), "rmi_whiten_row_stats")
    return out


def masked_whiten_stats_(x, stats):
    """masked_whiten of this shard's rows x f32[B, L] with batch statistics from all shards:
    stats f64[n, 3] = every rank's per-row partials in global row order (the multi-GPU form,
    ragen_amd.distributed.global_whiten_stats).  -> (x, scratch) as masked_whiten_."""
    _dev(x, stats)
    _dt(x, torch.float32, "values")
    _dt(stats, torch.float64, "stats")
    if x.dim() != 2 or stats.dim() != 2 or stats.shape[1] != 3:
        raise ValueError("x must be [B, L] and stats [n, 3]")
    B, L = x.shape
    scratch = torch.empty(64, dtype=torch.uint8, device=x.device)
    check(lib().rmi_masked_whiten_stats(_ptr(x), B, L, _ptr(stats), stats.shape[0], _ptr(scratch),
                                        _stream(x.device)), "rmi_masked_whiten_stats")
    return x, scratch


def reinforce_pp_returns(r, mask, gamma, row_stats=None):
    """verl compute_reinforce_plus_plus_outcome_advantage before its whitening: the masked
    discounted returns (adv = ret) -> (adv, ret) f32[B, L]; row_stats f64[B, 3] (optional)
    receives adv's per-row whitening partials."""
    _dev(r, mask, row_stats)
    _dt(r, torch.float32, "token_level_rewards")
    B, L = _rows(r, mask, names=("response_mask",))
    _row_stats(row_stats, B)
    m = _mask_u8(mask).contiguous()
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    check(lib().rmi_reinforce_pp_returns(_ptr(r), _ptr(m), B, L, float(gamma), _ptr(adv), _ptr(ret),
                                         _ptr(row_stats), _stream(r.device)), "rmi_reinforce_pp_returns")
    return adv, ret


def remax(r, mask, baseline):
    """verl compute_remax_outcome_advantage -> (adv, ret) f32[B, L]; baseline f32[B]."""
    _dev(r, mask, baseline)
    _dt(r, torch.float32, "token_level_rewards")
    _dt(baseline, torch.float32, "reward_baselines")
    B, L = _rows(r, mask, names=("response_mask",))
    if baseline.dim() != 1 or baseline.shape[0] != B:
        raise ValueError(f"reward_baselines must be [B={B}], got {tuple(baseline.shape)}")
    m = _mask_u8(mask).contiguous()
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    check(lib().rmi_remax(_ptr(r), _ptr(m), _ptr(baseline), B, L, _ptr(adv), _ptr(ret), _stream(r.device)),
          "rmi_remax")
    return adv, ret


def rloo_outcome(r, mask, seg):
    """verl compute_rloo_outcome_advantage over contiguous row groups seg -> (adv, ret)."""
    _dev(r, mask)
    _dt(r, torch.float32, "token_level_rewards")
    B, L = _rows(r, mask, names=("response_mask",))
    seg = segments(seg, B, r.device)
    if seg.device != r.device:
        raise ValueError("seg must be on the rows' device")
    m = _mask_u8(mask).contiguous()
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    check(lib().rmi_rloo_outcome(_ptr(r), _ptr(m), B, L, _ptr(seg), seg.numel() - 1, _ptr(adv), _ptr(ret),
                                 _stream(r.device)), "rmi_rloo_outcome")
    return adv, ret


def mask_mul_(x, mask):
    """x *= (mask != 0) in place (f32), the `* response_mask` after verl's masked_whiten."""
    _dev(x, mask)
    _dt(x, torch.float32, "values")
    if x.shape != mask.shape:
        raise ValueError(f"mask must match x {tuple(x.shape)}, got {tuple(mask.shape)}")
    m = _mask_u8(mask).contiguous()
    check(lib().rmi_mask_mul(_ptr(x), _ptr(m), x.numel(), _stream(x.device)), "rmi_mask_mul")
    return x


def segments(seg, B: int, device) -> torch.Tensor:
    """Contiguous group segments as i32[G+1] on `device`.  Host segments (list / numpy / CPU
    tensor) are validated (seg[0] == 0, non-decreasing, seg[-1] == B) before the upload; a
    device tensor is taken as is (the kernels never read outside [0, B) either way)."""
    if isinstance(seg, torch.Tensor) and seg.is_cuda:
        _dt(seg, torch.int32, "seg")
        if seg.dim() != 1 or seg.numel() < 1:
            raise ValueError("seg must be a 1-D i32 tensor of G+1 offsets")
        return seg.contiguous()
    h = np.asarray(seg.cpu().numpy() if isinstance(seg, torch.Tensor) else seg, np.int64).reshape(-1)
    if h.size < 1 or h[0] != 0 or h[-1] != B or (np.diff(h) < 0).any():
        raise ValueError(f"seg must be non-decreasing offsets from 0 to B={B}")
    return torch.from_numpy(h.astype(np.int32)).to(device)


def grpo_outcome(r, mask, seg, eps=1e-6, norm_by_std=True):
    """verl compute_grpo_outcome_advantage over contiguous row groups seg (App. A.4)."""
    _dev(r, mask)
    _dt(r, torch.float32, "token_level_rewards")
    B, L = _rows(r, mask, names=("response_mask",))
    seg = segments(seg, B, r.device)
    if seg.device != r.device:
        raise ValueError("seg must be on the rows' device")
    m = _mask_u8(mask).contiguous()
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    check(lib().rmi_grpo_outcome(_ptr(r), _ptr(m), B, L, _ptr(seg), seg.numel() - 1, float(eps), int(norm_by_std),
                                 _ptr(adv), _ptr(ret), _stream(r.device)), "rmi_grpo_outcome")
    return adv, ret
