"""Batched Sokoban (replaces ragen/env/sokoban/env.py + gym_sokoban step, App. A.1)."""
from typing import Optional

import numpy as np
import torch

from .. import _lib, ops
from ..torch_ops import direct, ep_args
from .base import BatchEnv
from .configs import SokobanEnvConfig


class SokobanBatch(BatchEnv):
    env_type = "sokoban"

    def __init__(self, config: SokobanEnvConfig, n_envs, max_turns, max_actions_per_turn, device=None):
        super().__init__(config or SokobanEnvConfig(), n_envs, max_turns, max_actions_per_turn, device)
        H, W = self.config.dim_room
        self.H, self.W = int(H), int(W)
        if self.H * self.W > 64:
            raise NotImplementedError("Sokoban kernel supports rooms of at most 64 cells")
        d = self.device
        B, HW = self.B, self.H * self.W
        self.room_fixed = torch.zeros(B, HW, dtype=torch.uint8, device=d)
        self.room_state = torch.zeros(B, HW, dtype=torch.uint8, device=d)
        self.player = torch.zeros(B, 2, dtype=torch.int8, device=d)
        self.num_env_steps = torch.zeros(B, dtype=torch.uint8, device=d)  # u8 (include/ragen_amd.h)
        self.boxes_on_target = torch.zeros(B, dtype=torch.int8, device=d)  # may go negative (App. A.1)
        # the generated rooms: reset() uploads here once, restore() re-initialises from them
        self.init_state = torch.zeros(B, HW, dtype=torch.uint8, device=d)
        self.init_player = torch.zeros(B, 2, dtype=torch.int8, device=d)
        # the turn kernel's optional board cache (enable_boards; include/ragen_amd.h)
        self.boards = None
        self.init_boards = None  # the reset state's entries (rmi_sokoban_step_turn_first)
        self._boards_valid = False
        self.init_boards_valid = False  # a first turn under BUILD wrote them since the last reset / load

    # 6x6 rooms at one lane per env (the plain turn launch's layout: 4097 <= B < 2^17)
    BOARDS_MIN_B, BOARDS_MAX_B = 4097, 1 << 17

    def enable_boards(self) -> bool:
        """Give the turn launches a board cache: 16 B per env holding each room's bitboards after
        its last turn, so a turn reads one entry instead of the two grid rows and skips their
        decode.  The cache is this batch's: every state write through its methods keeps it
        current or marks it stale (the next turn rebuilds it); a caller that writes room_state /
        room_fixed / player directly must call invalidate_boards().  -> whether the layout
        supports it (6x6 rooms, BOARDS_MIN_B <= B < BOARDS_MAX_B)."""
        if self.H * self.W != 36 or (self.H - 1) * self.W > 32 or not (self.BOARDS_MIN_B <= self.B < self.BOARDS_MAX_B):
            return False
        if self.boards is None:
            self.boards = torch.zeros(self.B, 16, dtype=torch.uint8, device=self.device)
            self.init_boards = torch.zeros(self.B, 16, dtype=torch.uint8, device=self.device)
        self._boards_valid = False
        self.init_boards_valid = False
        return True

    def invalidate_boards(self):
        """The state was written outside the cached turn launches: the next turn rebuilds (and,
        for a write to the reset rows or room_fixed, the next first turn)."""
        self._boards_valid = self.init_boards_valid = False

    def board_struct(self, mode: int) -> _lib.Sokoban:
        """struct() carrying the board cache in `mode` (_lib.BOARDS_BUILD / BOARDS_USE), for
        callers that sequence the turn launches themselves (a captured rollout: BUILD for a turn
        after any other state write, USE after a cached turn)."""
        if self.boards is None:
            raise RuntimeError("enable_boards() first")
        st = self.struct()
        st.boards, st.boards_mode, st.init_boards = self.boards.data_ptr(), int(mode), self.init_boards.data_ptr()
        return st

    def _turn_struct(self):
        """The state struct of a step_turn launch: with the cache when it is enabled (BUILD when
        stale, USE when current); the cache is current after the launch."""
        if self.boards is None:
            return self.struct()
        st = self.board_struct(_lib.BOARDS_USE if self._boards_valid else _lib.BOARDS_BUILD)
        self._boards_valid = True
        return st

    def struct(self) -> _lib.Sokoban:
        c = self.config
        return _lib.Sokoban(self.H, self.W, int(c.num_boxes), int(c.max_steps), self.room_fixed.data_ptr(),
                            self.room_state.data_ptr(), self.player.data_ptr(), self.num_env_steps.data_ptr(),
                            self.boxes_on_target.data_ptr())

    # SokobanEnv.reset (sokoban/env.py:28-42): generate_room under all_seed(seed); on
    # RuntimeError/RuntimeWarning reseed with abs(hash(str(seed))) % 2**32 and retry.
    # (hash() of a str depends on PYTHONHASHSEED — exactly as in the reference process.)
    reseed_fn = staticmethod(lambda s: abs(hash(str(s))) % (2 ** 32))

    @staticmethod
    def _distinct(seeds):
        """-> (distinct seeds, inv).  reset()'s seeds come sorted (seed + group id): no sort."""
        seeds = np.asarray(seeds, np.int64)
        if seeds.size and (seeds[1:] >= seeds[:-1]).all():
            first = np.empty(seeds.size, bool)
            first[0] = True
            np.not_equal(seeds[1:], seeds[:-1], out=first[1:])
            return seeds[first], np.cumsum(first) - 1
        return np.unique(seeds, return_inverse=True)

    @classmethod
    def _finish(cls, uniq, rooms, H, W, num_boxes, search_depth):
        """The generator's output for the distinct seeds -> rows u8[U, 2HW+2] (fixed | state |
        player bytes); a seed the reference would reject is reseeded (sokoban/env.py:41)."""
        fixed, state, player, status = rooms
        for i in np.nonzero(status)[0]:
            s = int(uniq[i])
            for _ in range(64):
                s = cls.reseed_fn(s)
                f, st, p, ok = ops.generate_sokoban_rooms([s], H, W, num_boxes, search_depth, 1)
                if ok[0] == 0:
                    fixed[i], state[i], player[i] = f[0], st[0], p[0]
                    break
            else:
                raise RuntimeError(f"Sokoban generation failed repeatedly for seed {uniq[i]}")
        HW = H * W
        rows = np.empty((len(uniq), 2 * HW + 2), np.uint8)
        rows[:, :HW], rows[:, HW:2 * HW], rows[:, 2 * HW:] = fixed, state, player.view(np.uint8)
        return rows

    @classmethod
    def generate_unique(cls, seeds, H, W, num_boxes, search_depth, n_threads=0):
        """Each distinct seed's room once -> (rows u8[U, 2HW+2] = fixed | state | player bytes,
        inv i64[B]: every env's row)."""
        uniq, inv = cls._distinct(seeds)
        rooms = ops.generate_sokoban_rooms(uniq, H, W, num_boxes, search_depth, n_threads)
        return cls._finish(uniq, rooms, H, W, num_boxes, search_depth), inv

    @classmethod
    def generate(cls, seeds, H, W, num_boxes, search_depth, n_threads=0):
        """-> (fixed u8[B, HW], state u8[B, HW], player i8[B, 2]) for every seed."""
        rows, inv = cls.generate_unique(seeds, H, W, num_boxes, search_depth, n_threads)
        r = np.take(rows, inv, axis=0)
        HW = H * W
        return (np.ascontiguousarray(r[:, :HW]), np.ascontiguousarray(r[:, HW:2 * HW]),
                np.ascontiguousarray(r[:, 2 * HW:]).view(np.int8))

    def prefetch(self, seeds):
        """Start generating the rooms of a later reset(seeds) on a native host thread
        (ops.RoomsJob; one core stays with the caller).  reset() with the same seeds takes them;
        other seeds generate afresh.  Rooms are a pure function of the seed, so the state after
        reset() is the same either way."""
        seeds = np.asarray(seeds, np.int64).copy()
        c = self.config
        uniq, inv = self._distinct(seeds)
        job = ops.RoomsJob(uniq, self.H, self.W, int(c.num_boxes), int(c.search_depth),
                           max(1, ops.host_threads() - 1))
        self._prefetched = (seeds, uniq, inv, job)

    def _rooms(self, seeds):
        """-> generate_unique(seeds): from the prefetch for these seeds if there is one."""
        c = self.config
        dims = (self.H, self.W, int(c.num_boxes), int(c.search_depth))
        pf, self._prefetched = getattr(self, "_prefetched", None), None
        self.reset_prefetched = False  # (whether the last reset took prefetched rooms)
        if pf is not None:
            pseeds, uniq, inv, job = pf
            if pseeds.shape == seeds.shape and np.array_equal(pseeds, seeds):
                rows = self._finish(uniq, job.wait(), *dims)
                self.reset_prefetched = True
                return rows, inv
            try:
                job.wait()  # not taken (its error, if any, with it)
            except ValueError:
                pass
        return self.generate_unique(seeds, *dims)

    def reset(self, seeds):
        self.seeds = np.asarray(seeds, np.int64).copy()
        rows, inv = self._rooms(self.seeds)
        # the distinct rooms and every env's row in them uploaded (pinned); one launch expands
        # them and resets (rmi_sokoban_load_rooms)
        room_of = None if len(rows) == self.B and np.array_equal(inv, np.arange(self.B)) else \
            ops.h2d(inv.astype(np.int32), self.device)
        ops.sokoban_load_rooms(self.struct(), self.ep, ops.h2d(rows, self.device), room_of, self.init_state,
                               self.init_player)
        self._boards_valid = self.init_boards_valid = False
        self._invalidate()

    def load_state(self, fixed, state, player):
        B, HW = self.B, self.H * self.W
        buf = np.empty((B, 2 * HW + 2), np.uint8)
        buf[:, :HW] = np.asarray(fixed).reshape(B, HW)
        buf[:, HW:2 * HW] = np.asarray(state).reshape(B, HW)
        buf[:, 2 * HW:] = np.asarray(player, np.int8).reshape(B, 2).view(np.uint8)
        self._load_rows(ops.h2d(buf, self.device))

    def _load_rows(self, d):
        """d u8[B, 2HW+2] on the device: [fixed | state | player] per env."""
        HW = self.H * self.W
        self.init_boards_valid = False
        self.room_fixed.copy_(d[:, :HW])
        self.init_state.copy_(d[:, HW:2 * HW])
        self.init_player.copy_(d[:, 2 * HW:].view(torch.int8))
        self.restore()

    # ---- the custom ops (torch.ops.ragen_amd.*) over this batch's tensors
    def state_args(self):
        """Tensor arguments of the Sokoban ops: the env SoA then the episode record."""
        return (self.room_fixed, self.room_state, self.player, self.num_env_steps, self.boxes_on_target) + \
            ep_args(self.ep)

    def dims(self):
        c = self.config
        return self.H, self.W, int(c.num_boxes), int(c.max_steps)

    def restore(self):
        """Back to the post-reset state of the last reset() (one fused launch)."""
        torch.ops.ragen_amd.sokoban_reset(*self.state_args(), self.init_state, self.init_player, *self.dims())
        self._boards_valid = False
        self._invalidate()

    # step_turn(render=True) renders every env's next observation in the same launch
    # (rmi_sokoban_step_turn_render); render_rows() then returns those rows without a launch
    fused_render = True

    def step_turn(self, turn, actions, n_actions, has_input, max_actions_per_traj, format_penalty, err=None,
                  render=False, **kw):
        if render and self.dispatch != "ctypes":
            H, W = self.H, self.W
            rows = ops.render_buffers(self.B, H, W, self.device)  # fresh: turn records keep each turn's rows
            direct.sokoban_step_turn_render(*self.state_args(), actions, n_actions, has_input, err, *rows,
                                            *self.glyph_lists(), int(turn), int(max_actions_per_traj),
                                            float(format_penalty), *self.dims())
            self._boards_valid = False  # (the render-fused turn keeps no cache)
            self._invalidate()
            self._rows = rows
            return
        if self.dispatch == "ctypes" or self.boards is not None:
            ops._dev(self.room_state, actions, n_actions, has_input, err)
            ops.sokoban_step_turn(self._turn_struct(), self.ep, ops.turn_struct(int(turn), actions, n_actions, has_input,
                                                                          int(max_actions_per_traj),
                                                                          float(format_penalty)), err)
        else:
            direct.sokoban_step_turn(*self.state_args(), actions, n_actions, has_input, err, int(turn),
                                                  int(max_actions_per_traj), float(format_penalty), *self.dims())
        self._invalidate()

    def render_rows(self):
        """SokobanEnv.render text mode (sokoban/env.py:53-61) of every env on the device:
        -> (UTF-8 rows u8[B, stride], lengths i32[B]) -- the rows the last step_turn(render=True)
        wrote, while the state has not changed since."""
        rows = self.__dict__.get("_rows")
        if rows is not None:
            return rows
        return direct.sokoban_render(self.room_fixed, self.room_state, self.H, self.W,
                                                  *self.glyph_lists())

    def obs_bound(self) -> int:
        """The longest render row (bytes) of a room with this config's box count: every cell a
        wall / floor / target glyph but the boxes' and the player's, plus the newlines (a
        hand-made room past it is built on the host by the device prompt path)."""
        g = self.config.grid_lookup or {}
        L = [len(str(g.get(c, "?")).encode("utf-8")) for c in range(7)]
        nb = max(0, min(int(self.config.num_boxes), self.H * self.W - 1))
        base = max(L[0], L[1], L[2])
        return (self.H * self.W - nb - 1) * base + nb * max(base, L[3], L[4]) + max(base, L[5], L[6]) + self.H - 1

    def render_all(self):
        if self._text is None:
            self._text = ops.decode_rows(*self.render_rows())
        return self._text
