"""Batched FrozenLake (replaces ragen/env/frozen_lake/env.py + gymnasium FrozenLakeEnv, App. A.2)."""
import numpy as np
import torch

from .. import _lib, ops
from ..torch_ops import ep_args
from .base import BatchEnv
from .configs import FrozenLakeEnvConfig



def _is_valid(board, max_size):  # frozen_lake/utils.py:6-22
    frontier, discovered = [], set()
    sr, sc = np.where(np.array(board) == "S")
    frontier.append((sr[0], sc[0]))
    while frontier:
        r, c = frontier.pop()
        if (r, c) not in discovered:
            discovered.add((r, c))
            for dr, dc in [(1, 0), (0, 1), (-1, 0), (0, -1)]:
                rn, cn = r + dr, c + dc
                if 0 <= rn < max_size and 0 <= cn < max_size:
                    if board[rn][cn] == "G":
                        return True
                    if board[rn][cn] != "H":
                        frontier.append((rn, cn))
    return False


def generate_random_map(size=8, p=0.8, seed=None):
    """frozen_lake/utils.py:25-47 (numpy Generator seeded like gymnasium seeding.np_random)."""
    rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
    while True:
        board = rng.choice(["F", "H"], (size, size), p=[p, 1 - p])
        start_r, start_c = rng.integers(size, size=2)
        goal_r, goal_c = rng.integers(size, size=2)
        if (start_r, start_c) != (goal_r, goal_c):
            board[start_r][start_c], board[goal_r][goal_c] = "S", "G"
            if _is_valid(board, size):
                break
    return ["".join(row) for row in board]


def slippery_cumsum(success_rate: float):
    """np.cumsum of the probabilities gymnasium lists for [(a-1)%4, a, (a+1)%4]."""
    other = (1.0 - success_rate) / 2.0
    return tuple(float(x) for x in np.cumsum([other, success_rate, other]))


class FrozenLakeBatch(BatchEnv):
    env_type = "frozen_lake"

    def __init__(self, config: FrozenLakeEnvConfig, n_envs, max_turns, max_actions_per_turn, device=None):
        super().__init__(config or FrozenLakeEnvConfig(), n_envs, max_turns, max_actions_per_turn, device)
        n = int(self.config.size)
        self.nrow = self.ncol = n
        if n * n > 64:
            raise NotImplementedError("FrozenLake kernel supports maps of at most 64 cells")
        d = self.device
        self.desc = torch.zeros(self.B, n * n, dtype=torch.uint8, device=d)
        self.s = torch.zeros(self.B, dtype=torch.int32, device=d)
        self.rng = torch.zeros(4, self.B, dtype=torch.int64, device=d)  # u64 bit patterns
        self.init_desc, self.init_s, self.init_rng = (torch.zeros_like(x) for x in (self.desc, self.s, self.rng))
        self.cs = slippery_cumsum(self.config.success_rate)

    def struct(self):
        return _lib.FrozenLake(self.nrow, self.ncol, int(bool(self.config.is_slippery)), self.cs[0], self.cs[1],
                               self.cs[2], self.desc.data_ptr(), self.s.data_ptr(), self.rng.data_ptr())

    # FrozenLakeEnv.reset (frozen_lake/env.py:28-37): map from seed (host, once per distinct
    # seed), env RNG reseeded with the same seed and one draw for the initial-state
    # categorical_sample (device, rmi_pcg64_seed).
    @staticmethod
    def reset_maps(seeds, size, p):
        seeds = np.asarray(seeds, np.int64)
        uniq, inv = np.unique(seeds, return_inverse=True)
        desc = np.zeros((len(uniq), size * size), np.uint8)
        s0 = np.zeros(len(uniq), np.int32)
        for i, sd in enumerate(uniq):
            m = generate_random_map(size=size, p=p, seed=int(sd))
            flat = "".join(m).encode()
            desc[i] = np.frombuffer(flat, np.uint8)
            s0[i] = flat.index(b"S")
        return desc[inv], s0[inv]

    def reset(self, seeds):
        self.seeds = np.asarray(seeds, np.int64).copy()
        desc, s0 = self.reset_maps(self.seeds, self.nrow, float(self.config.p))
        self.init_desc.copy_(torch.from_numpy(np.ascontiguousarray(desc)))
        self.init_s.copy_(torch.from_numpy(np.ascontiguousarray(s0, dtype=np.int32)))
        rng, _ = torch.ops.ragen_amd.pcg64_seed(torch.from_numpy(self.seeds).to(self.device), 1)
        self.init_rng.copy_(rng)
        self.restore()

    def load_state(self, desc, s0, rng):
        self.init_desc.copy_(torch.from_numpy(np.ascontiguousarray(desc)))
        self.init_s.copy_(torch.from_numpy(np.ascontiguousarray(s0, dtype=np.int32)))
        self.init_rng.copy_(torch.from_numpy(np.ascontiguousarray(rng).view(np.int64)))
        self.restore()

    # ---- the custom ops (torch.ops.ragen_amd.*) over this batch's tensors
    def state_args(self):
        return (self.desc, self.s, self.rng) + ep_args(self.ep)

    def dims(self):
        return self.nrow, self.ncol, bool(self.config.is_slippery), self.cs[0], self.cs[1], self.cs[2]

    def restore(self):
        """Back to the post-reset state of the last reset() (one fused launch)."""
        torch.ops.ragen_amd.frozenlake_reset(*self.state_args(), self.init_desc, self.init_s, self.init_rng,
                                             *self.dims())
        self._invalidate()

    def step_turn(self, turn, actions, n_actions, has_input, max_actions_per_traj, format_penalty, err=None, **kw):
        torch.ops.ragen_amd.frozenlake_step_turn(*self.state_args(), actions, n_actions, has_input, err, int(turn),
                                                 int(max_actions_per_traj), float(format_penalty), *self.dims())
        self._invalidate()

    def render_rows(self):
        """FrozenLakeEnv.render text mode (frozen_lake/env.py:47-61) of every env on the device."""
        return torch.ops.ragen_amd.frozenlake_render(self.desc, self.s, self.nrow, self.ncol, *self.glyph_lists())

    def obs_bound(self) -> int:
        """The longest render row (bytes): one player cell (codes 0 / 4 / 5), the other cells
        floor / hole / goal (1 / 2 / 3), plus the newlines."""
        g = self.config.grid_lookup or {}
        L = [len(str(g.get(c, "?")).encode("utf-8")) for c in range(6)]
        return (self.nrow * self.ncol - 1) * max(L[1], L[2], L[3]) + max(L) + self.nrow - 1

    def render_all(self):
        if self._text is None:
            self._text = ops.decode_rows(*self.render_rows())
        return self._text
