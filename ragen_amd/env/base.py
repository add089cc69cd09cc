"""Batched env plugin API.

The reference registers one Python object per env (ragen/env/base.py:5-73,
ragen/env/__init__.py:15-31).  Here one *batch* object owns the device SoA state of every
env of a tag; its ``step_turn`` runs one whole EnvStateManager turn for all of them in a
single HIP launch.  Per-env views (``render``, ``action_lookup``) keep the reference's
observable API for the Python facade (llm_agent/es_manager.py).
"""
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import ops


class BatchEnv:
    env_type = "base"
    # how a turn reaches the C ABI: "op" = the torch custom operator (torch.ops.ragen_amd.*,
    # dispatcher + schema checks), "ctypes" = the C entry point straight through ops (the
    # bench reports the facade both ways)
    dispatch = "op"

    def __init__(self, config, n_envs: int, max_turns: int, max_actions_per_turn: int, device=None):
        self.config = config
        self.B = int(n_envs)
        self.T = int(max_turns)
        self.K = int(max_actions_per_turn)
        self.device = torch.device(device if device is not None else "cuda")
        self.ep = ops.EpisodeState.empty(self.B, self.T, self.device)
        self.seeds = np.zeros(self.B, np.int64)
        self._host = None  # lazily synced host mirror (env-specific use)
        self._text = None  # this turn's observations, rendered on the device for every env at once
        self._rows = None

    # --- API ----------------------------------------------------------------------
    def reset(self, seeds) -> None:
        raise NotImplementedError

    def prefetch(self, seeds) -> None:
        """Hint: a later reset(seeds) will follow.  Envs whose reset does host work may start it
        in the background; the state reset() produces must not depend on whether it did."""

    def step_turn(self, turn: int, actions: torch.Tensor, n_actions: torch.Tensor, has_input: Optional[torch.Tensor],
                  max_actions_per_traj: int, format_penalty: float, err: Optional[torch.Tensor] = None,
                  **kw) -> None:
        raise NotImplementedError

    def render(self, i: int) -> str:
        return self.render_all()[i]

    def render_all(self) -> List[str]:
        """Observation text of every env, cached until the state changes."""
        raise NotImplementedError

    def action_lookup(self, i: int) -> Optional[Dict[int, str]]:
        return getattr(self.config, "action_lookup", None)

    def map_actions(self, i: int, actions: List[str]) -> List[int]:
        """Positional ids for es_manager._extract_map_valid_actions (es_manager.py:230-240):
        case-insensitive exact match against action_lookup; 0 = unknown (dropped by the kernel)."""
        lookup = self.action_lookup(i)
        rev = {v.lower(): k for k, v in lookup.items()}
        return [rev.get(a.lower(), 0) for a in actions]

    def map_actions_many(self, rows: List[int], actions: List[List[str]]) -> List[List[int]]:
        """map_actions for many envs of one turn; the reverse table is built once per lookup.
        With one lookup for every env (action_lookup not overridden) equal action lists map
        once: envs with the same actions share one (read-only) id list."""
        if type(self).action_lookup is BatchEnv.action_lookup:
            lookup = self.action_lookup(0)
            rev = {v.lower(): k for k, v in lookup.items()}
            memo = {}
            out = []
            for acts in actions:
                key = tuple(acts)
                ids = memo.get(key)
                if ids is None:
                    ids = memo[key] = [rev.get(a.lower(), 0) for a in acts]
                out.append(ids)
            return out
        revs = {}
        out = []
        for i, acts in zip(rows, actions):
            lookup = self.action_lookup(i)
            rev = revs.get(id(lookup))
            if rev is None:
                rev = revs[id(lookup)] = {v.lower(): k for k, v in lookup.items()}
            out.append([rev.get(a.lower(), 0) for a in acts])
        return out

    def get_all_actions(self):
        return list(self.action_lookup(0).keys())

    def parse_setup(self, enable_think: bool, action_sep: str, prepend: bool = True):
        """Device parse configuration of this env type (ops.parse_config) for the
        response -> action-id kernel: -> (rmi_parse_cfg_t, sel u8[B] | None, action-text bytes)."""
        from .. import ops
        return ops.parse_config(enable_think, self.K, action_sep, self.action_lookup(0), prepend=prepend), None, 0

    def glyph_lists(self):
        """config.grid_lookup as the render ops' glyph lists (ops.glyph_table), built once."""
        g = self.__dict__.get("_glyph_lists")
        if g is None:
            from .. import ops
            gb, gl = ops.glyph_table(self.config.grid_lookup)
            g = self._glyph_lists = (gb.tolist(), gl.tolist())
        return g

    def parse_sel(self):
        """The per-env lookup column of parse_setup (the part that changes with the episodes);
        the configuration itself depends on the arguments only."""
        return None

    def close(self):
        self._host = None
        self._text = None
        self._rows = None

    # --- helpers ------------------------------------------------------------------
    def _invalidate(self):
        self._host = None
        self._text = None
        self._rows = None  # device rows of a fused turn + render (SokobanBatch)

    def expand_seeds(self, base_seed: int, group_size: int, first_group: int = 0) -> np.ndarray:
        """es_manager.py:80-82: env i of the batch gets base + (global group index)."""
        g = first_group + np.arange(self.B) // group_size
        return (int(base_seed) + g).astype(np.int64)
