"""EnvStateManager — drop-in for ragen/llm_agent/es_manager.py:28-258 on the GPU engine.

Same constructor, ``reset(seed) -> rollout_cache``, ``step(all_env_inputs) -> env_outputs``,
``get_rollout_states()``, ``render()`` and ``close()``, same dict shapes.  All env state
lives in device SoA tensors owned by one batch object per tag; ``step`` maps the parsed
action strings to ids on the host (es_manager.py:230-240), runs ONE kernel launch per tag
for the whole turn, then reads back four small per-env vectors to build the dicts.

``step_tensor`` is the dict-free fast path (used by the benchmark's kernel variant).

Sharding: with ``rank`` / ``world_size`` (or a ``process_group``) the manager
owns the contiguous, group-aligned shard ``ragen_amd.distributed.shard_groups`` gives this
rank; env ids, group ids and seeds stay GLOBAL (seed + global env id // group_size,
es_manager.py:80-82), so a rank's envs are bit-identical to the same envs of a one-process
run.  The train seed drawn by ``random.randint`` (es_manager.py:88-89) is broadcast from rank
0 over the process group; without a group a sharded manager needs the seed passed in.
``rollout_cache`` holds this shard's envs in env order (``env_lo`` = global id of the first).
"""
import functools
import gc
import os
import random
import time
import warnings
from collections.abc import Sequence
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import _lib, ops
from .. import distributed as rd
from ..env import REGISTERED_ENV_CONFIGS, REGISTERED_ENVS
from ..env.base import BatchEnv
from ..torch_ops import direct, ep_args, parse_cfg_words


@dataclass
class EnvStatus:
    """Status of an environment (es_manager.py:17-24), materialised from the device record."""
    truncated: bool = False
    terminated: bool = False
    num_actions: int = 0
    rewards: List[float] = field(default_factory=list)
    seed: Optional[int] = None


STEP_STAMPS = None  # a list: _step_device appends (label, perf_counter) checkpoints (tools/prof_chain_stamps.py)


class LazyEnvOutputs:
    """What ``step`` returns on the device path: the rollout-cache entries of the envs still
    active after the turn, in input order (es_manager.py:168-169).  ``len()`` and ``env_ids``
    are known right away (one small device -> host copy per turn); the history dicts are
    materialised from the device record on first access."""

    def __init__(self, es, env_ids):
        self._es = es
        self.env_ids = np.asarray(env_ids, np.int64)

    def __len__(self):
        return len(self.env_ids)

    def __getitem__(self, k):
        self._es._materialize()
        rc, lo = self._es.rollout_cache, self._es.env_lo
        if isinstance(k, slice):
            return [rc[int(g) - lo] for g in self.env_ids[k]]
        return rc[int(self.env_ids[k]) - lo]

    def __iter__(self):
        rc, lo = self._es.rollout_cache, self._es.env_lo
        return iter([rc[int(g) - lo] for g in self.env_ids])


class LazyRolloutStates(Sequence):
    """get_rollout_states() on the device path: the rollout cache with its metrics, built on
    first element access (host parse of the generations, history dicts, per-env metrics).
    ContextManager.formulate_rollouts reads the device record instead and never builds them."""

    def __init__(self, es):
        self.es = es
        self.rollout_id = es.rollout_id
        self.env_ids = es.env_lo + np.arange(es.n_envs, dtype=np.int64)

    def _full(self):
        return self.es.rollout_cache

    def __len__(self):
        return self.es.n_envs

    def __getitem__(self, k):
        return self._full()[k]

    def __iter__(self):
        return iter(self._full())

    def __eq__(self, other):
        return list(self._full()) == list(other)


class _Tag:
    """One env tag of this shard = one contiguous GLOBAL env range [lo, hi) = one batch object."""

    def __init__(self, tag, lo, hi, batch, max_actions_per_traj, env_type):
        self.tag, self.lo, self.hi, self.batch = tag, lo, hi, batch
        self.max_actions_per_traj = int(max_actions_per_traj)
        self.env_type = env_type


def _make_env_config(env_type, env_config):
    cls = REGISTERED_ENV_CONFIGS[env_type]
    if env_config is None:
        return cls()
    return cls(**dict(env_config))


def shard_plan(n_groups_per_tag, group_size, rank, world_size):
    """Group-aligned shard of rank r: -> (first global group, n local groups, [(tag index,
    global env lo, global env hi)] of the tags it intersects).  Pure host logic."""
    G = sum(n_groups_per_tag)
    g0, ng = rd.shard_groups(G, world_size, rank)
    out, cur = [], 0
    for j, n in enumerate(n_groups_per_tag):
        lo, hi = max(cur, g0), min(cur + n, g0 + ng)
        if hi > lo:
            out.append((j, lo * group_size, hi * group_size))
        cur += n
    return g0, ng, out


def shard_sizes(n_groups_per_tag, tags, group_size, world_size, tag=None):
    """Every rank's env count (of ``tag``'s envs if given) under shard_plan, in rank order:
    host-known, so the collectives over the shards need no size exchange."""
    out = []
    for r in range(world_size):
        _, ng, parts = shard_plan(list(n_groups_per_tag), group_size, r, world_size)
        out.append(ng * group_size if tag is None else sum(hi - lo for j, lo, hi in parts if tags[j] == tag))
    return out


def _gc_paused(fn):
    """Run ``fn`` with Python's cyclic collector paused.  The host bookkeeping allocates tens of
    thousands of dicts and lists per turn (history entries, rollout-cache entries), none of them
    cyclic garbage; with a large heap in the process (a trainer's, or the bench's inputs) the
    collections those allocations trigger scanned the whole heap — ≈35 ms of a 8192-env turn's
    bookkeeping on the box, whether the loop ran in Python or in C.  The collector's state is
    restored afterwards; it runs again at its next threshold."""
    @functools.wraps(fn)
    def run(*a, **kw):
        was = gc.isenabled()
        gc.disable()
        try:
            return fn(*a, **kw)
        finally:
            if was:
                gc.enable()
    return run


_BOOK_CONSTS = (_lib.FLAG_TERMINATED, _lib.FLAG_TRUNCATED, _lib.FLAG_DONE, _lib.INFO_PRESENT, _lib.INFO_EFFECTIVE,
                _lib.INFO_VALID, _lib.INFO_SUCCESS)
_HOSTBOOK = []


def _hostbook():
    """The dict facade's bookkeeping extension (ragen_amd/_build/_hostbook*.so, built with the
    library); None when it was not built (the Python definition then runs, with a warning)."""
    if not _HOSTBOOK:
        import importlib.util
        from ..build import hostbook_path
        path = hostbook_path()
        mod = None
        if os.path.exists(path):
            spec = importlib.util.spec_from_file_location("_hostbook", path)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
        else:
            warnings.warn(f"{path} not built: the dict facade's bookkeeping runs in Python", RuntimeWarning)
        _HOSTBOOK.append(mod)
    return _HOSTBOOK[0]


class EnvStateManager:
    # after a rollout from a drawn train seed, prefetch_next() starts the next reset's host
    # work (Sokoban room generation) in the background, for the seed random will draw next
    prefetch_resets = True

    def __init__(self, config, mode: str = "train", device=None, rank: Optional[int] = None,
                 world_size: Optional[int] = None, process_group=None):
        self.sys_config = config
        self.mode = mode
        self.config = getattr(self.sys_config.es_manager, mode)
        self.env_groups = int(self.config.env_groups)
        self.group_size = int(self.config.group_size)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.process_group = process_group
        if process_group is not None:
            import torch.distributed as dist
            rank, world_size = dist.get_rank(process_group), dist.get_world_size(process_group)
        self.rank, self.world_size = int(rank or 0), int(world_size or 1)
        ap = self.sys_config.agent_proxy
        self.max_turn = int(ap.max_turn)
        self.K = int(ap.max_actions_per_turn)
        self.format_penalty = float(self.sys_config.es_manager.format_penalty)
        self._init_envs()
        self._rc = None
        self._reset_pending = False  # reset() ran, its rollout-cache dicts not built yet
        self._reset_rows = None
        # set by a ContextManager on the device path (set_device_vocab / attach_env_manager):
        # reset() then returns LazyEnvOutputs and builds the per-env dicts only when read
        self.lazy_outputs = False
        self._states_pending = False  # a LazyRolloutStates was handed out and not built yet
        self._formulated = False      # the device formulate_rollouts ran: drop the last states when built
        self._untrimmed = None
        self.rollout_id = 0
        self._ids_in_order = None  # the env-id array reset() handed out (all envs, in order)
        self._live_ids = None      # the env-id array the last turn handed out (its envs not done)
        self._turn = 0
        self._all_active = False
        self.reset_render = None
        # the device prompt builder whose next prompt a device turn appends before its readback
        # (prompts.DevicePrompts.advance_eager; set by the ContextManager), or None
        self._prompt_hook = None
        self._turn_records = []  # device-path turns (ContextManager's device prompts read them too)
        self._max_act = None  # i32[n_envs] max_actions_per_traj per env (device turn), built once
        self._mat_upto = 0       # records whose host bookkeeping is done

    def _init_envs(self):
        n_groups = list(self.config.env_configs.n_groups)
        tags = list(self.config.env_configs.tags)
        assert sum(n_groups) == self.env_groups, \
            f"Sum of n_groups must equal env_groups. Got sum({n_groups}) != {self.env_groups}"
        assert len(tags) == len(n_groups), \
            f"Number of tags must equal number of n_groups. Got {len(tags)} != {len(n_groups)}"
        g0, ng, parts = shard_plan(n_groups, self.group_size, self.rank, self.world_size)
        self.first_group, self.n_local_groups = g0, ng
        self.env_lo = g0 * self.group_size
        self.n_envs = ng * self.group_size
        self.tags: List[_Tag] = []
        for j, lo, hi in parts:
            tag = tags[j]
            cfg_t = self.sys_config.custom_envs[tag]
            env_type = cfg_t.env_type
            env_config = _make_env_config(env_type, cfg_t.get("env_config"))
            batch = REGISTERED_ENVS[env_type](env_config, hi - lo, self.max_turn, self.K, self.device)
            self.tags.append(_Tag(tag, lo, hi, batch, cfg_t.max_actions_per_traj, env_type))
        self._tag_of = np.zeros(self.n_envs, np.int32)
        for j, t in enumerate(self.tags):
            self._tag_of[t.lo - self.env_lo:t.hi - self.env_lo] = j
        # reference-shaped entries (es_manager.py:69-70); 'env' is the batch, 'local' its row
        self.envs = [{"tag": t.tag, "group_id": i // self.group_size, "env_id": i, "env": t.batch,
                      "local": i - t.lo, "config": t.batch.config, "status": EnvStatus(),
                      "max_actions_per_traj": t.max_actions_per_traj}
                     for t in self.tags for i in range(t.lo, t.hi)]

    def shard_sizes(self, tag: Optional[str] = None) -> List[int]:
        """Every rank's env count (of ``tag``'s envs if given), rank order (shard_sizes)."""
        return shard_sizes(self.config.env_configs.n_groups, self.config.env_configs.tags, self.group_size,
                           self.world_size, tag)

    @property
    def rollout_cache(self):
        """es_manager.py:85's rollout cache (this shard's envs): device-path turns and lazily
        handed-out rollout states are built into the dicts before it is read."""
        self._materialize()
        if self._states_pending:
            self._rollout_states_host()
        if self._formulated:  # formulate_rollouts dropped each history's last state (ctx_manager.py:236-237)
            self._formulated = False
            self._untrimmed = [c["history"] for c in self._rc]
            k = getattr(self, "_formulated_window", None)
            for cache in self._rc:
                if "state" in cache["history"][-1]:
                    cache["history"] = cache["history"][:-1]
                if k:  # and kept only the last max_context_window entries (ctx_manager.py:244-246)
                    cache["history"] = cache["history"][-k:]
        return self._rc

    # ---------------------------------------------------------------------- reset
    def _train_seed(self, seed):
        if seed is not None:
            return int(seed)
        if self.process_group is not None:
            import torch.distributed as dist
            box = [random.randint(0, 1000000) if self.rank == 0 else None]
            dist.broadcast_object_list(box, src=dist.get_global_rank(self.process_group, 0), group=self.process_group)
            return int(box[0])
        if self.world_size > 1:
            raise ValueError("a sharded EnvStateManager without a process group needs reset(seed=...) so that every "
                             "rank uses the same train seed")
        return random.randint(0, 1000000)

    def prefetch_next(self):
        """Start the next reset()'s host work (Sokoban room generation, on native host threads)
        for the train seed ``random`` will draw next, peeked without drawing it (its state is
        put back).  LLMAgentProxy.rollout calls it when the rollout is done, so the generation
        runs while the trainer updates the policy; the next reset() takes the rooms when its
        seeds match, and generates afresh when ``random`` was drawn from in between."""
        if not (self.prefetch_resets and getattr(self, "_seed_drawn", False)):
            return
        st = random.getstate()
        seed = random.randint(0, 1000000)
        random.setstate(st)
        nxt = seed + (self.env_lo + np.arange(self.n_envs)) // self.group_size
        for t in self.tags:
            t.batch.prefetch(nxt[t.lo - self.env_lo:t.hi - self.env_lo])

    def reset(self, seed: Optional[int] = None):
        """es_manager.py:75-103."""
        drawn = self.mode == "train" and seed is None and self.process_group is None
        seed = self._train_seed(seed) if self.mode == "train" else 123
        gids = self.env_lo + np.arange(self.n_envs)
        seeds = seed + gids // self.group_size  # _expand_seed, global ids
        for t in self.tags:
            t.batch.reset(seeds[t.lo - self.env_lo:t.hi - self.env_lo])
        self._seed_drawn = drawn  # (prefetch_next: the next reset draws its seed too)
        self._turn = 0
        self._turn_records = []
        self._mat_upto = 0
        self.rollout_id += 1
        self._seeds = seeds
        self._next_rows = self._asc_ids = None  # (a turn's device row list, turn_chain)
        self._live_ids = None  # the env ids the last turn handed out (its envs not done)
        self._states_pending = False
        self._formulated = False
        self._untrimmed = None
        self._rc = None
        self._reset_pending = True
        self._all_active = True  # every env may step (has_input = None) until a turn says otherwise
        if self.lazy_outputs:  # the device path reads env ids; the dicts wait for a reader
            # the initial observations rendered now, on the device (decoded when read; the
            # device prompts' first turn reads them too: reset_render)
            self._reset_rows = {j: tg.batch.render_rows() for j, tg in enumerate(self.tags)
                                if type(tg.batch).render is BatchEnv.render}
            self.reset_render = (self.rollout_id, self._reset_rows)
            self._ids_in_order = self._live_ids = self.env_lo + np.arange(self.n_envs, dtype=np.int64)
            return LazyEnvOutputs(self, self._ids_in_order)
        self._reset_rows = None
        self._reset_cache()
        return self._rc

    @_gc_paused
    def _reset_cache(self):
        """The rollout cache reset() hands out (es_manager.py:92-103): per env its EnvStatus and
        a history holding the initial observation; built once, when first read."""
        if not self._reset_pending:
            return
        self._reset_pending = False
        seeds = self._seeds
        self._rc = [{"env_id": e["env_id"], "history": [], "group_id": e["group_id"], "tag": e["tag"],
                     "penalty": 0} for e in self.envs]
        from .. import ops
        if self._reset_rows is not None:  # rendered at reset (the envs may have stepped since)
            obs = {j: ops.decode_rows(*rows) for j, rows in self._reset_rows.items()}
            self._reset_rows = None
        else:
            obs = {j: tg.batch.render_all() for j, tg in enumerate(self.tags) if type(tg.batch).render is BatchEnv.render}
        seeds_l, tag_l = seeds.tolist(), self._tag_of.tolist()  # python ints, one conversion
        for k, (e, cache) in enumerate(zip(self.envs, self._rc)):
            e["status"] = EnvStatus(seed=seeds_l[k])
            j = tag_l[k]
            state = obs[j][e["local"]] if j in obs else e["env"].render(e["local"])
            cache["history"] = self._update_cache_history(cache["history"], state, e["max_actions_per_traj"], None)

    # ----------------------------------------------------------------------- step
    @_gc_paused
    def step(self, all_env_inputs: List[Dict]):
        """es_manager.py:105-171: one kernel launch per tag for the whole turn.  Given the device
        form of the inputs (ContextManager.get_env_inputs on the device path) the turn runs
        without host round trips (``_step_device``)."""
        from .ctx_manager import DeviceEnvInputs
        if isinstance(all_env_inputs, DeviceEnvInputs):
            return self._step_device(all_env_inputs)
        self._materialize()
        if self._turn >= self.max_turn:
            raise RuntimeError(f"more than agent_proxy.max_turn={self.max_turn} turns in one rollout")
        self._all_active = False
        t = self._turn
        lo0 = self.env_lo
        gids_all = [int(inp["env_id"]) for inp in all_env_inputs]
        if len(self.tags) == 1:
            per_tag = {0: (all_env_inputs, gids_all)}
        else:
            per_tag = {j: ([], []) for j in range(len(self.tags))}
            tag_of = self._tag_of
            for inp, g in zip(all_env_inputs, gids_all):
                ins, gs = per_tag[int(tag_of[g - lo0])]
                ins.append(inp)
                gs.append(g)
        still_active = set()
        for j, tg in enumerate(self.tags):
            inputs, gids = per_tag[j]
            if not inputs:
                continue
            B, lo, K = tg.hi - tg.lo, tg.lo, self.K
            rows = [g - lo for g in gids]
            acts_l = [list(inp["actions"]) for inp in inputs]
            lens = [len(a) for a in acts_l]
            if max(lens) > K:
                k = lens.index(max(lens))
                raise ValueError(f"env {gids[k]}: {lens[k]} actions > max_actions_per_turn={K}")
            m_l = tg.batch.map_actions_many(rows, acts_l)
            # the turn's inputs as arrays: one scatter for every env's ids
            ids = np.zeros((B, K), np.int8)
            n = np.zeros(B, np.uint8)
            has = np.zeros(B, np.uint8)
            r = np.asarray(rows, np.int64)
            ln = np.asarray(lens, np.int64)
            n[r] = ln
            has[r] = 1
            if ln.sum():
                starts = np.repeat(np.cumsum(ln) - ln, ln)
                cols = np.arange(int(ln.sum())) - starts
                ids[np.repeat(r, ln), cols] = [x for m in m_l for x in m]
            is_cd = tg.env_type == "countdown"
            dev = self.device
            # one host -> device copy of the turn's inputs
            packed = torch.from_numpy(np.concatenate([ids.view(np.uint8).reshape(-1), n, has])).to(dev)
            ids_t = packed[:B * K].view(torch.int8).view(B, K)
            n_t, has_t = packed[B * K:B * K + B], packed[B * K + B:]
            kw = {}
            if is_cd:
                answers = [[] for _ in range(B)]
                for i, a in zip(rows, acts_l):
                    answers[i] = a
                buf, alens = tg.batch.encode_answers(answers)
                kw = {"answers": torch.from_numpy(buf).to(dev), "answer_len": torch.from_numpy(alens).to(dev)}
            err = torch.zeros(B, dtype=torch.uint8, device=dev)
            tg.batch.step_turn(t, ids_t, n_t, has_t, tg.max_actions_per_traj, self.format_penalty, err, **kw)
            ep = tg.batch.ep
            # one device -> host copy: flags, counters, info, exec count, error bits (as bytes)
            # and the turn reward / penalty (f64)
            host = torch.stack([ep.flags, ep.num_actions, ep.turn_info[t], ep.turn_exec[t], err]).cpu().numpy()
            f64 = torch.stack([ep.turn_reward[t], ep.penalty]).cpu().numpy()
            self._raise_errors(tg, host[4], rows, gids)
            # one host copy per turn, as Python lists (numpy scalar indexing per env is slower)
            flags, num_actions, info, n_exec = (x.tolist() for x in host[:4])
            # the text observation of every env at once unless the env type renders per env
            obs = tg.batch.render_all() if type(tg.batch).render is BatchEnv.render else None
            still_active |= self._book(tg, t, inputs, gids, rows, acts_l, m_l, flags, num_actions, info, n_exec,
                                       f64[0].tolist(), f64[1].tolist(), obs)
        self._turn += 1
        # only not-done envs go back for generation, in input order (es_manager.py:168-169)
        rc = self._rc
        return [rc[g - lo0] for g in gids_all if g in still_active]

    def _book(self, tg, t, inputs, gids, rows, acts_l, m_l, flags, num_actions, info, n_exec, rw, pen, obs):
        """The host side of one turn for one tag (es_manager.py:130-169), in the CPython extension
        csrc/hostbook.c: exactly _book_py (the definition; tests/test_hostbook.py compares the
        two).  -> the global ids of the envs still active."""
        hb = _hostbook()
        if hb is None:
            return self._book_py(tg, t, inputs, gids, rows, acts_l, m_l, flags, num_actions, info, n_exec, rw, pen, obs)
        return hb.book(int(t), inputs, gids, rows, acts_l, m_l, flags, num_actions, info, n_exec, rw, pen, obs,
                       self.envs, self._rc, int(self.env_lo), tg.env_type == "countdown",
                       getattr(tg.batch, "note_executed", None), tg.batch.render, _BOOK_CONSTS)

    def _book_py(self, tg, t, inputs, gids, rows, acts_l, m_l, flags, num_actions, info, n_exec, rw, pen, obs):
        """The host side of one turn for one tag (es_manager.py:130-169): EnvStatus, penalty and the
        history entries of the stepped envs, from the turn's device results (lists indexed by the
        tag-local row).  -> the global ids of the envs still active."""
        F_TERM, F_TRUNC, F_DONE = _lib.FLAG_TERMINATED, _lib.FLAG_TRUNCATED, _lib.FLAG_DONE
        I_PRES, I_EFF, I_VAL, I_SUCC = _lib.INFO_PRESENT, _lib.INFO_EFFECTIVE, _lib.INFO_VALID, _lib.INFO_SUCCESS
        is_cd = tg.env_type == "countdown"
        note = getattr(tg.batch, "note_executed", None)
        render = tg.batch.render
        envs, rcache, lo0 = self.envs, self._rc, self.env_lo
        still_active = set()
        for inp, gid, i, acts, m in zip(inputs, gids, rows, acts_l, m_l):
            entry, cache = envs[gid - lo0], rcache[gid - lo0]
            ne = n_exec[i]
            executed = (acts if is_cd else [a for a in m if a != 0])[:ne]
            if note is not None:
                note(t, i, executed)
            acc = rw[i] if ne else 0
            if is_cd and ne and acc in (0.0, 1.0):
                acc = int(acc)  # compute_reward returns int 0 / int score (countdown/env.py:73-78)
            inf = info[i]
            if inf & I_PRES:
                turn_info = {"action_is_effective": bool(inf & I_EFF), "action_is_valid": bool(inf & I_VAL),
                             "success": bool(inf & I_SUCC)}
            else:
                turn_info = {}
            st = entry["status"]
            na = num_actions[i]
            st.num_actions = na
            st.rewards.append(acc)
            fl = flags[i]
            st.terminated = bool(fl & F_TERM)
            st.truncated = bool(fl & F_TRUNC)
            if pen[i] != 0:
                cache["penalty"] = pen[i]
            hist = cache["history"]
            h = hist[-1]
            h["actions"] = executed
            h["reward"] = acc
            h["info"] = turn_info
            h["llm_response"] = inp["llm_response"]
            h["llm_raw_response"] = inp["llm_raw_response"]
            hist.append({"state": obs[i] if obs is not None else render(i),
                         "actions_left": entry["max_actions_per_traj"] - na})
            if not (fl & F_DONE):
                still_active.add(gid)
        return still_active

    def _raise_errors(self, tg, err, rows, gids):
        """Per-env error bits of the turn launch, as the reference would surface them: an action
        id outside the env's space is the AssertionError of bandit/env.py:63, a grid index numpy
        rejects is gym_sokoban's IndexError.  (The kernel leaves such an env untouched; the
        reference raises inside its per-env loop.)  A Countdown answer outside the evaluator's
        grammar was scored 'not correct' (DESIGN §5 deviation 4): counted and warned about."""
        if not err.any():
            return
        bad = [(g, int(err[i])) for i, g in zip(rows, gids) if err[i]]
        if any(e & _lib.ERR_ACTION for _, e in bad):
            raise AssertionError(f"env {next(g for g, e in bad if e & _lib.ERR_ACTION)}: invalid action")
        if any(e & (_lib.ERR_INDEX | _lib.ERR_STATE) for _, e in bad):
            raise IndexError(f"env {next(g for g, e in bad if e & (_lib.ERR_INDEX | _lib.ERR_STATE))}: "
                             "index out of range in the env step")
        n_unsup = sum(1 for _, e in bad if e & _lib.ERR_UNSUP)
        if n_unsup:
            tg.batch.unsupported_answers = getattr(tg.batch, "unsupported_answers", 0) + n_unsup
            warnings.warn(f"{n_unsup} Countdown answers outside the device evaluator's grammar were scored as not "
                          "correct (ragen_amd DESIGN §5, deviation 4)", RuntimeWarning)

    def step_tensor(self, actions: torch.Tensor, n_actions: torch.Tensor, has_input: Optional[torch.Tensor] = None,
                    tag_index: int = 0, **kw):
        """Dict-free turn on the device (kernel variant): ids i8[B,K] of one tag batch."""
        tg = self.tags[tag_index]
        self._all_active = False  # the active set is the caller's from here on
        tg.batch.step_turn(self._turn, actions, n_actions, has_input, tg.max_actions_per_traj, self.format_penalty,
                           **kw)
        self._turn += 1
        return tg.batch.ep

    def step_text(self, text: torch.Tensor, text_len: torch.Tensor, has_input: Optional[torch.Tensor] = None,
                  enable_think: bool = True, action_sep: str = "||", prepend: bool = True,
                  err: Optional[torch.Tensor] = None, render: bool = False):
        """Device-resident turn from response text (§8(f) rank 2): rows are this shard's envs in
        env-id order, text u8[n_envs, stride] / text_len i32[n_envs] the decoded generations
        (e.g. ops.detokenize of the response ids).  Per tag one parse launch
        (_parse_response + _extract_map_valid_actions, ctx_manager.py:148-173,
        es_manager.py:230-240) feeds one turn launch; nothing returns to the host.
        -> list of per-tag parse outputs (ops.parse_actions dicts)."""
        if self._turn >= self.max_turn:
            raise RuntimeError(f"more than agent_proxy.max_turn={self.max_turn} turns in one rollout")
        if text.shape[0] != self.n_envs or text_len.shape[0] != self.n_envs:
            raise ValueError(f"text rows must cover all {self.n_envs} envs")
        outs = []
        lo0 = self.env_lo
        for tg in self.tags:
            a, z = tg.lo - lo0, tg.hi - lo0
            cfg, sel, lact = self._parse_args(tg, enable_think, action_sep, prepend)
            acts, n_act, spans, at, al, perr = torch.ops.ragen_amd.parse_actions(
                cfg, text[a:z], text_len[a:z], sel, True, int(lact))
            outs.append({"actions": acts, "n_actions": n_act, "spans": spans, "action_text": at if lact else None,
                         "action_len": al if lact else None, "err": perr})
        self._parsed_turn(outs, has_input, err, render)
        return outs

    def _parse_args(self, tg, enable_think, action_sep, prepend):
        """tg.batch.parse_setup as the parse ops take it (cfg words, sel, action-text bytes); the
        configuration is built once per argument set, the per-env column read every turn."""
        cache = tg.batch.__dict__.setdefault("_parse_cache", {})
        key = (bool(enable_think), action_sep, bool(prepend))
        if key not in cache:
            cfg, _, lact = tg.batch.parse_setup(enable_think, action_sep, prepend)
            cache[key] = (parse_cfg_words(cfg), int(lact))
        words, lact = cache[key]
        return words, tg.batch.parse_sel(), lact

    def _parsed_turn(self, parsed, has_input, err, render=False):
        """One turn launch per tag from the tag's parse outputs (ops.parse_actions dicts); with
        ``render`` a batch that can renders its next observations in the same launch
        (SokobanBatch.fused_render: render_rows() then reads them)."""
        self._all_active = False  # _step_device sets it again from the turn's active set
        lo0 = self.env_lo
        for tg, p in zip(self.tags, parsed):
            a, z = tg.lo - lo0, tg.hi - lo0
            has = None if has_input is None else has_input[a:z]
            kw = {}
            if p["action_text"] is not None:
                kw = {"answers": p["action_text"], "answer_len": p["action_len"]}
            if render and getattr(tg.batch, "fused_render", False):
                kw["render"] = True
            tg.batch.step_turn(self._turn, p["actions"], p["n_actions"], has, tg.max_actions_per_traj,
                               self.format_penalty, None if err is None else err[a:z], **kw)
        self._turn += 1

    def _decode_parse(self, inp, enable_think, action_sep):
        """The device decode of the turn's generations fused with each tag's parse
        (rmi_detok_parse, one launch per tag): -> per-tag parse dicts; the decoded rows go into
        ``inp`` (the prompts and the history read them)."""
        v = inp.vocab
        lo0 = self.env_lo
        outs, texts, lens, derrs = [], [], [], []
        for tg in self.tags:
            a, z = tg.lo - lo0, tg.hi - lo0
            cfg, sel, lact = self._parse_args(tg, enable_think, action_sep, True)
            text, tlen, derr, acts, n_act, spans, at, al, perr = direct.detok_parse(
                inp.ids[a:z], None if inp.n_ids is None else inp.n_ids[a:z], v.packed, v.data, inp.stride, cfg, sel, True, int(lact))
            outs.append({"actions": acts, "n_actions": n_act, "spans": spans, "action_text": at if lact else None,
                         "action_len": al if lact else None, "err": perr})
            texts.append(text)
            lens.append(tlen)
            derrs.append(derr)
        inp.set_decoded(self._cat(texts), self._cat(lens), self._cat(derrs))
        return outs

    def _cat(self, xs):
        return xs[0] if len(xs) == 1 else torch.cat(xs)

    def _step_device(self, inp):
        """One turn from the decoded generations on the device: parse + turn per tag (step_text),
        the next observation rendered on the device, the active set read back.  The host
        bookkeeping (EnvStatus, history dicts, penalties) is deferred to ``_materialize``; the
        turn's record (inputs, spans, observation, flags, actions left) is kept for it and for
        the device prompt path (prompts.DevicePrompts.advance).  ONE readback per turn: the
        decode's row size comes from a hint (ContextManager._device_env_inputs), and a
        generation longer than it is masked out of this pass and stepped by a second pass over
        those envs, sized from the lengths the first pass read back (rare: the hint keeps a
        margin over every length seen)."""
        if self._turn >= self.max_turn:
            raise RuntimeError(f"more than agent_proxy.max_turn={self.max_turn} turns in one rollout")
        t = self._turn
        n = self.n_envs
        # the whole turn in one call into the library where it applies (turn_chain.py), else
        # launch by launch; either way one device -> host copy (pinned, then the stream waited
        # on): the active set and the turn's per-env error bits, raised in the step where they
        # happen, as the reference raises inside its per-env loop
        chain = self._turn_chain()
        res = chain.run(inp, t) if chain is not None else None
        slot = None
        if res is not None:
            rec, host, slot = res
            hook, eager = self._prompt_hook, True
        else:
            if inp.pad_counted:  # the generation batch's left-cut rows, counted into this readback
                ops.count_nonzero_into(inp.pad_err, ops.readback_pad(inp.pack, n))
            rec, pack, hook, eager = self._device_pass(inp, t, None)
            host = ops.d2h(pack, self)
        asc = self._ascending(inp.env_ids)
        _cp = STEP_STAMPS.append if STEP_STAMPS is not None else None  # (diagnostic checkpoints)
        self._next_rows = None
        o = (3 * n + 3) & ~3
        # max text / obs, the next batch's stats, raw max, pad count (and from the chain: the
        # OR of the error bytes, the done count -- the numpy passes below skipped when clean)
        tail = host[o:o + 36].view(np.int32)
        if getattr(inp, "pad_counted", False) and tail[6]:
            raise RuntimeError(f"{int(tail[6])} rows of this turn's generation batch were longer than its width "
                               "(rmi_pad_rows RMI_ERR_UNSUP): the actor was given left-cut prompts")
        if inp.raw_max is None:
            inp.ctx.note_raw(int(tail[5]))
        if _cp:
            _cp(("t1", time.perf_counter()))
        summ = ops.readback_summary(tail) if slot is not None else None
        err_h = host[n:2 * n]
        dec_h = host[2 * n:3 * n]
        if summ is None or summ[1]:
            over = ((dec_h & _lib.ERR_UNSUP) != 0) & ((dec_h & _lib.ERR_INDEX) == 0)
        else:
            over = None
        if over is not None and over.any() and inp.raw_max is None and not (dec_h & _lib.ERR_INDEX).any():
            slot = summ = None  # (the chain's row list and summary count the first pass only)
            err_h = err_h.copy()
            if self._prompt_hook is not None:  # (this pass appends more rows: the batch is built later)
                self._prompt_hook._eager_pad = None
            # the second pass: every row decoded again at the size the lengths ask for (the
            # rows of the first pass decode and parse the same), only the overflowed envs step
            from .ctx_manager import decode_stride
            raw = int(tail[5])
            over_t = ops.h2d(over.astype(np.uint8), self.device)
            inp2 = type(inp)(inp.ctx, inp.env_ids, over_t, inp.ids, inp.n_ids, decode_stride(raw, 3))
            inp2.raw_max, inp2.raw_dev = raw, inp.raw_dev
            self._turn = t
            rec2, pack2, hook, eager2 = self._device_pass(inp2, t, rec)
            host = ops.d2h(pack2, self)
            tail = host[o:o + 36].view(np.int32)
            err_h |= host[n:2 * n]
            dec_h = host[2 * n:3 * n]
            eager = eager and eager2
            rec = rec2
        if _cp:
            _cp(("t2", time.perf_counter()))
        rec["text_max"], rec["obs_max"] = int(tail[0]), (int(tail[1]) if rec.pop("_obs_known") else None)
        self._turn_records.append(rec)
        n_in = len(inp.env_ids)
        fl_h = host[:n]
        if (summ[1] if summ is not None else dec_h.any()):
            bad = int(np.nonzero(dec_h)[0][0])
            raise ValueError(f"env {self.env_lo + bad}: the decoded generation exceeded the device row buffer or held "
                             "an id outside the vocabulary (rmi_detokenize RMI_ERR_UNSUP); its env was not stepped")
        if summ is not None and asc and inp.env_ids is self._live_ids:
            # the envs outside this turn's ids were all done before it (the ids are the last
            # turn's survivors, ascending): the inputs that go on are the envs not done
            all_still = summ[2] == n - n_in
            if not all_still:  # the survivors' ids from the flags in one C pass (rmi_host_live_ids)
                still = None
                out_local = np.empty(n - summ[2], np.int64)
                # (the flags from the chain's pinned buffer: the same bytes as fl_h, pointer at hand)
                k = _lib.lib().rmi_host_live_ids(self._chain.host_p, n, _lib.FLAG_DONE, self.env_lo,
                                                 out_local.ctypes.data, out_local.size)
                if k != out_local.size:
                    raise RuntimeError(f"the turn's done count ({summ[2]}) disagrees with its flags")
        else:
            if inp.env_ids is self._ids_in_order:  # every env, in order (no gather)
                still = (fl_h & _lib.FLAG_DONE) == 0
            else:
                still = (fl_h[inp.env_ids - self.env_lo] & _lib.FLAG_DONE) == 0
            all_still = bool(still.all())
        if _cp:
            _cp(("t3", time.perf_counter()))
        self._all_active = n_in == self.n_envs and all_still
        if all_still:
            out_ids = inp.env_ids
        elif still is None:
            out_ids = out_local  # (env_lo added by rmi_host_live_ids)
        else:
            out_ids = inp.env_ids[still]
        self._live_ids = out_ids
        if _cp:
            _cp(("t4", time.perf_counter()))
        if eager:  # the next batch's stats, valid for exactly the env-id array handed out below
            hook.set_next_stats(t, tail[2:5], out_ids)
        if slot is not None and asc:  # the chain listed these envs (ascending) on the device
            self._next_rows = (out_ids, slot.next_rows, slot.next_src)
            self._asc_ids = out_ids
        if (summ[0] if summ is not None else err_h.any()):
            err_h = err_h.copy()
            for tg in self.tags:
                gids = [int(g) for g in inp.env_ids if tg.lo <= g < tg.hi]
                self._raise_errors(tg, err_h[tg.lo - self.env_lo:tg.hi - self.env_lo], [g - tg.lo for g in gids],
                                   gids)
            self._turn_records[-1]["err_seen"] = True
        if _cp:
            _cp(("t5", time.perf_counter()))
        return LazyEnvOutputs(self, out_ids)

    use_turn_chain = True  # (tests compare the chained turn with the step-by-step one)

    def _turn_chain(self):
        """The turn chain of this manager and its device prompts (turn_chain.TurnChain), built
        on first use; None where it does not apply."""
        hook = self._prompt_hook
        if not self.use_turn_chain or hook is None:
            return None
        ch = self.__dict__.get("_chain")
        if ch is None or ch.pr is not hook:
            from .turn_chain import TurnChain
            ch = self._chain = TurnChain(self, hook.ctx, hook) if TurnChain.applies(self, hook) else None
        return ch

    def _ascending(self, ids) -> bool:
        """Whether a turn's env ids are strictly ascending (the order the chain lists the next
        batch's rows in): reset's ids and the ids a chained turn handed out are, by construction."""
        if ids is self._ids_in_order or ids is self.__dict__.get("_asc_ids"):
            return True
        return ids.size < 2 or bool((ids[1:] > ids[:-1]).all())

    def _device_pass(self, inp, t, first):
        """The device launches of one pass of turn t over the envs with a generation in ``inp``
        (all of them, or inp.has_t) that decode: decode + parse, the turn with its render, the
        record's columns and the packed readback buffer (rmi_turn_readback, then the next
        prompt's append and the next batch's stats, DevicePrompts.advance_eager).  ``first``:
        the record of the turn's first pass when this is its second (the overflowed envs):
        the record returned then covers both.  -> (record, readback buffer, prompt hook,
        whether the hook appended)."""
        dev = self.device
        n = self.n_envs
        ap = self.sys_config.agent_proxy
        # decode + parse in one launch per tag unless the rows were decoded already
        parsed = None if inp.is_decoded else self._decode_parse(inp, bool(ap.enable_think), ap.action_sep)
        # a generation the device decode truncated (row stride) or could not decode (an id
        # outside the vocabulary) is not stepped on: masked out of the turn on the device and
        # handled after it, from the turn's readback (no host synchronisation before the turn)
        # the envs with a generation (all of them, or has_t written by rmi_gen_rows) minus the
        # undecodable ones, and the zeroed step-error bytes: one launch (rmi_turn_inputs)
        has = torch.empty(n, dtype=torch.uint8, device=dev)
        err = torch.empty(n, dtype=torch.uint8, device=dev)
        ops.turn_inputs(inp.has_t, inp.err, has, err)
        if parsed is None:
            parsed = self.step_text(inp.text, inp.text_len, has, bool(ap.enable_think), ap.action_sep, True, err=err,
                                    render=True)
        else:
            self._parsed_turn(parsed, has, err, render=True)
        obs = {j: tg.batch.render_rows() for j, tg in enumerate(self.tags) if type(tg.batch).render is BatchEnv.render}
        flags = self._cat([tg.batch.ep.flags for tg in self.tags])
        num_actions = self._cat([tg.batch.ep.num_actions for tg in self.tags])
        obs_len = self._cat([obs[j][1] for j in sorted(obs)]) if len(obs) == len(self.tags) else None
        if self._max_act is None:  # per-env max_actions_per_traj (the "actions left" base)
            self._max_act = torch.tensor(np.concatenate([np.full(tg.hi - tg.lo, tg.max_actions_per_traj, np.int32)
                                                         for tg in self.tags]), device=dev)
        flags_copy = torch.empty(n, dtype=torch.uint8, device=dev)
        left = torch.empty(n, dtype=torch.int32, device=dev)
        pack = getattr(inp, "pack", None) if first is None else None  # (rmi_gen_rows wrote the raw max there)
        if pack is None:
            pack = torch.empty(ops.readback_bytes(n), dtype=torch.uint8, device=dev)
        # the record's flags and actions-left columns, and the one packed readback: flags, step
        # and decode errors, the longest decoded response and observation (rmi_turn_readback)
        ops.turn_readback(flags, err, inp.err, num_actions, self._max_act, inp.text_len, obs_len, flags_copy, left,
                          pack)
        raw_v = ops.readback_raw(pack, n)
        if inp.raw_max is None and inp.raw_dev.data_ptr() != raw_v.data_ptr():
            raw_v.copy_(inp.raw_dev)  # the longest generation's raw bytes ride along (the next hint)
        rec = {"turn": t, "inp": inp, "has": has, "err": err, "obs": obs, "spans": [p["spans"] for p in parsed],
               "flags": flags_copy, "left": left, "_obs_known": obs_len is not None}
        has_next = has
        if first is not None:  # the second pass: this pass's envs and the first's
            has_next = has | first["has"]
        # with device prompts the next prompt's text and ids are appended by this turn's own
        # launches, and the next generation batch's row stats land in the readback buffer
        # (DevicePrompts.advance_eager): the turn's one readback serves the prompt batch too
        hook = self._prompt_hook
        eager = hook is not None and hook.advance_eager(rec, ops.readback_stats(pack, n), has_next=has_next,
                                                        again=first is not None)
        if first is not None:
            rec["has"], rec["err"] = has_next, err | first["err"]
        return rec, pack, hook, eager

    @_gc_paused
    def _materialize(self):
        """The host side of the pending device-path turns, in turn order: exactly what ``step``
        records per turn (``_book``), from the device record — the per-turn rewards / info /
        executed counts, the final flags and penalties, num_actions as the running sum of the
        executed counts — plus the host parse of each decoded generation for the history
        strings (llm_response, llm_raw_response, the executed action names)."""
        self._reset_cache()
        if self._mat_upto >= len(self._turn_records):
            return
        from .. import ops
        from .ctx_manager import parse_response_spans
        turns = self._turn_records[self._mat_upto:]
        self._mat_upto = len(self._turn_records)
        ap = self.sys_config.agent_proxy
        prefix = "<think>" if ap.enable_think else "<answer>"
        rec = []
        for tg in self.tags:
            ep = tg.batch.ep
            rec.append((ep.turn_reward.cpu().numpy(), ep.turn_info.cpu().numpy(), ep.turn_exec.cpu().numpy(),
                        ep.flags.cpu().numpy(), ep.penalty.cpu().numpy()))
        lo0 = self.env_lo
        for d in turns:
            t, inp = d["turn"], d["inp"]
            texts = inp.decoded()
            err = d["err"].cpu().numpy()
            for j, tg in enumerate(self.tags):
                gids = [int(g) for g in inp.env_ids if tg.lo <= g < tg.hi]
                if not gids:
                    continue
                rows = [g - tg.lo for g in gids]
                raws = [prefix + texts[g - lo0] for g in gids]
                spans = d["spans"][j].cpu().numpy()  # the device parse's regex match, per tag row
                parsed = [parse_response_spans(r, spans[i], bool(ap.enable_think), ap.action_sep, self.K)
                          for r, i in zip(raws, rows)]
                inputs = [{"llm_response": lr, "llm_raw_response": raw} for (lr, _), raw in zip(parsed, raws)]
                acts_l = [a for _, a in parsed]
                m_l = tg.batch.map_actions_many(rows, acts_l)
                if not d.get("err_seen"):
                    self._raise_errors(tg, err[tg.lo - lo0:tg.hi - lo0], rows, gids)
                tr, ti, te, fl, pen = rec[j]
                num_actions = te[:t + 1].astype(np.int64).sum(0)
                obs = ops.decode_rows(*d["obs"][j]) if j in d["obs"] else None
                self._book(tg, t, inputs, gids, rows, acts_l, m_l, fl.tolist(), num_actions.tolist(), ti[t].tolist(),
                           te[t].tolist(), tr[t].tolist(), pen.tolist(), obs)

    # ------------------------------------------------------- get_rollout_states
    def metric_arrays(self, extra: Optional[torch.Tensor] = None):
        """Per-env rollout metrics of this shard from the device record, one copy for every tag:
        -> list of (tag, m f64[B_tag, 4] = success, num_actions, action_is_effective mean,
        action_is_valid mean, custom bool[B_tag] = some turn carried an info dict,
        info u8[T_seen, B_tag]).  extra (u8 on the device, or a list of them; optional): read back
        in the same copy -> (list, extra's host bytes, concatenated)."""
        T = min(self._turn, self.max_turn)
        extras = [] if extra is None else [x.reshape(-1) for x in (extra if isinstance(extra, (list, tuple)) else [extra])]
        n_extra = sum(x.numel() for x in extras)
        parts, shapes = list(extras), []
        for tg in self.tags:
            ep = tg.batch.ep
            m = direct.rollout_metrics(*ep_args(ep))
            info = ep.turn_info[:T]
            parts += [m.view(torch.uint8).reshape(-1), info.reshape(-1)]
            shapes.append((tg, m.shape, m.numel() * 8, info.numel()))
        flat = parts[0] if len(parts) == 1 else torch.cat(parts)
        host = ops.d2h(flat, self)
        o = n_extra
        out = []
        for tg, mshape, nm, ni in shapes:
            mh = host[o:o + nm].view(np.float64).reshape(mshape)
            ih = host[o + nm:o + nm + ni].reshape(T, -1)
            o += nm + ni
            custom = (ih & _lib.INFO_PRESENT).any(0) if T else np.zeros(mh.shape[0], bool)
            out.append((tg.tag, mh, custom, ih))
        return out if extra is None else (out, host[:n_extra])

    def get_rollout_states(self):
        """es_manager.py:173-207.  On the device path (turns taken from device token ids) the
        states are lazy (LazyRolloutStates): ContextManager.formulate_rollouts reads the device
        record, and the dicts are built only when a caller reads them."""
        if self._turn_records:
            self._states_pending = True
            return LazyRolloutStates(self)
        return self._rollout_states_host()

    @_gc_paused
    def _rollout_states_host(self):
        """The per-env metrics dicts (es_manager.py:180-205) from one device -> host copy per
        tag; the per-env lists are built from whole-array numpy results."""
        self._materialize()
        self._states_pending = False
        eff_k, val_k = "action_is_effective", "action_is_valid"
        for tg, (tag, m, custom, info) in zip(self.tags, self.metric_arrays()):  # one entry per config entry
            succ = m[:, 0].tolist()
            na = m[:, 1].astype(np.int64).tolist()
            eff, val = m[:, 2].tolist(), m[:, 3].tolist()
            present = (info & _lib.INFO_PRESENT) != 0
            eff_b = ((info & _lib.INFO_EFFECTIVE) != 0).T.tolist()
            val_b = ((info & _lib.INFO_VALID) != 0).T.tolist()
            pres = present.T.tolist()
            cust = custom.tolist()
            k_s, k_n, k_e, k_v = f"{tag}/success", f"{tag}/num_actions", f"{tag}/{eff_k}", f"{tag}/{val_k}"
            base = tg.lo - self.env_lo
            for i in range(tg.hi - tg.lo):
                cache = self._rc[base + i]
                metrics = {k_s: succ[i], k_n: na[i]}
                if cust[i]:
                    p = pres[i]
                    metrics[k_e] = np.float64(eff[i])
                    metrics[k_v] = np.float64(val[i])
                    cache["history"][-1]["metrics"] = {
                        eff_k: [float(x) for x, q in zip(eff_b[i], p) if q],
                        val_k: [float(x) for x, q in zip(val_b[i], p) if q]}
                else:
                    cache["history"][-1]["metrics"] = {}
                cache["metrics"] = metrics
        return self._rc

    def _rollout_states_full(self):
        """Shallow copies of the rollout cache entries with every history entry (as
        formulate_rollouts found them, before its trim)."""
        self._materialize()
        if self._states_pending:
            self._rollout_states_host()
        if self._untrimmed is not None:
            return [dict(c, history=h) for c, h in zip(self._rc, self._untrimmed)]
        return [dict(c) for c in self._rc]

    @staticmethod
    def _update_cache_history(history, next_state, actions_left, num_actions_info=None):
        """es_manager.py:212-228."""
        if num_actions_info is not None:
            assert len(history), "History should not be empty"
            history[-1].update(num_actions_info)
        history.append({"state": next_state, "actions_left": actions_left})
        return history

    def render(self):
        return [e["env"].render(e["local"]) for e in self.envs]

    def close(self):
        for t in self.tags:
            t.batch.close()
