"""One device turn of LLMAgentProxy.rollout as ONE call into the library (rmi_turn_chain).

The turn of the device path (EnvStateManager._step_device) is ten launches: the generations onto
the env rows, the fused decode + parse, the step inputs, the turn with its render, the record's
columns and readback, the next prompt's text, its BPE ids, the commit with the next batch's
stats, and the readback copy.  Driven from Python each launch cost 10-60 us of interpreter and
dispatcher time, and an 8192-env turn spent ~400 us on the host against ~290 us of kernels
(profiles/r04_api_host_stamps.txt): the GPU sat idle between launches.  Here every pointer and
shape of the turn is kept in one rmi_turn_chain_t per turn slot (buffers allocated once per
manager and reused by every rollout), a turn sets the handful of fields that change (the
generations, their env map, the decode row) and makes one ctypes call, which enqueues the ten
steps back to back, copies the readback and waits.

Applies to a shard with one env tag whose batch renders on the device in the turn (Sokoban,
FrozenLake), with device prompts in append mode; anything else takes the step-by-step path of
EnvStateManager._step_device.  Both paths produce the same record, prompt arena and readback,
bit for bit (tests/test_gpu_turn_chain.py runs rollouts both ways and compares every tensor).
"""
import ctypes

import torch

from .. import _lib, ops
from ..torch_ops import _parse_cfg, _render_struct, prompt_struct


class _Slot:
    """The buffers of one turn number, reused by every rollout (the turn record of that turn
    points at them until the next reset)."""

    def __init__(self, n, K, dev):
        e = lambda *s, dt: torch.empty(*s, dtype=dt, device=dev)  # noqa: E731
        self.has, self.err, self.flags_copy, self.derr, self.perr = (e(n, dt=torch.uint8) for _ in range(5))
        self.left, self.tlen = e(n, dt=torch.int32), e(n, dt=torch.int32)
        self.acts, self.n_act, self.spans = e(n, K, dt=torch.int8), e(n, dt=torch.uint8), e(n, 4, dt=torch.int32)
        self.n_ids, self.has_t = e(n, dt=torch.int32), e(n, dt=torch.uint8)
        self.ptext_len, self.pmark, self.mark_tok = (e(n, dt=torch.int32) for _ in range(3))
        self.pterr, self.bpe_err, self.bad = (e(n, dt=torch.uint8) for _ in range(3))
        self.text = None      # u8[n, stride], sized by the decode row
        self.ptext = None     # u8[n, pstride], sized by the prompt row bound
        self.ids = None       # i64[n, R] (generations scattered onto the envs), sized by R
        self.obs = None       # (rows, lengths) of the render
        self.render = None    # its rmi_render_t
        self.prompt = None    # (key, rmi_prompt_t, pstride, bpe_stride)
        self.c = _lib.TurnChain()


class TurnChain:
    """rmi_turn_chain for one EnvStateManager / DevicePrompts pair (module docstring)."""

    @staticmethod
    def applies(es, pr) -> bool:
        if pr is None or pr.window or len(es.tags) != 1:
            return False
        tg = es.tags[0]
        return tg.env_type in ("sokoban", "frozen_lake") and getattr(tg.batch, "dispatch", "op") != "ctypes" \
            and tg.batch.B == es.n_envs

    def __init__(self, es, ctx, pr):
        self.es, self.ctx, self.pr = es, ctx, pr
        tg = es.tags[0]
        self.tg, self.batch = tg, tg.batch
        self.n = es.n_envs
        self.K = es.K
        self.dev = es.device
        self.kind = _lib.CHAIN_SOKOBAN if tg.env_type == "sokoban" else _lib.CHAIN_FROZENLAKE
        self.slots = {}
        self.env = self.batch.struct()          # the batch's tensors live as long as the batch
        self.ep_struct = self.batch.ep.struct()
        if es._max_act is None:
            es._max_act = torch.full((self.n,), tg.max_actions_per_traj, dtype=torch.int32, device=self.dev)
        self.vocab = None
        self.parse = None
        self.runs = 0  # turns taken through the chain

    # ------------------------------------------------------------------ per slot
    def _slot(self, t):
        s = self.slots.get(t)
        if s is None:
            s = self.slots[t] = _Slot(self.n, self.K, self.dev)
            c = s.c
            es, tg = self.es, self.tg
            c.n_envs = self.n
            c.dec_err, c.text_len, c.actions, c.n_actions = (x.data_ptr() for x in (s.derr, s.tlen, s.acts, s.n_act))
            c.spans, c.parse_err, c.has, c.err = (x.data_ptr() for x in (s.spans, s.perr, s.has, s.err))
            c.env_kind = self.kind
            ptr = ctypes.addressof(self.env)
            c.sokoban, c.frozenlake = (ptr, None) if self.kind == _lib.CHAIN_SOKOBAN else (None, ptr)
            c.ep = ctypes.addressof(self.ep_struct)
            c.turn, c.K = int(t), self.K
            c.max_actions_per_traj, c.format_penalty = tg.max_actions_per_traj, es.format_penalty
            c.max_actions, c.flags_copy, c.left = es._max_act.data_ptr(), s.flags_copy.data_ptr(), s.left.data_ptr()
            c.pmark, c.ptext_len, c.pterr = s.pmark.data_ptr(), s.ptext_len.data_ptr(), s.pterr.data_ptr()
            c.mark_tok, c.bpe_err, c.bad = s.mark_tok.data_ptr(), s.bpe_err.data_ptr(), s.bad.data_ptr()
            b = self.batch
            if self.kind == _lib.CHAIN_SOKOBAN:
                s.obs = ops.render_buffers(self.n, b.H, b.W, self.dev)
            else:
                st = (b.nrow * b.ncol * 4 + b.nrow - 1 + 3) // 4 * 4
                s.obs = (torch.empty(self.n, st, dtype=torch.uint8, device=self.dev),
                         torch.empty(self.n, dtype=torch.int32, device=self.dev))
            s.render = _render_struct(*b.glyph_lists(), *s.obs)
            c.obs = ctypes.addressof(s.render)
        return s

    def _vocab(self, v):
        if self.vocab is None or self.vocab[0] is not v:
            self.vocab = (v, v.packed.data_ptr(), v.data.data_ptr(), int(v.data.numel()), int(v.packed.shape[0]))
        return self.vocab

    def _parse(self):
        ap = self.es.sys_config.agent_proxy
        words, _, lact = self.es._parse_args(self.tg, bool(ap.enable_think), ap.action_sep, True)
        if lact:
            return None  # answers as text (Countdown): not a chain env
        if self.parse is None or self.parse[0] != words:
            cfg = _parse_cfg(words)
            self.parse = (words, cfg, ctypes.addressof(cfg))
        return self.parse[2]

    # ------------------------------------------------------------------- the turn
    def run(self, inp, t):
        """Turn t over the generations of ``inp`` (ctx_manager.DeviceEnvInputs), the next
        prompt appended: -> (record, host copy of the readback pack) or None when the chain does
        not apply to this turn (the caller takes the step-by-step path; nothing was launched)."""
        es, pr, n = self.es, self.pr, self.n
        if pr.rollout != es.rollout_id or pr.turns_done != t or pr._pending is not None:
            return None
        parse = self._parse()
        if parse is None:
            return None
        obs_max = pr._obs_bound({0: None})
        if obs_max is None:
            return None
        s = self._slot(t)
        c = s.c
        v, packed, vbytes, nbytes, V = self._vocab(inp.vocab)
        c.vocab_packed, c.vocab_bytes, c.vocab_n_bytes, c.V = packed, vbytes, nbytes, V
        sel = self.batch.parse_sel()
        c.parse, c.sel = parse, ops._ptr(sel)
        s.sel = sel
        # the generations: scattered onto the envs by the chain's first launch (deferred by
        # get_env_inputs), or already on the device
        pend = inp.pending_gen
        if pend is not None and inp.raw_next is None:
            return None  # (a hand-made DeviceEnvInputs: the chained scatter needs the other raw slot)
        if pend is not None:
            resp, src = pend
            R = int(resp.shape[1])
            c.resp, c.n_resp, c.R = resp.data_ptr(), int(resp.shape[0]), R
            if src is None:
                c.src, c.ids, c.n_ids, c.has_t = None, resp.data_ptr(), None, None
                inp.ids, inp.n_ids, inp.has_t = resp, None, None
            else:
                if s.ids is None or s.ids.shape[1] < R:
                    s.ids = torch.empty(n, R, dtype=torch.int64, device=self.dev)
                ids = s.ids if s.ids.shape[1] == R else s.ids[:, :R]
                if not ids.is_contiguous():
                    s.ids = torch.empty(n, R, dtype=torch.int64, device=self.dev)
                    ids = s.ids
                s.src_dev = ops.h2d(src, self.dev)  # (held: the allocator must not hand its block on)
                c.src = s.src_dev.data_ptr()
                c.ids, c.n_ids, c.has_t = ids.data_ptr(), s.n_ids.data_ptr(), s.has_t.data_ptr()
                inp.ids, inp.n_ids, inp.has_t = ids, s.n_ids, s.has_t
            inp.pending_gen = None
        else:
            c.resp, c.src = None, None
            c.R = int(inp.ids.shape[1])
            c.ids, c.n_ids, c.has_t = inp.ids.data_ptr(), ops._ptr(inp.n_ids), ops._ptr(inp.has_t)
        c.raw_max, c.raw_next = inp.raw_dev.data_ptr(), inp.raw_next.data_ptr() if inp.raw_next is not None else None
        # the decode row
        stride = (int(inp.stride) + 3) // 4 * 4
        if s.text is None or s.text.shape[1] != stride:
            s.text = torch.empty(n, stride, dtype=torch.uint8, device=self.dev)
            s.prompt = None
        c.text, c.stride = s.text.data_ptr(), stride
        # the next prompt's program: turn t's text (DevicePrompts._turn_text), sized from the
        # host's bounds (the decode row, the widest render row)
        resp_max = inp.raw_max if inp.raw_max is not None else stride
        pieces, last = pr.turn_pieces(t, t + 2)
        prog, pool, tc = pr._program(pieces)
        bound = pr._text_bound(prog, obs_max, resp_max)
        if bound is None:
            return None
        pstride = pr._stride(bound + 4)
        key = (stride, pstride, id(pool), id(tc), last)
        if s.prompt is None or s.prompt[0] != key:
            if s.ptext is None or s.ptext.shape[1] != pstride:
                s.ptext = torch.empty(n, pstride, dtype=torch.uint8, device=self.dev)
            ep = self.batch.ep
            rows, obs_len = s.obs
            flat = [len(prog)] + [x for p in prog for x in p] + [pr.n_tags, rows.shape[1], stride,
                                                                  int(pr.enable_think), pr.K]
            reward, ne = ep.turn_reward[t], ep.turn_exec[t]
            P = prompt_struct(flat, pr.sep, (pool, tc, pr.tag, rows, obs_len, s.left, reward, None, s.text, s.tlen,
                                             s.spans, None, s.has),
                              (ne, s.flags_copy, pr.int_reward_tags, int(last)))
            mx = min(int(bound), pstride)
            # (the tensors behind the struct's pointers held with it: ids in the key stay unique)
            s.prompt = (key, P, pstride, max((mx + 3) // 4 * 4, 4), (reward, ne, pool, tc))
        _, P, pstride, bpe_stride, _ = s.prompt
        c.prompt = ctypes.addressof(P)
        c.ptext, c.pstride = s.ptext.data_ptr(), pstride
        bpe = pr.dt.bpe_struct()
        c.bpe, c.bpe_stride = ctypes.addressof(bpe), bpe_stride
        c.arena, c.arena_stride = pr.arena.data_ptr(), int(pr.arena.shape[1])
        c.arena_len, c.len_upd = pr.len.data_ptr(), pr.len_upd.data_ptr()
        pack = inp.pack
        c.pack, c.stats = pack.data_ptr(), ops.readback_stats(pack, n).data_ptr()
        nb = ops.readback_bytes(n)
        host = es.__dict__.get("_pin_buf")
        if host is None or host.numel() < nb:
            host = es._pin_buf = torch.empty(max(nb, 1 << 16), dtype=torch.uint8, pin_memory=True)
        c.host, c.pack_bytes = host.data_ptr(), nb
        stream = ops._stream(self.dev)
        ops.D2H_COUNT[0] += 1
        ops.check(_lib.lib().rmi_turn_chain(ctypes.byref(c), stream), "rmi_turn_chain")
        self.runs += 1
        if ops._RING:  # the chain waited on the stream: the upload ring's slices are free
            ops._RING[0].reset_after_sync(stream)
        # the batch's state and the host-side records, as the step-by-step path leaves them
        b = self.batch
        b._invalidate()
        b._rows = s.obs
        inp.set_decoded(s.text, s.tlen, s.derr)
        es._turn += 1
        rec = {"turn": t, "inp": inp, "has": s.has, "err": s.err, "obs": {0: s.obs}, "spans": [s.spans],
               "flags": s.flags_copy, "left": s.left, "_obs_known": True}
        flags = s.flags_copy
        pr._pending = (s.bad, lambda e: pr._host_turn(e, t, not last and not int(flags[e]) & _lib.FLAG_DONE))
        pr.turns_done = t + 1
        pr.eager_turns += 1
        pr._next_stats = None
        return rec, host[:nb].numpy().copy()
