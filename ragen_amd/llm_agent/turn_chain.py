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

import numpy as np
import torch

from .. import _lib, ops
from ..torch_ops import _parse_cfg, _render_struct, prompt_struct


def ref_f32_mean(total: int, n: int, counts) -> float:
    """``response_mask.sum(-1).float().mean()`` (ctx_manager.py:305) from the integer total of the
    n row counts.  Below 2^24 every f32 partial sum of integers is exact, whatever the order, so the
    mean is f32(total) / f32(n), one rounding, as torch's.  From 2^24 up the partial sums round and
    the result depends on the reduction order: ``counts()`` (the per-row counts, any device) then
    goes through the reference's own op, torch's CPU f32 mean."""
    if n < 1:
        return float("nan")
    if total < (1 << 24):
        return float(np.float32(total) / np.float32(n))
    return float(counts().to("cpu", torch.int64).float().mean().item())


class _Slot:
    """The buffers of one turn number, reused by every rollout (the turn record of that turn
    points at them until the next reset)."""

    def __init__(self, n, K, dev):
        e = lambda *s, dt: torch.empty(*s, dtype=dt, device=dev)  # noqa: E731
        self.has, self.err, self.flags_copy, self.derr, self.perr = (e(n, dt=torch.uint8) for _ in range(5))
        self.left, self.tlen = e(n, dt=torch.int32), e(n, dt=torch.int32)
        self.acts, self.n_act, self.spans = e(n, K, dt=torch.int8), e(n, dt=torch.uint8), e(n, 4, dt=torch.int32)
        self.n_ids, self.has_t = e(n, dt=torch.int32), e(n, dt=torch.uint8)
        self.n_ids_p, self.has_t_p = self.n_ids.data_ptr(), self.has_t.data_ptr()
        self.next_rows, self.next_src = e(n, dt=torch.int64), e(n, dt=torch.int64)  # the next batch's rows
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
        self.parse = None
        self.runs = 0  # turns taken through the chain
        n = self.n
        self.pack_bytes = ops.readback_bytes(n)
        self.stats_off = ((3 * n + 3) & ~3) + 8   # ops.readback_stats
        # the pinned host copy of the readback (numpy view over it)
        self.host = torch.empty(self.pack_bytes, dtype=torch.uint8, pin_memory=True)
        self.host_p, self.host_np = self.host.data_ptr(), self.host.numpy()
        self.pad_S = ctypes.c_int64(0)  # the width the chain padded the next batch to (0: not)
        self.padded = 0  # next batches the chain padded

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
            c.next_rows, c.next_src = s.next_rows.data_ptr(), s.next_src.data_ptr()
            c.pack_bytes = self.pack_bytes
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
    def _static(self, inp):
        """The per-manager constants of the call (parse configuration, env column, the widest
        render row, the vocabulary), once; None when the chain cannot run this manager."""
        st = self.__dict__.get("_st")
        if st is None or st[0] is not inp.vocab:
            parse = self._parse()
            ob = self.batch.obs_bound() if hasattr(self.batch, "obs_bound") else None
            if parse is None or ob is None:
                return None
            v = inp.vocab
            st = self._st = (v, parse, self.batch.parse_sel(), int(ob), v.packed.data_ptr(), v.data.data_ptr(),
                             int(v.data.numel()), int(v.packed.shape[0]))
        return st

    # the two-pass form of rmi_bpe_encode measured no faster than the one-kernel form on the
    # API turn's text (78 vs 75 us): off by default, kept as a tested option
    two_pass_bpe = False

    def _bpe(self, stride):
        """The tokenizer's current rmi_bpe_t (rebuilt when an expansion grew its tables or the
        two-pass scratch grew: rows x the BPE row bound)."""
        dt = self.pr.dt
        grew = self.two_pass_bpe and dt.ensure_two_pass(self.n, stride)
        b = self.__dict__.get("_bpe_c")
        if b is None or b[0] is not dt.added_bytes or grew or b[2] is not dt.pre or b[3] != self.two_pass_bpe:
            b = self._bpe_c = (dt.added_bytes, dt.bpe_struct(self.two_pass_bpe), dt.pre, self.two_pass_bpe)
        return ctypes.addressof(b[1])

    def _plan(self, s, t, stride, resp_max, obs_max):
        """Turn t's prompt program against this slot's buffers (DevicePrompts._turn_text), sized
        from the host's bounds: -> (rmi_prompt_t, pstride, BPE row bound), cached per slot for
        one (decode row, response bound, render bound) -- the program's constants stay valid
        as the pool grows (append-only, the old pool tensor is held)."""
        key = (stride, resp_max, obs_max)
        if s.prompt is not None and s.prompt[0] == key:
            return s.prompt
        pr, n = self.pr, self.n
        pieces, last = pr.turn_pieces(t, t + 2)
        prog, pool, tc = pr._program(pieces)
        bound = pr._text_bound(prog, obs_max, resp_max)
        if bound is None:
            return None
        pstride = pr._stride(bound + 4)
        if s.ptext is None or s.ptext.shape[1] != pstride:
            s.ptext = torch.empty(n, pstride, dtype=torch.uint8, device=self.dev)
        ep = self.batch.ep
        rows, obs_len = s.obs
        flat = [len(prog)] + [x for p in prog for x in p] + [pr.n_tags, rows.shape[1], stride, int(pr.enable_think),
                                                              pr.K]
        reward, ne = ep.turn_reward[t], ep.turn_exec[t]
        P = prompt_struct(flat, pr.sep, (pool, tc, pr.tag, rows, obs_len, s.left, reward, None, s.text, s.tlen,
                                         s.spans, None, s.has),
                          (ne, s.flags_copy, pr.int_reward_tags, int(last)))
        P.num_cache, P.num_cache_mask = pr.num_cache.data_ptr(), pr.num_cache.numel() // 16 - 1  # (held by pr)
        mx = min(int(bound), pstride)
        # (the tensors behind the struct's pointers are held with it)
        s.prompt = (key, ctypes.addressof(P), pstride, max((mx + 3) // 4 * 4, 4), last, (P, reward, ne, pool, tc))
        return s.prompt

    def run(self, inp, t):
        """Turn t over the generations of ``inp`` (ctx_manager.DeviceEnvInputs), the next
        prompt appended: -> (record, host copy of the readback pack, slot) or None when the chain
        does not apply to this turn (the caller takes the step-by-step path; nothing was
        launched)."""
        es, pr, n = self.es, self.pr, self.n
        if pr.rollout != es.rollout_id or pr.turns_done != t or pr._pending is not None:
            return None
        st = self._static(inp)
        if st is None:
            return None
        _, parse, sel, ob, packed, vbytes, nbytes, V = st
        pend = inp.pending_gen
        if pend is not None and inp.raw_next is None:
            return None  # (a hand-made DeviceEnvInputs: the chained scatter needs the other raw slot)
        stride = (int(inp.stride) + 3) // 4 * 4
        resp_max = inp.raw_max if inp.raw_max is not None else stride
        s = self._slot(t)
        if s.text is None or s.text.shape[1] != stride:
            s.text = torch.empty(n, stride, dtype=torch.uint8, device=self.dev)
            s.prompt = None
        plan = self._plan(s, t, stride, resp_max, max(ob, pr._reset_obs_max))
        if plan is None:
            return None
        _, P, pstride, bpe_stride, last, _ = plan
        c = s.c
        bpe = self._bpe(bpe_stride)
        # the fields that stay the same from rollout to rollout (vocabulary, parse, the slot's
        # rows, the prompt program, the tokenizer, the arena): set when they change only
        skey = (id(st), s.text.data_ptr(), stride, P, bpe)
        if s.__dict__.get("static_key") != skey:
            c.vocab_packed, c.vocab_bytes, c.vocab_n_bytes, c.V = packed, vbytes, nbytes, V
            c.parse, c.sel = parse, ops._ptr(sel)
            c.text, c.stride = s.text.data_ptr(), stride
            c.prompt, c.ptext, c.pstride = P, s.ptext.data_ptr(), pstride
            c.bpe, c.bpe_stride = bpe, bpe_stride
            c.arena, c.arena_stride = pr.arena_p, pr.arena_stride
            c.arena_len, c.len_upd = pr.len_p, pr.len_upd_p
            c.host = self.host_p
            c.pad_tail, c.pad_tail_n, c.pad_id = pr.tail_p, pr.tail_n, int(pr.pad_id)
            c.pad_S_out = ctypes.addressof(self.pad_S)
            s.static_key = skey
        # the generations: scattered onto the envs by the chain's first launch (deferred by
        # get_env_inputs), or already on the device
        if pend is not None:
            resp, src, src_dev = pend
            R = int(resp.shape[1])
            c.resp, c.n_resp, c.R = resp.data_ptr(), int(resp.shape[0]), R
            if src is None and src_dev is None:
                c.src, c.ids, c.n_ids, c.has_t = None, resp.data_ptr(), None, None
                inp.ids, inp.n_ids, inp.has_t = resp, None, None
            else:
                if s.ids is None or s.ids.shape[1] != R:
                    s.ids = torch.empty(n, R, dtype=torch.int64, device=self.dev)
                if src_dev is None:
                    src_dev = ops.h2d(src, self.dev)
                s.src_dev = src_dev  # (held: the allocator must not hand its block on)
                c.src = src_dev.data_ptr()
                c.ids, c.n_ids, c.has_t = s.ids.data_ptr(), s.n_ids_p, s.has_t_p
                inp.ids, inp.n_ids, inp.has_t = s.ids, s.n_ids, s.has_t
            inp.pending_gen = None
        else:
            c.resp, c.src = None, None
            c.R = int(inp.ids.shape[1])
            c.ids, c.n_ids, c.has_t = inp.ids.data_ptr(), ops._ptr(inp.n_ids), ops._ptr(inp.has_t)
        c.raw_max, c.raw_next = inp.raw_dev.data_ptr(), inp.raw_next.data_ptr() if inp.raw_next is not None else None
        pack = inp.pack
        pk = pack.data_ptr()
        c.pack, c.stats = pk, pk + self.stats_off
        # the generation batch's flagged rows counted into this readback (DevicePrompts.gen_batch)
        pad = inp.pad_err if inp.pad_counted else None
        c.pad_err, c.n_pad = (pad.data_ptr(), pad.numel()) if pad is not None else (None, 0)
        # the next generation batch padded by the chain itself, into the block of that turn
        # number's batch when nothing outside holds it (DevicePrompts.gen_batch takes it)
        blk = None if last else pr.batch_block(t + 1)
        if blk is not None:
            c.pad_block, c.pad_cap, c.pad_err_next = blk[0].data_ptr(), blk[0].numel(), blk[1].data_ptr()
        else:
            c.pad_block = None
        stream = ops._stream(self.dev)
        ops.D2H_COUNT[0] += 1
        if getattr(self.batch, "boards", None) is not None:
            self.batch.invalidate_boards()  # (the chain's token turn keeps no board cache)
        ops.check(_lib.lib().rmi_turn_chain(ctypes.byref(c), stream), "rmi_turn_chain")
        self.runs += 1
        if ops._RING:  # the chain waited for its copy: every upload enqueued before it has run
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
        host = self.host_np.copy()
        S = self.pad_S.value if blk is not None else 0
        if S:
            o = (3 * n + 3) & ~3
            count = int(host[o + 16:o + 20].view(np.int32)[0])
            pr._eager_pad = ((pr.rollout, t + 1), S, count, blk[0], blk[1])
            self.padded += 1
        else:
            pr._eager_pad = None
        return rec, host, s


class FormulateChain:
    """ContextManager.formulate_rollouts on the device path as two waits on the library
    (rmi_formulate_chain_part): the batch width (rmi_formulate_stats) with the finalize (per-env
    metrics, normalised scores) and the copies of both, then the assembly (left-padded batch,
    masks, the normalised score in place, per-row response counts) and the reductions, during
    which the host reduces the metric rows -- where the step-by-step form made ~20 launches and
    torch glue kernels between two readbacks.  Applies to one env tag, unsharded, without per-turn scores or a context
    window; ContextManager.formulate_device takes the step-by-step form otherwise (the same
    outputs: tests/test_gpu_turn_chain.py)."""

    overlap = True  # the metric rows reduced on the host while the assembly runs

    @staticmethod
    def applies(ctx, es, pr) -> bool:
        ap = ctx.config.agent_proxy
        return (pr is not None and not pr.window and len(es.tags) == 1 and not ap.use_turn_scores
                and not (ctx.process_group is not None and ctx.world_size > 1) and es.n_envs > 0)

    def __init__(self, ctx, es, pr):
        from ..torch_ops import NORM
        self.ctx, self.es, self.pr = ctx, es, pr
        n, dev = es.n_envs, es.device
        self.n, self.dev = n, dev
        tg = es.tags[0]
        self.ep = tg.batch.ep
        self.ep_struct = self.ep.struct()
        rn = ctx.config.agent_proxy.reward_normalization
        if rn.method not in NORM:
            raise ValueError(f"Invalid normalization method: {rn.method}")
        if rn.grouping == "state":
            gs = es.group_size
            seg = np.arange(0, n + 1, gs, dtype=np.int32)
        elif rn.grouping in ("batch", "inductive"):  # one tag: one group either way
            seg = np.array([0, n], np.int32)
        else:
            raise ValueError(f"Invalid grouping: {rn.grouping}")
        self.seg = torch.from_numpy(seg).to(dev)
        i32, u8 = torch.int32, torch.uint8
        self.n_sc = torch.empty(n, dtype=i32, device=dev)
        self.stats = torch.empty(4, dtype=i32, device=dev)
        self.norm = torch.empty(n, dtype=torch.float32, device=dev)
        self.resp_count = torch.empty(n, dtype=i32, device=dev)
        self.err = torch.empty(n, dtype=u8, device=dev)
        self.block = torch.empty(16 + 32 * n, dtype=u8, device=dev)  # tail i64[2] | metrics f64[n, 4]
        self.h_stats = torch.empty(16, dtype=u8, pin_memory=True)
        self.h_tail = torch.empty(16, dtype=u8, pin_memory=True)
        self.h_met = torch.empty(32 * n, dtype=u8, pin_memory=True)
        self.h_info = torch.empty(max(1, self.ep.T * n), dtype=u8, pin_memory=True)
        self.rmask = None  # the response mask (internal: only its row counts leave)
        c = self.c = _lib.FormulateChain()
        c.ep, c.seg, c.G, c.method = ctypes.addressof(self.ep_struct), self.seg.data_ptr(), len(seg) - 1, NORM[rn.method]
        c.metrics, c.norm = self.block.data_ptr() + 16, self.norm.data_ptr()
        c.B, c.pad_id = n, int(pr.pad_id)
        c.scores, c.n_scores, c.T = self.ep.turn_reward.data_ptr(), self.n_sc.data_ptr(), int(self.ep.T)
        c.resp_count, c.err, c.tail = self.resp_count.data_ptr(), self.err.data_ptr(), self.block.data_ptr()
        # copies 0-2 (the metric rows, turn_info, the width stats) after part 1 (the finalize, with
        # rmi_formulate_stats before it), copy 3 (the tail) after part 2 (rmi_formulate_chain_part)
        c.n_copies = 4
        c.host[0], c.dev[0], c.bytes[0] = self.h_met.data_ptr(), self.block.data_ptr() + 16, 32 * n
        c.host[1], c.dev[1] = self.h_info.data_ptr(), self.ep.turn_info.data_ptr()
        c.host[2], c.dev[2], c.bytes[2] = self.h_stats.data_ptr(), self.stats.data_ptr(), 12
        c.host[3], c.dev[3], c.bytes[3] = self.h_tail.data_ptr(), self.block.data_ptr(), 16
        self.runs = 0

    def run(self):
        """-> the formulated DataProto (as ContextManager.formulate_device)."""
        from .ctx_manager import LazyDataProto, _raise_assemble_errors, get_special_tokens
        ctx, es, pr, n, dev = self.ctx, self.es, self.pr, self.n, self.dev
        ap = ctx.config.agent_proxy
        pend = pr._pending[0] if pr._pending is not None else None
        tokens, start, row_len = pr.update_rows(resolve=False)
        L = _lib.lib()
        stream = ops._stream(dev)
        T = min(es._turn, es.max_turn)
        c = self.c
        c.bytes[1] = T * n
        # 1. the width, the pending host rows, zip_longest's length (rmi_formulate_stats) and the
        #    finalize (per-env metrics, normalised scores; part 1), their copies, one wait
        ops.check(L.rmi_formulate_stats(row_len.data_ptr(), ops._ptr(pend), self.ep.n_turns.data_ptr(), n,
                                        self.n_sc.data_ptr(), self.stats.data_ptr(), stream), "rmi_formulate_stats")
        ops.D2H_COUNT[0] += 1
        ops.check(L.rmi_formulate_chain_part(ctypes.byref(c), 1, 3, stream), "rmi_formulate_chain_part")
        ops.check(L.rmi_formulate_chain_wait(stream), "rmi_formulate_chain_wait")
        S, any_bad, n_slots = (int(x) for x in self.h_stats.numpy()[:12].view(np.int32))
        if pend is not None:
            pr._resolve(bool(any_bad))
            if any_bad:  # host rows were written: the longest row again
                S = int(row_len.max())
        S = max(S, 1)
        if ctx.__dict__.get("_special") is None:  # a tokenizer call: once per manager
            ctx._special = get_special_tokens(ctx.tokenizer)
        special_token, reward_token = ctx._special
        # 2. the batch: one block for the id tensors, the score, the loss mask
        So = S - 1
        ids, am, pos = torch.empty(3, n, S, dtype=torch.int64, device=dev).unbind(0)
        score = torch.empty(n, So, dtype=torch.float32, device=dev)
        lm = torch.empty(n, So, dtype=torch.bool, device=dev)
        if self.rmask is None or self.rmask.numel() < n * So:
            self.rmask = torch.empty(max(1, n * So + n * So // 4), dtype=torch.uint8, device=dev)
        c.tokens, c.row_start, c.row_len = tokens.data_ptr(), start.data_ptr(), row_len.data_ptr()
        c.S, c.special_token, c.reward_token = S, int(special_token), int(reward_token)
        c.n_slots = n_slots
        c.flags = (_lib.MS_RESPONSE_MASK if ctx.config.enable_response_mask else 0) | \
            (_lib.MS_ROLL if "qwen" in ctx.tokenizer.name_or_path.lower() else 0)
        c.input_ids, c.attention_mask, c.position_ids = ids.data_ptr(), am.data_ptr(), pos.data_ptr()
        c.score_out, c.loss_mask, c.response_mask = score.data_ptr(), lm.data_ptr(), self.rmask.data_ptr()
        # the assembly and the tail (part 2), not waited on: the host reduces the metric rows
        # meanwhile, then waits for the tail
        ops.D2H_COUNT[0] += 1
        ops.check(L.rmi_formulate_chain_part(ctypes.byref(c), 2, 3, stream), "rmi_formulate_chain_part")
        self.runs += 1
        if not self.overlap:  # (A/B: the host's reductions after the assembly, not beside it)
            ops.check(L.rmi_formulate_chain_wait(stream), "rmi_formulate_chain_wait")
        # the metric rows as columns (one copy; device_metrics reduces each column contiguously)
        m = np.ascontiguousarray(self.h_met.numpy().view(np.float64).reshape(n, 4).T).T
        info = self.h_info.numpy()[:T * n].reshape(T, n)
        custom = (info & _lib.INFO_PRESENT).any(0) if T else np.zeros(n, bool)
        batch = {"input_ids": ids, "attention_mask": am, "position_ids": pos, "responses": ids[:, 1:],
                 "loss_mask": lm, "rm_scores": score, "original_rm_scores": score}
        env_ids = es.env_lo + np.arange(n, dtype=np.int64)
        out = LazyDataProto(env_ids, lambda: ctx._messages_only(es._rollout_states_full(), True))
        out.set_device_batch(batch, env_ids, es.group_size)
        metrics = ctx.device_metrics(es, [(es.tags[0].tag, m, custom, None)])
        ops.check(L.rmi_formulate_chain_wait(stream), "rmi_formulate_chain_wait")
        total, bits = (int(x) for x in self.h_tail.numpy().view(np.int64))
        _raise_assemble_errors(None, S, (bool(bits & _lib.ERR_UNSUP), bool(bits & _lib.ERR_STATE)))
        # response_length: the f32 mean of the row counts (ctx_manager.py:305); exact while the
        # total stays below 2^24, where f32 sums of integers are exact in any order.  Above it the
        # partial sums round, so the counts go through the reference's own op: torch's CPU f32 mean
        response_length = ref_f32_mean(total, n, lambda: self.resp_count[:n])
        metrics["response_length"] = response_length
        out.meta_info = {"metrics": metrics}
        es._formulated = True
        es._formulated_window = pr.window
        return out
