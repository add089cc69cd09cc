"""Prompt token ids built on the device, turn by turn (§8(f) ranks 1-2).

The reference rebuilds every env's whole conversation each turn — chat messages from the
history, ``apply_chat_template``, then the tokenizer over all of it (ctx_manager.py:228-278) —
and once more for the update batch (formulate_rollouts, :354-356 -> :278-306).  Here each env
keeps its prompt as token ids in a device arena, and a turn APPENDS the ids of the text it
adds, built and tokenized on the device:

* the chat template is cut once (``ChatTemplate``) into the pieces the reference's messages
  produce: the system block and the first user opening (``head``), the user / assistant
  openings and closings, the generation prompt;
* a reset writes ``head + first user message + user closing`` per env (rmi_prompt_text with
  the env's instruction prefix, ``Turn 1``, its rendered state, actions left, the format and
  length lines), then tokenizes it (rmi_bpe_encode);
* a turn writes ``assistant opening + llm_response + assistant closing`` (llm_response rebuilt
  from the parse kernel's spans, exactly _parse_response, ctx_manager.py:148-173) and, for an
  env that goes on, ``user opening + Reward / Turn / State / actions-left block + user
  closing``, and appends their ids; the position after the assistant block is kept (the
  update batch ends there: prepare_for_update drops the last state and reward,
  ctx_manager.py:236-237, :258-262);
* the generation batch is the arena rows of the active envs plus the ids of the generation
  prompt (``gen`` + "<think>"), left-padded (rmi_pad_rows); the update batch is the arena rows
  up to the kept positions with masks and scores (rmi_assemble_rows).

Exactness: tokenizing a concatenation equals concatenating the tokenizations whenever every
cut falls right before an added token (the tokenizer splits on added tokens first, and the
pre-tokenizer and BPE never look across that split).  ``ChatTemplate`` checks that each
appended piece starts with one, and the whole construction against the host tokenizer on a
probe conversation; otherwise the device path raises NotImplementedError at construction and
the ContextManager keeps the host path.  A row the kernels flag (text past the row buffer, a
code point NFC may change, a reward outside the formatter's range) is built and tokenized on
the host for that env alone (``host_rows``), and counted in ``self.host_rows_used``.

``agent_proxy.max_context_window`` = k (history truncation with re-numbered turns,
ctx_manager.py:244-246) changes every prompt each turn (the window slides and the ``Turn i``
headers renumber), so it is not an append: the rows are REBUILT on the device from the kept
turn records (``window`` mode) -- the first kept entry's block (``Turn 1`` and its state, as a
reset writes it) and, per later entry, the assistant block and the reward / next-state block
with its renumbered header, each through rmi_prompt_text + rmi_bpe_encode into the env's arena
row.  The generation batch rebuilds the active envs' windows each turn; the update batch
rebuilds each env's last k complete entries (envs grouped by their turn count).  A row the
kernels flag is rebuilt on the host from the env's history (the reference's own message code).
"""
import warnings
from typing import List, Optional

import numpy as np
import torch

from .. import _lib, ops
from ..tokenizer import DeviceTokenizer
from ..torch_ops import direct

SYSTEM = "You're a helpful assistant. "


def _storage_uses(t: torch.Tensor) -> int:
    """References to t's storage (t itself and a temporary count 2: no view of it is alive)."""
    f = getattr(torch._C, "_storage_Use_Count", None)
    return f(t.untyped_storage()._cdata) if f is not None else 1 << 30


_USE_COUNT = getattr(torch._C, "_storage_Use_Count", None)


def _uses(st) -> int:
    """References to a held storage object's storage (its tensor and the object itself count
    2: no view of it is alive)."""
    return _USE_COUNT(st._cdata) if _USE_COUNT is not None else 1 << 30
_P = ("@@RMI_S@@", "@@RMI_U1@@", "@@RMI_A1@@", "@@RMI_U2@@", "@@RMI_A2@@")


def format_prompt(enable_think: bool) -> str:
    return ("<think> [Your thoughts] </think> <answer> [your answer] </answer>" if enable_think
            else "<answer> [your answer] </answer>")


class ChatTemplate:
    """The tokenizer's chat template cut into concatenable pieces (module docstring)."""

    def __init__(self, tokenizer, system: str = SYSTEM):
        _, U1, A1, U2, A2 = _P

        def ap(msgs, gen):
            return tokenizer.apply_chat_template(msgs, add_generation_prompt=gen, tokenize=False)
        sysm = {"role": "system", "content": system}
        u = lambda c: {"role": "user", "content": c}  # noqa: E731
        a = lambda c: {"role": "assistant", "content": c}  # noqa: E731
        r_u, r_ug = ap([sysm, u(U1)], False), ap([sysm, u(U1)], True)
        r_a = ap([sysm, u(U1), a(A1)], False)
        r_aug = ap([sysm, u(U1), a(A1), u(U2)], True)
        r_aua = ap([sysm, u(U1), a(A1), u(U2), a(A2)], False)
        try:
            i = r_u.index(U1)
            self.head, self.u_suf = r_u[:i], r_u[i + len(U1):]
            assert r_ug.startswith(r_u)
            self.gen = r_ug[len(r_u):]
            assert r_a.startswith(r_u)
            rest = r_a[len(r_u):]
            j = rest.index(A1)
            self.a_pre, self.a_suf = rest[:j], rest[j + len(A1):]
            assert r_aug.startswith(r_a)
            rest = r_aug[len(r_a):]
            k = rest.index(U2)
            self.u_pre = rest[:k]
            assert rest[k + len(U2):] == self.u_suf + self.gen
            assert r_aua == r_a + self.u_pre + U2 + self.u_suf + self.a_pre + A2 + self.a_suf
        except (AssertionError, ValueError):
            raise NotImplementedError("the chat template is not a concatenation of per-message blocks; the device "
                                      "prompt path does not apply") from None


# Context probes of the expansion analysis: every text that may stand next to a constant stretch
# of a prompt (an LLM response, a rendered state, a reward, an int) is arbitrary, so a cut must
# hold against every class the Qwen2 pre-tokenizer regex tells apart on either side: letters
# (and the contraction letters after an apostrophe), digits, other numerics, punctuation, the
# space, other whitespace, newlines, CR, wide and astral characters -- alone, doubled, tripled
# and in every ordered pair, plus the shapes the prompts actually carry.  (Combining marks and
# other NFC-unsafe code points never reach the device encoder: their rows go to the host.)
_PROBE_CHARS = ["a", "Z", "s", "t", "e", "é", "中", "1", "9", "½", "_", ".", ",", "<", ">", "'", '"', "-", "#", "|",
                " ", "\t", "\n", "\r", "\u00a0", "\u3000", "\U0001F600"]
_PROBE_EXTRA = ["'s", "'re", "'ll", "x ", "x\n", " \n", "\n ", "\r\n", "1.5", "-0.1", "10.0", "1e-05", "</answer>",
                "<answer>", "</think>", "Up || Down", "#_P\n##", "  x", "x  ", "abc def", "<|im_end|>", "<|im_start|>"]


def _probes():
    c = _PROBE_CHARS
    runs = [w * k for w in (" ", "\t", "\n", "\r\n", "-", "=", "#", "a", "1") for k in (4, 5, 6, 8, 12, 16, 24)]
    return [""] + c + [x * 2 for x in c] + [x * 3 for x in c] + [a + b for a in c for b in c] + runs + _PROBE_EXTRA


class ExpansionSplitter:
    """Finds, in a constant stretch X of prompt text, the longest middle X[q1:q2] whose token ids
    did not depend on the text around X in any of the probe contexts:  ids(L + X + R) ==
    ids(L + X[:q1]) + I + ids(X[q2:] + R) for every probe L, R -- exactly what the device
    encoder computes when the middle is replaced by an added-token placeholder standing for I
    (the placeholder cuts the regex segments there).  This is CHECKED against a finite probe
    set, not proven for every context: the generic probes (``_probes``: every pre-tokenizer
    class alone, doubled, tripled and in pairs, runs, and prompt shapes) plus the texts that can
    actually stand next to a stretch in this run's prompts (``extra``: the env tags' render
    glyphs and rendered rows, the reward and integer forms, the chat template's added tokens).
    Cuts are tried at X's own token boundaries, outermost first.  The tokenizer's own
    `tokenizers` backend encodes (batched); results are cached per text."""

    _by_tok = {}
    MIN_BYTES = 12  # a shorter middle is not worth a placeholder (2 bytes)

    def __init__(self, backend, extra=()):
        self.bt = backend
        base = _probes()
        seen = set(base)
        self.probes = base + [x for x in dict.fromkeys(extra) if x not in seen]
        self.cache = {}

    @classmethod
    def for_tokenizer(cls, tokenizer, extra=()):
        bt = getattr(tokenizer, "backend_tokenizer", None)
        if bt is None or not hasattr(bt, "encode_batch"):
            return None
        key = (id(bt), tuple(dict.fromkeys(extra)))
        if key not in cls._by_tok:
            cls._by_tok[key] = cls(bt, extra)
        return cls._by_tok[key]


    def _ids(self, texts):
        return [e.ids for e in self.bt.encode_batch(list(texts), add_special_tokens=False)]

    def split(self, x: str, right_free: bool = False):
        """-> (q1, ids of X[q1:q2], q2) in characters, or None.  right_free: nothing but an
        added token or the row end ever follows X."""
        key = (x, right_free)
        if key not in self.cache:
            self.cache[key] = self._split(x, right_free)
        return self.cache[key]

    def _split(self, x, right_free):
        if len(x.encode("utf-8")) < self.MIN_BYTES:
            return None
        enc = self.bt.encode(x, add_special_tokens=False)
        ids, starts = list(enc.ids), [o[0] for o in enc.offsets]
        cuts = sorted(set(starts) | {0, len(x)})
        P = self.probes
        whole_l = self._ids([p + x for p in P])
        q1 = k1 = None
        for q in cuts:  # the leftmost cut every left context agrees with
            k = next((i for i, st in enumerate(starts) if st >= q), len(ids))
            pre = self._ids([p + x[:q] for p in P])
            if all(w == a + ids[k:] for w, a in zip(whole_l, pre)):
                q1, k1 = q, k
                break
        if q1 is None:
            return None
        R = [""] if right_free else P
        whole_r = self._ids([x + r for r in R])
        q2 = k2 = None
        for q in reversed(cuts):  # the rightmost cut every right context agrees with
            if q < q1:
                break
            k = next((i for i, st in enumerate(starts) if st >= q), len(ids))
            post = self._ids([x[q:] + r for r in R])
            if all(w == ids[:k] + b for w, b in zip(whole_r, post)):
                q2, k2 = q, k
                break
        if q2 is None or len(x[q1:q2].encode("utf-8")) < self.MIN_BYTES or k2 <= k1:
            return None
        mid = ids[k1:k2]
        # both sides at once, on a spread of pairs
        pairs = [(P[i], R[(7 * i + 3) % len(R)]) for i in range(0, len(P), 3)]
        whole = self._ids([l + x + r for l, r in pairs])
        lefts = self._ids([l + x[:q1] for l, _ in pairs])
        rights = self._ids([x[q2:] + r for _, r in pairs])
        if any(w != a + mid + b for w, a, b in zip(whole, lefts, rights)):
            return None
        return q1, mid, q2


def context_probes(es, tpl, added) -> list:
    """The texts that can stand next to a constant stretch of this run's prompts, beyond the
    generic probes: each tag's render glyphs (alone, doubled, as a row), a rendered state of each
    env batch, the reward forms a turn prints (ints, step sums, successes), integers, and the
    chat template's pieces and added tokens."""
    out = []
    for tg in es.tags:
        g = getattr(tg.batch.config, "grid_lookup", None) or {}
        glyphs = [str(v) for v in g.values()]
        out += glyphs + [x * 2 for x in glyphs] + ["".join(glyphs), "\n".join(glyphs)]
        if hasattr(tg.batch, "render"):
            try:
                out.append(tg.batch.render(0))
            except Exception:  # (a batch not reset yet renders nothing useful)
                pass
    out += ["0", "1", "-1", "0.0", "1.0", "-0.1", "-0.2", "-0.30000000000000004", "0.9", "10.9", "-1.1", "9.9",
            "0.7999999999999999", "10", "100", "255", "4294967295"]
    out += [tpl.head, tpl.u_suf, tpl.a_pre, tpl.a_suf, tpl.u_pre, tpl.gen] + list(added)
    return [x for x in out if x]


class DevicePrompts:
    """Per-env prompt ids on the device for one ContextManager / EnvStateManager pair."""

    first_bound = True  # the first prompt's BPE row size from the host's bound (A/B: read back)

    def __init__(self, ctx, es, tokenizer, device, capacity: Optional[int] = None, window: Optional[int] = None,
                 expansions: bool = True):
        ap = ctx.config.agent_proxy
        self.window = int(window) if window else None  # max_context_window (k > 0), or None
        self.ctx, self.es, self.tok = ctx, es, tokenizer
        self.device = torch.device(device)
        self.enable_think = bool(ap.enable_think)
        self.tpl = ChatTemplate(tokenizer)
        self.dt = DeviceTokenizer.from_hf(tokenizer, self.device)
        self.splitter = ExpansionSplitter.for_tokenizer(
            tokenizer, context_probes(es, self.tpl, list(self.dt.added))) if expansions else None
        starts = [s for s in self.dt.added]
        for nm in ("a_pre", "u_pre", "gen"):
            piece = getattr(self.tpl, nm)
            if not any(piece.startswith(s) for s in starts):
                raise NotImplementedError(f"template piece {nm}={piece!r} does not start with an added token")
        self.pad_id = tokenizer.pad_token_id if getattr(tokenizer, "pad_token_id", None) is not None else 0
        self.prefix = "<think>" if self.enable_think else "<answer>"
        self.sep = list(ap.action_sep.encode("utf-8"))
        self.K = int(ap.max_actions_per_turn)
        self.max_turn = int(ap.max_turn)
        cfg_len = getattr(getattr(getattr(ctx.config, "actor_rollout_ref", None), "rollout", None), "max_model_len",
                          None)
        self.cap = int(capacity or cfg_len or 8192)
        n = es.n_envs
        self.n_envs = n
        # per-env tag index and per-tag strings (instruction prefix, length line, actions cap)
        tags = es.tags
        self.n_tags = len(tags)
        tag = np.zeros(n, np.uint8)
        for j, tg in enumerate(tags):
            tag[tg.lo - es.env_lo:tg.hi - es.env_lo] = j
        self.tag = torch.from_numpy(tag).to(self.device)
        # tags whose 0 / 1 rewards print as ints (Countdown's integer rewards), as a bit mask
        if any(tg.env_type == "countdown" for tg in tags[32:]):
            raise NotImplementedError("a Countdown tag past the 32nd tag of a shard")
        self.int_reward_tags = sum(1 << j for j, tg in enumerate(tags) if tg.env_type == "countdown")
        prefixes = [ctx.prefix_lookup[tg.lo] for tg in tags]
        self._max_prefix = max(len(p) for p in ctx.prefix_lookup.values())  # the start row's width bound
        lengths = [f"Max response length: {ctx.env_config_lookup[tg.lo]['max_tokens']} words (tokens)." for tg in tags]
        self._pool = bytearray()
        self._const_at = {}
        self._pool_dev = None
        self._tag_tables = []
        self._tag_strings = []   # the tables' strings (the expansion analysis reads them)
        self._exp_cache = {}     # program -> program with expansions (_with_expansions)
        self._tag_table(prefixes)  # table 0: instruction prefix
        self._tag_table(lengths)   # table 1: length line
        self.mapt = torch.tensor([tg.max_actions_per_traj for tg in tags], dtype=torch.int32,
                                 device=self.device)[self.tag.long()]
        fmt = format_prompt(self.enable_think)
        self._c_mid = f" actions left. Always output: {fmt} with no extra text. Strictly follow this format. "
        # device buffers
        self.arena = torch.zeros(n, self.cap, dtype=torch.int64, device=self.device)
        self.len = torch.zeros(n, dtype=torch.int32, device=self.device)
        self.len_upd = torch.zeros(n, dtype=torch.int32, device=self.device)
        # (kept for the life of the builder: the turn chain takes their pointers once)
        self.arena_p, self.arena_stride = self.arena.data_ptr(), int(self.arena.shape[1])
        self.len_p, self.len_upd_p = self.len.data_ptr(), self.len_upd.data_ptr()
        self._all_idx = np.arange(n, dtype=np.int64)
        self._all_rows = torch.arange(n, dtype=torch.int64, device=self.device)
        # the reward text cache of the chained prompt launches (rmi_prompt_t.num_cache): 64 KB
        self.num_cache = torch.zeros(1024 * 16, dtype=torch.int32, device=self.device)
        tail = self.dt.encode([self.tpl.gen + self.prefix])[0]
        if tail is None or tail != self._host_ids(self.tpl.gen + self.prefix):
            raise NotImplementedError("the generation prompt does not encode like the host tokenizer")
        self.tail = torch.tensor(tail, dtype=torch.int64, device=self.device)
        self.tail_p, self.tail_n = self.tail.data_ptr(), int(self.tail.numel())
        self._batch_bufs = {}  # turn number -> gen_batch's output block and error bytes (_pad_rows)
        self.last_rows = None  # the device rows of the last generation batch
        self.host_rows_used = 0
        self._pending = None  # (bad rows u8/bool[B] on the device, their host builder), not read back yet
        self._next_stats = None  # (turns done, longest row, any host row, rows) of advance_eager
        self._eager_pad = None   # ((rollout, turns done), S, rows, block, err) the turn chain padded
        self.chain_padded = 0    # generation batches taken from the turn chain's pad
        self.eager_turns = 0     # turns appended by advance_eager (the rest at get_lm_inputs)
        self._reset_obs_max = 0
        self.rollout = None
        self.turns_done = 0
        self._verify()

    def _host_ids(self, text: str) -> List[int]:
        """The host tokenizer's ids of one text (the reference's call, ctx_manager.py:265-278)."""
        return [int(x) for x in self.tok([text], padding=False, truncation=False).input_ids[0]]

    # ---------------------------------------------------------------- constant pool
    def _const(self, s):
        """The pool (offset, length) of a str (UTF-8) or bytes constant (an expansion placeholder
        is not valid UTF-8)."""
        if s not in self._const_at:
            b = s.encode("utf-8") if isinstance(s, str) else bytes(s)
            self._const_at[s] = (len(self._pool), len(b))
            self._pool += b
        return self._const_at[s]

    def _tag_table(self, strings):
        """A per-tag constant table (one entry per tag) -> its index (RMI_PT_TAG_CONST's a)."""
        tab = []
        for s in strings:
            tab += list(self._const(s))
        self._tag_tables.append(tab)
        self._tag_strings.append(list(strings))
        return len(self._tag_tables) - 1

    def _program(self, pieces):
        """pieces: (kind, a, b) triples, CONST given as a str -> (program ints, pool, tag_const).
        Long constant stretches become expansion placeholders (_with_expansions)."""
        pieces = self._with_expansions(pieces)
        prog = []
        for p in pieces:
            if isinstance(p, str):
                off, ln = self._const(p)
                prog.append((_lib.PT_CONST, off, ln))
            else:
                prog.append(p)
        key = (len(self._pool), len(self._tag_tables))
        if self._pool_dev is None or self._pool_dev[0] != key:  # upload when the pool or the tables grew
            pad = 4 + (-len(self._pool)) % 4  # whole dwords: the kernel stages the pool with dword loads
            pool = torch.frombuffer(bytearray(self._pool) + b"\0" * pad, dtype=torch.uint8).to(self.device)
            tc = torch.tensor([x for t in self._tag_tables for x in t], dtype=torch.int32, device=self.device)
            self._pool_dev = (key, pool, tc)
        return prog, self._pool_dev[1], self._pool_dev[2]

    # ------------------------------------------------------------ expansions
    @staticmethod
    def _is_const(p):
        return isinstance(p, (str, bytes)) or p[0] in (_lib.PT_CONST, _lib.PT_TAG_CONST)

    def _const_text(self, p, tag):
        if isinstance(p, str):
            return p
        if p[0] == _lib.PT_TAG_CONST:
            return self._tag_strings[p[1]][tag]
        raise ValueError("pool-offset CONST pieces are not analysed")

    def _with_expansions(self, pieces):
        """Each maximal run of constant pieces (between variable pieces, MARK and IF) whose middle
        tokenized the same in every context it was checked against (ExpansionSplitter: the
        generic and this run's probes, per tag) becomes prefix + placeholder + suffix: the placeholder is an
        added token of the device tokenizer standing for the middle's ids (rmi_bpe_t
        expansions), so the BPE kernel skips those bytes.  Cached per program."""
        key = tuple(pieces)
        hit = self._exp_cache.get(key)
        if hit is not None:
            return hit
        out, i, n = [], 0, len(pieces)
        split = self.splitter
        while i < n:
            if not self._is_const(pieces[i]) or split is None:
                out.append(pieces[i])
                i += 1
                continue
            j = i
            while j < n and self._is_const(pieces[j]):
                j += 1
            run = pieces[i:j]
            texts = ["".join(self._const_text(p, tg) for p in run) for tg in range(self.n_tags)]
            res = [split.split(t, right_free=(j == n)) for t in texts]
            if any(r is not None for r in res):
                pre, ph, post = [], [], []
                for t, r in zip(texts, res):
                    mark = self.dt.add_expansion(r[1]) if r is not None else None
                    if mark is None:
                        pre.append(t)
                        ph.append("")
                        post.append("")
                    else:
                        q1, _, q2 = r
                        pre.append(t[:q1])
                        ph.append(mark)
                        post.append(t[q2:])
                out += [(_lib.PT_TAG_CONST, self._tag_table(x), 0) for x in (pre, ph, post) if any(x)]
            else:
                out += run
            i = j
        self._exp_cache[key] = out
        return out

    def _text_bound(self, prog, obs_max, resp_max):
        """An upper bound on the longest row a program writes, from the host: the constants'
        lengths (a tag table's longest entry), the longest observation and decoded response of
        the turn (rmi_turn_readback), and each number's widest form -> the BPE launch's row size
        with no device round trip.  None when a length it needs is unknown.  (A row past the
        bound would be flagged by the encoder and rebuilt on the host, never mis-encoded.)"""
        n = 0
        for k, a, b in prog:
            if k == _lib.PT_CONST:
                n += b
            elif k == _lib.PT_TAG_CONST:
                n += max(self._tag_tables[a][1::2])
            elif k == _lib.PT_OBS:
                if obs_max is None:
                    return None
                n += obs_max
            elif k == _lib.PT_INT:
                n += 11    # str of an int32
            elif k == _lib.PT_REWARD:
                n += 32    # repr of a double: at most 24 characters; an int reward fewer
            elif k == _lib.PT_RESPONSE:
                if resp_max is None:
                    return None
                # the prefix tag, the text, and llm_response's re-join (" sep " around each of at
                # most K - 1 separators: two spaces each) over the raw answer
                n += len(self.prefix) + resp_max + 2 * self.K + 8
        return n

    def _run_text(self, pieces, stride, obs, obs_len, ints, reward=None, reward_int=None, resp=None, resp_len=None,
                  spans=None, cond=None, active=None, turn=None):
        prog, pool, tc = self._program(pieces)
        self._prog_last = prog  # (the caller's _text_bound)
        flat = [len(prog)] + [x for p in prog for x in p] + [self.n_tags, obs.shape[1], 0 if resp is None else
                                                             resp.shape[1], int(self.enable_think), self.K]
        if turn is None:
            return direct.prompt_text(flat, self.sep, self.n_envs, stride, pool, tc, self.tag, obs,
                                                   obs_len, ints, reward, reward_int, resp, resp_len, spans, cond,
                                                   active)
        ne, flags, last = turn
        return direct.prompt_text(flat, self.sep, self.n_envs, stride, pool, tc, self.tag, obs, obs_len,
                                               ints, reward, None, resp, resp_len, spans, None, active, ne, flags,
                                               self.int_reward_tags, int(last))

    # ------------------------------------------------------------------ rollout steps
    def _obs(self, rows_by_tag):
        """Every env's observation text as one [n_envs, stride] buffer: the device render of the
        tags that have one (``rows_by_tag[j]``), else the env's text at reset."""
        parts, lens = [], []
        st = max([r[0].shape[1] for r in rows_by_tag.values()] + [self._reset_obs[0].shape[1]])
        for j, tg in enumerate(self.es.tags):
            if j in rows_by_tag:
                r, ln = rows_by_tag[j]
            else:
                r, ln = self._reset_obs[0][tg.lo - self.es.env_lo:tg.hi - self.es.env_lo], \
                    self._reset_obs[1][tg.lo - self.es.env_lo:tg.hi - self.es.env_lo]
            parts.append(r if r.shape[1] == st else torch.nn.functional.pad(r, (0, st - r.shape[1])))
            lens.append(ln)
        if len(parts) == 1:
            return parts[0].contiguous(), lens[0].contiguous()
        return torch.cat(parts).contiguous(), torch.cat(lens).contiguous()

    def start(self):
        """After es.reset(): every env's first prompt (ctx_manager.py:248-263 for history[0])."""
        es = self.es
        self.rollout = es.rollout_id
        self.turns_done = 0
        self._pending = None  # a previous rollout's unread host rows: its arena is rebuilt now
        self._next_stats = self._eager_pad = None
        # the reset text of the tags without a device render, as host rows (the others' rows stay
        # empty: their observation comes from render_rows)
        host_tags = [tg for tg in es.tags if not hasattr(tg.batch, "render_rows")]
        if not host_tags:
            # every tag renders on the device: the host rows are all empty -- device zeros, kept
            # across rollouts (two pageable uploads cost ~70 us of host time per reset)
            z = self.__dict__.get("_reset_obs_zero")
            if z is None:
                z = self._reset_obs_zero = (torch.zeros(self.n_envs, 4, dtype=torch.uint8, device=self.device),
                                            torch.zeros(self.n_envs, dtype=torch.int32, device=self.device))
            self._reset_obs_max = 0
            self._reset_obs = z
        else:
            lens = np.zeros(self.n_envs, np.int32)
            rows = []
            for tg in host_tags:
                for i in range(tg.hi - tg.lo):
                    b = tg.batch.render(i).encode("utf-8")
                    rows.append((tg.lo - es.env_lo + i, b))
                    lens[tg.lo - es.env_lo + i] = len(b)
            st = max(4, (int(lens.max()) + 3) // 4 * 4)
            self._reset_obs_max = int(lens.max()) if lens.size else 0
            buf = np.zeros((self.n_envs, st), np.uint8)
            for e, b in rows:
                buf[e, :len(b)] = np.frombuffer(b, np.uint8)
            self._reset_obs = (torch.from_numpy(buf).to(self.device), torch.from_numpy(lens).to(self.device))
        rr = getattr(es, "reset_render", None)  # the rows es.reset rendered, when it did
        rows = rr[1] if rr is not None and rr[0] == es.rollout_id else \
            {j: tg.batch.render_rows() for j, tg in enumerate(es.tags) if hasattr(tg.batch, "render_rows")}
        obs, obs_len = self._obs(rows)
        ints = self.mapt.clone()
        self.len.zero_()
        if self.window:  # rows are rebuilt per batch from the turn records (_build_window)
            self._obs0 = (obs, obs_len, ints)
            self.len_upd.zero_()
            return
        text, tlen, terr, stride = self._first_text(obs, obs_len, ints)
        # the BPE launch's row size from the host's bound (no device round trip for the longest
        # row; None when a length it needs is unknown: then the longest row is read back)
        bound = self._text_bound(self._prog_last, self._obs_bound(rows), None) if self.first_bound else None
        self._encode(text, tlen, terr, None, stride, lambda e: self._host_first(e), bound=bound)
        self.len_upd.copy_(self.len)

    def _first_text(self, obs, obs_len, ints, active=None):
        """The first user block (system + instruction prefix + ``Turn 1`` + the state; at reset,
        and as the first kept entry of a window) -> (text, len, err, stride)."""
        pieces = [self.tpl.head, (_lib.PT_TAG_CONST, 0, 0), "\nTurn 1:\nState:\n", (_lib.PT_OBS, 0, 0),
                  "\nYou have ", (_lib.PT_INT, 0, 0), self._c_mid, (_lib.PT_TAG_CONST, 1, 0), "\n" + self.tpl.u_suf]
        stride = self._stride(obs.shape[1] + self._max_prefix + 1024)
        text, tlen, _, terr = self._run_text(pieces, stride, obs, obs_len, ints, active=active)
        return text, tlen, terr, stride

    def advance(self, d, bounds=None, merge=False, stats=None):
        """Append turn d["turn"] (a device-path turn record of EnvStateManager._step_device).
        bounds: (longest observation, longest response) in bytes when the record does not carry
        them yet (advance_eager); merge: the rows of a turn's second pass (their host rows join
        the first pass's, unresolved)."""
        t = d["turn"]
        if self.window:  # window mode: the rows are rebuilt per batch (_build_window)
            self.turns_done = t + 1
            return
        text, tlen, mark, terr, stride, last, flags, bound = self._turn_text(d, t + 2, d["has"], bounds)
        self._encode(text, tlen, terr, mark, stride,
                     lambda e: self._host_turn(e, t, not last and not int(flags[e]) & _lib.FLAG_DONE),
                     active=d["has"], bound=bound, merge=merge, stats=stats)
        self.turns_done = t + 1

    def advance_eager(self, d, stats, has_next=None, again=False) -> bool:
        """Turn d's append launched from inside the turn (EnvStateManager._step_device), BEFORE the
        turn's readback: the row sizes come from host bounds (the longest generation's raw bytes,
        rmi_gen_rows; each env type's widest render row) instead of the readback's exact maxima
        (a row past them is flagged by the encoder and built on the host, never mis-encoded),
        and rmi_next_rows_stats writes the next generation batch's longest row, whether a row
        waits for the host and the row count into ``stats`` (inside the readback buffer) -- so
        gen_batch needs no readback of its own.  has_next: the envs that had a generation this
        turn (default d["has"]); again: d is the turn's second pass (the envs whose generation
        overflowed the first pass's decode), appended after the first.  -> False when it does
        not apply (window mode, a stale rollout, unknown bounds): the prompt is then appended at
        the next get_lm_inputs."""
        es = self.es
        t = d["turn"]
        if self.window or self.rollout != es.rollout_id or self.turns_done != (t + 1 if again else t):
            return False
        inp = d["inp"]
        # a generation's decoded length: at most the decode's row (rows past it were not stepped)
        resp_max = inp.raw_max if inp.raw_max is not None else inp.stride
        obs_max = self._obs_bound(d["obs"])
        if obs_max is None and not again:
            return False
        has_n = d["has"] if has_next is None else has_next
        # the first pass: the commit and the next batch's stats in one launch (the rows the
        # commit flags are the only pending ones: an earlier turn's were resolved first)
        self.advance(d, bounds=(obs_max, resp_max), merge=again, stats=None if again else (has_n, d["flags"], stats))
        self.eager_turns += 0 if again else 1
        if again:
            pend = self._pending[0] if self._pending is not None else None
            ops.next_rows_stats(self.len, has_n, d["flags"], pend, stats)
        self._next_stats = None
        return True

    def set_next_stats(self, turn, vals, env_ids):
        """advance_eager's stats as read back with the turn: (turns done, longest row, any host
        row, row count, the env-id array they were counted over -- EnvStateManager hands that
        very array out; gen_batch takes the stats only for it)."""
        self._next_stats = (turn + 1, int(vals[0]), int(vals[1]), int(vals[2]), env_ids)

    def _obs_bound(self, rows_by_tag):
        """The widest observation row (bytes) this turn's rows can hold, from the host: each
        rendering tag's bound (its batch's obs_bound), the reset text of the others."""
        b = self._reset_obs_max
        for j, tg in enumerate(self.es.tags):
            if j in rows_by_tag:
                f = getattr(tg.batch, "obs_bound", None)
                x = f() if f is not None else None
                if x is None:
                    return None
                b = max(b, int(x))
        return b

    def _turn_text(self, d, number, active, bounds=None):
        """The text turn d["turn"] appends: the assistant block (its end marked: the update rows
        stop there) and, for an env that goes on, the user block with the reward and the next
        state under the header ``Turn {number}``.  -> (text, len, mark, err, stride, last, flags,
        the host's bound on the longest row or None)."""
        t = d["turn"]
        inp = d["inp"]
        obs, obs_len = self._obs(d["obs"])
        resp, resp_len = inp.text, inp.text_len
        spans = torch.cat(d["spans"]) if len(d["spans"]) > 1 else d["spans"][0]
        eps = [tg.batch.ep for tg in self.es.tags]
        cat = (lambda xs: torch.cat(xs)) if len(eps) > 1 else (lambda xs: xs[0])  # noqa: E731
        reward = cat([ep.turn_reward[t] for ep in eps]).contiguous()
        ne = cat([ep.turn_exec[t] for ep in eps]).contiguous()
        # the reward's int form and the next block's condition come from the turn record on the
        # device (the prompt op's turn form): turn_exec, flags, the Countdown tags, the last turn
        flags = d["flags"]
        ints = d["left"]
        pieces, last = self.turn_pieces(t, number)
        obs_max, resp_max = bounds if bounds is not None else (d.get("obs_max"), d.get("text_max"))
        # the text rows sized from the host's bound on the longest row when it has one (the
        # kernel's LDS grows with the row: a tight row keeps more waves resident); a row past it
        # is flagged by the kernel and built on the host
        bound = self._text_bound(self._program(pieces)[0], obs_max, resp_max)
        stride = self._stride(bound + 4) if bound is not None else self._stride(resp.shape[1] + obs.shape[1] + 1024)
        text, tlen, mark, terr = self._run_text(pieces, stride, obs, obs_len, ints, reward, None, resp,
                                                resp_len, spans, None, active, turn=(ne, flags, last))
        return text, tlen, mark, terr, stride, last, flags, bound

    def turn_pieces(self, t, number):
        """The program of the text turn t appends (the assistant block, its end marked, then --
        unless the env is done or t is the rollout's last turn -- the user block with the reward
        and the state under ``Turn {number}``): -> (pieces, last turn)."""
        pieces = [self.tpl.a_pre, (_lib.PT_RESPONSE, 0, 0), self.tpl.a_suf, (_lib.PT_MARK, 0, 0),
                  (_lib.PT_IF, 0, 0), self.tpl.u_pre + "Reward:\n", (_lib.PT_REWARD, 0, 0),
                  f"\n\nTurn {number}:\nState:\n", (_lib.PT_OBS, 0, 0), "\nYou have ", (_lib.PT_INT, 0, 0),
                  self._c_mid, (_lib.PT_TAG_CONST, 1, 0), "\n" + self.tpl.u_suf]
        return pieces, t + 1 >= self.max_turn

    # ----------------------------------------------------------- max_context_window
    def _entry_state(self, j):
        """(obs, obs_len, actions_left) of history entry j: the reset's, or the turn j-1 record's."""
        if j == 0:
            return self._obs0
        d = self.es._turn_records[j - 1]
        obs, obs_len = self._obs(d["obs"])
        return obs, obs_len, d["left"]

    def _build_window(self, sel, n_done, update):
        """Rebuild the arena rows of the envs in ``sel`` (u8/bool[n_envs] on the device), every one
        with ``n_done`` completed turns, as their last-k history window (ctx_manager.py:244-246):
        generation rows keep entries 0..n_done (the last holds the current state only), update
        rows entries 0..n_done-1 (prepare_for_update drops the last state, :240-241).  The
        kept entries are renumbered ``Turn 1..``.  Rows a kernel flags are rebuilt on the host."""
        k = self.window
        n_entries = n_done if update else n_done + 1
        j0 = max(0, n_entries - k)
        sel = sel.to(torch.uint8)
        keep = sel == 0
        self.len.copy_(torch.where(keep, self.len, torch.zeros_like(self.len)))
        self.len_upd_w = self.len_upd.clone()  # the marks this rebuild records
        obs, obs_len, ints = self._entry_state(j0)
        text, tlen, terr, stride = self._first_text(obs, obs_len, ints, active=sel)
        bad = self._encode_window(text, tlen, terr, None, stride, sel)
        for j in range(j0, n_done):
            d = self.es._turn_records[j]
            act = sel & d["has"].to(torch.uint8) if d["has"] is not None else sel
            text, tlen, mark, terr, stride, _, _, _ = self._turn_text(d, j - j0 + 2, act)
            bad |= self._encode_window(text, tlen, terr, mark, stride, act)
        if update:
            self.len_upd.copy_(torch.where(keep, self.len_upd, self.len_upd_w))
        if bool(bad.any()):
            idx = torch.nonzero(bad).flatten().cpu().tolist()
            self.host_rows_used += len(idx)
            warnings.warn(f"{len(idx)} prompt rows built on the host (text past the device row buffer, an NFC-changing "
                          "code point, or an unsupported reward)", RuntimeWarning)
            for e in idx:
                self._host_window(e, update)

    def _encode_window(self, text, tlen, terr, mark, stride, active):
        """Append one block of a window rebuild; -> the rows the device could not build."""
        mx = int(tlen.max()) if tlen.numel() else 0
        n_tok, mark_tok, err = self.dt.encode_rows(text, tlen, self.arena, self.len, mark, max_len=max(mx, 4))
        if mark is not None:
            self.len_upd_w = torch.where(active.bool(), mark_tok, self.len_upd_w)
        return ((err != 0) | (terr != 0)) & active.bool()

    def _host_window(self, e, update):
        """Env e's window row tokenized on the host: the reference's messages for its history
        (ContextManager._build_messages applies max_context_window), the generation tail cut off
        (pad_rows appends it) -- or, for an update row, the whole text."""
        self.es._materialize()
        entry = dict(self.es.rollout_cache[e])
        entry["history"] = list(entry["history"])
        texts, _ = self.ctx._build_messages([entry], update)
        ids = self._host_ids(texts[0])
        if not update:
            tail = self.tail.tolist()
            if ids[-len(tail):] != tail:
                raise RuntimeError("the host prompt does not end with the generation tail")
            ids = ids[:-len(tail)]
        if len(ids) > self.cap:
            raise RuntimeError(f"env {e}: prompt longer than the device arena ({self.cap} tokens)")
        self.arena[e, :len(ids)] = torch.tensor(ids, dtype=torch.int64, device=self.device)
        self.len[e] = len(ids)
        if update:
            self.len_upd[e] = len(ids)

    @staticmethod
    def _stride(n):
        return min(3072, (int(n) + 3) // 4 * 4)

    def _encode(self, text, tlen, terr, mark, stride, host_fn, active=None, bound=None, merge=False, stats=None):
        """Tokenize the rows onto the arena; the rows the device could not build are left for
        the host (``_resolve``), read back with the next readback of the arena lengths.  The
        launch's row size is ``bound`` (the host's, _text_bound) when given, else the longest
        row read back.  merge: other rows of the same turn (its second pass): the pending host
        rows stay pending and are joined by these."""
        prev = self._pending if merge else None
        if not merge:
            self._resolve()  # an earlier turn's host rows come first in the arena
        if bound is not None:
            mx = min(int(bound), text.shape[1])
        else:
            mx = int(tlen.max()) if tlen.numel() else 0
        n_tok, mark_tok, err = self.dt.encode_rows(text, tlen, self.arena, self.len, mark,
                                                   max_len=max((mx + 3) // 4 * 4, 4))
        # the rows left for the host and the update batch's row ends (after the assistant block):
        # one launch (rmi_prompt_commit)
        bad = torch.empty(self.n_envs, dtype=torch.uint8, device=self.device)
        act = None if active is None else (active if active.dtype == torch.uint8 else active.to(torch.uint8))
        if stats is not None and prev is None:  # (has, flags, out): rmi_next_rows_stats fused in
            ops.prompt_commit_stats(err, terr, act, mark_tok if mark is not None else None, self.len_upd, bad,
                                    self.len, stats[0], stats[1], stats[2])
        else:
            ops.prompt_commit(err, terr, act, mark_tok if mark is not None else None, self.len_upd, bad)
        if prev is not None:
            bad = bad | prev[0]
        self._pending = (bad, host_fn)

    def _resolve(self, any_bad=None):
        """Build the pending host rows (``any_bad``: their any() already read back)."""
        if self._pending is None:
            return
        bad, host_fn = self._pending
        self._pending = None
        if any_bad is False:
            return
        if any_bad is None:  # read the any() first (one small kernel): nonzero() is a sort-based pass
            stats = torch.empty(2, dtype=torch.int32, device=self.device)
            ops.rows_stats(self.len, None, 0, bad, stats)
            if not int(ops.d2h(stats, self)[1]):
                return
        idx = torch.nonzero(bad).flatten().cpu().tolist()
        if idx:
            self.host_rows_used += len(idx)
            warnings.warn(f"{len(idx)} prompt rows built on the host (text past the device row buffer, an NFC-changing "
                          "code point, or an unsupported reward)", RuntimeWarning)
            for e in idx:
                host_fn(e)

    # ---------------------------------------------------------------- host rows
    def _write_host(self, e, ids_a, ids_b=None):
        """Append ids for env e (a host-tokenized row); ids_b after the update mark."""
        cur = int(self.len[e])
        ids = list(ids_a) + list(ids_b or [])
        if cur + len(ids) > self.cap:
            raise RuntimeError(f"env {e}: prompt longer than the device arena ({self.cap} tokens)")
        self.arena[e, cur:cur + len(ids)] = torch.tensor(ids, dtype=torch.int64, device=self.device)
        self.len[e] = cur + len(ids)
        if ids_b is not None:
            self.len_upd[e] = cur + len(ids_a)

    def _host_first(self, e):
        g = self.es.env_lo + e
        cache = self.es.rollout_cache[e]
        ap = self.ctx.config.agent_proxy
        h = cache["history"][0]
        length = f"Max response length: {self.ctx.env_config_lookup[g]['max_tokens']} words (tokens)."
        text = (self.tpl.head + self.ctx.prefix_lookup[g] + f"\nTurn 1:\nState:\n{h['state']}\nYou have "
                f"{h['actions_left']}" + self._c_mid + length + "\n" + self.tpl.u_suf)
        del ap
        self._write_host(e, self._host_ids(text))

    def host_turn_text(self, e, t, cont):
        """The text turn t appends to env e's prompt, built on the host from its history
        (ctx_manager.py:248-263 under the chat template): (assistant block, user block or "")."""
        self.es._materialize()
        g = self.es.env_lo + e
        hist = self.es.rollout_cache[e]["history"]
        h = hist[t]
        a = self.tpl.a_pre + h["llm_response"] + self.tpl.a_suf
        b = ""
        if cont:
            nxt = hist[t + 1]
            length = f"Max response length: {self.ctx.env_config_lookup[g]['max_tokens']} words (tokens)."
            b = (self.tpl.u_pre + f"Reward:\n{h['reward']}\n\nTurn {t + 2}:\nState:\n{nxt['state']}\n"
                 f"You have {nxt['actions_left']}" + self._c_mid + length + "\n" + self.tpl.u_suf)
        return a, b

    def _host_turn(self, e, t, cont):
        a, b = self.host_turn_text(e, t, cont)
        self._write_host(e, self._host_ids(a), self._host_ids(b) if cont else [])

    # ------------------------------------------------------------------- batches
    def gen_batch(self, env_ids: np.ndarray):
        """get_lm_inputs(prepare_for_update=False)'s tensors for these envs (device)."""
        nr = self.es.__dict__.get("_next_rows")
        asc = True  # rows ascending (a device-resident actor may take them as its gather index)
        if nr is not None and env_ids is nr[0]:  # the ids the last turn handed out: their rows are on the device
            rows = nr[1][:len(env_ids)]
        elif env_ids is self.es._ids_in_order:
            rows = self._all_rows
        else:
            local = np.asarray(env_ids, np.int64) - self.es.env_lo
            if len(local) == self.n_envs and np.array_equal(local, self._all_idx):
                rows = self._all_rows  # every env in order (no host -> device copy)
            else:
                rows = ops.h2d(local, self.device)
                asc = False
        self.last_rows = rows if asc else None
        if self.window and rows.numel():  # every active env has the same turn count
            sel = torch.zeros(self.n_envs, dtype=torch.uint8, device=self.device)
            sel[rows] = 1
            self._build_window(sel, self.turns_done, update=False)
        if not rows.numel():
            self._resolve()
            S = 1
        else:
            ns, self._next_stats = self._next_stats, None
            if ns is not None and ns[0] == self.turns_done and ns[4] is env_ids and ns[3] == rows.numel():
                # the stats came with the turn's readback (advance_eager) for exactly these env
                # ids (the array the turn handed out: the envs that went on, the ones it counted)
                mx, any_bad = ns[1], ns[2]
                self._resolve(bool(any_bad))
            else:  # one readback: the longest row and whether any row is the host's (rmi_rows_stats)
                stats = torch.empty(2, dtype=torch.int32, device=self.device)
                pend = self._pending[0] if self._pending is not None else None
                ops.rows_stats(self.len, rows, rows.numel(), pend, stats)
                mx, any_bad = (int(x) for x in ops.d2h(stats, self))
                if pend is not None:
                    self._resolve(bool(any_bad))
            if any_bad:  # host rows were written: the longest row again
                stats = torch.empty(2, dtype=torch.int32, device=self.device)
                ops.rows_stats(self.len, rows, rows.numel(), None, stats)
                mx = int(ops.d2h(stats, self)[0])
            S = mx + self.tail.numel()
        ep, self._eager_pad = self._eager_pad, None
        if (ep is not None and nr is not None and env_ids is nr[0] and rows.numel() and not any_bad
                and ep[0] == (self.rollout, self.turns_done) and ep[1] == S and ep[2] == rows.numel()):
            # padded by the turn chain right after its readback (the same rmi_pad_rows launch
            # over the same rows, width and block: TurnChain.run)
            n = rows.numel()
            blk = ep[3]
            P = (n * S + 1) & ~1  # the outputs at k * P (rmi_turn_chain's step 8)
            ids, am, pos = (blk.as_strided((n, S), (S, 1), blk.storage_offset() + k * P) for k in range(3))
            err = ep[4][:n]
            self.chain_padded += 1
        else:
            ids, am, pos, err = self._pad_rows(rows, S)
        if rows.numel():  # rows longer than S would be left-cut: counted into the next turn's readback
            self.ctx._pad_pending = (self.ctx.turn_packs()[0], err)
        return {"input_ids": ids, "attention_mask": am, "position_ids": pos, "responses": ids[:, 1:]}

    def batch_block(self, slot, n=None, S=None):
        """The output block (i64, >= 3 n S) and error bytes of turn number ``slot``'s generation
        batch: the block the previous batch of that turn number used when nothing outside holds
        it any more (its storage's use count), else a fresh one with room for every env's row at
        1.25 S (the turn chain pads the next rollout's batch of this turn number into it: its row
        count varies with the envs done, its width a little with the rooms).  n=None: the free
        block as it is, or None when there is none (TurnChain.run)."""
        # (each block kept with its storage object: the use count of a held storage is the
        # block, that object and any view; untyped_storage() per check cost ~2 us)
        buf, err, bst, est = self._batch_bufs.get(slot, (None, None, None, None))
        if n is None:
            if buf is None or _uses(bst) > 2 or _uses(est) > 2:
                return None
            return buf, err
        if buf is None or buf.numel() < 3 * (n * S + 1) or _uses(bst) > 2:
            buf = torch.empty(3 * (max(n, self.n_envs) * (S + S // 4) + 1), dtype=torch.int64, device=self.device)
            bst = buf.untyped_storage()
        if err is None or _uses(est) > 2:
            err = torch.empty(self.n_envs, dtype=torch.uint8, device=self.device)
            est = err.untyped_storage()
        self._batch_bufs[slot] = (buf, err, bst, est)
        return buf, err

    def _pad_rows(self, rows, S):
        """rmi_pad_rows into the batch's own tensors (ops.pad_rows without its argument checks:
        every operand is this builder's).  The outputs are views of one block at k * P (P = n S
        rounded up to even); the block the
        previous batch of the same shape class used is taken again when nothing outside holds
        it any more (its storage's use count), else a fresh one is allocated."""
        n = rows.numel()
        P = (n * S + 1) & ~1  # the three outputs at k * P: 16-B aligned alike (rmi_pad_rows' column pairs)
        buf, err = self.batch_block(self.turns_done, n, S)
        ids, am, pos = (buf[k * P:k * P + n * S].view(n, S) for k in range(3))
        err = err[:n]
        ops.check(_lib.lib().rmi_pad_rows(self.arena_p, self.arena_stride, self.len_p, rows.data_ptr(), n,
                                          self.tail_p, self.tail_n, int(S), int(self.pad_id), ids.data_ptr(),
                                          am.data_ptr(), pos.data_ptr(), err.data_ptr(), ops._stream(self.device)),
                  "rmi_pad_rows")
        return ids, am, pos, err

    def update_rows(self, resolve=True):
        """(tokens, row_start, row_len) of formulate_rollouts' rows, env order.  resolve=False:
        pending host rows stay pending (the caller reads their any() with its own readback and
        calls _resolve)."""
        if resolve or self.window:
            self._resolve()
        if self.window:  # each env's last k complete entries: envs grouped by their turn count
            eps = [tg.batch.ep for tg in self.es.tags]
            n_t = (eps[0].n_turns if len(eps) == 1 else torch.cat([ep.n_turns for ep in eps])).to(torch.int32)
            for n in sorted(set(n_t.cpu().tolist())):
                if n > 0:
                    self._build_window(n_t == n, int(n), update=True)
        if getattr(self, "_row_start", None) is None:
            self._row_start = torch.arange(self.n_envs, dtype=torch.int64, device=self.device) * self.cap
        return self.arena.view(-1), self._row_start, self.len_upd

    # ------------------------------------------------------------------ self-check
    def _verify(self):
        """The concatenation rule on a probe conversation, against the host tokenizer."""
        fmt = self._c_mid
        first = "instr\nTurn 1:\nState:\n#_P#\nYou have 9" + fmt + "x.\n"
        resp = "<think>a b</think><answer>Up || Down</answer>"
        user2 = "Reward:\n-0.1\n\nTurn 2:\nState:\n#P_#\nYou have 7" + fmt + "x.\n"
        parts = [self.tpl.head + first + self.tpl.u_suf, self.tpl.a_pre + resp + self.tpl.a_suf,
                 self.tpl.u_pre + user2 + self.tpl.u_suf, self.tpl.gen + self.prefix]
        whole = self._host_ids("".join(parts))
        pieces: List[int] = []
        for p in parts:
            pieces += self._host_ids(p)
        if whole != pieces:
            raise NotImplementedError("the tokenizer does not split the chat template at its blocks")
