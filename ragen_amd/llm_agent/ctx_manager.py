"""ContextManager — drop-in for ragen/llm_agent/ctx_manager.py:74-356.

Text in/out stays on the host (prompt building, tokenizer, response regex: the LLM owns
those bytes).  The numeric hot path runs on the GPU engine:
  * ``get_masks_and_scores`` (ctx_manager.py:35-70) as torch device ops on the token ids
    (cumsum / compare / scatter on the GPU tensor);
  * ``_normalize_score_tensor`` (ctx_manager.py:175-226) through rmi_group_normalize;
  * trajectory scores come straight from the device episode record when the rollout came
    from this package's EnvStateManager.
"""
import re
import warnings
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import _lib, ops
from ..env import REGISTERED_ENV_CONFIGS
from ..torch_ops import NORM, direct
from ..protocol import DataProto


def get_special_tokens(tokenizer):
    """ctx_manager.py:24-33."""
    if "qwen" in tokenizer.name_or_path.lower():
        return tokenizer.encode("<|im_start|>")[0], tokenizer.encode("<|im_end|>")[0]
    if "llama-3" in tokenizer.name_or_path.lower():
        return 128006, 128009
    raise ValueError(f"Unsupported model: {tokenizer.name_or_path}")


def _score_table(all_scores, B, dev):
    """all_scores (per row a list of turn rewards) -> (f64[T, B] turn-major, i32[B] lengths, T)."""
    all_scores = all_scores if all_scores is not None else [[] for _ in range(B)]
    n = [len(x) for x in all_scores]
    T = max(n) if n else 0
    tab = np.zeros((max(T, 1), B), np.float64)
    for b, row in enumerate(all_scores):
        tab[:len(row), b] = row
    return torch.from_numpy(tab).to(dev), torch.tensor(n, dtype=torch.int32, device=dev), T


def get_masks_and_scores(input_ids: torch.Tensor, tokenizer, all_scores: List[List[float]] = None,
                         use_turn_scores: bool = False, enable_response_mask: bool = False):
    """ctx_manager.py:35-70 on the device holding ``input_ids``: one HIP kernel
    (rmi_masks_and_scores) — turn prefix scan, both masks, score placement incl. the Qwen roll
    and the last-column fallback.  Raises RuntimeError where the reference's boolean-mask
    assignment would (a turn with more than one reward-token position)."""
    special_token, reward_token = get_special_tokens(tokenizer)
    B = input_ids.shape[0]
    dev = input_ids.device
    tab, n, T = _score_table(all_scores, B, dev)
    score, lm, rm, err = torch.ops.ragen_amd.masks_and_scores(
        input_ids.to(torch.int64).contiguous(), int(special_token), int(reward_token), tab, n, T,
        bool(use_turn_scores), bool(enable_response_mask), "qwen" in tokenizer.name_or_path.lower())
    if use_turn_scores and bool(err.any()):
        raise RuntimeError("shape mismatch: a turn has more than one reward-token position "
                           "(reference score_tensor[reward_position] = scores)")
    return score, lm, rm


def assemble_batch(rows, tokenizer, all_scores, use_turn_scores: bool, enable_response_mask: bool, device, S=None):
    """The tokenizer's left-padded batch + attention_mask + position_ids (ctx_manager.py:278-306)
    and get_masks_and_scores on it, from ragged token rows (lists / arrays of ids), in one device
    pass (rmi_assemble_batch).  -> device tensors (input_ids, attention_mask, position_ids,
    score, loss_mask, response_mask)."""
    special_token, reward_token = get_special_tokens(tokenizer)
    lens = np.array([len(r) for r in rows], np.int64)
    B = len(rows)
    off = np.zeros(B + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    flat = np.concatenate([np.asarray(r, np.int64) for r in rows]) if B else np.zeros(0, np.int64)
    S = (int(lens.max()) if B else 0) if S is None else int(S)  # the tokenizer pads to the longest row
    pad = tokenizer.pad_token_id if getattr(tokenizer, "pad_token_id", None) is not None else 0
    tab, n, T = _score_table(all_scores, B, device)
    out = torch.ops.ragen_amd.assemble_batch(
        torch.from_numpy(flat if flat.size else np.zeros(1, np.int64)).to(device), torch.from_numpy(off).to(device),
        S, int(pad), int(special_token), int(reward_token), tab, n, T, bool(use_turn_scores),
        bool(enable_response_mask), "qwen" in tokenizer.name_or_path.lower())
    ids, am, pos, score, lm, rm, err = out
    _raise_assemble_errors(err, S)
    return ids, am, pos, score, lm, rm


def _raise_assemble_errors(err, S, bits=None):
    """rmi_assemble_batch's per-row bits: RMI_ERR_UNSUP = a row longer than the batch width S
    (it would have been truncated), RMI_ERR_STATE = a turn with more than one reward-token
    position (the reference's boolean-mask score assignment raises there)."""
    overlong, multi = bits if bits is not None else \
        torch.stack([(err & _lib.ERR_UNSUP).any(), (err & _lib.ERR_STATE).any()]).cpu().tolist()
    if overlong:
        raise ValueError(f"a token row is longer than the batch width S={S}")
    if multi:
        raise RuntimeError("shape mismatch: a turn has more than one reward-token position "
                           "(reference score_tensor[reward_position] = scores)")


SPECIAL_TOKENS = ["<think>", "</think>", "<answer>", "</answer>", "<|im_start|>", "<|im_end|>"]
PARSE_MAX_ROW = 8192  # rmi_parse_actions' row limit (bytes of a decoded generation)


def decode_stride(raw: int, factor: int) -> int:
    """The decode's row (bytes): factor x raw, whole dwords, within the parse's row limit."""
    return max(4, min(PARSE_MAX_ROW, (factor * int(raw) + 7) // 4 * 4))


def parse_response(response: str, enable_think: bool, action_sep: str, max_actions_per_turn: int):
    """ContextManager._parse_response (ctx_manager.py:148-173) as a function of the agent_proxy
    settings: -> (llm_response, actions).  The device path (rmi_parse_actions) computes the
    same actions; this host form rebuilds the history strings when a device-path rollout is
    materialised (EnvStateManager._materialize)."""
    pattern = r"<think>(.*?)</think>\s*<answer>(.*?)</answer>" if enable_think else r"<answer>(.*?)</answer>"
    match = re.search(pattern, response, re.DOTALL)
    if not match:
        return response, []
    think_content, action_content = (match.group(1), match.group(2)) if enable_think else ("", match.group(1))
    for tok in SPECIAL_TOKENS:
        action_content = action_content.replace(tok, "").strip()
        think_content = think_content.replace(tok, "").strip()
    actions = [a.strip() for a in action_content.split(action_sep) if a.strip()]
    if len(actions) > max_actions_per_turn:
        actions = actions[:max_actions_per_turn]
        action_content = (" " + action_sep + " ").join(actions)
    llm_response = (f"<think>{think_content}</think><answer>{action_content}</answer>" if enable_think
                    else f"<answer>{action_content}</answer>")
    return llm_response, actions


def parse_response_spans(raw: str, span, enable_think: bool, action_sep: str, max_actions_per_turn: int):
    """parse_response with the regex match taken from the device parse (rmi_parse_actions'
    spans: think [start, end), answer [start, end) in the UTF-8 bytes of ``raw``, -1 = no
    match; tested against the reference's match on every parse vector).  The rest is
    parse_response's own string code; a content holding a '<' runs the special-token cascade,
    any other content only needs its strip (the cascade is a no-op on it)."""
    ts, te, a0, a1 = (int(x) for x in span)
    if a0 < 0:
        return raw, []
    rb = raw.encode("utf-8")
    think_content = rb[ts:te].decode("utf-8") if enable_think else ""
    action_content = rb[a0:a1].decode("utf-8")
    if "<" in action_content or "<" in think_content:
        for tok in SPECIAL_TOKENS:
            action_content = action_content.replace(tok, "").strip()
            think_content = think_content.replace(tok, "").strip()
    else:
        action_content = action_content.strip()
        think_content = think_content.strip()
    actions = [a.strip() for a in action_content.split(action_sep) if a.strip()]
    if len(actions) > max_actions_per_turn:
        actions = actions[:max_actions_per_turn]
        action_content = (" " + action_sep + " ").join(actions)
    llm_response = (f"<think>{think_content}</think><answer>{action_content}</answer>" if enable_think
                    else f"<answer>{action_content}</answer>")
    return llm_response, actions


def segments_for(grouping: str, env_outputs: List[Dict]):
    """Group ids of ctx_manager.py:184-191 as contiguous segments (first-seen order)."""
    if grouping == "state":
        tags = [o["group_id"] for o in env_outputs]
    elif grouping == "inductive":
        tags = [o["tag"] for o in env_outputs]
    elif grouping == "batch":
        tags = [1] * len(env_outputs)
    else:
        raise ValueError(f"Invalid grouping: {grouping}")
    order, seen = {}, []
    for i, t in enumerate(tags):
        if t not in order:
            order[t] = []
            seen.append(t)
        order[t].append(i)
    perm = np.concatenate([np.asarray(order[t], np.int64) for t in seen]) if tags else np.zeros(0, np.int64)
    seg = np.zeros(len(seen) + 1, np.int32)
    seg[1:] = np.cumsum([len(order[t]) for t in seen])
    return perm, seg


def tag_segments(tags, n_groups, group_size: int):
    """The "inductive" grouping (ctx_manager.py:184-191: one group per tag NAME, first-seen
    order) over the env order the config's entries lay down (entry i owns n_groups[i] *
    group_size contiguous envs).  A tag listed more than once gathers all of its entries' envs.
    -> (perm i64[B] or None when every tag's envs are already contiguous, seg i32[n_tags+1]);
    equal to segments_for("inductive", ...) on the per-env tags."""
    first = {}
    for t in tags:
        first.setdefault(t, len(first))
    sizes = [int(n) * int(group_size) for n in n_groups]
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    order = sorted(range(len(sizes)), key=lambda i: first[tags[i]])  # stable: config order within a tag
    per_tag = np.zeros(len(first), np.int64)
    for i, t in enumerate(tags):
        per_tag[first[t]] += sizes[i]
    seg = np.concatenate([[0], np.cumsum(per_tag)]).astype(np.int32)
    if order == list(range(len(sizes))):
        return None, seg
    perm = np.concatenate([np.arange(starts[i], starts[i + 1]) for i in order]) if order else np.zeros(0, np.int64)
    return perm.astype(np.int64), seg


class DeviceEnvInputs:
    """What ``get_env_inputs`` returns on the device path: the generations of the active envs as
    token ids of the FULL env batch (rows of envs without a generation are empty and carry no
    input), decoded on the device (rmi_detokenize, = batch_decode(skip_special_tokens=True),
    ctx_manager.py:334-337) into UTF-8 rows — by EnvStateManager.step's device turn, fused with
    the parse (rmi_detok_parse), or on first access to ``text`` / ``text_len`` / ``err``.
    Iterating it yields the reference's env-input dicts (host decode + parse), built lazily."""

    def __init__(self, ctx, env_ids, has_t, ids, n_ids, stride):
        # has_t: u8[n_envs] 1 for the envs with a generation (device), None = every env in order
        self.ctx, self.env_ids, self._has_t = ctx, env_ids, has_t
        self._ids, self._n_ids, self.stride = ids, n_ids, stride
        self.raw_max = None  # host int: the longest generation's raw bytes, when known
        self.raw_dev = None  # the same on the device (i32[1], rmi_gen_rows)
        self.raw_next = None  # the other readback buffer's raw slot (rmi_gen_rows_chained zeroes it)
        self.pack = None     # the turn's readback buffer raw_dev lives in
        # (resp, src host array or None, src on the device or None): the generations not yet
        # scattered onto the envs -- the turn's first launch does it (llm_agent/turn_chain.py),
        # or flush() on first use
        self.pending_gen = None
        self.pad_counted, self.pad_err = False, None  # the generation batch's error bytes (gen_batch)
        self.vocab = ctx.device_vocab
        self._text = self._text_len = self._err = None
        self._decoded = None

    def flush(self):
        """Launch the deferred rmi_gen_rows (the step-by-step path, or a reader before the turn)."""
        if self.pending_gen is None:
            return
        resp, src, src_dev = self.pending_gen
        self.pending_gen = None
        n, dev, v = self.ctx.n_envs, resp.device, self.vocab
        if src is None and src_dev is None:
            direct.gen_rows(resp, None, n, v.packed, None, None, self.raw_dev, None, self.raw_next)
            self._ids, self._n_ids, self._has_t = resp, None, None
            return
        R = resp.shape[1]
        self._ids = torch.empty(n, R, dtype=torch.int64, device=dev)
        self._n_ids = torch.empty(n, dtype=torch.int32, device=dev)
        self._has_t = torch.empty(n, dtype=torch.uint8, device=dev)
        direct.gen_rows(resp, src_dev if src_dev is not None else ops.h2d(src, dev), n, v.packed, self._ids,
                        self._n_ids, self.raw_dev, self._has_t, self.raw_next)

    @property
    def ids(self):
        self.flush()
        return self._ids

    @ids.setter
    def ids(self, v):
        self._ids = v

    @property
    def n_ids(self):
        self.flush()
        return self._n_ids

    @n_ids.setter
    def n_ids(self, v):
        self._n_ids = v

    @property
    def has_t(self):
        self.flush()
        return self._has_t

    @has_t.setter
    def has_t(self, v):
        self._has_t = v

    def set_decoded(self, text, text_len, err):
        self._text, self._text_len, self._err = text, text_len, err

    @property
    def is_decoded(self):
        return self._text is not None

    def _ensure(self):
        if self._text is None:
            v = self.vocab
            self.set_decoded(*torch.ops.ragen_amd.detokenize(self.ids, self.n_ids, v.packed, v.data, self.stride))

    @property
    def text(self):
        self._ensure()
        return self._text

    @property
    def text_len(self):
        self._ensure()
        return self._text_len

    @property
    def err(self):
        self._ensure()
        return self._err

    def __len__(self):
        return len(self.env_ids)

    def decoded(self):
        """-> list[str] of every env's decoded generation (host copy; index = env id)."""
        if self._decoded is None:
            if bool(self.err.any()):
                raise ValueError("a decoded generation exceeded the device row buffer (rmi_detokenize RMI_ERR_UNSUP)")
            self._decoded = ops.decode_rows(self.text, self.text_len)
        return self._decoded

    def __iter__(self):
        ap = self.ctx.config.agent_proxy
        prefix = "<think>" if ap.enable_think else "<answer>"
        texts = self.decoded()
        for e in self.env_ids:
            raw = prefix + texts[int(e)]
            llm_response, actions = parse_response(raw, ap.enable_think, ap.action_sep, ap.max_actions_per_turn)
            yield {"env_id": int(e), "llm_raw_response": raw, "llm_response": llm_response, "actions": actions}


class _LazyState:
    """What a LazyDataProto and its non_tensor_batch share: the ids, the group size, the build
    function and its result.  Neither of the two is referenced from here, so the pair holds no
    reference cycle: a batch is freed when its last user lets go (a cycle kept the generation
    batch's tensors alive until the cyclic GC ran, and its block could not be taken again by
    the next rollout, DevicePrompts.batch_block)."""
    __slots__ = ("env_ids_i64", "group_size", "build_fn", "built", "batch", "device_batch")

    def __init__(self, env_ids_i64, build_fn):
        self.env_ids_i64, self.build_fn = env_ids_i64, build_fn
        self.group_size, self.built, self.batch, self.device_batch = 0, False, None, False

    def build(self, nt: dict):
        """Run the build once; its non-tensor entries go into ``nt``."""
        if self.built:
            return
        self.built = True
        real = self.build_fn()
        if self.device_batch:  # only the host strings are missing
            dict.__setitem__(nt, "messages_list", real.non_tensor_batch["messages_list"])
            return
        self.batch = real.batch
        dict.update(nt, real.non_tensor_batch)


class _LazyNonTensor(dict):
    """non_tensor_batch of a LazyDataProto: 'env_ids' (and, with a device batch, 'group_ids')
    as the reference's object arrays, converted from the owner's int64 ids on first read; any
    other access builds the batch."""

    _IDS = ("env_ids", "group_ids")

    def __init__(self, st: _LazyState):
        super().__init__()
        self._st = st

    def _ids(self, k):
        st = self._st
        if k == "env_ids":
            v = st.env_ids_i64.astype(object)
        elif st.group_size:
            v = (st.env_ids_i64 // st.group_size).astype(object)
        else:
            return None
        dict.__setitem__(self, k, v)
        return v

    def __missing__(self, k):
        if k in self._IDS and self._ids(k) is not None:
            return dict.__getitem__(self, k)
        self._st.build(self)
        return dict.__getitem__(self, k)

    def __contains__(self, k):
        return dict.__contains__(self, k) or k == "env_ids" or (k == "group_ids" and bool(self._st.group_size))

    def get(self, k, default=None):
        return self[k] if k in self else default

    def __len__(self):
        return dict.__len__(self._full())

    def _full(self):
        for k in self._IDS:
            if not dict.__contains__(self, k):
                self._ids(k)
        self._st.build(self)
        return self

    def keys(self):
        return dict.keys(self._full())

    def items(self):
        return dict.items(self._full())

    def values(self):
        return dict.values(self._full())

    def __iter__(self):
        return dict.__iter__(self._full())


class LazyDataProto(DataProto):
    """The per-turn LM inputs on the device path (get_lm_inputs, ctx_manager.py:228-330): the env
    ids right away, the chat-templated prompts and their token ids built on first access.  An
    actor that reads only the env ids (a device-resident policy) never pays for them."""

    def __init__(self, env_ids, build):
        # the ids as int64 (what the device path and a device-resident actor read); the
        # reference's object arrays are made from them on first read of non_tensor_batch
        self._st = _LazyState(np.asarray(env_ids, np.int64), build)
        self.env_rows_device, self.env_rows_lo = None, 0
        self.non_tensor_batch = _LazyNonTensor(self._st)
        self.meta_info = {}

    @property
    def env_ids_i64(self):
        return self._st.env_ids_i64

    def __len__(self):
        return len(self._st.env_ids_i64)

    def set_device_batch(self, batch: dict, env_ids, group_size: int):
        """The device prompt path: the tensors are built already (on the GPU), and so are
        env_ids / group_ids; only messages_list (host strings) is left to the lazy build."""
        from ..protocol import TensorBatch
        st = self._st
        st.batch = TensorBatch(batch)
        st.device_batch = True
        ids = np.asarray(env_ids, np.int64)
        if ids is not st.env_ids_i64 and not np.array_equal(ids, st.env_ids_i64):
            st.env_ids_i64 = ids
            dict.pop(self.non_tensor_batch, "env_ids", None)
        st.group_size = int(group_size)
        dict.pop(self.non_tensor_batch, "group_ids", None)

    @property
    def batch(self):
        if not self._st.device_batch:
            self._build()
        return self._st.batch

    @batch.setter
    def batch(self, v):
        self._st.batch = v

    def _build(self):
        nt = self.non_tensor_batch
        self._st.build(nt if isinstance(nt, dict) else {})


class ContextManager:
    def __init__(self, config, tokenizer, processor=None, mode: str = "train", device=None,
                 rank: Optional[int] = None, world_size: Optional[int] = None, process_group=None):
        self.config = config
        self.tokenizer = tokenizer
        self.processor = processor
        self.action_sep = self.config.agent_proxy.action_sep
        self.special_token_list = list(SPECIAL_TOKENS)
        self.es_cfg = self.config.es_manager[mode]
        self.env_nums = {tag: n * self.es_cfg.group_size  # GLOBAL counts (the metric denominators)
                         for n, tag in zip(self.es_cfg.env_configs.n_groups, self.es_cfg.env_configs.tags)}
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.process_group = process_group
        if process_group is not None:
            import torch.distributed as dist
            rank, world_size = dist.get_rank(process_group), dist.get_world_size(process_group)
        self.rank, self.world_size = int(rank or 0), int(world_size or 1)
        from .. import distributed as rd
        g0, ng = rd.shard_groups(int(self.es_cfg.env_groups), self.world_size, self.rank)
        self.env_lo = g0 * int(self.es_cfg.group_size)
        self.n_envs = ng * int(self.es_cfg.group_size)  # this shard's envs (all of them unsharded)
        self.device_vocab = None
        self._raw_hint = None      # decode row hint (raw bytes), note_raw
        self._raw_hint_pin = None  # (tests) a fixed hint for every turn
        self.device_prompts = True  # build prompt ids on the device when the device path is on
        self._es = None
        self._prompts = None
        self._init_prefix_lookup()

    def shard_sizes(self, tag: Optional[str] = None) -> List[int]:
        """Every rank's env count (of ``tag``'s if given), rank order (es_manager.shard_sizes)."""
        from .es_manager import shard_sizes
        ec = self.es_cfg.env_configs
        return shard_sizes(ec.n_groups, list(ec.tags), int(self.es_cfg.group_size), self.world_size, tag)

    def set_device_vocab(self, vocab: "ops.VocabTable"):
        """Turn on the device path: generations that arrive as token ids on the GPU are decoded by
        rmi_detokenize against this byte table (ops.VocabTable.from_tokenizer for a byte-level
        BPE tokenizer), the turn runs on the device, and — once an EnvStateManager is attached
        (attach_env_manager; LLMAgentProxy does it) — the prompt ids are built on the device
        turn by turn (prompts.DevicePrompts)."""
        self.device_vocab = vocab
        if self._es is not None:
            self._es.lazy_outputs = vocab is not None
        return self

    def attach_env_manager(self, es):
        """The EnvStateManager whose device record this manager reads on the device path."""
        self._es = es
        self._prompts = None
        es.lazy_outputs = self.device_vocab is not None  # reset() hands out env ids, dicts on demand
        return self

    def prompts(self):
        """The device prompt builder, or None where it does not apply (no device vocab or env
        manager, or a tokenizer / chat template outside prompts.DevicePrompts' envelope: the
        reason is warned once).  max_context_window > 0 selects its window mode."""
        if self._prompts is not None:
            return self._prompts or None
        if self.device_vocab is None or self._es is None or not self.device_prompts:
            return None
        max_k = getattr(self.config.agent_proxy, "max_context_window", None)
        window = max_k if isinstance(max_k, int) and max_k > 0 else None  # ctx_manager.py:244-246
        from .prompts import DevicePrompts
        try:
            self._prompts = DevicePrompts(self, self._es, self.tokenizer, self.device, window=window)
        except NotImplementedError as e:
            warnings.warn(f"device prompt ids off, host tokenizer used: {e}", RuntimeWarning)
            self._prompts = False
            return None
        return self._prompts

    def _sync_prompts(self, pr):
        """Bring the prompt arena up to the env manager's turns (and let the env manager's device
        turns append the next prompt themselves, DevicePrompts.advance_eager)."""
        es = self._es
        es._prompt_hook = pr if not pr.window else None
        if pr.rollout != es.rollout_id:
            pr.start()
        for d in es._turn_records[pr.turns_done:]:
            pr.advance(d)

    def _init_prefix_lookup(self):
        """ctx_manager.py:107-146."""
        from dataclasses import asdict
        prefixes, env_config_lookup = {}, {}
        for env_tag, env_config in self.config.custom_envs.items():
            if env_tag not in self.es_cfg.env_configs.tags:
                continue
            if env_config.env_type not in REGISTERED_ENV_CONFIGS:
                raise ValueError(f"Environment {env_config.env_type} is not installed.")
            new = asdict(REGISTERED_ENV_CONFIGS[env_config.env_type]())
            for k, v in env_config.items():
                new[k] = v
            instr = new.get("env_instruction", "")
            if new.get("grid_vocab", False):
                instr += "\nThe meaning of each symbol in the state is:\n" + ", ".join(
                    f"{k}: {v}" for k, v in new["grid_vocab"].items())
            if new.get("action_lookup", False):
                instr += "\nYour available actions are:\n" + ", ".join(f"{v}" for k, v in new["action_lookup"].items())
                instr += (f"\nYou can make up to {new['max_actions_per_traj']} actions, separated by the action "
                          f"separator \" " + self.action_sep + " \"\n")
            prefixes[env_tag] = instr
            env_config_lookup[env_tag] = {"max_tokens": env_config.get(
                "max_tokens", self.config.actor_rollout_ref.rollout.response_length)}
        self.prefix_lookup, self.env_config_lookup = {}, {}
        cur = 0
        gs = self.es_cfg.group_size
        for tag, ng in zip(self.es_cfg.env_configs.tags, self.es_cfg.env_configs.n_groups):
            for i in range(cur * gs, (cur + ng) * gs):
                self.prefix_lookup[i] = prefixes[tag]
                self.env_config_lookup[i] = env_config_lookup[tag]
            cur += ng

    def _parse_response(self, response: str):
        """ctx_manager.py:148-173."""
        ap = self.config.agent_proxy
        return parse_response(response, ap.enable_think, self.action_sep, ap.max_actions_per_turn)

    def _normalize_score_tensor(self, score_tensor: torch.Tensor, env_outputs: List[Dict]) -> torch.Tensor:
        """ctx_manager.py:175-226 on the GPU (in place on score_tensor[:, -1], as the reference)."""
        assert self.config.agent_proxy.use_turn_scores is False, \
            "Reward normalization is not supported for use_turn_scores == True"
        rn = self.config.agent_proxy.reward_normalization
        if rn.method not in ("mean_std", "mean", "asym_clip", "identity"):
            raise ValueError(f"Invalid normalization method: {rn.method}")
        if rn.grouping not in ("state", "inductive", "batch"):
            raise ValueError(f"Invalid grouping: {rn.grouping}")
        dev = self.device
        acc = score_tensor[:, -1].to(dev, torch.float32)
        pen = torch.tensor([o.get("penalty", 0) for o in env_outputs], dtype=torch.float32).to(dev)
        off = 0
        rows = env_outputs
        if self._sharded() and rn.grouping != "state":
            # "inductive" / "batch" group over the WHOLE batch: every rank's scores, penalties and
            # tags gathered in rank order (= global env order), normalised identically on every
            # rank, own rows kept ("state" groups are group-aligned shards: rank-local)
            from .. import distributed as rd
            names = list(dict.fromkeys(self.es_cfg.env_configs.tags))
            tid = torch.tensor([names.index(o["tag"]) if rn.grouping == "inductive" else 0 for o in env_outputs],
                               dtype=torch.int64, device=dev)
            acc, off = rd.all_gather_rows(acc, with_offset=True, group=self.process_group)
            pen = rd.all_gather_rows(pen, group=self.process_group)
            rows = [{"tag": names[int(t)]} for t in rd.all_gather_rows(tid, group=self.process_group).cpu().tolist()]
        perm, seg = segments_for(rn.grouping, rows)
        identity_perm = np.array_equal(perm, np.arange(len(perm)))
        p = None if identity_perm else torch.from_numpy(perm).to(dev)
        a = acc if p is None else acc[p].contiguous()
        b = pen if p is None else pen[p].contiguous()
        out = self._group_norm(a.contiguous(), b.contiguous(), ops.segments(seg, len(perm), dev), rn.method)
        if p is not None:
            res = torch.empty_like(out)
            res[p] = out
            out = res
        out = out[off:off + score_tensor.shape[0]]
        score_tensor[:, -1] = out.to(score_tensor.device)
        return score_tensor

    @staticmethod
    def _group_norm(acc, pen, seg, method):
        """rmi_group_normalize (group normalisation of ctx_manager.py:193-218) on device tensors."""
        return direct.group_normalize(acc, pen, seg, NORM[method])

    def _sharded(self) -> bool:
        return self.process_group is not None and self.world_size > 1

    def get_lm_inputs(self, env_outputs: List[Dict], prepare_for_update: bool) -> DataProto:
        """ctx_manager.py:228-330.  On the device path with device prompts the generation batch
        is built from the device prompt arena (input_ids / attention_mask / position_ids on the
        GPU; messages_list built on the host only when read); without them the inputs are lazy
        (LazyDataProto): env ids now, the host-tokenized batch when the actor reads it."""
        if self.device_vocab is not None and not prepare_for_update:
            env_ids = env_outputs.env_ids if hasattr(env_outputs, "env_ids") else \
                np.array([o["env_id"] for o in env_outputs], np.int64)
            pr = self.prompts()
            if pr is not None:
                self._sync_prompts(pr)
                batch = pr.gen_batch(env_ids)
                out = LazyDataProto(env_ids, lambda: self._messages_only(list(env_outputs), False))
                out.set_device_batch(batch, env_ids, self.es_cfg.group_size)
                # the batch rows' env indices (local to this shard, ascending) on the device, for
                # an actor that gathers per-env state by them (TokenActor)
                out.env_rows_device, out.env_rows_lo = pr.last_rows, self.env_lo
                return out
            return LazyDataProto(env_ids, lambda: self.get_lm_inputs_eager(list(env_outputs)))
        return self.get_lm_inputs_eager(env_outputs, prepare_for_update)

    def _build_messages(self, env_outputs: List[Dict], prepare_for_update: bool):
        """ctx_manager.py:236-276: the chat messages of every env's history and their templated
        text (the histories are trimmed in place as the reference does).  -> (texts, messages)."""
        ap = self.config.agent_proxy
        llm_input_texts, messages_list = [], []
        for env_output in env_outputs:
            if "state" in env_output["history"][-1] and prepare_for_update:
                env_output["history"] = env_output["history"][:-1]
            max_k = getattr(ap, "max_context_window", None)
            if max_k is not None and isinstance(max_k, int) and max_k > 0:
                env_output["history"] = env_output["history"][-max_k:]
            messages = [{"role": "system", "content": "You're a helpful assistant. "},
                        {"role": "user", "content": self.prefix_lookup[env_output["env_id"]]}]
            for idx, content in enumerate(env_output["history"]):
                messages[-1]["content"] += f"\nTurn {idx + 1}:\n"
                if "state" in content:
                    fmt = ("<think> [Your thoughts] </think> <answer> [your answer] </answer>" if ap.enable_think
                           else "<answer> [your answer] </answer>")
                    length = (f"Max response length: {self.env_config_lookup[env_output['env_id']]['max_tokens']} "
                              "words (tokens).")
                    messages[-1]["content"] += (f"State:\n{content['state']}\nYou have {content['actions_left']} "
                                                f"actions left. Always output: {fmt} with no extra text. Strictly "
                                                f"follow this format. {length}\n")
                if "llm_response" in content:
                    messages.append({"role": "assistant", "content": content["llm_response"]})
                if "reward" in content and not (prepare_for_update and idx == len(env_output["history"]) - 1):
                    messages.append({"role": "user", "content": f"Reward:\n{content['reward']}\n"})
            assert all(msg["role"] == "assistant" for msg in messages[2::2])
            text = self.tokenizer.apply_chat_template(messages, add_generation_prompt=(not prepare_for_update),
                                                      tokenize=False)
            if not prepare_for_update:
                text += "<think>" if ap.enable_think else "<answer>"
            llm_input_texts.append(text)
            messages_list.append(messages)
        return llm_input_texts, messages_list

    def _messages_only(self, env_outputs, prepare_for_update):
        """messages_list for a device-built batch (on shallow copies: the caller's histories are
        trimmed by the device path's own bookkeeping)."""
        copies = [dict(o) for o in env_outputs]
        _, msgs = self._build_messages(copies, prepare_for_update)
        return DataProto(None, {"messages_list": np.array(msgs, dtype=object)})

    def get_lm_inputs_eager(self, env_outputs: List[Dict], prepare_for_update: bool = False) -> DataProto:
        ap = self.config.agent_proxy
        llm_input_texts, messages_list = self._build_messages(env_outputs, prepare_for_update)
        if prepare_for_update:
            # ragged token rows -> the padded batch, masks and scores in one device pass
            # (rmi_assemble_batch); the batch is copied to the CPU, single-device like the
            # reference's (ctx_manager.py:290-301)
            scores = [[i.get("reward", 0.0) for i in o["history"]] for o in env_outputs]
            enc = self.tokenizer(llm_input_texts, padding=False, truncation=False)
            ids, am, pos, score_tensor, loss_mask, response_mask = assemble_batch(
                enc.input_ids, self.tokenizer, scores, ap.use_turn_scores, self.config.enable_response_mask,
                self.device)
            normalized = score_tensor
            if not ap.use_turn_scores:
                normalized = self._normalize_score_tensor(score_tensor, env_outputs)
            row_resp = response_mask.sum(dim=-1).float()
            if self._sharded():  # the mean over the WHOLE batch (ctx_manager.py:305)
                from .. import distributed as rd
                row_resp = rd.all_gather_rows(row_resp, group=self.process_group)
            response_length = row_resp.mean().item()
            input_ids = ids.cpu()
            batch = {"input_ids": input_ids, "attention_mask": am.cpu(), "position_ids": pos.cpu(),
                     "responses": input_ids[:, 1:]}
            scores_host = normalized.cpu()
            batch["loss_mask"] = loss_mask.cpu()
            batch["rm_scores"] = scores_host
            batch["original_rm_scores"] = scores_host  # aliases rm_scores, as in the reference
        else:
            inputs = self.tokenizer(llm_input_texts, return_tensors="pt", padding=True, padding_side="left",
                                    truncation=False)
            input_ids, attention_mask = inputs.input_ids, inputs.attention_mask
            position_ids = attention_mask.cumsum(dim=-1)
            batch = {"input_ids": input_ids, "attention_mask": attention_mask, "position_ids": position_ids,
                     "responses": input_ids[:, 1:]}
        out = DataProto(batch)
        out.non_tensor_batch = {
            "env_ids": np.array([o["env_id"] for o in env_outputs], dtype=object),
            "group_ids": np.array([o["group_id"] for o in env_outputs], dtype=object),
            "messages_list": np.array(messages_list, dtype=object),
        }
        if prepare_for_update:
            metrics = self._gather_metric_lists(env_outputs)
            mean_metrics = {k: np.sum(v) / self.env_nums[k.split("/")[0]] for k, v in metrics.items()}
            for k, values in metrics.items():
                prefix, suffix = k.split("/", 1)
                nz = [v for v in values if v != 0]
                if nz:
                    mean_metrics[f"{prefix}/non-zero/{suffix}"] = np.mean(nz)
            mean_metrics["response_length"] = response_length
            out.meta_info = {"metrics": mean_metrics}
        return out

    def _gather_metric_lists(self, env_outputs) -> Dict[str, list]:
        """The per-env metric values of ctx_manager.py:308-312 as {key: [values in env order]};
        sharded, every rank's lists are all-gathered (host objects, rank order = global env
        order) and concatenated, so the means and non-zero means are the whole batch's."""
        metrics = {}
        for o in env_outputs:
            for k, v in o["metrics"].items():
                metrics.setdefault(k, []).append(v)
        if not self._sharded():
            return metrics
        import torch.distributed as dist
        parts = [None] * self.world_size
        dist.all_gather_object(parts, metrics, group=self.process_group)
        merged = {}
        for part in parts:
            for k, v in part.items():
                merged.setdefault(k, []).extend(v)
        return merged

    def get_env_inputs(self, lm_outputs: DataProto) -> List[Dict]:
        """ctx_manager.py:332-352.  Generations that arrive as token ids on the GPU with the device
        path on are decoded there (-> DeviceEnvInputs, no host round trip)."""
        if self.device_vocab is not None and lm_outputs.batch is not None and "responses" in lm_outputs.batch \
                and lm_outputs.batch["responses"].is_cuda:
            return self._device_env_inputs(lm_outputs)
        if lm_outputs.batch is not None and "responses" in lm_outputs.batch.keys():
            responses = self.tokenizer.batch_decode(lm_outputs.batch["responses"], skip_special_tokens=True)
        else:
            responses = lm_outputs.non_tensor_batch["response_texts"]
        prefix = "<think>" if self.config.agent_proxy.enable_think else "<answer>"
        responses = [prefix + r for r in responses]
        env_inputs = []
        for env_id, response in zip(lm_outputs.non_tensor_batch["env_ids"], responses):
            llm_response, actions = self._parse_response(response)
            env_inputs.append({"env_id": env_id, "llm_raw_response": response, "llm_response": llm_response,
                               "actions": actions})
        return env_inputs

    def _device_env_inputs(self, lm_outputs: DataProto) -> DeviceEnvInputs:
        vocab = self.device_vocab
        dev = self.device
        resp = lm_outputs.batch["responses"]
        if resp.device != dev or resp.dtype != torch.int64 or not resp.is_contiguous():
            resp = resp.to(dev, torch.int64).contiguous()
        env_ids = np.asarray(lm_outputs.non_tensor_batch["env_ids"], dtype=np.int64)
        R = resp.shape[1]
        lo, n = self.env_lo, self.n_envs
        es = getattr(self, "_es", None)
        in_order = es is not None and env_ids is es._ids_in_order  # reset()'s own array: every env, in order
        # the ids the last turn handed out (ascending): their rows' map is on the device already
        nr = es.__dict__.get("_next_rows") if es is not None else None
        src_dev = nr[2] if nr is not None and env_ids is nr[0] and resp.shape[0] == len(env_ids) else None
        # the turn's readback buffer, here so rmi_gen_rows writes the longest generation's raw
        # bytes straight into it (EnvStateManager._device_pass reads it back).  Two buffers,
        # alternating by turn: each turn's gen_rows zeroes the other's raw slot for the next turn
        # (rmi_gen_rows_chained: no zeroing launch); a turn's buffer is read back (and done with)
        # before the turn after next reuses it.
        pack, nxt = self.turn_packs()
        raw, raw_next = ops.readback_raw(pack, n), ops.readback_raw(nxt, n)
        if in_order or (src_dev is None and len(env_ids) == n and n and env_ids[0] == lo
                        and np.array_equal(env_ids, lo + np.arange(n))):
            src, src_dev = None, None  # every env in order: the generations are the rows (n_ids None: R each)
        elif src_dev is not None:
            src = None
        else:  # one launch: the rows scattered onto the batch, n_ids, has_t, the raw width
            local = env_ids - lo
            if local.size and (local.min() < 0 or local.max() >= n):
                raise ValueError(f"env ids outside this manager's envs [{lo}, {lo + n})")
            src = np.full(n, -1, np.int64)  # src[e]: env e's row (-1: none)
            src[local] = np.arange(len(env_ids))
            if np.count_nonzero(src >= 0) != local.size:  # (a sort-free duplicate check)
                raise ValueError("duplicate env ids in the generation batch")
        self._pack_i ^= 1  # (the launch below zeroes the other buffer's slot before it is used again)
        # the decoded rows' width.  With a hint from the turns before (the longest generation
        # seen, with a margin) no readback: a longer generation overflows the decode's row, is
        # masked out of the turn's first pass and stepped by a second pass sized from the
        # lengths the turn reads back (EnvStateManager._step_device).  Without one (a manager's
        # first turn): the longest row's raw bytes read back now (x3 for U+FFFD replacements of
        # invalid UTF-8).  Either way within the parse kernel's row limit; a generation past it
        # is flagged by the decode and refused by the step (ValueError).
        hint = self._raw_hint_pin if self._raw_hint_pin is not None else self._raw_hint
        inp = DeviceEnvInputs(self, env_ids, None, None, None, 0)
        inp.raw_dev = raw      # i32[1] on the device: the longest row's raw bytes (read back with the turn)
        inp.raw_next = raw_next
        inp.pack = pack
        # the generation batch's error bytes, counted into this pack with the turn (gen_batch)
        pp, self._pad_pending = self._pad_pending, None
        if pp is not None and pp[0] is pack:
            inp.pad_counted, inp.pad_err = True, pp[1]
        inp.pending_gen = (resp, src, src_dev)
        if hint is None or not resp.numel():  # the rows now: the decode is sized from their read-back width
            inp.flush()
            raw_max = int(ops.d2h(raw, self)[0]) if resp.numel() else 0
            stride = decode_stride(raw_max, 3)
            self.note_raw(raw_max)
        else:  # the scatter waits for the turn's own launches (turn_chain), or its first reader
            raw_max = None
            stride = decode_stride(hint, 1)
        inp.stride = stride
        inp.raw_max = raw_max  # the decoded rows' length bound (longer only with U+FFFD replacements)
        return inp

    _pad_pending = None  # (the next turn's readback pack, the last generation batch's error bytes)

    def turn_packs(self):
        """(this turn's readback buffer, the other one): two, alternating by turn (allocated on
        first use)."""
        n, dev = self.n_envs, self.device
        nb = ops.readback_bytes(n)
        packs = getattr(self, "_packs", None)
        if packs is None or packs[0].numel() != nb:
            packs = self._packs = [torch.zeros(nb, dtype=torch.uint8, device=dev) for _ in range(2)]
            self._pack_i = 0
        return packs[self._pack_i], packs[1 - self._pack_i]

    RAW_HINT_MARGIN = 1.1  # the decode's row over the longest generation seen (+ 32 bytes)

    def note_raw(self, raw_max: int):
        """A turn's longest generation (raw bytes, read back) -> the next turns' decode hint."""
        h = int(raw_max * self.RAW_HINT_MARGIN) + 32
        self._raw_hint = h if self._raw_hint is None else max(self._raw_hint, h)

    def formulate_rollouts(self, env_outputs: List[Dict]) -> DataProto:
        """ctx_manager.py:354-356.  The rollout states of the attached env manager's device path
        (LazyRolloutStates) with device prompts are formulated on the device (formulate_device);
        anything else through the reference's host code."""
        from .es_manager import LazyRolloutStates
        pr = self.prompts()
        if (pr is not None and isinstance(env_outputs, LazyRolloutStates) and env_outputs.es is self._es
                and env_outputs.rollout_id == self._es.rollout_id):
            return self.formulate_device(pr)
        return self.get_lm_inputs_eager(env_outputs, prepare_for_update=True)

    def formulate_device(self, pr) -> DataProto:
        """formulate_rollouts (get_lm_inputs(prepare_for_update=True), ctx_manager.py:228-330) from
        the device record: the update rows of the prompt arena (each env's conversation up to its
        last assistant block) assembled with masks and scores in one pass (rmi_assemble_rows),
        scores = the turn rewards (n_turns per env), the reward normalisation on the device, and
        the metrics (ctx_manager.py:308-329) from one copy of the per-env metric rows.  The
        batch stays on the GPU; messages_list is built on the host only when read."""
        es = self._es
        self._sync_prompts(pr)
        fc = self._formulate_chain(es, pr)
        if fc is not None:
            return fc.run()
        ap = self.config.agent_proxy
        dev = self.device
        # the rows the device could not build are resolved after the readback below, which
        # carries their any() (one readback fewer)
        pend = pr._pending[0] if pr._pending is not None and not pr.window else None
        tokens, start, row_len = pr.update_rows(resolve=pend is None)
        eps = [tg.batch.ep for tg in es.tags]
        tab = (eps[0].turn_reward if len(eps) == 1 else torch.cat([ep.turn_reward for ep in eps], 1)).contiguous()
        n_sc = (eps[0].n_turns if len(eps) == 1 else torch.cat([ep.n_turns for ep in eps])).to(torch.int32)
        if pr.window:  # the kept entries' rewards only: the reference reads the TRIMMED history (:282)
            k = pr.window
            j0 = (n_sc - k).clamp(min=0)
            n_w = n_sc - j0
            i = torch.arange(k, device=dev, dtype=torch.int32)[:, None]
            src = (j0[None, :] + i).clamp(max=tab.shape[0] - 1).long()
            tab = torch.gather(tab, 0, src).masked_fill(i >= n_w[None, :], 0.0).contiguous()
            n_sc = n_w.to(torch.int32)
        if getattr(self, "_special", None) is None:  # a tokenizer call: once per manager
            self._special = get_special_tokens(self.tokenizer)
        special_token, reward_token = self._special
        # the longest row, the most turns and whether a row waits for the host, in one readback
        if row_len.numel():
            st = torch.empty(3, dtype=torch.int32, device=dev)
            ops.rows_stats(row_len, None, row_len.numel(), pend, st)  # (max row, any pending)
            st[2:].copy_(n_sc.max().view(1))
            S, any_bad, n_slots = (int(x) for x in ops.d2h(st, es))
            if pend is not None:
                pr._resolve(bool(any_bad))
                if any_bad:  # host rows were written: the longest row again
                    S = int(row_len.max())
        else:
            pr._resolve()
            S, n_slots = 1, 0
        # zip_longest's length over the WHOLE batch (ctx_manager.py:52-62): every rank's longest
        from .. import distributed as rd
        if self.process_group is not None and self.world_size > 1:
            n_slots = rd.all_reduce_max_int(n_slots, self.process_group, dev)
        ids, am, pos, score_tensor, loss_mask, response_mask, err = direct.assemble_rows(
            tokens, start, row_len, max(S, 1), int(pr.pad_id), int(special_token), int(reward_token), tab, n_sc,
            n_slots, bool(ap.use_turn_scores), bool(self.config.enable_response_mask),
            "qwen" in self.tokenizer.name_or_path.lower())
        normalized = score_tensor
        if not ap.use_turn_scores:
            normalized = self._normalize_device(score_tensor, es)
        # the mean over the WHOLE batch (ctx_manager.py:305): every rank's row lengths, rank order
        # (rmi_row_counts: the values of response_mask.sum(-1), without torch's widening copy)
        row_resp = ops.row_counts(response_mask).float()
        if self.process_group is not None and self.world_size > 1:
            row_resp = rd.all_gather_rows(row_resp, group=self.process_group, sizes=self.shard_sizes())
        # the mean, the assembly's per-row error bytes and the metric rows in one readback (the
        # error bits reduced on the host: no launches for them)
        mean = row_resp.mean().double().reshape(1).view(torch.uint8)
        parts, ext = es.metric_arrays([mean, err])
        response_length = float(ext[:8].view(np.float64)[0])
        if row_resp.numel() * max(S, 1) >= (1 << 24):
            # partial f32 sums of the counts may round here, and the device's reduction order is
            # not torch CPU's: the reference's own op on the counts (exact below 2^24 either way)
            response_length = float(row_resp.cpu().mean().item())
        err_h = ext[8:]
        _raise_assemble_errors(None, S, (bool((err_h & _lib.ERR_UNSUP).any()), bool((err_h & _lib.ERR_STATE).any())))
        batch = {"input_ids": ids, "attention_mask": am, "position_ids": pos, "responses": ids[:, 1:],
                 "loss_mask": loss_mask, "rm_scores": normalized, "original_rm_scores": normalized}
        env_ids = es.env_lo + np.arange(es.n_envs, dtype=np.int64)
        out = LazyDataProto(env_ids, lambda: self._messages_only(es._rollout_states_full(), True))
        out.set_device_batch(batch, env_ids, es.group_size)
        metrics = self.device_metrics(es, parts)
        metrics["response_length"] = response_length
        out.meta_info = {"metrics": metrics}
        es._formulated = True
        es._formulated_window = pr.window
        return out

    use_formulate_chain = True  # (tests compare the chained form with the step-by-step one)

    def _formulate_chain(self, es, pr):
        """turn_chain.FormulateChain for this manager's env manager and prompts, or None."""
        from .turn_chain import FormulateChain
        if not self.use_formulate_chain or not FormulateChain.applies(self, es, pr):
            return None
        fc = self.__dict__.get("_fchain")
        if fc is None or fc.es is not es or fc.pr is not pr:
            fc = self._fchain = FormulateChain(self, es, pr)
        return fc

    def _normalize_device(self, score_tensor, es):
        """_normalize_score_tensor (ctx_manager.py:175-226) from the device record: penalties from
        the episode arena, groups by grouping (state: group ids, contiguous; inductive: tags;
        batch: all).  Under sharding the "state" groups are rank-local; the other groupings
        need every rank's scores (ragen_amd.distributed: gathered, normalised identically on
        every rank, the own rows kept)."""
        rn = self.config.agent_proxy.reward_normalization
        if rn.method not in ("mean_std", "mean", "asym_clip", "identity"):
            raise ValueError(f"Invalid normalization method: {rn.method}")
        if rn.grouping not in ("state", "inductive", "batch"):
            raise ValueError(f"Invalid grouping: {rn.grouping}")
        from .. import distributed as rd
        eps = [tg.batch.ep for tg in es.tags]
        pen = (eps[0].penalty if len(eps) == 1 else torch.cat([ep.penalty for ep in eps])).to(torch.float32)
        acc = score_tensor[:, -1].contiguous()
        dev = acc.device
        gs = es.group_size
        if rn.grouping == "state":
            seg = np.arange(0, es.n_envs + 1, gs, dtype=np.int32)
            out = self._group_norm(acc, pen.contiguous(), ops.segments(seg, es.n_envs, dev), rn.method)
        else:
            sharded = self._sharded()
            sz = self.shard_sizes() if sharded else None
            a_all = rd.all_gather_rows(acc, group=self.process_group, sizes=sz) if sharded else acc
            p_all = rd.all_gather_rows(pen.contiguous(), group=self.process_group, sizes=sz) if sharded else pen
            n_all = a_all.numel()
            perm = None
            if rn.grouping == "batch":
                seg = np.array([0, n_all], np.int32)
            else:  # one group per tag NAME (a tag listed twice in the config is one group)
                ec = self.es_cfg.env_configs
                perm, seg = tag_segments(list(ec.tags), list(ec.n_groups), gs)
            if perm is not None:
                p = torch.from_numpy(perm).to(dev)
                a_all, p_all = a_all[p], p_all[p]
            res = self._group_norm(a_all.contiguous(), p_all.contiguous(), ops.segments(seg, n_all, dev), rn.method)
            if perm is not None:
                back = torch.empty_like(res)
                back[p] = res
                res = back
            out = res[es.env_lo:es.env_lo + es.n_envs] if sharded else res
        score_tensor[:, -1] = out
        return score_tensor

    def device_metrics(self, es, parts=None) -> Dict:
        """The mean / non-zero metrics of get_lm_inputs (ctx_manager.py:308-329) from the device
        metric rows (es.metric_arrays: one copy; ``parts`` when read already), with numpy over
        whole arrays in env order — the same values and summation order as the reference's
        lists.  Under sharding every rank's rows are gathered first, so each rank reports the
        global metrics."""
        from .. import distributed as rd
        if parts is None:
            parts = es.metric_arrays()
        sharded = self.process_group is not None and self.world_size > 1
        local = {}  # per tag NAME, env order (a tag listed twice in the config: its entries' rows in order)
        for tag, m, custom, _ in parts:
            if tag not in local and not sharded:
                local[tag] = (m, custom)  # (one entry: the metric rows and the custom mask as they are)
                continue
            rows = np.concatenate([m, custom[:, None].astype(np.float64)], 1)
            if tag in local and isinstance(local[tag], tuple):
                m0, c0 = local[tag]
                local[tag] = np.concatenate([m0, c0[:, None].astype(np.float64)], 1)
            local[tag] = np.concatenate([local[tag], rows]) if tag in local else rows
        per_tag = {}
        for tag in dict.fromkeys(self.es_cfg.env_configs.tags):  # every rank, same order (collectives)
            rows = local.get(tag, np.zeros((0, 5), np.float64))
            if sharded:
                rows = rd.all_gather_rows(torch.from_numpy(rows).to(self.device), group=self.process_group,
                                          sizes=self.shard_sizes(tag)).cpu().numpy()
            if len(rows[0] if isinstance(rows, tuple) else rows):
                per_tag[tag] = rows
        metrics, nz = {}, []
        for tag in dict.fromkeys(self.es_cfg.env_configs.tags):
            if tag not in per_tag:
                continue
            rows = per_tag[tag]
            if isinstance(rows, tuple):  # the metric rows [n, 4] and the custom mask, unconcatenated
                m, cust = rows
                m = np.ascontiguousarray(m.T)  # one pass: each column contiguous for its reductions
            else:
                m, cust = np.ascontiguousarray(rows[:, :4].T), rows[:, 4] != 0
            # success and num_actions hold integers (the finalize's 0 / 1 and action counts): their
            # sums are exact in any order, so their non-zero means are sum / count -- the values
            # np.mean over the non-zero entries gives -- with two reductions for both columns
            tot, cnt = m[:2].sum(axis=1), np.count_nonzero(m[:2], axis=1)
            metrics[f"{tag}/success"] = tot[0] / self.env_nums[tag]
            metrics[f"{tag}/num_actions"] = np.int64(tot[1]) / self.env_nums[tag]
            nz += [(f"{tag}/non-zero/success", tot[0], cnt[0]), (f"{tag}/non-zero/num_actions", tot[1], cnt[1])]
            if cust.any():
                all_c = bool(cust.all())
                for k, v in (("action_is_effective", m[2] if all_c else m[2][cust]),
                             ("action_is_valid", m[3] if all_c else m[3][cust])):
                    metrics[f"{tag}/{k}"] = np.sum(v) / self.env_nums[tag]
                    v = v[v != 0]  # (fractions: the reference's order of summation over the non-zero ones)
                    nz.append((f"{tag}/non-zero/{k}", np.sum(v), len(v)))
        for k, t, c in nz:
            if c:
                metrics[k] = np.float64(t) / c
        return metrics
