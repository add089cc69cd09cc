"""Device-side encoding for byte-level BPE tokenizers (§8(f) ranks 1-2): the tables
``rmi_bpe_encode`` (csrc/bpe.hip) reads, built from the tokenizer's own serialized form.

Replaces the tokenizer call of ContextManager.get_lm_inputs (ctx_manager.py:265-278,
``self.tokenizer(llm_input_texts, ...)``) for the tokenizers RAGEN runs with: a HF fast
tokenizer whose backend (the ``tokenizers`` library) is

* model ``BPE`` without dropout, byte fallback, subword prefixes or ``ignore_merges``;
* normalizer ``NFC`` or none;
* pre-tokenizer ``Split(<Qwen2 regex>, Isolated) + ByteLevel(use_regex=False)`` (Qwen2 / 2.5),
  or ``Split(<one character>, Isolated) + ByteLevel`` (character-level test tokenizers);
* added tokens without lstrip / rstrip / single_word (matched leftmost-longest);
* no post-processor that adds ids.

Anything else raises ``NotImplementedError`` at construction: the prompt path then stays on
the host tokenizer (ContextManager.get_lm_inputs_eager), never a silent approximation.

Code-point classes (``\\p{L}``, ``\\p{N}``, ``\\s`` as the pre-tokenizer's regex engine sees
them) are read off the ``tokenizers`` pre-tokenizer itself: one probe string per class over
every code point, so the table follows the library's own Unicode tables, whatever their
version.  ``RMI_CP_UNSAFE`` marks code points NFC may change in context (a nonzero canonical
combining class, a character NFC rewrites, the second half of a canonical composition, Hangul
jamo); a row that holds one is flagged instead of encoded, and the caller encodes it on the
host.
"""
import ctypes
import functools
import json
import os
import unicodedata
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib

QWEN2_PATTERN = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}| ?[^\s\p{L}\p{N}]+[\r\n]*|"
                 r"\s*[\r\n]+|\s+(?!\S)|\s+")
CHAR_PATTERNS = (".", "(?s:.)", "(?m:.)")
PRETOK_QWEN2, PRETOK_CHARS = 0, 1
CP_L, CP_N, CP_W, CP_NL, CP_UNSAFE = 1, 2, 4, 8, 16
MAX_STRIDE = 3072


@functools.lru_cache(maxsize=None)
def bytes_to_unicode():
    """GPT-2's byte <-> printable character map (the ByteLevel pre-tokenizer / decoder)."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {b: chr(c) for b, c in zip(bs, cs)}


def _code_points():
    """Planes 0-3 and 14 (every assigned code point); planes 4-13 are unassigned and 15-16
    private use: \\p{L}, \\p{N} and \\s hold none of them, so they stay "other"."""
    return [c for c in range(0x40000) if not 0xD800 <= c <= 0xDFFF] + list(range(0xE0000, 0xF0000))


def _probe(pretok, fmt, sep, cps, at):
    """Pre-tokenize one string holding fmt(c) for every code point c, joined by sep; -> bool
    array: is there a pre-token boundary at offset ``at`` of each probe (in characters)."""
    parts = [fmt(chr(c)) for c in cps]
    text = sep.join(parts)
    starts = set()
    for _, (s, _e) in pretok.pre_tokenize_str(text):
        starts.add(s)
    out = np.zeros(len(cps), bool)
    pos = 0
    step = [len(p) + len(sep) for p in parts]
    for i in range(len(cps)):
        out[i] = (pos + at) in starts
        pos += step[i]
    return out


DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "qwen2_cp_classes.npz")


@functools.lru_cache(maxsize=None)
def class_table():
    """The Qwen2 code-point class table: the committed ``data/qwen2_cp_classes.npz`` when it
    was probed with the installed tokenizers version (tests/test_tokenizer.py re-probes and
    compares), else probed now (a few seconds)."""
    import tokenizers
    if os.path.exists(DATA):
        z = np.load(DATA, allow_pickle=False)
        if str(z["tokenizers_version"]) == tokenizers.__version__:
            return z["cp_block"].astype(np.uint16), z["cp_class"].astype(np.uint8)
    return probe_class_table()


def save_class_table(path=DATA):
    import tokenizers
    blk, cls = probe_class_table()
    os.makedirs(os.path.dirname(path), exist_ok=True)
    np.savez_compressed(path, cp_block=blk, cp_class=cls, tokenizers_version=np.array(tokenizers.__version__))


def probe_class_table():
    """-> (cp_block u16[0x1100], cp_class u8[n_blocks*256]) for the Qwen2 regex classes, read
    off the tokenizers library's Split pre-tokenizer (Isolated) with probe strings:
      L: "x" + c   joined  <=> c in \\p{L}          (alternative 2: \\p{L}+)
      O: "!" + c   joined  <=> c in \\p{L} or other (alternatives 2 and 4)
      W: c + " \\n" joined <=> c in \\s             (alternative 5: \\s*[\\r\\n]+)
    N is what is none of them (the remaining class of [^\\s\\p{L}\\p{N}]'s complement)."""
    from tokenizers import Regex, pre_tokenizers
    pre = pre_tokenizers.Split(Regex(QWEN2_PATTERN), behavior="isolated", invert=False)
    cps = _code_points()
    # separators that force a boundary before the next probe: "0" is \p{N} (a one-char match)
    is_l = ~_probe(pre, lambda c: "x" + c, "0", cps, 1)
    joins_o = ~_probe(pre, lambda c: "!" + c, "0", cps, 1)
    is_w = ~_probe(pre, lambda c: c + " \n", "0", cps, 1)
    cls = np.zeros(0x110000, np.uint8)
    idx = np.asarray(cps)
    is_o = joins_o & ~is_l
    cls[idx[is_l]] |= CP_L
    cls[idx[is_w & ~is_l]] |= CP_W
    cls[idx[~is_l & ~is_o & ~is_w]] |= CP_N
    cls[0x0A] |= CP_NL | CP_W
    cls[0x0D] |= CP_NL | CP_W
    cls[_nfc_unsafe()] |= CP_UNSAFE
    # two-stage table: identical 256-entry blocks shared
    blocks, block_of = {}, np.zeros(0x1100, np.uint16)
    data = []
    for hi in range(0x1100):
        blk = cls[hi * 256:(hi + 1) * 256].tobytes()
        if blk not in blocks:
            blocks[blk] = len(blocks)
            data.append(blk)
        block_of[hi] = blocks[blk]
    return block_of, np.frombuffer(b"".join(data), np.uint8).copy()


@functools.lru_cache(maxsize=None)
def _nfc_unsafe():
    """Code points whose presence lets NFC change a string (conservative)."""
    out = set()
    for c in _code_points():
        ch = chr(c)
        if unicodedata.combining(ch) or unicodedata.normalize("NFC", ch) != ch:
            out.add(c)
        d = unicodedata.decomposition(ch)
        if d and not d.startswith("<"):
            parts = d.split()
            if len(parts) == 2:
                out.add(int(parts[1], 16))  # may compose with what precedes it
    out.update(range(0x1100, 0x1200))  # Hangul jamo (algorithmic composition)
    out.update(range(0xA960, 0xA980))
    out.update(range(0xD7B0, 0xD800))
    return np.asarray(sorted(out), np.int64)


class Bpe(ctypes.Structure):
    """rmi_bpe_t."""
    _fields_ = [("cp_block", ctypes.c_void_p), ("cp_class", ctypes.c_void_p), ("byte_id", ctypes.c_void_p),
                ("merges", ctypes.c_void_p), ("merge_mask", ctypes.c_uint32), ("merge_shift", ctypes.c_uint32),
                ("pretok", ctypes.c_int32), ("nfc", ctypes.c_int32), ("n_added", ctypes.c_int32),
                ("added_bytes", ctypes.c_void_p), ("added_off", ctypes.c_void_p), ("added_id", ctypes.c_void_p),
                ("added_first", ctypes.c_uint32 * 8), ("word_cache", ctypes.c_void_p),
                ("word_cache_mask", ctypes.c_uint32), ("n_exp", ctypes.c_int32), ("exp_off", ctypes.c_void_p),
                ("exp_ids", ctypes.c_void_p), ("added_words", ctypes.c_void_p), ("ascii_class", ctypes.c_void_p),
                ("n_exp_ids", ctypes.c_int32), ("pre", ctypes.c_void_p), ("pre_gid", ctypes.c_void_p),
                ("pre_np", ctypes.c_void_p), ("pre_retry", ctypes.c_void_p), ("pre_cap", ctypes.c_int64)]


def _backend_json(tokenizer) -> dict:
    for obj in (getattr(tokenizer, "backend_tokenizer", None), tokenizer):
        if obj is not None and hasattr(obj, "to_str"):
            return json.loads(obj.to_str())
    raise NotImplementedError("device encoding needs a HF fast tokenizer (a `tokenizers` backend)")


def _post_processor_adds_nothing(pp) -> bool:
    """ByteLevel (offsets only), or a TemplateProcessing whose single-sequence template is the
    sequence alone (what transformers installs without BOS / EOS)."""
    if pp.get("type") == "ByteLevel":
        return True
    if pp.get("type") == "TemplateProcessing":
        return all("Sequence" in piece for piece in pp.get("single", []))
    if pp.get("type") == "Sequence":
        return all(_post_processor_adds_nothing(x) for x in pp.get("processors", []))
    return False


def _pretok_mode(pt) -> int:
    if not pt or pt.get("type") != "Sequence" or len(pt.get("pretokenizers", [])) != 2:
        raise NotImplementedError(f"pre-tokenizer {pt and pt.get('type')} is not supported on the device")
    split, bl = pt["pretokenizers"]
    if bl.get("type") != "ByteLevel" or bl.get("use_regex", True) or bl.get("add_prefix_space", False):
        raise NotImplementedError("the device path needs ByteLevel(use_regex=False, add_prefix_space=False)")
    if split.get("type") != "Split" or split.get("behavior") != "Isolated" or split.get("invert"):
        raise NotImplementedError("the device path needs Split(..., behavior=Isolated, invert=False)")
    pat = (split.get("pattern") or {}).get("Regex")
    if pat == QWEN2_PATTERN:
        return PRETOK_QWEN2
    if pat in CHAR_PATTERNS:
        return PRETOK_CHARS
    raise NotImplementedError(f"pre-tokenizer regex {pat!r} is not supported on the device")


def _merge_table(pairs: np.ndarray, ranks: np.ndarray, new_ids: np.ndarray):
    """Open-addressed (key, value) table: key = left << 32 | right, value = rank << 32 | new id,
    slot = (key * 0x9E3779B97F4A7C15) >> shift, linear probing; the lowest rank wins a
    duplicated pair (the tokenizers crate keeps the first).  -> (u64[2*cap], mask, shift)."""
    n = len(pairs)
    bits = max(4, int(np.ceil(np.log2(max(2 * n, 16)))))
    cap = 1 << bits
    keys = np.full(cap, np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64)
    vals = np.zeros(cap, np.uint64)
    k = (pairs[:, 0].astype(np.uint64) << np.uint64(32)) | pairs[:, 1].astype(np.uint64)
    v = (ranks.astype(np.uint64) << np.uint64(32)) | new_ids.astype(np.uint64)
    with np.errstate(over="ignore"):
        slot = ((k * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(64 - bits)).astype(np.int64)
    order = np.argsort(ranks, kind="stable")
    seen = set()
    mask = cap - 1
    for i in order.tolist():
        key = int(k[i])
        if key in seen:
            continue
        seen.add(key)
        h = int(slot[i])
        while keys[h] != np.uint64(0xFFFFFFFFFFFFFFFF):
            h = (h + 1) & mask
        keys[h] = k[i]
        vals[h] = v[i]
    table = np.empty(2 * cap, np.uint64)
    table[0::2], table[1::2] = keys, vals
    return table, mask, 64 - bits


@dataclass
class DeviceTokenizer:
    """The device tables of one tokenizer (module docstring)."""
    cp_block: torch.Tensor
    cp_class: torch.Tensor
    byte_id: torch.Tensor
    merges: torch.Tensor
    merge_mask: int
    merge_shift: int
    pretok: int
    nfc: int
    added_bytes: torch.Tensor
    added_off: torch.Tensor
    added_id: torch.Tensor
    added_first: List[int]
    added: dict  # content -> id
    # the word cache (rmi_bpe_t.word_cache): i32[(mask + 1) * 16], zeroed once; None = off
    word_cache: Optional[torch.Tensor] = None
    # expansions (rmi_bpe_t.n_exp / exp_off / exp_ids): placeholder added tokens standing for a
    # precomputed id sequence (add_expansion); the tables below are rebuilt when one is added
    exp: Optional[list] = None
    exp_off: Optional[torch.Tensor] = None
    exp_ids: Optional[torch.Tensor] = None
    # staging tables (rmi_bpe_t.added_words / ascii_class; _build_staging)
    added_words: Optional[torch.Tensor] = None
    ascii_class: Optional[torch.Tensor] = None
    # the two-pass form's scratch (rmi_bpe_t.pre*; ensure_two_pass): None = one kernel per call
    pre: Optional[tuple] = None

    MAX_EXPANSIONS = 64

    WORD_CACHE_ENTRIES = 1 << 15  # 2 MB: the distinct pre-tokens of the prompts with room to spare

    @staticmethod
    def from_hf(tokenizer, device) -> "DeviceTokenizer":
        j = _backend_json(tokenizer)
        m = j.get("model") or {}
        if m.get("type") != "BPE":
            raise NotImplementedError(f"model {m.get('type')} is not supported on the device (BPE only)")
        for k in ("dropout", "continuing_subword_prefix", "end_of_word_suffix"):
            if m.get(k):
                raise NotImplementedError(f"BPE {k}={m.get(k)!r} is not supported on the device")
        if m.get("byte_fallback") or m.get("ignore_merges"):
            raise NotImplementedError("BPE byte_fallback / ignore_merges are not supported on the device")
        norm = j.get("normalizer")
        if norm is not None and norm.get("type") != "NFC":
            raise NotImplementedError(f"normalizer {norm.get('type')} is not supported on the device")
        pp = j.get("post_processor")
        if pp is not None and not _post_processor_adds_nothing(pp):
            raise NotImplementedError(f"post-processor {pp.get('type')} adds ids; not supported on the device")
        pretok = _pretok_mode(j.get("pre_tokenizer"))
        vocab = m["vocab"]
        b2u = bytes_to_unicode()
        try:
            byte_id = np.array([vocab[b2u[b]] for b in range(256)], np.int32)
        except KeyError as e:
            raise NotImplementedError(f"byte-level symbol {e} missing from the vocabulary") from None
        merges = m.get("merges") or []
        pairs, new_ids = np.zeros((len(merges), 2), np.int64), np.zeros(len(merges), np.int64)
        keep = np.ones(len(merges), bool)
        for r, mg in enumerate(merges):
            a, b = mg.split(" ", 1) if isinstance(mg, str) else mg
            ia, ib, ic = vocab.get(a), vocab.get(b), vocab.get(a + b)
            if ia is None or ib is None or ic is None:
                keep[r] = False
                continue
            pairs[r] = (ia, ib)
            new_ids[r] = ic
        ranks = np.arange(len(merges), dtype=np.int64)
        table, mask, shift = _merge_table(pairs[keep], ranks[keep], new_ids[keep])
        added = {}
        for at in j.get("added_tokens") or []:
            if at.get("lstrip") or at.get("rstrip") or at.get("single_word"):
                raise NotImplementedError(f"added token {at['content']!r}: lstrip / rstrip / single_word")
            added[at["content"]] = int(at["id"])
        blobs = [c.encode("utf-8") for c in added]
        off = np.zeros(len(blobs) + 1, np.int32)
        np.cumsum([len(x) for x in blobs], out=off[1:])
        first = [0] * 8
        for x in blobs:
            first[x[0] >> 5] |= 1 << (x[0] & 31)
        blk, cls = class_table() if pretok == PRETOK_QWEN2 else _char_class_table()
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        data = b"".join(blobs) + b"\0" * 4
        dt = DeviceTokenizer(
            t(blk.astype(np.int16).view(np.int16)), t(cls), t(byte_id), t(table.view(np.int64)), mask, shift, pretok,
            int(norm is not None), t(np.frombuffer(data, np.uint8).copy()), t(off),
            t(np.array(list(added.values()) or [0], np.int32)), first, added,
            torch.zeros(DeviceTokenizer.WORD_CACHE_ENTRIES * 16, dtype=torch.int32, device=device))
        dt.ascii_class = t(np.ascontiguousarray(cls[int(blk[0]) * 256:int(blk[0]) * 256 + 128]).astype(np.uint8))
        dt._build_staging(blobs)
        return dt

    def _build_staging(self, blobs):
        """The added tokens as zero-padded 32-byte words (rmi_bpe_t.added_words), when every
        one fits (<= 32 bytes, <= 64 tokens); else None (the kernel compares from the tables)."""
        if not blobs or len(blobs) > 64 or any(len(x) > 32 for x in blobs):
            self.added_words = None
            return
        w = np.zeros((len(blobs), 32), np.uint8)
        for i, x in enumerate(blobs):
            w[i, :len(x)] = np.frombuffer(x, np.uint8)
        self.added_words = torch.from_numpy(w.view(np.int64).reshape(-1).copy()).to(self.byte_id.device)

    def add_expansion(self, ids) -> bytes:
        """The placeholder bytes (0xFF, 0x80 + e) of the expansion whose tokens are ``ids`` (a
        constant stretch of prompt text proven context-free by prompts.py); registered once per
        distinct id sequence.  The added-token tables grow by the placeholder, with id -(e + 1)."""
        ids = tuple(int(x) for x in ids)
        if self.exp is None:
            self.exp = []
        if ids in self.exp:
            e = self.exp.index(ids)
        else:
            if len(self.exp) >= self.MAX_EXPANSIONS or not ids or len(ids) > 1024:
                return None
            self.exp.append(ids)
            e = len(self.exp) - 1
            self._rebuild_added()
        return bytes([0xFF, 0x80 + e])

    def _rebuild_added(self):
        dev = self.byte_id.device
        blobs = [c.encode("utf-8") for c in self.added] + [bytes([0xFF, 0x80 + e]) for e in range(len(self.exp))]
        id_list = list(self.added.values()) + [-(e + 1) for e in range(len(self.exp))]
        off = np.zeros(len(blobs) + 1, np.int32)
        np.cumsum([len(x) for x in blobs], out=off[1:])
        first = [0] * 8
        for x in blobs:
            first[x[0] >> 5] |= 1 << (x[0] & 31)
        self.added_bytes = torch.from_numpy(np.frombuffer(b"".join(blobs) + b"\0" * 4, np.uint8).copy()).to(dev)
        self.added_off = torch.from_numpy(off).to(dev)
        self.added_id = torch.from_numpy(np.array(id_list, np.int32)).to(dev)
        self.added_first = first
        eo = np.zeros(len(self.exp) + 1, np.int32)
        np.cumsum([len(x) for x in self.exp], out=eo[1:])
        self.exp_off = torch.from_numpy(eo).to(dev)
        self.exp_ids = torch.from_numpy(np.array([i for x in self.exp for i in x], np.int32)).to(dev)
        self._build_staging(blobs)

    @property
    def n_added(self) -> int:
        return len(self.added) + (len(self.exp) if self.exp else 0)

    def struct(self) -> Bpe:
        s = Bpe(self.cp_block.data_ptr(), self.cp_class.data_ptr(), self.byte_id.data_ptr(), self.merges.data_ptr(),
                self.merge_mask, self.merge_shift, self.pretok, self.nfc, self.n_added,
                self.added_bytes.data_ptr(), self.added_off.data_ptr(), self.added_id.data_ptr())
        if self.exp:
            s.n_exp, s.exp_off, s.exp_ids = len(self.exp), self.exp_off.data_ptr(), self.exp_ids.data_ptr()
            s.n_exp_ids = int(self.exp_ids.numel())
        for i, w in enumerate(self.added_first):
            s.added_first[i] = w
        if self.word_cache is not None:
            s.word_cache, s.word_cache_mask = self.word_cache.data_ptr(), self.word_cache.numel() // 16 - 1
        if self.added_words is not None:
            s.added_words = self.added_words.data_ptr()
        if self.ascii_class is not None:
            s.ascii_class = self.ascii_class.data_ptr()
        return s

    def args(self):
        """The tables in the order torch.ops.ragen_amd.bpe_encode takes them."""
        return (self.cp_block, self.cp_class, self.byte_id, self.merges, self.added_bytes, self.added_off,
                self.added_id, [self.merge_mask, self.merge_shift, self.pretok, self.nfc, self.n_added]
                + list(self.added_first))

    def bpe_struct(self, two_pass: bool = True):
        """The validated rmi_bpe_t of the current tables (expansions included), built once per
        set of tables (torch_ops._bpe_struct): what rmi_bpe_encode / rmi_turn_chain take; with
        the two-pass scratch when it is allocated (ensure_two_pass) and ``two_pass``."""
        from .torch_ops import _bpe_struct
        return _bpe_struct(*self.args(), self.word_cache, self.exp_off if self.exp else None,
                           self.exp_ids if self.exp else None, self.added_words, self.ascii_class,
                           self.pre if two_pass else None)

    def ensure_two_pass(self, rows: int, stride: int) -> bool:
        """Scratch for the two-pass form of rmi_bpe_encode over ``rows`` rows of at most
        ``stride`` bytes (pre-token lists and added ids: 8 B per row byte), grown when too small.
        -> whether it was (re)allocated (a cached rmi_bpe_t must be rebuilt)."""
        need = int(rows) * int(stride)
        if self.pre is not None and self.pre[0].numel() >= need:
            return False
        cap = max(need, 1)
        dev = self.byte_id.device
        # (the per-row arrays hold cap / 4 entries: every call the C side accepts has rows <= cap / 4)
        self.pre = (torch.empty(cap, dtype=torch.int32, device=dev), torch.empty(cap, dtype=torch.int32, device=dev),
                    torch.empty(max(cap // 4, 1), dtype=torch.int32, device=dev),
                    torch.empty(max(cap // 4, 1), dtype=torch.uint8, device=dev))
        return True

    def encode_two_pass(self, text: torch.Tensor, text_len: torch.Tensor, out: torch.Tensor, stride: int):
        """rmi_bpe_encode in its two-pass form (ensure_two_pass's scratch) over every row of
        ``text`` (u8 [rows, pitch], rows of at most ``stride`` bytes): -> (n_tok, err)."""
        import ctypes
        from . import _lib, ops
        B = int(text.shape[0])
        self.ensure_two_pass(B, stride)
        st = self.bpe_struct(True)
        n_tok = torch.empty(B, dtype=torch.int32, device=text.device)
        err = torch.empty(B, dtype=torch.uint8, device=text.device)
        ops.check(_lib.lib().rmi_bpe_encode(ctypes.addressof(st), text.data_ptr(), int(text.shape[1]), int(stride),
                                            text_len.data_ptr(), B, out.data_ptr(), int(out.shape[1]), None,
                                            n_tok.data_ptr(), None, None, err.data_ptr(), ops._stream(text.device)),
                  "rmi_bpe_encode")
        return n_tok, err

    def encode_rows(self, text: torch.Tensor, text_len: torch.Tensor, out: torch.Tensor,
                    out_len: Optional[torch.Tensor] = None, mark_byte: Optional[torch.Tensor] = None,
                    max_len: int = 0):
        """Append the ids of every text row to ``out`` (rmi_bpe_encode); max_len (0: the row
        pitch) bounds the rows' length.  -> (n_tok, mark_tok, err)."""
        from .torch_ops import direct
        return direct.bpe_encode(*self.args(), text, text_len, out, out_len, mark_byte, int(max_len),
                                 self.word_cache, self.exp_off if self.exp else None,
                                 self.exp_ids if self.exp else None, self.added_words, self.ascii_class)

    def encode(self, texts: Sequence[str], stride: int = None, two_pass: bool = False) -> List[Optional[List[int]]]:
        """Convenience (tests, tools): ids of each text, or None for a row the device flagged.
        two_pass: through the two-pass form of rmi_bpe_encode (the turn chain's)."""
        dev = self.byte_id.device
        rows = [t.encode("utf-8") for t in texts]
        stride = stride or max(4, (max((len(r) for r in rows), default=0) + 3) // 4 * 4)
        buf = np.zeros((len(rows), stride), np.uint8)
        for i, r in enumerate(rows):
            buf[i, :len(r)] = np.frombuffer(r, np.uint8)
        lens = torch.tensor([len(r) for r in rows], dtype=torch.int32, device=dev)
        out = torch.zeros(len(rows), max(stride, 1), dtype=torch.int64, device=dev)
        if two_pass:
            n_tok, err = self.encode_two_pass(torch.from_numpy(buf).to(dev), lens, out, stride)
        else:
            n_tok, _, err = self.encode_rows(torch.from_numpy(buf).to(dev), lens, out)
        n_tok, err, out = n_tok.cpu().tolist(), err.cpu().tolist(), out.cpu().numpy()
        return [None if e else out[i, :n].tolist() for i, (n, e) in enumerate(zip(n_tok, err))]


@functools.lru_cache(maxsize=None)
def _char_class_table():
    """Character pre-tokenizer: no class is read; only the NFC flag matters."""
    cls = np.zeros(0x110000, np.uint8)
    cls[_nfc_unsafe()] |= CP_UNSAFE
    blocks, block_of, data = {}, np.zeros(0x1100, np.uint16), []
    for hi in range(0x1100):
        blk = cls[hi * 256:(hi + 1) * 256].tobytes()
        if blk not in blocks:
            blocks[blk] = len(blocks)
            data.append(blk)
        block_of[hi] = blocks[blk]
    return block_of, np.frombuffer(b"".join(data), np.uint8).copy()
