"""CPU restatement of rmi_bpe_encode (ragen_amd/csrc/bpe.hip) — TEST INFRASTRUCTURE.

Only tests/ may import it, as a checker.  It states, in plain Python over the same device
tables (ragen_amd.tokenizer.DeviceTokenizer's numpy sources), the algorithm the kernel runs:
leftmost-longest added tokens, the Qwen2 pre-tokenizer regex written as its seven
alternatives over code-point classes (the kernel's match_serial), and BPE merging by the
lowest (rank, position) pair through the open-addressed merge table.  tests/test_tokenizer.py
checks it against the `tokenizers` library itself (the reference tokenizer RAGEN calls at
ctx_manager.py:265-278), so the tables and the rules are pinned on the CPU; the GPU tests
then compare the kernel with the library directly.
"""
import numpy as np

L, N, W, NL, UNSAFE = 1, 2, 4, 8, 16


class Tables:
    def __init__(self, cp_block, cp_class, byte_id, merges, merge_mask, merge_shift, pretok, nfc, added):
        self.cp_block, self.cp_class = np.asarray(cp_block, np.int64), np.asarray(cp_class, np.uint8)
        self.byte_id = np.asarray(byte_id, np.int64)
        m = np.asarray(merges).view(np.uint64)
        self.keys, self.vals = m[0::2], m[1::2]
        self.mask, self.shift = int(merge_mask), int(merge_shift)
        self.pretok, self.nfc = int(pretok), int(nfc)
        self.added = sorted(((c.encode("utf-8"), i) for c, i in added.items()), key=lambda x: -len(x[0]))

    def cls(self, cp):
        return int(self.cp_class[self.cp_block[cp >> 8] * 256 + (cp & 255)])

    def lookup(self, a, b):
        key = (a << 32) | b
        h = ((key * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF) >> self.shift
        while True:
            k = int(self.keys[h])
            if k == key:
                v = int(self.vals[h])
                return v >> 32, v & 0xFFFFFFFF
            if k == 0xFFFFFFFFFFFFFFFF:
                return None
            h = (h + 1) & self.mask


def _contraction(t, p, lim):
    if p + 1 >= lim:
        return 0
    a = t[p + 1]
    a_is = 65 <= (a & 0xDF) <= 90
    if a_is and (a | 0x20) in b"stmd":
        return 2
    if a == 0xC5 and p + 2 < lim and t[p + 2] == 0xBF:
        return 3
    if p + 2 >= lim:
        return 0
    b = t[p + 2]
    if not (a_is and 65 <= (b & 0xDF) <= 90):
        return 0
    return 3 if bytes([a | 0x20, b | 0x20]) in (b"re", b"ve", b"ll") else 0


def _match(t, C, start, p, s1):
    """bpe.hip match_serial: the Qwen2 regex at char start p of the segment [.., s1)."""
    cat = lambda q: C[q] if q < s1 else 0  # noqa: E731
    is_o = lambda q: q < s1 and not (C[q] & (L | N | W))  # noqa: E731

    def run(q, bit):
        while q < s1 and C[q] & bit:
            q += 1
        return q

    def run_o(q):
        while is_o(q):
            q += 1
        return q
    if t[p] == 0x27:
        ln = _contraction(t, p, s1)
        if ln:
            return ln
    n0 = p + 1
    while n0 < s1 and not start[n0]:
        n0 += 1
    c = cat(p)
    if c & L:
        return run(p, L) - p
    if not (c & (NL | N)) and cat(n0) & L:
        return run(n0, L) - p
    if c & N:
        return n0 - p
    if t[p] == 0x20 and is_o(n0):
        return run(run_o(n0), NL) - p
    if not (c & W):
        return run(run_o(p), NL) - p
    e = run(p, W)
    nls = [q for q in range(p, e) if C[q] & NL]
    if nls:
        return nls[-1] + 1 - p
    if e == s1:
        return e - p
    ls = max(q for q in range(p, e) if start[q])
    return ls - p if ls > p else e - p


def encode(tab: Tables, text: str):
    """-> list of ids, or None where the kernel flags the row (an NFC-unsafe code point)."""
    t = text.encode("utf-8")
    n = len(t)
    C = [0] * n
    start = [False] * n
    p = 0
    for ch in text:
        cls = tab.cls(ord(ch))
        if tab.nfc and cls & UNSAFE:
            return None
        ln = len(ch.encode("utf-8"))
        start[p] = True
        for k in range(ln):
            C[p + k] = cls & (L | N | W | NL)
        p += ln
    # added tokens, leftmost-longest
    spans, cur = [], 0
    for q in range(n):
        if q < cur or not start[q]:
            continue
        for blob, tid in tab.added:
            if t.startswith(blob, q):
                spans.append((q, len(blob), tid))
                cur = q + len(blob)
                break
    pieces, q, si = [], 0, 0
    while q < n:
        if si < len(spans) and spans[si][0] == q:
            pieces.append(("added", spans[si][2]))
            q += spans[si][1]
            si += 1
            continue
        s1 = spans[si][0] if si < len(spans) else n
        ln = len(text_char_at(t, q)) if tab.pretok == 1 else _match(t, C, start, q, s1)
        pieces.append(("text", t[q:q + ln]))
        q += ln
    out = []
    for kind, v in pieces:
        if kind == "added":
            out.append(v)
            continue
        sym = [int(tab.byte_id[x]) for x in v]
        while len(sym) > 1:
            best = None
            for i in range(len(sym) - 1):
                r = tab.lookup(sym[i], sym[i + 1])
                if r is not None and (best is None or r[0] < best[0]):
                    best = (r[0], i, r[1])
            if best is None:
                break
            _, i, nid = best
            sym[i:i + 2] = [nid]
        out.extend(sym)
    return out


def text_char_at(t: bytes, q: int) -> bytes:
    b = t[q]
    ln = 1 if b < 0x80 else 2 if b < 0xE0 else 3 if b < 0xF0 else 4
    return t[q:q + ln]


def tables_of(dt) -> Tables:
    """A Tables from a ragen_amd.tokenizer.DeviceTokenizer (its tensors copied to the host)."""
    return Tables(dt.cp_block.cpu().numpy().view(np.uint16), dt.cp_class.cpu().numpy(), dt.byte_id.cpu().numpy(),
                  dt.merges.cpu().numpy(), dt.merge_mask, dt.merge_shift, dt.pretok, dt.nfc, dt.added)
