"""The decode's UTF-8 validity test (parse_core.hpp utf8_dword_bad: SWAR over 4 bytes per lane)
restated bit for bit in Python, against CPython's strict UTF-8 decode on random byte strings
(biased to the boundary bytes of Unicode Table 3-7) and on valid texts of 1- to 4-byte
characters.  The device function itself is pinned by tests/test_gpu_parse.py (invalid UTF-8
vocabularies, the lossy rewrite) and the token-turn tests."""
import random

H, M = 0x80808080, 0xFFFFFFFF


def zero(z):  # bit 7 of each zero byte
    return ~((((z & 0x7F7F7F7F) + 0x7F7F7F7F) | z) & H) & H & M


def eq(x, k):
    return zero(x ^ (k * 0x01010101))


def shl(x, s):
    return (x << s) & M


def alignbyte(hi, lo, s):  # v_alignbyte_b32
    return ((hi << 32 | lo) >> (8 * s)) & M


def dword_bad(w, wp):
    """utf8_dword_bad: bit 7 of each bad byte of dword w (wp: the dword before it)."""
    c = w
    p1, p2, p3 = alignbyte(w, wp, 3), alignbyte(w, wp, 2), alignbyte(w, wp, 1)
    cont = c & ~shl(c, 1) & H
    expect = (p1 & shl(p1, 1)) | (p2 & shl(p2, 1) & shl(p2, 2)) | (p3 & shl(p3, 1) & shl(p3, 2) & shl(p3, 3))
    err = (cont ^ expect) & H
    err |= zero((c & 0xFEFEFEFE) ^ 0xC0C0C0C0)  # C0, C1
    err |= c & shl(c, 1) & shl(c, 2) & shl(c, 3) & shl(c, 4)  # F8..FF
    err |= zero((c & 0xF8F8F8F8) ^ 0xF0F0F0F0) & shl(c, 5) & (shl(c, 6) | shl(c, 7))  # F5..F7
    b5, b4 = shl(c, 2), shl(c, 3)
    err |= eq(p1, 0xE0) & ~b5
    err |= eq(p1, 0xED) & b5
    err |= eq(p1, 0xF0) & ~(b5 | b4)
    err |= eq(p1, 0xF4) & (b5 | b4)
    return err & H


def invalid(bs):
    """The row loop of detok_row: dwords q with 4q < n + 3, zero bytes before and after the row."""
    n = len(bs)
    buf = bytes(4) + bs + bytes(12)
    for q in range((n + 3 + 3) // 4):
        w = int.from_bytes(buf[4 + 4 * q: 8 + 4 * q], "little")
        wp = int.from_bytes(buf[4 * q: 4 + 4 * q], "little")
        if dword_bad(w, wp):
            return True
    return False


def strict_invalid(bs):
    try:
        bs.decode("utf-8")
        return False
    except UnicodeDecodeError:
        return True


POOL = [0x41, 0x80, 0x8F, 0x90, 0x9F, 0xA0, 0xBF, 0xC0, 0xC1, 0xC2, 0xDF, 0xE0, 0xE1, 0xEC, 0xED, 0xEE, 0xEF,
        0xF0, 0xF1, 0xF3, 0xF4, 0xF5, 0xF7, 0xF8, 0xFF, 0x00, 0x7F]


def test_swar_validity_equals_strict_decode():
    rng = random.Random(1)
    for _ in range(60000):
        bs = bytes(rng.choice(POOL) if rng.random() < 0.8 else rng.randint(0, 255) for _ in range(rng.randint(0, 12)))
        assert invalid(bs) == strict_invalid(bs), bs.hex()


def test_swar_validity_accepts_valid_text():
    rng = random.Random(2)
    for _ in range(5000):
        s = "".join(chr(rng.choice([rng.randint(0x20, 0x7E), rng.randint(0x80, 0x7FF), rng.randint(0x800, 0xD7FF),
                                    rng.randint(0xE000, 0xFFFF), rng.randint(0x10000, 0x10FFFF)]))
                    for _ in range(rng.randint(0, 20)))
        assert not invalid(s.encode())
