import random
H = 0x80808080
M = 0xFFFFFFFF
def nz(z):  # bit 7 set in each nonzero byte
    return ((((z & 0x7F7F7F7F) + 0x7F7F7F7F) | z) & H) & M
def zero(z): return ~nz(z) & H & M
def eq(x, k): return zero(x ^ (k * 0x01010101))
def shl(x, s): return (x << s) & M
def alignbyte(hi, lo, s): return ((hi << 32 | lo) >> (8 * s)) & M
def dword_bad(w, wp):
    c = w
    p1, p2, p3 = alignbyte(w, wp, 3), alignbyte(w, wp, 2), alignbyte(w, wp, 1)
    ge_c0 = lambda x: x & shl(x, 1) & H
    ge_e0 = lambda x: x & shl(x, 1) & shl(x, 2) & H
    ge_f0 = lambda x: x & shl(x, 1) & shl(x, 2) & shl(x, 3) & H
    ge_f8 = lambda x: x & shl(x, 1) & shl(x, 2) & shl(x, 3) & shl(x, 4) & H
    cont = c & ~shl(c, 1) & H
    exp = ge_c0(p1) | ge_e0(p2) | ge_f0(p3)
    err = (cont ^ exp) & H
    err |= zero((c & 0xFEFEFEFE) ^ 0xC0C0C0C0)                       # C0, C1
    err |= ge_f8(c) | (zero((c & 0xF8F8F8F8) ^ 0xF0F0F0F0) & shl(c, 5) & (shl(c, 6) | shl(c, 7)) & H)  # F5..FF
    b5, b4 = shl(c, 2), shl(c, 3)
    err |= eq(p1, 0xE0) & ~b5 & H
    err |= eq(p1, 0xED) & b5 & H
    err |= eq(p1, 0xF0) & ~(b5 | b4) & H
    err |= eq(p1, 0xF4) & (b5 | b4) & H
    return err & M
def invalid(bs):
    n = len(bs)
    buf = bytes(4) + bs + bytes(8 + 4)
    for q in range((n + 3 + 3) // 4):
        if 4 * q >= n + 3: break
        w = int.from_bytes(buf[4 + 4 * q: 8 + 4 * q], 'little')
        wp = int.from_bytes(buf[4 * q: 4 + 4 * q], 'little')
        if dword_bad(w, wp): return True
    return False
def ref(bs):
    try: bs.decode('utf-8'); return False
    except UnicodeDecodeError: return True
rng = random.Random(1)
pool = [0x41, 0x80, 0x8F, 0x90, 0x9F, 0xA0, 0xBF, 0xC0, 0xC1, 0xC2, 0xDF, 0xE0, 0xE1, 0xEC, 0xED, 0xEE, 0xEF, 0xF0, 0xF1, 0xF3, 0xF4, 0xF5, 0xF7, 0xF8, 0xFF, 0x00, 0x7F]
bad = 0
for it in range(300000):
    L = rng.randint(0, 12)
    bs = bytes(rng.choice(pool) if rng.random() < 0.8 else rng.randint(0, 255) for _ in range(L))
    if invalid(bs) != ref(bs):
        bad += 1
        if bad < 10: print("MISMATCH", bs.hex(), invalid(bs), ref(bs))
# valid texts
for it in range(20000):
    s = ''.join(chr(rng.choice([rng.randint(0x20, 0x7e), rng.randint(0x80, 0x7ff), rng.randint(0x800, 0xd7ff), rng.randint(0xe000, 0xffff), rng.randint(0x10000, 0x10ffff)])) for _ in range(rng.randint(0, 20)))
    bs = s.encode()
    if invalid(bs): bad += 1; print("FALSE POS", bs.hex())
print("mismatches", bad)
