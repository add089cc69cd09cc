// bigint.hpp — bounded Python-int arithmetic for the Countdown evaluator (countdown.hip).
//
// check_correctness (countdown/env.py:16-21) runs Python's eval, whose ints are unbounded: an
// answer like (a**b)//(c**d) passes through intermediates far past 64 bits and may still land
// on the target.  This header gives the evaluator's slow path exact integers up to 1024 bits of
// magnitude (Python semantics for + - * // % ** << >> & | ^ ~, unary -, int -> float and int / int
// correctly rounded as CPython does); a result past 1024 bits is reported as out of range (the
// caller flags RMI_ERR_UNSUP there, as before for 64 bits).
//
// A value is sign + magnitude in 32-bit limbs, least significant first, stored in caller-owned
// words (LDS on the device): w[0] = limb count n (0 = zero), w[1] = 1 if negative, w[2..2+n)
// the limbs, normalised (top limb nonzero).  Capacity kBigCap limbs (one more than the 1024-bit
// bound, so a product's carry limb lands inside the value before the bound is checked).
//
// Every routine is __host__ __device__ and allocation-free, so tests/native/bigint_driver.cpp
// runs the same code on the host against Python's ints (tests/test_bigint.py).
#pragma once
#include <math.h>
#include <stdint.h>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define RMI_BHD __host__ __device__ __forceinline__
#define RMI_BHDN __host__ __device__ __attribute__((noinline))
#else
#define RMI_BHD inline
#define RMI_BHDN inline
#endif

namespace rmi {

constexpr int kBigLimbs = 32;               // magnitudes below 2^1024
constexpr int kBigCap = kBigLimbs + 1;      // limbs of storage per value
constexpr int kBigWords = kBigCap + 2;      // + count and sign words
constexpr int kDivU = 2 * kBigLimbs + 4;    // true division's shifted dividend (<= 2100 bits) + 1
constexpr int kDivQ = 2 * kBigLimbs + 4;    // its quotient limbs before trimming

enum BigStatus : int { BIG_OK = 0, BIG_RANGE = 1, BIG_OVERFLOW = 2, BIG_ZERODIV = 3 };

RMI_BHD int bit_len32(uint32_t x) { return x ? 32 - __builtin_clz(x) : 0; }
RMI_BHD int big_n(const uint32_t* w) { return (int)w[0]; }
RMI_BHD bool big_neg(const uint32_t* w) { return w[1] != 0; }
RMI_BHD uint32_t* big_d(uint32_t* w) { return w + 2; }
RMI_BHD const uint32_t* big_d(const uint32_t* w) { return w + 2; }

RMI_BHD void big_norm(uint32_t* w, int n) {
  const uint32_t* d = w + 2;
  while (n > 0 && d[n - 1] == 0) --n;
  w[0] = (uint32_t)n;
  if (n == 0) w[1] = 0;
}
RMI_BHD int big_bits(const uint32_t* w) {
  const int n = big_n(w);
  return n ? 32 * (n - 1) + bit_len32(big_d(w)[n - 1]) : 0;
}
RMI_BHD void big_set_i64(uint32_t* w, long long v) {
  const unsigned long long m = v < 0 ? 0ull - (unsigned long long)v : (unsigned long long)v;
  w[2] = (uint32_t)m;
  w[3] = (uint32_t)(m >> 32);
  w[1] = v < 0 ? 1u : 0u;
  big_norm(w, 2);
}
RMI_BHD void big_copy(uint32_t* dst, const uint32_t* src) {
  const int n = big_n(src);
  for (int i = 0; i < n + 2; ++i) dst[i] = src[i];
}
// the value as an int64 when it is one
RMI_BHD bool big_to_i64(const uint32_t* w, long long& v) {
  const int n = big_n(w);
  if (n > 2) return false;
  const unsigned long long m = (n > 0 ? big_d(w)[0] : 0u) | (n > 1 ? (unsigned long long)big_d(w)[1] << 32 : 0ull);
  if (big_neg(w)) {
    if (m > 9223372036854775808ull) return false;
    v = (long long)(0ull - m);
  } else {
    if (m > 9223372036854775807ull) return false;
    v = (long long)m;
  }
  return true;
}
RMI_BHD int mag_cmp(const uint32_t* a, int an, const uint32_t* b, int bn) {
  if (an != bn) return an < bn ? -1 : 1;
  for (int i = an - 1; i >= 0; --i)
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return 0;
}

// ---- + and - (out may not alias a or b)
RMI_BHDN int big_add(const uint32_t* a, const uint32_t* b, bool sub, uint32_t* out) {
  const bool an = big_neg(a), bn = big_neg(b) != sub;
  const int na = big_n(a), nb = big_n(b);
  const uint32_t *da = big_d(a), *db = big_d(b);
  uint32_t* o = big_d(out);
  if (an == bn) {  // magnitudes add
    const int n = na > nb ? na : nb;
    unsigned long long c = 0;
    for (int i = 0; i < n; ++i) {
      c += (unsigned long long)(i < na ? da[i] : 0u) + (i < nb ? db[i] : 0u);
      o[i] = (uint32_t)c;
      c >>= 32;
    }
    o[n] = (uint32_t)c;
    out[1] = an ? 1u : 0u;
    big_norm(out, n + 1);
  } else {  // the larger magnitude minus the smaller, its sign
    const int c = mag_cmp(da, na, db, nb);
    const uint32_t *x = c >= 0 ? da : db, *y = c >= 0 ? db : da;
    const int nx = c >= 0 ? na : nb, ny = c >= 0 ? nb : na;
    long long br = 0;
    for (int i = 0; i < nx; ++i) {
      long long t = (long long)x[i] - (i < ny ? (long long)y[i] : 0) - br;
      br = t < 0;
      o[i] = (uint32_t)(t + (br << 32));
    }
    out[1] = (c >= 0 ? an : bn) ? 1u : 0u;
    big_norm(out, nx);
  }
  return big_bits(out) > 32 * kBigLimbs ? BIG_RANGE : BIG_OK;
}

// ---- magnitude product into out (no aliasing); BIG_RANGE past the bound
RMI_BHDN int big_mul(const uint32_t* a, const uint32_t* b, uint32_t* out) {
  const int na = big_n(a), nb = big_n(b);
  if (na == 0 || nb == 0) {
    out[0] = out[1] = 0;
    return BIG_OK;
  }
  if (na + nb - 1 > kBigLimbs) return BIG_RANGE;  // >= 2^(32 (na + nb - 2)) >= 2^1024
  const uint32_t *da = big_d(a), *db = big_d(b);
  uint32_t* o = big_d(out);
  const int n = na + nb;  // <= kBigCap
  for (int i = 0; i < n; ++i) o[i] = 0;
  for (int i = 0; i < na; ++i) {
    unsigned long long c = 0;
    for (int j = 0; j < nb; ++j) {
      c += (unsigned long long)da[i] * db[j] + o[i + j];
      o[i + j] = (uint32_t)c;
      c >>= 32;
    }
    o[i + nb] = (uint32_t)c;
  }
  out[1] = (big_neg(a) != big_neg(b)) ? 1u : 0u;
  big_norm(out, n);
  return big_bits(out) > 32 * kBigLimbs ? BIG_RANGE : BIG_OK;
}

// ---- magnitude division (Knuth D, Hacker's Delight divmnu with 32-bit limbs):
// u[0..m) / v[0..n) -> q[0..m-n+1) (if q), r[0..n) (if r); v[n-1] != 0, m >= n >= 1.
// un: scratch of m + 1 limbs, vn: scratch of n limbs.
RMI_BHDN void mag_divmod(const uint32_t* u, int m, const uint32_t* v, int n, uint32_t* q, uint32_t* r, uint32_t* un,
                         uint32_t* vn) {
  const unsigned long long b = 1ull << 32;
  if (n == 1) {
    unsigned long long k = 0;
    for (int j = m - 1; j >= 0; --j) {
      const unsigned long long t = k * b + u[j];
      if (q) q[j] = (uint32_t)(t / v[0]);
      k = t - (t / v[0]) * v[0];
    }
    if (r) r[0] = (uint32_t)k;
    return;
  }
  const int s = __builtin_clz(v[n - 1]);  // normalise: the divisor's top bit set
  for (int i = n - 1; i > 0; --i) vn[i] = s ? (v[i] << s) | (v[i - 1] >> (32 - s)) : v[i];
  vn[0] = v[0] << s;
  un[m] = s ? u[m - 1] >> (32 - s) : 0u;
  for (int i = m - 1; i > 0; --i) un[i] = s ? (u[i] << s) | (u[i - 1] >> (32 - s)) : u[i];
  un[0] = u[0] << s;
  for (int j = m - n; j >= 0; --j) {
    const unsigned long long num = (unsigned long long)un[j + n] * b + un[j + n - 1];
    unsigned long long qhat = num / vn[n - 1], rhat = num - qhat * vn[n - 1];
    while (qhat >= b || qhat * vn[n - 2] > b * rhat + un[j + n - 2]) {
      qhat -= 1;
      rhat += vn[n - 1];
      if (rhat >= b) break;
    }
    long long t, k = 0;
    for (int i = 0; i < n; ++i) {
      const unsigned long long p = qhat * vn[i];
      t = (long long)un[i + j] - k - (long long)(p & 0xFFFFFFFFull);
      un[i + j] = (uint32_t)t;
      k = (long long)(p >> 32) - (t >> 32);
    }
    t = (long long)un[j + n] - k;
    un[j + n] = (uint32_t)t;
    if (t < 0) {  // subtracted too much: add back
      qhat -= 1;
      unsigned long long c = 0;
      for (int i = 0; i < n; ++i) {
        c += (unsigned long long)un[i + j] + vn[i];
        un[i + j] = (uint32_t)c;
        c >>= 32;
      }
      un[j + n] += (uint32_t)c;
    }
    if (q) q[j] = (uint32_t)qhat;
  }
  if (r)
    for (int i = 0; i < n; ++i) r[i] = s ? (un[i] >> s) | (un[i + 1] << (32 - s)) : un[i];
}

// ---- Python floor division and modulo: q = a // b, r = a % b (either may be null; they may
// not alias a, b or each other).  un: kDivU + 1 limbs, vn: 2 kBigCap limbs of scratch (the
// second half holds the remainder magnitude).
RMI_BHDN int big_floordiv(const uint32_t* a, const uint32_t* b, uint32_t* q, uint32_t* r, uint32_t* un,
                          uint32_t* vn) {
  const int na = big_n(a), nb = big_n(b);
  if (nb == 0) return BIG_ZERODIV;
  const bool sa = big_neg(a), sb = big_neg(b);
  uint32_t* rem = vn + kBigCap;
  int nq = 0, nr;
  if (mag_cmp(big_d(a), na, big_d(b), nb) < 0) {  // |a| < |b|: quotient 0, remainder |a|
    for (int i = 0; i < na; ++i) rem[i] = big_d(a)[i];
    nr = na;
  } else {
    mag_divmod(big_d(a), na, big_d(b), nb, q ? big_d(q) : nullptr, rem, un, vn);
    nq = na - nb + 1;
    nr = nb;
  }
  bool rz = true;
  for (int i = 0; i < nr; ++i) rz &= rem[i] == 0;
  if (q) {
    if (nq == 0) q[0] = q[1] = 0;
    else {
      q[1] = 0;
      big_norm(q, nq);
    }
  }
  const bool flip = sa != sb && !rz;  // floor differs from truncation
  if (q && sa != sb) {
    if (flip) {  // q = -(|q| + 1)
      uint32_t* d = big_d(q);
      int n = big_n(q), i = 0;
      for (; i < n; ++i)
        if (++d[i] != 0) break;
      if (i == n) d[n++] = 1;
      big_norm(q, n);
    }
    if (big_n(q)) q[1] = 1;
  }
  if (r) {
    uint32_t* d = big_d(r);
    if (flip) {  // r = sign(b) * (|b| - |rem|)
      const uint32_t* db = big_d(b);
      long long br = 0;
      for (int i = 0; i < nb; ++i) {
        const long long t = (long long)db[i] - (i < nr ? (long long)rem[i] : 0) - br;
        br = t < 0;
        d[i] = (uint32_t)(t + (br << 32));
      }
      nr = nb;
    } else {  // r = sign(a) * |rem| (a and b share the sign, or the division is exact)
      for (int i = 0; i < nr; ++i) d[i] = rem[i];
    }
    r[1] = sb ? 1u : 0u;  // Python: the remainder takes the divisor's sign
    big_norm(r, nr);
  }
  return BIG_OK;
}

// ---- a ** e for an int exponent e >= 0 (Python long_pow): square and multiply through two
// scratch values t1, t2 (kBigWords each); out may not alias a, t1 or t2.
RMI_BHDN int big_pow(const uint32_t* a, unsigned long long e, uint32_t* out, uint32_t* t1, uint32_t* t2) {
  const bool neg = big_neg(a) && (e & 1);
  big_set_i64(out, 1);
  if (e == 0) return BIG_OK;
  const int bits = big_bits(a);
  if (bits == 0) {
    out[0] = out[1] = 0;
    return BIG_OK;
  }
  if (bits > 1 && e > 32ull * kBigLimbs) return BIG_RANGE;  // |a| >= 2: a ** e >= 2^e
  if (bits > 1) {
    uint32_t *base = t1, *tmp = t2;
    big_copy(base, a);
    base[1] = 0;
    for (;;) {
      if (e & 1) {
        const int st = big_mul(out, base, tmp);
        if (st) return st;
        big_copy(out, tmp);
      }
      e >>= 1;
      if (!e) break;
      const int st = big_mul(base, base, tmp);
      if (st) return st;
      uint32_t* sw = base;
      base = tmp;
      tmp = sw;
    }
  }
  out[1] = neg && big_n(out) ? 1u : 0u;
  return BIG_OK;
}

// ---- shifts (Python: a << k, a >> k = floor(a / 2^k)); out may not alias a
RMI_BHDN int big_shl(const uint32_t* a, unsigned long long k, uint32_t* out) {
  const int na = big_n(a);
  if (na == 0) {
    out[0] = out[1] = 0;
    return BIG_OK;
  }
  if ((unsigned long long)big_bits(a) + k > 32ull * kBigLimbs) return BIG_RANGE;
  const int lw = (int)(k >> 5), lb = (int)(k & 31);
  uint32_t* o = big_d(out);
  const uint32_t* d = big_d(a);
  for (int i = 0; i < lw; ++i) o[i] = 0;
  uint32_t carry = 0;
  for (int i = 0; i < na; ++i) {
    o[i + lw] = lb ? (d[i] << lb) | carry : d[i];
    carry = lb ? d[i] >> (32 - lb) : 0u;
  }
  o[na + lw] = carry;
  out[1] = a[1];
  big_norm(out, na + lw + 1);
  return BIG_OK;
}
RMI_BHDN void big_shr_floor(const uint32_t* a, unsigned long long k, uint32_t* out) {
  const int na = big_n(a);
  const bool neg = big_neg(a);
  const uint32_t* d = big_d(a);
  uint32_t* o = big_d(out);
  if (k >= 32ull * na) {  // every bit shifted out
    if (neg) big_set_i64(out, -1);
    else out[0] = out[1] = 0;
    return;
  }
  const int lw = (int)(k >> 5), lb = (int)(k & 31);
  bool lost = false;  // nonzero bits shifted out (floor rounds a negative value down)
  for (int i = 0; i < lw; ++i) lost |= d[i] != 0;
  if (lb) lost |= (d[lw] & ((1u << lb) - 1)) != 0;
  const int n = na - lw;
  for (int i = 0; i < n; ++i) {
    const uint32_t hi = i + lw + 1 < na ? d[i + lw + 1] : 0u;
    o[i] = lb ? (d[i + lw] >> lb) | (hi << (32 - lb)) : d[i + lw];
  }
  out[1] = neg ? 1u : 0u;
  big_norm(out, n);
  if (neg && lost) {  // -(|a| >> k) - 1
    int m = big_n(out), i = 0;
    for (; i < m; ++i)
      if (++o[i] != 0) break;
    if (i == m) o[m++] = 1;
    out[1] = 1;
    big_norm(out, m);
  }
}

// ---- & | ^ on two's complement values (infinite sign extension); out may not alias.
// op: 0 and, 1 or, 2 xor
RMI_BHDN int big_bitop(int op, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  const int na = big_n(a), nb = big_n(b);
  const int n = (na > nb ? na : nb) + 1;
  const bool sa = big_neg(a), sb = big_neg(b);
  // two's complement limbs on the fly: neg -> ~(|x| - 1)
  long long bra = 1, brb = 1;  // borrows of |x| - 1
  uint32_t* o = big_d(out);
  for (int i = 0; i < n; ++i) {
    uint32_t x = i < na ? big_d(a)[i] : 0u, y = i < nb ? big_d(b)[i] : 0u;
    if (sa) {
      const long long t = (long long)x - bra;
      bra = t < 0;
      x = ~(uint32_t)(t + (bra << 32));
    }
    if (sb) {
      const long long t = (long long)y - brb;
      brb = t < 0;
      y = ~(uint32_t)(t + (brb << 32));
    }
    o[i] = op == 0 ? (x & y) : (op == 1 ? (x | y) : (x ^ y));
  }
  const bool sr = op == 0 ? (sa && sb) : (op == 1 ? (sa || sb) : (sa != sb));
  if (sr) {  // back to magnitude: |r| = ~r + 1
    unsigned long long c = 1;
    for (int i = 0; i < n; ++i) {
      c += (uint32_t)~o[i];
      o[i] = (uint32_t)c;
      c >>= 32;
    }
  }
  out[1] = sr ? 1u : 0u;
  big_norm(out, n);
  return big_bits(out) > 32 * kBigLimbs ? BIG_RANGE : BIG_OK;
}

// ---- int -> float (PyLong_AsDouble: correctly rounded, half to even); BIG_OVERFLOW past DBL_MAX
RMI_BHDN int big_to_double(const uint32_t* a, double& out) {
  const int bits = big_bits(a);
  if (bits == 0) {
    out = 0.0;
    return BIG_OK;
  }
  const uint32_t* d = big_d(a);
  // the top 55 bits of |a| (or all of them) and a sticky bit for the rest
  const int sh = bits > 55 ? bits - 55 : 0;
  unsigned long long top = 0;
  bool sticky = false;
  for (int i = big_n(a) - 1; i >= 0; --i) {  // top = |a| >> sh, sticky = low bits != 0
    const int lo = 32 * i;
    if (lo + 32 <= sh) {
      sticky |= d[i] != 0;
      continue;
    }
    if (lo >= sh) top |= (unsigned long long)d[i] << (lo - sh);
    else {
      top |= (unsigned long long)d[i] >> (sh - lo);
      sticky |= (d[i] & ((1u << (sh - lo)) - 1)) != 0;
    }
  }
  if (sh > 0) {  // round 55 -> 53 bits, half to even
    const unsigned long long low = (top & 3) | (sticky ? 1u : 0u);
    top >>= 2;
    if ((low & 2) && ((low & 1) || (top & 1))) top += 1;
    const int e = sh + 2;
    if (top == (1ull << 53)) {
      top >>= 1;
      if (e + 1 + 53 > 1024) return BIG_OVERFLOW;
      out = ldexp((double)top, e + 1);
    } else {
      if (e + 53 > 1024) return BIG_OVERFLOW;
      out = ldexp((double)top, e);
    }
  } else {
    out = (double)top;
  }
  if (big_neg(a)) out = -out;
  return BIG_OK;
}

// ---- int / int (CPython long_true_divide: correctly rounded, subnormals included, OverflowError
// past DBL_MAX).  un: kDivU + 1 limbs, vn: kBigCap, qs: kDivQ, xs: kDivU limbs of scratch.
RMI_BHDN int big_true_div(const uint32_t* a, const uint32_t* b, double& out, uint32_t* un, uint32_t* vn, uint32_t* qs,
                          uint32_t* xs) {
  const int nb = big_n(b);
  if (nb == 0) return BIG_ZERODIV;
  const bool negate = big_neg(a) != big_neg(b);
  const int abits = big_bits(a), bbits = big_bits(b);
  if (abits == 0) {
    out = negate ? -0.0 : 0.0;
    return BIG_OK;
  }
  const int DBL_MANT = 53, DBL_MINE = -1021, DBL_MAXE = 1024;
  const int diff = abits - bbits;
  if (diff > DBL_MAXE) return BIG_OVERFLOW;
  if (diff < DBL_MINE - DBL_MANT - 1) {
    out = negate ? -0.0 : 0.0;
    return BIG_OK;
  }
  const int shift = (diff > DBL_MINE ? diff : DBL_MINE) - DBL_MANT - 2;
  bool inexact = false;
  // x = |a| * 2^-shift into xs
  const uint32_t* da = big_d(a);
  const int na = big_n(a);
  int nx;
  if (shift <= 0) {
    const int k = -shift, lw = k >> 5, lb = k & 31;
    for (int i = 0; i < lw; ++i) xs[i] = 0;
    uint32_t carry = 0;
    for (int i = 0; i < na; ++i) {
      xs[i + lw] = lb ? (da[i] << lb) | carry : da[i];
      carry = lb ? da[i] >> (32 - lb) : 0u;
    }
    xs[na + lw] = carry;
    nx = na + lw + 1;
  } else {
    const int lw = shift >> 5, lb = shift & 31;
    for (int i = 0; i < lw && i < na; ++i) inexact |= da[i] != 0;
    if (lb && lw < na) inexact |= (da[lw] & ((1u << lb) - 1)) != 0;
    nx = na - lw;
    for (int i = 0; i < nx; ++i) {
      const uint32_t hi = i + lw + 1 < na ? da[i + lw + 1] : 0u;
      xs[i] = lb ? (da[i + lw] >> lb) | (hi << (32 - lb)) : da[i + lw];
    }
  }
  while (nx > 0 && xs[nx - 1] == 0) --nx;
  // x //= |b|, inexact |= remainder != 0
  unsigned long long x = 0;
  if (nx < nb) {  // quotient 0 cannot happen (x has >= 54 bits more than b)... guard anyway
    inexact |= nx > 0;
  } else {
    uint32_t* rem = vn + kBigCap;  // callers give vn 2 kBigCap limbs
    mag_divmod(xs, nx, big_d(b), nb, qs, rem, un, vn);
    for (int i = 0; i < nb; ++i) inexact |= rem[i] != 0;
    const int nq = nx - nb + 1;
    for (int i = nq - 1; i >= 2; --i)
      if (qs[i]) return BIG_OVERFLOW;  // cannot happen: the quotient has <= 56 bits
    x = (unsigned long long)qs[0] | (nq > 1 ? (unsigned long long)qs[1] << 32 : 0ull);
  }
  const int x_bits = x ? 64 - __builtin_clzll(x) : 0;
  if (x_bits == 0) {
    out = negate ? -0.0 : 0.0;
    return BIG_OK;
  }
  const int extra = (x_bits > DBL_MINE - shift ? x_bits : DBL_MINE - shift) - DBL_MANT;
  const unsigned long long mask = 1ull << (extra - 1);
  unsigned long long low = x | (inexact ? 1ull : 0ull);
  if ((low & mask) && (low & (3ull * mask - 1ull))) low += mask;
  x = low & ~(2ull * mask - 1ull);
  const double dx = (double)x;
  if (shift + x_bits >= DBL_MAXE && (shift + x_bits > DBL_MAXE || dx == ldexp(1.0, x_bits))) return BIG_OVERFLOW;
  const double r = ldexp(dx, shift);
  out = negate ? -r : r;
  return BIG_OK;
}

// ---- a decimal literal (digits and '_') -> out; BIG_RANGE past the bound
RMI_BHDN int big_from_dec(const uint8_t* s, int n, uint32_t* out) {
  out[0] = out[1] = 0;
  uint32_t* d = big_d(out);
  int m = 0;
  for (int i = 0; i < n; ++i) {
    if (s[i] == '_') continue;
    unsigned long long c = (unsigned long long)(s[i] - '0');
    for (int k = 0; k < m; ++k) {
      c += (unsigned long long)d[k] * 10u;
      d[k] = (uint32_t)c;
      c >>= 32;
    }
    if (c) {
      if (m >= kBigCap) return BIG_RANGE;
      d[m++] = (uint32_t)c;
    }
    out[0] = (uint32_t)m;
    if (big_bits(out) > 32 * kBigLimbs) return BIG_RANGE;
  }
  big_norm(out, m);
  return BIG_OK;
}

}  // namespace rmi
