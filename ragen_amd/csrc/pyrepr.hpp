// pyrepr.hpp — CPython's str() of a float and of an int, for the prompt text built on the device.
//
// The prompt's "Reward:\n{reward}\n" block (ctx_manager.py:260-262) prints the turn reward with
// Python's str(): for a float that is repr (float_repr_style 'short': the SHORTEST decimal string
// that reads back as the same double, the nearest of those to the value, round-half-even on a
// tie — David Gay's dtoa mode 0), then PyOS_double_to_string's 'r' layout: exponent form when
// the decimal point position is <= -4 or > 16 ("1e-05", "1.5e+16"), else fixed with ".0" added
// to integral values ("10.0", "0.0001").
//
// A double-arithmetic fast path settles every value whose repr has at most 15 significant
// digits (see py_float_repr); the rest takes the exact integer search, starting at the digit
// count the fast path reached (16 when it ruled out every shorter one: a sum like
// -0.1 + -0.1 + -0.1 = -0.30000000000000004 costs two rounds of it, not seventeen).
// Exact integer arithmetic: the rounding interval of x (the half-way points to its neighbours)
// is scaled by 10^s and 2^K into 128-bit integers, and for n = 1, 2, ... the first n whose
// n-digit grid has a point inside the interval gives the digits.  That needs
// 1e-5 <= |x| < 2^53 (every reward RAGEN's envs produce); other finite values return -1 and
// the row is left to the host.  No 128-bit division (shifts and 64-bit division only), so the
// same code runs on the device and in the host test driver (tests/test_pyrepr.py).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define RMI_HD __host__ __device__ __forceinline__
#else
#define RMI_HD inline
#endif

namespace rmi {

typedef unsigned __int128 u128;

RMI_HD u128 pow10_u128(int k) {
  u128 r = 1;
  for (int i = 0; i < k; ++i) r *= 10u;
  return r;
}

// floor / ceil of a / 2^k for k >= 0 (k may exceed 127)
RMI_HD u128 shr_floor(u128 a, int k) { return k >= 128 ? (u128)0 : (a >> k); }
RMI_HD u128 shr_ceil(u128 a, int k) {
  if (k >= 128) return a ? 1 : 0;
  const u128 q = a >> k;
  return (q << k) == a ? q : q + 1;
}

// Decimal digits of v (v > 0) into out, most significant first; -> count.
RMI_HD void reverse_chars(char* a, int n) {
  for (int i = 0, j = n - 1; i < j; ++i, --j) {
    const char t = a[i];
    a[i] = a[j];
    a[j] = t;
  }
}

RMI_HD int u128_digits(u128 v, char* out) {  // (no local array: out may be LDS on the device)
  int n = 0;
  // every value formatted here is below 10^18 (17 significant digits, or an integer below
  // 2^53): 64-bit division by 10, which compiles to a multiply-high; a 128-bit division on the
  // device is a bit-serial loop (it made the reward piece of a prompt row cost ~25 k cycles)
  uint64_t u = (uint64_t)v;
  while (v >> 64) {
    out[n++] = (char)('0' + (uint64_t)(v % 10u));
    v /= 10u;
    u = (uint64_t)v;
  }
  while (u) {
    out[n++] = (char)('0' + u % 10u);
    u /= 10u;
  }
  reverse_chars(out, n);
  return n;
}

// str(int) for |v| < 2^63.
RMI_HD int py_int_repr(int64_t v, char* out) {
  int n = 0;
  uint64_t u = (uint64_t)v;
  if (v < 0) {
    out[n++] = '-';
    u = 0 - u;
  }
  if (u == 0) {
    out[n++] = '0';
    return n;
  }
  int k = 0;
  while (u) {
    out[n + k++] = (char)('0' + u % 10u);
    u /= 10u;
  }
  reverse_chars(out + n, k);
  return n + k;
}

// Lay out digits d[0..nd) with the decimal point at position decpt as PyOS_double_to_string
// 'r' does; -> length.
RMI_HD int py_layout(bool neg, const char* d, int nd, int decpt, char* out) {
  int n = 0;
  if (neg) out[n++] = '-';
  if (decpt <= -4 || decpt > 16) {
    out[n++] = d[0];
    if (nd > 1) {
      out[n++] = '.';
      for (int i = 1; i < nd; ++i) out[n++] = d[i];
    }
    int e = decpt - 1;
    out[n++] = 'e';
    out[n++] = e < 0 ? '-' : '+';
    if (e < 0) e = -e;
    if (e >= 100) out[n++] = (char)('0' + e / 100);
    out[n++] = (char)('0' + (e / 10) % 10);
    out[n++] = (char)('0' + e % 10);
  } else if (decpt <= 0) {
    out[n++] = '0';
    out[n++] = '.';
    for (int i = 0; i < -decpt; ++i) out[n++] = '0';
    for (int i = 0; i < nd; ++i) out[n++] = d[i];
  } else if (decpt >= nd) {
    for (int i = 0; i < nd; ++i) out[n++] = d[i];
    for (int i = nd; i < decpt; ++i) out[n++] = '0';
    out[n++] = '.';
    out[n++] = '0';
  } else {
    for (int i = 0; i < decpt; ++i) out[n++] = d[i];
    out[n++] = '.';
    for (int i = decpt; i < nd; ++i) out[n++] = d[i];
  }
  return n;
}

// repr(float(x)); -> length written to out (<= 32), or -1 outside 1e-5 <= |x| < 2^53.
// scratch: >= 40 bytes for the digits (LDS on the device: no per-lane register array).
RMI_HD int py_float_repr(double x, char* out, char* scratch) {
  const uint64_t bits = __builtin_bit_cast(uint64_t, x);
  const bool neg = bits >> 63;
  const int bexp = (int)((bits >> 52) & 0x7FF);
  const uint64_t frac = bits & ((1ull << 52) - 1);
  int n = 0;
  if (bexp == 0x7FF) {
    if (frac) {
      out[0] = 'n', out[1] = 'a', out[2] = 'n';
      return 3;
    }
    if (neg) out[n++] = '-';
    out[n++] = 'i', out[n++] = 'n', out[n++] = 'f';
    return n;
  }
  if (bexp == 0 && frac == 0) {
    if (neg) out[n++] = '-';
    out[n++] = '0', out[n++] = '.', out[n++] = '0';
    return n;
  }
  const double ax = neg ? -x : x;
  if (!(ax >= 1e-5 && ax < 9007199254740992.0)) return -1;
  const uint64_t f = frac | (1ull << 52);  // normal: |x| >= 1e-5
  const int e = bexp - 1075;               // |x| = f * 2^e
  char* d = scratch;
  if (e >= 0) {  // 2^52 <= |x| < 2^53: an integer, alone in its rounding interval
    const int nd0 = u128_digits((u128)f << e, d);
    int nd = nd0;
    while (nd > 1 && d[nd - 1] == '0') --nd;
    return py_layout(neg, d, nd, nd0, out);
  }
  // Fast path, exact, for reprs of at most 15 significant digits (every reward RAGEN's envs
  // produce): at scale 10^s the rounding interval of |x| is narrower than 10^15 * 2^-52 < 0.23,
  // so at most one integer c lies in it, and float(c * 10^-s) is the IEEE quotient c / 10^s
  // (or product c * 10^-s): c < 2^53 and 10^|s| <= 10^22 are exact doubles and the operation
  // is correctly rounded.  The scales are tried upward from the one where c first reaches 1,
  // so the first hit has the fewest digits.  Anything else takes the exact search below.
  int nd_min = 1;  // the exact search's first digit count: fewer were ruled out here
  {
    int D0 = 0;  // floor(log10 |x|), possibly off by one: only where the scan starts
    for (double t = ax; t >= 10.0; t /= 10.0) ++D0;
    for (double t = ax; t < 1.0; t *= 10.0) --D0;
    int s = -D0 - 1;  // in [-16, 4] over the supported range
    double pw = 1.0;  // 10^|s|, exact (every power of ten up to 10^22 is a double)
    for (int i = 0; i < (s < 0 ? -s : s); ++i) pw *= 10.0;
    for (; s <= 22; pw = s >= 0 ? pw * 10.0 : pw / 10.0, ++s) {
      const double y = s >= 0 ? ax * pw : ax / pw;
      if (y >= 1e15) {  // more than 15 digits: every shorter repr was tried and failed
        nd_min = 16;
        break;
      }
      const double m = __builtin_rint(y);
      int hits = 0;
      double hit = 0.0;
      for (int dm = -1; dm <= 1; ++dm) {
        const double c = m + dm;
        if (c < 1.0) continue;
        if ((s >= 0 ? c / pw : c * pw) == ax) {
          ++hits;
          hit = c;
        }
      }
      if (hits > 1) {  // two candidates at this scale: the exact search decides, from about here
        int dm = 0;
        for (uint64_t u = (uint64_t)m; u; u /= 10u) ++dm;
        nd_min = dm > 2 ? dm - 1 : 1;
        break;
      }
      if (hits == 1) {
        int k = 0;
        for (uint64_t u = (uint64_t)hit; u; u /= 10u) d[k++] = (char)('0' + u % 10u);
        reverse_chars(d, k);
        const int decpt = k - s;
        while (k > 1 && d[k - 1] == '0') --k;
        return py_layout(neg, d, k, decpt, out);
      }
    }
  }
  // |x| = V / 2^K with V = 4f; interval [(4f - dl) / 2^K, (4f + 2) / 2^K], closed iff f even
  const int K = 2 - e;
  const u128 V = (u128)f << 2;
  const u128 lo = V - ((f == (1ull << 52) && bexp > 1) ? 1u : 2u), hi = V + 2u;
  const bool closed = (f & 1) == 0;
  // D = floor(log10 |x|), exact: 10^D <= |x| < 10^(D+1)
  int D = 0;
  {
    double t = ax;
    while (t >= 10.0) t /= 10.0, ++D;
    while (t < 1.0) t *= 10.0, --D;
    auto ge_pow10 = [&](int p) -> bool {  // |x| >= 10^p ?
      return p >= 0 ? V >= (pow10_u128(p) << K) : V * pow10_u128(-p) >= ((u128)1 << K);
    };
    while (!ge_pow10(D)) --D;
    while (ge_pow10(D + 1)) ++D;
  }
  for (int nd = nd_min; nd <= 17; ++nd) {
    const int s = nd - 1 - D;  // candidates: integers c with c / 10^s in the interval
    u128 cmin, cmax, cnear;
    bool tie;
    if (s >= 0) {
      const u128 p = pow10_u128(s);
      const u128 L = lo * p, H = hi * p, X = V * p;
      cmin = shr_ceil(L, K);
      cmax = shr_floor(H, K);
      if (!closed && (cmin << K) == L) ++cmin;
      if (!closed && (cmax << K) == H) --cmax;
      cnear = shr_floor(X, K);
      const u128 r = X - (cnear << K), half = (u128)1 << (K - 1);
      tie = r == half;
      if (r > half || (tie && (cnear & 1))) ++cnear;
    } else {
      // c * 10^-s * 2^K in [lo, hi]: the quotient of lo, hi, V by 2^K, then by 10^-s
      const uint64_t q10 = (uint64_t)pow10_u128(-s);
      auto div_floor = [&](u128 a) -> u128 { return shr_floor(a, K) / q10; };
      auto exact = [&](u128 a, u128 c) -> bool { return ((c * q10) << K) == a; };
      cmin = div_floor(lo);
      if (!exact(lo, cmin) || !closed) ++cmin;
      if (exact(lo, cmin - 1) && closed) --cmin;
      cmax = div_floor(hi);
      if (!closed && exact(hi, cmax)) --cmax;
      cnear = div_floor(V);
      const u128 base = (cnear * q10) << K, unit = (u128)q10 << K;
      const u128 r = V - base;
      tie = 2 * r == unit;
      if (2 * r > unit || (tie && (cnear & 1))) ++cnear;
    }
    if (cmin > cmax) continue;
    u128 c = cnear < cmin ? cmin : (cnear > cmax ? cmax : cnear);
    int decpt = D + 1;
    int k = u128_digits(c, d);
    if (k > nd) decpt += k - nd;  // c == 10^nd: one more integer digit
    while (k > 1 && d[k - 1] == '0') --k;
    return py_layout(neg, d, k, decpt, out);
  }
  return -1;
}

}  // namespace rmi
