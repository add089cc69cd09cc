// countdown.hip — Countdown rule reward on device (gfx950), one thread per answer.
//
// Replaces CountdownEnv.step/compute_reward (countdown/env.py:58-78) with
//   check_format      (:9-14)  re.findall(r'\d+') multiset == nums   -> exact, incl. every
//                               Unicode Nd digit (Python 3.10 / Unicode 13.0 table below)
//   check_correctness (:16-21) eval(expr, {"__builtins__": None}, {}) within 1e-5 of target
// The evaluator implements Python's expression semantics for the grammar an arithmetic
// answer can use: int literals (underscores, no leading zeros), float literals, + - * / //
// % ** << >> & | ^, unary + - ~, parentheses, whitespace, '#' comments, Python int/float
// rules (true division, floor division/modulo signs, int**negative -> float, ZeroDivision
// -> not correct).  Bytes whose eval result the evaluator does not model (letters and
// keywords, quotes, '[', '{', '.', comparisons, '\\') make the answer "not correct" AND set
// RMI_ERR_UNSUP in err[] so a caller can see the envelope was left; bare names are modelled
// (every lookup raises under {"__builtins__": None}: not correct, see name_outcome);
// every other byte only yields errors in Python too (SyntaxError/TypeError -> False).
// Python's ints are unbounded: an int past 64 bits (a literal, or an intermediate such as the
// a**b of (a**b)//(c**d)) continues in bounded multi-word arithmetic (bigint.hpp, magnitudes
// below 2^1024, in the row's LDS); only a value past that bound is flagged RMI_ERR_UNSUP.
#include <math.h>

#include "bigint.hpp"
#include "common.hpp"

namespace rmi {
namespace {

__constant__ uint32_t kNdStarts[65] = {
    0x30,    0x660,   0x6f0,   0x7c0,   0x966,   0x9e6,   0xa66,   0xae6,   0xb66,   0xbe6,   0xc66,   0xce6,   0xd66,
    0xde6,   0xe50,   0xed0,   0xf20,   0x1040,  0x1090,  0x17e0,  0x1810,  0x1946,  0x19d0,  0x1a80,  0x1a90,  0x1b50,
    0x1bb0,  0x1c40,  0x1c50,  0xa620,  0xa8d0,  0xa900,  0xa9d0,  0xa9f0,  0xaa50,  0xabf0,  0xff10,  0x104a0, 0x10d30,
    0x11066, 0x110f0, 0x11136, 0x111d0, 0x112f0, 0x11450, 0x114d0, 0x11650, 0x116c0, 0x11730, 0x118e0, 0x11950, 0x11c50,
    0x11d50, 0x11da0, 0x16a60, 0x16b50, 0x1d7ce, 0x1d7d8, 0x1d7e2, 0x1d7ec, 0x1d7f6, 0x1e140, 0x1e2f0, 0x1e950, 0x1fbf0};

__device__ __forceinline__ int nd_value(uint32_t cp) {  // -1 if not a decimal digit
  if (cp < 0x30) return -1;
  if (cp <= 0x39) return (int)(cp - 0x30);
  if (cp < 0x660) return -1;
#pragma unroll 1
  for (int i = 1; i < 65; ++i)
    if (cp >= kNdStarts[i] && cp < kNdStarts[i] + 10) return (int)(cp - kNdStarts[i]);
  return -1;
}

// decode one UTF-8 code point at s[i]; returns its length (invalid bytes decode as themselves)
__device__ __forceinline__ int utf8_next(const uint8_t* s, int n, int i, uint32_t& cp) {
  const uint8_t c = s[i];
  if (c < 0x80) {
    cp = c;
    return 1;
  }
  int len = (c >= 0xF0) ? 4 : (c >= 0xE0) ? 3 : (c >= 0xC0) ? 2 : 1;
  if (i + len > n || len == 1) {
    cp = c;
    return 1;
  }
  cp = c & (0x7F >> len);
  for (int k = 1; k < len; ++k) cp = (cp << 6) | (s[i + k] & 0x3F);
  return len;
}

// check_format: sorted([int(x) for x in re.findall(r'\d+', eq)]) == sorted(nums).
// The digit runs and the numbers live in registers (every array index is a compile-time
// constant after unrolling), so nothing of this goes through scratch memory.
constexpr int kMaxNums = 8;
__device__ __forceinline__ bool same_multiset(const uint64_t (&found)[kMaxNums], int nf, bool too_many,
                                              const int32_t (&nums)[kMaxNums], int n_nums);
__device__ bool check_format(const uint8_t* s, int n, const int32_t (&nums)[kMaxNums], int n_nums) {
  uint64_t found[kMaxNums];
#pragma unroll
  for (int k = 0; k < kMaxNums; ++k) found[k] = 0;
  int nf = 0;
  bool in_run = false, overflow = false, too_many = false;
  uint64_t cur = 0;
  auto close_run = [&]() {
    if (nf < kMaxNums) {
      const uint64_t val = overflow ? 0xFFFFFFFFFFFFFFFFull : cur;
#pragma unroll
      for (int k = 0; k < kMaxNums; ++k)
        if (k == nf) found[k] = val;
      nf++;
    } else {
      too_many = true;
    }
  };
  for (int i = 0; i < n;) {
    uint32_t cp;
    const int len = utf8_next(s, n, i, cp);
    const int d = nd_value(cp);
    if (d >= 0) {
      if (!in_run) {
        in_run = true;
        cur = 0;
        overflow = false;
      }
      if (cur > (0xFFFFFFFFFFFFFFFFull - 9) / 10) overflow = true;
      else cur = cur * 10 + (uint64_t)d;
    } else if (in_run) {
      in_run = false;
      close_run();
    }
    i += len;
  }
  if (in_run) close_run();
  return same_multiset(found, nf, too_many, nums, n_nums);
}

// sorted(found[:nf]) == sorted(nums[:n_nums])  (nums may be negative -> never equal a digit run)
__device__ __forceinline__ bool same_multiset(const uint64_t (&found)[kMaxNums], int nf, bool too_many,
                                              const int32_t (&nums)[kMaxNums], int n_nums) {
  if (too_many || nf != n_nums) return false;
  uint32_t used = 0;
#pragma unroll
  for (int j = 0; j < kMaxNums; ++j) {
    if (j < n_nums) {
      bool hit = false;
#pragma unroll
      for (int k = 0; k < kMaxNums; ++k) {
        if (!hit && k < nf && !((used >> k) & 1) && nums[j] >= 0 && found[k] == (uint64_t)nums[j]) {
          used |= 1u << k;
          hit = true;
        }
      }
      if (!hit) return false;
    }
  }
  return true;
}

// ------------------------------------------------------------------ evaluator
struct Val {  // no padding: copies stay in registers
  long long i;   // an int64, or the pool slot of a big int (is_f == kBig)
  double f;
  int is_f;      // 0 int64, 1 float, kBig big int
  __device__ double as_f() const { return is_f ? f : (double)i; }
};
constexpr int kBig = 3;

// The big ints of one evaluation: kBigLive value slots plus the scratch of one operation, in
// the row's LDS (bigint.hpp's layout).  A value that fits int64 never stays big (demoted after
// every operation), so the int64 code paths keep every answer that does not need more.
constexpr int kBigLive = 6;
constexpr int kBigScratch = (kDivU + 2) + 2 * kBigCap + (kDivU + 2);  // un, vn (+ remainder), xs (= qs)
constexpr int kBigPoolWords = kBigLive * kBigWords + 2 * 4 + kBigScratch;
constexpr int kBigPoolBytes = 4 * kBigPoolWords;
static_assert(2 * kBigWords <= kBigScratch, "big_pow's two temporaries fit the scratch");
struct BigCtx {
  uint32_t* slots = nullptr;  // [kBigLive][kBigWords]
  uint32_t* imm = nullptr;    // [2][4]: int64 operands in big form (two limbs)
  uint32_t* un = nullptr;     // kDivU + 2
  uint32_t* vn = nullptr;     // 2 kBigCap
  uint32_t* xs = nullptr;     // kDivU + 2 (true division's dividend and quotient; big_pow's temporaries)
  uint32_t free_mask = (1u << kBigLive) - 1;
  __device__ void init(uint8_t* base) {  // base: 4-B aligned, kBigPoolBytes
    uint32_t* w = reinterpret_cast<uint32_t*>(base);
    slots = w;
    imm = slots + kBigLive * kBigWords;
    un = imm + 8;
    vn = un + kDivU + 2;
    xs = vn + 2 * kBigCap;
    free_mask = (1u << kBigLive) - 1;
  }
  __device__ uint32_t* at(int s) const { return slots + s * kBigWords; }
  __device__ int alloc() {
    if (!free_mask) return -1;
    const int s = __builtin_ctz(free_mask);
    free_mask &= free_mask - 1;
    return s;
  }
  __device__ void release(const struct Val& v) {
    if (v.is_f == kBig) free_mask |= 1u << (int)v.i;
  }
  // an int operand (int64 or big) as a big value (which: 0 / 1, the imm slot for an int64)
  __device__ const uint32_t* view(const struct Val& v, int which) {
    if (v.is_f == kBig) return at((int)v.i);
    uint32_t* w = imm + 4 * which;
    big_set_i64(w, v.i);
    return w;
  }
  // slot s holds a result: demote it to an int64 when it is one
  __device__ void finish(int s, Val& out) {
    long long x;
    if (big_to_i64(at(s), x)) {
      free_mask |= 1u << s;
      out.is_f = 0;
      out.i = x;
    } else {
      out.is_f = kBig;
      out.i = s;
    }
    out.f = 0.0;
  }
};
__device__ __forceinline__ int big_status(int st) {  // bigint status -> evaluator status
  return st == BIG_OK ? 0 : (st == BIG_RANGE ? 2 : 1);  // RANGE: outside the model; overflow, /0: raises
}

enum Op : int8_t {
  OP_LPAREN = 0,
  OP_OR, OP_XOR, OP_AND, OP_SHL, OP_SHR, OP_ADD, OP_SUB, OP_MUL, OP_DIV, OP_FDIV, OP_MOD,
  OP_NEG, OP_POS, OP_INV, OP_POW
};
__device__ __forceinline__ int prec(int op) {
  switch (op) {
    case OP_OR: return 1;
    case OP_XOR: return 2;
    case OP_AND: return 3;
    case OP_SHL: case OP_SHR: return 4;
    case OP_ADD: case OP_SUB: return 5;
    case OP_MUL: case OP_DIV: case OP_FDIV: case OP_MOD: return 6;
    case OP_NEG: case OP_POS: case OP_INV: return 7;
    case OP_POW: return 8;
    default: return 0;
  }
}

enum EvalStatus { EV_OK = 0, EV_ERR = 1, EV_UNSUP = 2 };

__device__ double py_floor_div_f(double vx, double wx, double* modp) {  // CPython float_divmod
  double mod = fmod(vx, wx);
  double div = (vx - mod) / wx;
  if (mod != 0.0) {
    if ((wx < 0) != (mod < 0)) {
      mod += wx;
      div -= 1.0;
    }
  } else {
    mod = copysign(0.0, wx);
  }
  double floordiv;
  if (div != 0.0) {
    floordiv = floor(div);
    if (div - floordiv > 0.5) floordiv += 1.0;
  } else {
    floordiv = copysign(0.0, vx / wx);
  }
  *modp = mod;
  return floordiv;
}

__device__ int apply_unary(int op, Val& a, BigCtx& bc) {
  if (op == OP_POS) return EV_OK;
  if (a.is_f == 1) {
    if (op == OP_INV) return EV_ERR;  // ~float -> TypeError
    a.f = -a.f;
    return EV_OK;
  }
  if (a.is_f == 0 && !(op == OP_NEG && a.i == (-9223372036854775807LL - 1))) {
    a.i = op == OP_NEG ? -a.i : ~a.i;
    return EV_OK;
  }
  // a big int, or -(-2^63): -a, ~a = -(a + 1)
  const int s = bc.alloc();
  if (s < 0) return EV_UNSUP;
  uint32_t* w = bc.at(s);
  int st = BIG_OK;
  if (op == OP_NEG) {
    big_copy(w, bc.view(a, 0));
    if (big_n(w)) w[1] ^= 1u;
  } else {
    uint32_t* one = bc.imm + 4;
    big_set_i64(one, 1);
    st = big_add(bc.view(a, 0), one, false, w);
    if (big_n(w)) w[1] ^= 1u;
  }
  bc.release(a);
  if (st) return big_status(st);
  bc.finish(s, a);
  return EV_OK;
}

__device__ int float_pow(double iv, double iw, double& out) {  // CPython float_pow (non-complex cases)
  if (iw == 0.0) { out = 1.0; return EV_OK; }
  if (iv != iv) { out = iv; return EV_OK; }
  if (iw != iw) { out = iv == 1.0 ? 1.0 : iw; return EV_OK; }
  if (iv == 1.0) { out = 1.0; return EV_OK; }
  if (iv == 0.0) {
    if (iw < 0.0) return EV_ERR;  // ZeroDivisionError
    const bool odd = floor(iw) == iw && fmod(fabs(iw), 2.0) == 1.0;
    out = odd ? iv : 0.0;
    return EV_OK;
  }
  bool negate = false;
  if (iv < 0.0) {
    if (iw != floor(iw)) return EV_UNSUP;  // Python returns a complex number
    iv = -iv;
    negate = fmod(fabs(iw), 2.0) == 1.0;
  }
  double r = pow(iv, iw);
  if (negate) r = -r;
  if (isinf(r) && !isinf(iv) && !isinf(iw)) return EV_ERR;  // OverflowError
  out = r;
  return EV_OK;
}

// int / int past 2**53 (CPython long_true_divide): the correctly rounded (half-even) quotient.
// q = floor(|a| 2^s / |b|) with s chosen so that q has 55 or 56 bits (128-bit restoring
// division), then 53 bits kept, rounded with the dropped bits and the remainder as sticky.
// |a / b| lies in [2^-63, 2^63]: no overflow, no subnormal.  b != 0.
__device__ double int_true_div(long long a, long long b) {
  const bool neg = (a < 0) != (b < 0);
  const unsigned long long x = a < 0 ? 0ull - (unsigned long long)a : (unsigned long long)a;
  const unsigned long long y = b < 0 ? 0ull - (unsigned long long)b : (unsigned long long)b;
  if (x == 0) return neg ? -0.0 : 0.0;
  const int lx = 64 - __builtin_clzll(x), ly = 64 - __builtin_clzll(y);
  const int s = 55 - (lx - ly);
  const unsigned __int128 N = s >= 0 ? (unsigned __int128)x << s : (unsigned __int128)x;
  const unsigned __int128 D = s < 0 ? (unsigned __int128)y << -s : (unsigned __int128)y;
  unsigned __int128 rem = N;
  unsigned long long q = 0;
  for (int i = 55; i >= 0; --i) {
    const unsigned __int128 t = D << i;
    if (rem >= t) {
      rem -= t;
      q |= 1ull << i;
    }
  }
  const int extra = (64 - __builtin_clzll(q)) - 53;  // 2 or 3
  unsigned long long mant = q >> extra;
  const unsigned long long dropped = q & ((1ull << extra) - 1), half = 1ull << (extra - 1);
  const bool up = dropped > half || (dropped == half && (rem != 0 || (mant & 1)));
  mant += up;
  const double v = ldexp((double)mant, extra - s);
  return neg ? -v : v;
}

// float(x) of an int or float operand (PyLong_AsDouble for a big int: OverflowError past DBL_MAX)
__device__ __forceinline__ int to_f(const Val& v, BigCtx& bc, double& out) {
  if (v.is_f != kBig) {
    out = v.as_f();
    return EV_OK;
  }
  return big_status(big_to_double(bc.at((int)v.i), out));
}

// int (op) int past int64, or with a big operand: bigint.hpp into a fresh slot
__device__ int big_binary(int op, const Val& a, const Val& b, Val& out, BigCtx& bc) {
  const int s = bc.alloc();
  if (s < 0) return EV_UNSUP;
  uint32_t* w = bc.at(s);
  const uint32_t* A = bc.view(a, 0);
  const uint32_t* Bv = bc.view(b, 1);
  int st = BIG_OK;
  switch (op) {
    case OP_ADD: st = big_add(A, Bv, false, w); break;
    case OP_SUB: st = big_add(A, Bv, true, w); break;
    case OP_MUL: st = big_mul(A, Bv, w); break;
    case OP_FDIV: st = big_floordiv(A, Bv, w, nullptr, bc.un, bc.vn); break;
    case OP_MOD: st = big_floordiv(A, Bv, nullptr, w, bc.un, bc.vn); break;
    case OP_AND: st = big_bitop(0, A, Bv, w); break;
    case OP_OR: st = big_bitop(1, A, Bv, w); break;
    case OP_XOR: st = big_bitop(2, A, Bv, w); break;
    case OP_POW: {  // b >= 0 here
      unsigned long long e;
      if (big_n(Bv) > 2) e = ~0ull;  // past 2^64: only |a| <= 1 stays in range
      else e = (big_n(Bv) > 0 ? big_d(Bv)[0] : 0u) | (big_n(Bv) > 1 ? (unsigned long long)big_d(Bv)[1] << 32 : 0ull);
      if (e == ~0ull && big_bits(A) <= 1) e = (big_n(Bv) ? (big_d(Bv)[0] & 1u) : 0u) + 2;  // same parity, >= 2
      st = big_pow(A, e, w, bc.xs, bc.xs + kBigWords);
      break;
    }
    case OP_SHL:
    case OP_SHR: {  // b >= 0 here
      const bool huge = big_n(Bv) > 2 || (big_n(Bv) == 2 && big_d(Bv)[1] >= 0x80000000u);
      const unsigned long long k = huge ? (1ull << 62)
                                        : (big_n(Bv) > 0 ? big_d(Bv)[0] : 0u) |
                                              (big_n(Bv) > 1 ? (unsigned long long)big_d(Bv)[1] << 32 : 0ull);
      if (op == OP_SHL) st = big_shl(A, k, w);
      else big_shr_floor(A, k, w);
      break;
    }
    default: st = BIG_RANGE;
  }
  bc.release(a);
  bc.release(b);
  if (st) {
    bc.free_mask |= 1u << s;
    return big_status(st);
  }
  bc.finish(s, out);
  return EV_OK;
}

__device__ int apply_binary(int op, const Val& a, const Val& b, Val& out, BigCtx& bc) {
  const bool fl = a.is_f == 1 || b.is_f == 1;
  const bool big = a.is_f == kBig || b.is_f == kBig;
  out.is_f = false;
  out.i = 0;
  out.f = 0;
  double x = 0.0, y = 0.0;
  if (fl) {  // float arithmetic: an int operand converts (OverflowError for a big int past DBL_MAX)
    int st = to_f(a, bc, x);
    if (st == EV_OK) st = to_f(b, bc, y);
    bc.release(a);
    bc.release(b);
    if (st != EV_OK) return st;
  }
  switch (op) {
    case OP_ADD:
    case OP_SUB:
    case OP_MUL:
      if (fl) {
        out.is_f = true;
        out.f = op == OP_ADD ? x + y : (op == OP_SUB ? x - y : x * y);
        return EV_OK;
      } else {
        long long r;
        if (!big) {
          bool ov = op == OP_ADD ? __builtin_add_overflow(a.i, b.i, &r)
                                 : (op == OP_SUB ? __builtin_sub_overflow(a.i, b.i, &r)
                                                 : __builtin_mul_overflow(a.i, b.i, &r));
          if (!ov) {
            out.i = r;
            return EV_OK;
          }
        }
        return big_binary(op, a, b, out, bc);
      }
    case OP_DIV: {
      if (!fl) {
        if (big) {  // CPython long_true_divide on the big values (the result is a float: no slot)
          const uint32_t* A = bc.view(a, 0);
          const uint32_t* Bv = bc.view(b, 1);
          double r;
          const int st = big_true_div(A, Bv, r, bc.un, bc.vn, bc.xs, bc.xs);
          bc.release(a);
          bc.release(b);
          if (st) return big_status(st);
          out.is_f = true;
          out.f = r;
          return EV_OK;
        }
        if (b.i == 0) return EV_ERR;
        const long long lim = 9007199254740992LL;
        if (a.i > lim || a.i < -lim || b.i > lim || b.i < -lim) {
          out.is_f = true;
          out.f = int_true_div(a.i, b.i);
          return EV_OK;
        }
        x = (double)a.i;
        y = (double)b.i;
      }
      if (y == 0.0) return EV_ERR;
      out.is_f = true;
      out.f = x / y;
      return EV_OK;
    }
    case OP_FDIV:
    case OP_MOD:
      if (fl) {
        if (y == 0.0) return EV_ERR;
        double mod;
        const double q = py_floor_div_f(x, y, &mod);
        out.is_f = true;
        out.f = op == OP_FDIV ? q : mod;
        return EV_OK;
      } else {
        if (!big) {
          if (b.i == 0) return EV_ERR;
          if (!(a.i == (-9223372036854775807LL - 1) && b.i == -1)) {
            long long q = a.i / b.i, r = a.i % b.i;
            if (r != 0 && ((r < 0) != (b.i < 0))) {
              q -= 1;
              r += b.i;
            }
            out.i = op == OP_FDIV ? q : r;
            return EV_OK;
          }
        }
        return big_binary(op, a, b, out, bc);  // ZeroDivisionError from bigint.hpp for a zero divisor
      }
    case OP_POW: {
      const bool bneg = b.is_f == kBig ? big_neg(bc.at((int)b.i)) : b.i < 0;
      if (!fl && !bneg) {
        if (!big) {
          long long base = a.i, e = b.i, acc = 1;
          bool ov = false;
          while (e) {
            if ((e & 1) && __builtin_mul_overflow(acc, base, &acc)) {
              ov = true;
              break;
            }
            e >>= 1;
            if (e && __builtin_mul_overflow(base, base, &base)) {  // base overflow matters only if a bit remains
              ov = true;
              break;
            }
          }
          if (!ov) {
            out.i = acc;
            return EV_OK;
          }
        }
        return big_binary(op, a, b, out, bc);
      } else {
        if (!fl) {  // int ** negative int: float(a) ** float(b) (CPython long_pow -> float_pow)
          if (a.is_f == 0 && a.i == 0) {
            bc.release(b);
            return EV_ERR;  // 0 ** negative int -> ZeroDivisionError
          }
          int st = to_f(a, bc, x);
          if (st == EV_OK) st = to_f(b, bc, y);
          bc.release(a);
          bc.release(b);
          if (st != EV_OK) return st;
        }
        out.is_f = true;
        return float_pow(x, y, out.f);
      }
    }
    case OP_SHL:
    case OP_SHR:
      if (fl) return EV_ERR;
      if (b.is_f == kBig ? big_neg(bc.at((int)b.i)) : b.i < 0) return EV_ERR;  // ValueError: negative shift count
      if (!big) {
        if (op == OP_SHR) {
          out.i = b.i >= 64 ? (a.i < 0 ? -1 : 0) : (a.i >> b.i);
          return EV_OK;
        }
        if (a.i == 0) {
          out.i = 0;
          return EV_OK;
        }
        long long r;  // (a * 2^b without signed-overflow UB: the compiler may not assume it away)
        if (b.i < 63 && !__builtin_mul_overflow(a.i, 1LL << b.i, &r)) {
          out.i = r;
          return EV_OK;
        }
      }
      return big_binary(op, a, b, out, bc);
    case OP_AND:
    case OP_OR:
    case OP_XOR:
      if (fl) return EV_ERR;
      if (!big) {
        out.i = op == OP_AND ? (a.i & b.i) : (op == OP_OR ? (a.i | b.i) : (a.i ^ b.i));
        return EV_OK;
      }
      return big_binary(op, a, b, out, bc);
  }
  return EV_ERR;
}

constexpr int kStack = 32;  // deeper expressions are flagged RMI_ERR_UNSUP (host re-evaluates)

// A stack slot: 16 B (value bits + kind) — the stacks live in the thread's LDS slice, not in
// scratch: a private array indexed at run time would spill every push/pop to memory.
struct SVal {
  long long bits;
  int is_f, pad;
};
__device__ __forceinline__ SVal pack(const Val& v) {
  SVal s;
  s.bits = v.is_f == 1 ? __double_as_longlong(v.f) : v.i;  // a big int keeps its slot index
  s.is_f = v.is_f;
  s.pad = 0;
  return s;
}
__device__ __forceinline__ Val unpack(const SVal& s) {
  Val v;
  v.is_f = s.is_f;
  v.i = s.is_f == 1 ? 0 : s.bits;
  v.f = s.is_f == 1 ? __longlong_as_double(s.bits) : 0.0;
  return v;
}
constexpr int kMachineBytes = kStack * (int)sizeof(SVal) + kStack;  // per thread, in LDS

struct Machine {
  SVal* vals;    // [kStack] in LDS
  int8_t* ops;   // [kStack] in LDS
  int nv = 0, no = 0;
  int status = EV_OK;
  bool ev = true;  // false: the syntax pass (stack shapes only, no arithmetic)
  BigCtx big;      // ints past int64

  __device__ bool reduce_one() {
    const int op = ops[--no];
    if (!ev) {
      const int need = (op == OP_NEG || op == OP_POS || op == OP_INV) ? 1 : 2;
      if (nv < need) { status = EV_ERR; return false; }
      nv -= need - 1;
      return true;
    }
    if (op == OP_NEG || op == OP_POS || op == OP_INV) {
      if (nv < 1) { status = EV_ERR; return false; }
      Val a = unpack(vals[nv - 1]);
      const int st = apply_unary(op, a, big);
      if (st != EV_OK) { status = st; return false; }
      vals[nv - 1] = pack(a);
      return true;
    }
    if (nv < 2) { status = EV_ERR; return false; }
    Val r;
    const int st = apply_binary(op, unpack(vals[nv - 2]), unpack(vals[nv - 1]), r, big);
    if (st != EV_OK) { status = st; return false; }
    vals[nv - 2] = pack(r);
    nv -= 1;
    return true;
  }
  __device__ bool push_op(int op) {
    if (no >= kStack) { status = EV_UNSUP; return false; }
    ops[no++] = (int8_t)op;
    return true;
  }
  __device__ bool push_val(const Val& v) {
    if (nv >= kStack) { status = EV_UNSUP; return false; }
    vals[nv++] = pack(v);
    return true;
  }
  __device__ bool binary(int op) {  // pop higher/equal-precedence operators, then push
    const int p = prec(op);
    const bool right = op == OP_POW;
    while (no > 0 && ops[no - 1] != OP_LPAREN) {
      const int q = prec(ops[no - 1]);
      if (q > p || (q == p && !right)) {
        if (!reduce_one()) return false;
      } else {
        break;
      }
    }
    return push_op(op);
  }
};

__device__ __forceinline__ bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
__device__ __forceinline__ bool is_alpha(uint8_t c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }

__device__ const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                      1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Lex a number literal at s[i]; returns the index after it.  status EV_ERR = SyntaxError;
// EV_UNSUP with v.is_f == kValidLit: a valid literal whose value is outside the model;
// EV_UNSUP with v.is_f == kBigLit: an int literal past int64 (v.i = its first byte), which the
// evaluation builds as a big int.
constexpr int kValidLit = 2;
constexpr int kBigLit = 4;
__device__ int lex_number(const uint8_t* s, int n, int i, Val& v, int& status) {
  const int start = i;
  uint64_t mant = 0;
  int ndig = 0, frac = 0, exp10 = 0;
  bool is_float = false, overflow = false, leading_zero = false, nonzero_digit = false;
  bool first = true;
  auto digits = [&](bool in_frac) {
    bool prev_digit = false;
    while (i < n && (is_digit(s[i]) || (s[i] == '_' && prev_digit && i + 1 < n && is_digit(s[i + 1])))) {
      if (s[i] == '_') {
        i++;
        prev_digit = false;
        continue;
      }
      const int d = s[i] - '0';
      if (first && !in_frac) {
        leading_zero = d == 0;
        first = false;
      }
      if (d) nonzero_digit = true;
      if (mant > (0xFFFFFFFFFFFFFFFFull - 9) / 10) overflow = true;
      else {
        mant = mant * 10 + (uint64_t)d;
        if (mant || ndig) ndig++;
      }
      if (in_frac) frac++;
      prev_digit = true;
      i++;
    }
    return prev_digit;
  };
  const bool had_int = digits(false);
  if (i < n && s[i] == '.') {
    is_float = true;
    i++;
    digits(true);
  }
  (void)had_int;
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    int j = i + 1;
    int sign = 1;
    if (j < n && (s[j] == '+' || s[j] == '-')) {
      sign = s[j] == '-' ? -1 : 1;
      j++;
    }
    if (j < n && is_digit(s[j])) {
      int e = 0;
      bool prev = false;
      while (j < n && (is_digit(s[j]) || (s[j] == '_' && prev && j + 1 < n && is_digit(s[j + 1])))) {
        if (s[j] != '_') {
          if (e < 100000) e = e * 10 + (s[j] - '0');
          prev = true;
        } else {
          prev = false;
        }
        j++;
      }
      exp10 = sign * e;
      is_float = true;
      i = j;
    } else {
      status = EV_UNSUP;  // "1e" / "1ex": name-like tail
      return i;
    }
  }
  if (i < n && (is_alpha(s[i]) || s[i] == '_' || s[i] == '.' || s[i] >= 0x80)) {
    status = EV_UNSUP;  // 1j, 0x.., 1if.., attribute access: outside the modelled grammar
    return i;
  }
  if (!is_float) {
    if (leading_zero && nonzero_digit) {
      status = EV_ERR;  // leading zeros in decimal integer literals are not permitted
      return i;
    }
    if (overflow || mant > 9223372036854775807ull) {
      status = EV_UNSUP;  // a Python big int: built by the evaluation (bigint.hpp)
      v.is_f = kBigLit;
      v.i = start;
      return i;
    }
    v.is_f = false;
    v.i = (long long)mant;
    return i;
  }
  // float literal: exact when mantissa <= 2^53 and |power of ten| <= 22 (one rounding)
  const int e10 = exp10 - frac;
  if (overflow || mant > 9007199254740992ull || e10 > 22 || e10 < -22) {
    if (mant == 0 && !overflow) {
      v.is_f = true;
      v.f = 0.0;
      return i;
    }
    status = EV_UNSUP;  // a float literal this parser does not round exactly
    v.is_f = kValidLit;
    return i;
  }
  v.is_f = true;
  v.f = e10 >= 0 ? (double)mant * kPow10[e10] : (double)mant / kPow10[-e10];
  return i;
}

// Python 3.10 keyword.kwlist, each packed little-endian into a u64
__constant__ uint64_t kPyKeywords[35] = {
    0x00000065736c6146ull /* False */,
    0x00000000656e6f4eull /* None */,
    0x0000000065757254ull /* True */,
    0x0000000000646e61ull /* and */,
    0x0000000000007361ull /* as */,
    0x0000747265737361ull /* assert */,
    0x000000636e797361ull /* async */,
    0x0000007469617761ull /* await */,
    0x0000006b61657262ull /* break */,
    0x0000007373616c63ull /* class */,
    0x65756e69746e6f63ull /* continue */,
    0x0000000000666564ull /* def */,
    0x00000000006c6564ull /* del */,
    0x0000000066696c65ull /* elif */,
    0x0000000065736c65ull /* else */,
    0x0000747065637865ull /* except */,
    0x00796c6c616e6966ull /* finally */,
    0x0000000000726f66ull /* for */,
    0x000000006d6f7266ull /* from */,
    0x00006c61626f6c67ull /* global */,
    0x0000000000006669ull /* if */,
    0x000074726f706d69ull /* import */,
    0x0000000000006e69ull /* in */,
    0x0000000000007369ull /* is */,
    0x00006164626d616cull /* lambda */,
    0x6c61636f6c6e6f6eull /* nonlocal */,
    0x0000000000746f6eull /* not */,
    0x000000000000726full /* or */,
    0x0000000073736170ull /* pass */,
    0x0000006573696172ull /* raise */,
    0x00006e7275746572ull /* return */,
    0x0000000000797274ull /* try */,
    0x000000656c696877ull /* while */,
    0x0000000068746977ull /* with */,
    0x000000646c656979ull /* yield */};

// A bare name in the answer (countdown/env.py:16-21 evaluates with {"__builtins__": None}):
// every name lookup raises there (TypeError: None is not subscriptable), so an answer whose
// names are all plain identifiers and whose other bytes only form strict operators cannot be
// correct — every operand is evaluated, the name included, or the parse fails.  The answer
// stays outside the model (EV_UNSUP) when something could bind or skip a name: a keyword
// (lambda, if/else, and/or, not, in, is, True/False/None ...), ':' (walrus, slices, dicts),
// '.' (attribute names, floats), comparisons ('<' '>' '=' '!': chains short-circuit), quotes,
// '\\', non-ASCII bytes (Unicode identifiers), or a digit run fused with letters (1if, 0x10).
__device__ int name_outcome(const uint8_t* s, int n) {
  int i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    if (c >= 0x80 || c == ':' || c == '\'' || c == '"' || c == '\\' || c == '.' || c == '<' || c == '>' ||
        c == '=' || c == '!')
      return EV_UNSUP;
    if (is_alpha(c) || c == '_' || is_digit(c)) {
      const bool digit_start = is_digit(c);
      bool letters = false;
      uint64_t packed = 0;
      int j = i;
      while (j < n && (is_alpha(s[j]) || s[j] == '_' || is_digit(s[j]))) {
        letters |= !is_digit(s[j]);
        if (j - i < 8) packed |= (uint64_t)s[j] << (8 * (j - i));
        j++;
      }
      if (digit_start && letters) return EV_UNSUP;
      if (!digit_start && j - i <= 8) {
#pragma unroll 1
        for (int k = 0; k < 35; ++k)
          if (packed == kPyKeywords[k]) return EV_UNSUP;
      }
      i = j;
      continue;
    }
    i++;
  }
  return EV_ERR;
}

// returns EV_OK with value in out, EV_ERR (Python raises), EV_UNSUP (outside the model).
// evaluate = false: the syntax pass.  Python compiles before it evaluates, so a syntax error
// anywhere wins over whatever the evaluation would meet first (an int past int64: EV_UNSUP);
// countdown_reward runs this pass first and evaluates only a well-formed answer.
__device__ int py_eval(const uint8_t* s, int n, Val& out, uint8_t* work, uint8_t* pool, bool evaluate = true) {
  Machine m;
  m.ev = evaluate;
  if (evaluate) m.big.init(pool);
  m.vals = reinterpret_cast<SVal*>(work);
  m.ops = reinterpret_cast<int8_t*>(work + kStack * sizeof(SVal));
  bool expect_operand = true;
  int depth = 0;
  // eval() strips leading spaces/tabs; ctx_manager already .strip()s the action
  int i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    if (c == ' ' || c == '\t' || c == '\f') { i++; continue; }
    if (c == '#') {  // comment to end of line
      while (i < n && s[i] != '\n' && s[i] != '\r') i++;
      continue;
    }
    if (c == '\n' || c == '\r') {
      if (depth > 0) { i++; continue; }
      // a newline at depth 0 ends the expression: only whitespace/comments may follow
      int j = i;
      while (j < n) {
        const uint8_t d = s[j];
        if (d == ' ' || d == '\t' || d == '\f' || d == '\n' || d == '\r') { j++; continue; }
        if (d == '#') { while (j < n && s[j] != '\n' && s[j] != '\r') j++; continue; }
        return EV_ERR;
      }
      i = n;
      break;
    }
    if (is_digit(c) || (c == '.' && i + 1 < n && is_digit(s[i + 1]))) {
      if (!expect_operand) return EV_ERR;
      Val v;
      int st = EV_OK;
      i = lex_number(s, n, i, v, st);
      if (st == EV_UNSUP && !evaluate && (v.is_f == kValidLit || v.is_f == kBigLit)) {
        st = EV_OK;  // a valid literal (the syntax pass needs no value)
        v.is_f = 0;
      }
      if (st == EV_UNSUP && v.is_f == kBigLit) {  // an int literal past int64
        const int slot = m.big.alloc();
        if (slot < 0) return EV_UNSUP;
        const int bst = big_from_dec(s + v.i, i - (int)v.i, m.big.at(slot));
        if (bst) return EV_UNSUP;  // past the bound
        m.big.finish(slot, v);
        st = EV_OK;
      }
      if (st != EV_OK) return st;
      if (!m.push_val(v)) return m.status;
      expect_operand = false;
      continue;
    }
    if (c == '(') {
      if (!expect_operand) return EV_ERR;  // call of a number -> TypeError (not correct either way)
      if (!m.push_op(OP_LPAREN)) return m.status;
      depth++;
      i++;
      continue;
    }
    if (c == ')') {
      if (expect_operand || depth == 0) return EV_ERR;  // "()" is an empty tuple -> TypeError
      while (m.no > 0 && m.ops[m.no - 1] != OP_LPAREN)
        if (!m.reduce_one()) return m.status;
      m.no--;  // pop '('
      depth--;
      i++;
      continue;
    }
    if (expect_operand) {
      int op = -1;
      if (c == '-') op = OP_NEG;
      else if (c == '+') op = OP_POS;
      else if (c == '~') op = OP_INV;
      if (op >= 0) {
        if (!m.push_op(op)) return m.status;
        i++;
        continue;
      }
    } else {
      int op = -1, len = 1;
      const uint8_t d = i + 1 < n ? s[i + 1] : 0;
      switch (c) {
        case '+': op = OP_ADD; break;
        case '-': op = OP_SUB; break;
        case '*': if (d == '*') { op = OP_POW; len = 2; } else op = OP_MUL; break;
        case '/': if (d == '/') { op = OP_FDIV; len = 2; } else op = OP_DIV; break;
        case '%': op = OP_MOD; break;
        case '&': op = OP_AND; break;
        case '|': op = OP_OR; break;
        case '^': op = OP_XOR; break;
        case '<': if (d == '<') { op = OP_SHL; len = 2; } break;
        case '>': if (d == '>') { op = OP_SHR; len = 2; } break;
        default: break;
      }
      if (op >= 0) {
        // augmented assignment ("+=") and '==' etc. are not expressions
        if (i + len < n && s[i + len] == '=') {
          if (c == '<' || c == '>') return EV_UNSUP;  // "<<=" / ">>=" vs comparisons: leave the model
          return EV_ERR;
        }
        if (!m.binary(op)) return m.status;
        expect_operand = true;
        i += len;
        continue;
      }
    }
    // anything else
    if (is_alpha(c) || c == '_') return name_outcome(s, n);
    if (c == '"' || c == '\'' || c == '[' || c == '{' || c == '.' || c == '<' ||
        c == '>' || c == '=' || c == '!' || c == '\\' || c >= 0x80)
      return (c == '=' && !(i + 1 < n && s[i + 1] == '=')) ? EV_ERR : EV_UNSUP;
    return EV_ERR;  // ',', ';', ':', '@', '$', '?', '`', ']', '}', control chars ...
  }
  if (expect_operand || depth != 0) return EV_ERR;
  while (m.no > 0) {
    if (m.ops[m.no - 1] == OP_LPAREN) return EV_ERR;
    if (!m.reduce_one()) return m.status;
  }
  if (m.nv != 1) return EV_ERR;
  out = unpack(m.vals[0]);
  return EV_OK;
}

// Fast path for answers of at most 64 bytes over "0-9 +-*/()" and ' ' (the usual arithmetic
// answer): check_format and the evaluation in ONE pass over the answer's TOKENS, with no
// per-byte loop and (almost) no branches, so the lanes of a wave (one answer each) run one
// straight-line body per token whatever their answers look like.
//  * Structure from bit masks: SWAR over the staged row gives a 64-bit digit mask D and a
//    space mask SP; token starts are the non-space bytes that do not continue a digit run.
//    A token is found with one ctz, its bytes with two aligned 8-B LDS reads, a literal's
//    value (<= 8 digits) with three SWAR multiply steps.
//  * One value representation: every value is an f64 plus an is-float bit.  Python int
//    arithmetic on ints below 2**53 in magnitude is exact in f64, and true division of two
//    such ints is CPython's single correctly rounded double division (long_true_divide's
//    small-int case), so every result is bit-identical to Python's as long as every int
//    result stays below 2**53; one that reaches it leaves the fast path.
//  * The evaluator is the two-level form of the grammar
//      expr := term (('+'|'-') term)* ; term := factor (('*'|'/') factor)* ;
//      factor := ('+'|'-')* (literal | '(' expr ')')
//    computed eagerly left to right: acc (aop) term (mop) operand — the same operations in
//    the same order as Python's AST evaluation (and py_eval's postfix).  At most ONE
//    arithmetic operation per token at ONE code site; ')' hands its group's value to the
//    next iteration as an operand token.  Parentheses save the outer level in the thread's
//    LDS stack (the push slot is always written, the pop slot always read, so neither
//    needs a branch).  Syntax is checked exactly as py_eval does (expect-operand, depth).
// Returns false when the answer leaves the subset (longer than 64 bytes, another byte,
// '**', '//', a literal of more than 8 digits or with a leading 0, nesting deeper than
// kFastDepth, an int result >= 2**53): the caller then runs check_format + py_eval.
// fmt = check_format; st / out = the evaluation.
constexpr int kFastDepth = 16;
constexpr int kFastMax = 64;       // answer bytes covered by the masks
constexpr int kSlotBytes = 24;     // stack slot: acc f64, term f64, state word
static_assert((kFastDepth + 1) * kSlotBytes + (kMaxNums + 1) * 8 <= kStack * (int)sizeof(SVal) + kStack,
              "the fast path's stack and digit runs fit the LDS work area");
enum : int { F_NONE = 0, F_ADD, F_SUB, F_MUL, F_DIV };
// Per-lane state is kept in integer words, not bools: a bool that merges at a join of
// divergent control flow is a 64-bit lane mask, and keeping a dozen of them costs more
// scalar instructions than the evaluation itself.
enum : int { S_EXPECT = 1, S_SLOW = 2, S_GROUP = 4, S_NEG = 8, S_NEGANY = 16, S_TOOMANY = 32 };
__device__ __forceinline__ uint32_t nib4(uint32_t hi) {  // bit 7 of each byte -> a 4-bit mask
  return ((hi >> 7) * 0x01020408u) >> 24;
}
__device__ __forceinline__ uint32_t digit4(uint32_t x) {  // bytes '0'..'9' (ASCII only)
  const uint32_t h = x & 0x7F7F7F7Fu;
  return nib4((h + 0x50505050u) & ~(h + 0x46464646u) & ~x & 0x80808080u);
}
__device__ __forceinline__ uint32_t space4(uint32_t x) {  // bytes == ' '
  const uint32_t y = x ^ 0x20202020u;
  return nib4(~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u);
}
__device__ __forceinline__ int ctz64(uint64_t x) { return x ? __builtin_ctzll(x) : 64; }

__device__ __forceinline__ uint64_t load8(const uint8_t* row, int p) {  // bytes [p, p+8) of a staged row
  const uint64_t* r8 = reinterpret_cast<const uint64_t*>(row);
  const int pw = p >> 3, ps = (p & 7) * 8;
  const uint64_t lo = r8[pw], hi = r8[pw + 1];
  return (lo >> ps) | ((hi << 1) << (63 - ps));  // branch-free funnel shift (ps = 0 included)
}

// row: the answer staged in LDS, 16-B aligned, readable 80 bytes past its start.
// work: the thread's LDS work area (the parenthesis stack, then the digit runs found).
// The loop body has no data-dependent branch: the token tests are 0/1 ints combined with
// bitwise operators (C's && and || would become divergent control flow), every state word
// is updated by selects, the stack slot is always written and read, and the next token's
// bytes are read one iteration ahead.
__device__ __forceinline__ bool fast_reward(const uint8_t* row, int n, const int32_t (&nums)[kMaxNums], int n_nums,
                                            bool& fmt, int& st_out, Val& out, uint8_t* work) {
  if (n > kFastMax) return false;
  const uint4* r16 = reinterpret_cast<const uint4*>(row);
  uint64_t D = 0, SP = 0;
#pragma unroll
  for (int c = 0; c < kFastMax / 16; ++c) {
    const uint4 q = r16[c];
    D |= (uint64_t)(digit4(q.x) | digit4(q.y) << 4 | digit4(q.z) << 8 | digit4(q.w) << 12) << (16 * c);
    SP |= (uint64_t)(space4(q.x) | space4(q.y) << 4 | space4(q.z) << 8 | space4(q.w) << 12) << (16 * c);
  }
  const uint64_t lm = n >= 64 ? ~0ull : ((1ull << n) - 1);
  D &= lm;
  uint64_t TS = lm & ~SP & ~(D & (D << 1));  // token starts
  uint8_t* lits = work + (kFastDepth + 1) * kSlotBytes;  // the digit runs (kMaxNums + 1 slots of 8 B)
  int p = ctz64(TS);
  TS &= TS - 1;
  uint64_t w = load8(row, p);
  int nf = 0, depth = 0, sf = S_EXPECT, aop = F_NONE, mop = F_NONE, st = EV_OK;
  double acc = 0.0, term = 0.0, gv = 0.0, res = 0.0;
  int accf = 0, termf = 0, gvf = 0, resf = 0;
  // at most 64 tokens + 32 group operands + the end: the cap is only a guard every wave reaches
  for (int it = 0;; ++it) {
    if (it > 2 * kFastMax + 2) {
      sf |= S_SLOW;
      break;
    }
    const int grp = (sf >> 2) & 1;  // S_GROUP
    sf &= ~S_GROUP;
    // the slot a ')' pops, and the next token's bytes (both reads issued up front)
    const uint8_t* pslot = work + (depth > 0 ? depth - 1 : 0) * kSlotBytes;
    const double pacc = *reinterpret_cast<const double*>(pslot);
    const double pterm = *reinterpret_cast<const double*>(pslot + 8);
    const uint32_t pword = *reinterpret_cast<const uint32_t*>(pslot + 16);
    const int cp = p;
    const uint64_t cw = w;
    p = grp ? p : ctz64(TS);
    TS = grp ? TS : TS & (TS - 1);
    w = load8(row, p);
    // ---- this iteration's token: an operand (a digit run, or the group value after ')'),
    //      the end, or one of ( ) * + - /
    const int b0 = (int)(cw & 0xFF), b1 = cp + 1 < n ? (int)((cw >> 8) & 0xFF) : 0;
    const int nogrp = grp ^ 1;
    const int end = nogrp & (cp >= n);
    const int lit = nogrp & (end ^ 1) & ((unsigned)(b0 - '0') < 10u);
    const int tok = nogrp & (end ^ 1) & (lit ^ 1);
    const unsigned kc = (unsigned)(b0 - '(');
    const int kind = (kc < 8u ? (int)((0x60504321u >> (4 * kc)) & 15u) : 0) * tok;  // ( ) * + , - . /
    const int lp = kind == 1, rp = kind == 2, star = kind == 3, plus = kind == 4, minus = kind == 5,
              slash = kind == 6, md = star | slash, pm = plus | minus;
    const int L = lit ? ctz64(~(D >> (cp & 63))) : 0;
    const int Lc = L < 1 ? 1 : L > 8 ? 8 : L;
    uint64_t x8 = (cw & (~0ull >> (64 - 8 * Lc))) << (8 * (8 - Lc));
    x8 &= 0x0F0F0F0F0F0F0F0Full;
    x8 = (x8 * 10 + (x8 >> 8)) & 0x00FF00FF00FF00FFull;
    x8 = (x8 * 100 + (x8 >> 16)) & 0x0000FFFF0000FFFFull;
    x8 = (x8 * 10000 + (x8 >> 32)) & 0xFFFFFFFFull;
    const int slow_tok = (lit & (((b0 == '0') & (L > 1)) | (L > 8))) | (tok & (kind == 0)) | (md & (b1 == b0));
    // a check_format digit run (the slot past the last run is free: written unconditionally)
    *reinterpret_cast<uint64_t*>(lits + 8 * nf) = x8;
    sf |= (lit & (nf == kMaxNums)) ? S_TOOMANY : 0;
    nf += lit & (nf < kMaxNums);
    // ---- syntax (py_eval's checks) and this token's effect
    const int expect = sf & S_EXPECT, noexp = expect ^ 1;
    const int err = (lit & noexp) | (end & (expect | (depth != 0))) | (lp & noexp) | (rp & (expect | (depth == 0))) |
                    (md & expect);
    const int stok = st == EV_OK;
    const int go = stok & (err ^ 1);
    st = (stok & err) ? EV_ERR : st;
    const int g_opnd = go & (lit | grp), g_end = go & end, g_rp = go & rp;
    const int g_lp = go & lp & (depth < kFastDepth);
    const int g_neg = go & expect & minus;
    const int g_md = go & noexp & md, g_pm = go & noexp & pm;
    const int slow = slow_tok | (go & lp & (depth == kFastDepth));
    double v = grp ? gv : (double)(uint32_t)x8;
    const int vf = grp ? gvf : 0;
    v = (sf & S_NEG) ? (vf ? -v : 0.0 - v) : v;  // an int -0 is 0
    // the push slot is free whether or not this token opens a group
    {
      uint8_t* s = work + depth * kSlotBytes;
      *reinterpret_cast<double*>(s) = acc;
      *reinterpret_cast<double*>(s + 8) = term;
      *reinterpret_cast<uint32_t*>(s + 16) =
          (uint32_t)(aop | (mop << 3) | ((sf & (S_NEG | S_NEGANY)) << 3) | (accf << 8) | (termf << 9));
    }
    // at most one operation: operand -> term (mop) v; end / ')' / binary +- -> acc (aop) term
    const int opc = g_opnd ? mop : (g_end | g_rp | g_pm) ? aop : F_NONE;
    const double x = g_opnd ? term : acc, y = g_opnd ? v : term;
    const int xf = g_opnd ? termf : accf, yf = g_opnd ? vf : termf;
    const int did = opc != F_NONE, dv = opc == F_DIV;
    const double sm = x + (opc == F_SUB ? -y : y), pr = x * y, qt = x / y;
    double r = opc == F_MUL ? pr : dv ? qt : sm;
    const int rf = xf | yf | (int)dv;
    r = rf ? r : r + 0.0;  // an int -0 is 0
    st = (did & dv & (y == 0.0)) ? EV_ERR : st;  // ZeroDivisionError
    const int big = did & (rf ^ 1) & (fabs(r) >= 9007199254740992.0);  // an int past 2**53: leave the f64 model
    const double val = did ? r : g_opnd ? v : term;                 // the token's result
    const int valf = did ? rf : g_opnd ? vf : termf;
    term = g_opnd ? val : term;
    termf = g_opnd ? valf : termf;
    acc = g_pm ? val : acc;
    accf = g_pm ? valf : accf;
    gv = g_rp ? val : gv;
    gvf = g_rp ? valf : gvf;
    res = g_end ? val : res;
    resf = g_end ? valf : resf;
    // state words
    int nsf = sf;
    nsf = g_opnd ? nsf & ~(S_EXPECT | S_NEG | S_NEGANY) : nsf;
    nsf = g_lp ? nsf & ~(S_NEG | S_NEGANY) : nsf;
    nsf = g_neg ? (nsf ^ S_NEG) | S_NEGANY : nsf;
    nsf = g_md | g_pm ? nsf | S_EXPECT : nsf;
    nsf = g_rp ? nsf | S_GROUP : nsf;
    nsf |= slow | big ? S_SLOW : 0;
    mop = g_opnd | g_lp ? F_NONE : g_md ? (star ? F_MUL : F_DIV) : mop;
    aop = g_lp ? F_NONE : g_pm ? (plus ? F_ADD : F_SUB) : aop;
    depth += g_lp ? 1 : 0;
    // ')': the enclosing level comes back (its operation has read it)
    const int rs = g_rp & (st == EV_OK);
    depth -= rs ? 1 : 0;
    acc = rs ? pacc : acc;
    term = rs ? pterm : term;
    accf = rs ? (int)((pword >> 8) & 1) : accf;
    termf = rs ? (int)((pword >> 9) & 1) : termf;
    aop = rs ? (int)(pword & 7) : aop;
    mop = rs ? (int)((pword >> 3) & 7) : mop;
    nsf |= rs ? (int)((pword >> 3) & (S_NEG | S_NEGANY)) : 0;
    sf = nsf;
    if ((sf & S_SLOW) | end) break;
  }
  if (sf & S_SLOW) return false;
  uint64_t found[kMaxNums];
#pragma unroll
  for (int k = 0; k < kMaxNums; ++k) found[k] = *reinterpret_cast<const uint64_t*>(lits + 8 * k);
  st_out = st;
  out.is_f = resf;
  out.f = resf ? res : 0.0;
  out.i = resf ? 0 : (long long)res;
  fmt = same_multiset(found, nf, (sf & S_TOOMANY) != 0, nums, n_nums);
  return true;
}

// compute_reward (countdown/env.py:69-78): 0 | format_score | score ; flags bit0 format bit1 correct
// staged: s is the answer in this thread's LDS row (the fast path reads it there)
__device__ double countdown_reward(const uint8_t* s, int n, bool staged, const int32_t (&nums)[kMaxNums],
                                   int n_nums, int32_t target, double score, double format_score, uint8_t& flags,
                                   uint8_t& err, uint8_t* work, uint8_t* pool) {
  flags = 0;
  Val v;
  bool fmt = false;
  int st = EV_ERR;
  if (!staged || !fast_reward(s, n, nums, n_nums, fmt, st, v, work)) {
    fmt = check_format(s, n, nums, n_nums);
    if (fmt) st = py_eval(s, n, v, work, pool, false);
    if (fmt && st == EV_OK) st = py_eval(s, n, v, work, pool, true);
  }
  if (!fmt) return 0.0;
  flags |= 1;
  bool correct = false;
  if (st == EV_UNSUP) err |= RMI_ERR_UNSUP;
  if (st == EV_OK) {
    if (v.is_f == 1) correct = fabs(v.f - (double)target) < 1e-5;  // abs(result - target) < 1e-5
    else if (v.is_f == 0) correct = v.i == (long long)target;
    // a big int (past int64) never equals an int32 target; Python compares int and float exactly
  }
  if (!correct) return format_score;
  flags |= 2;
  return score;
}

// ================================================================ 16 lanes per answer
// A turn's answers are few next to the machine (16 384 envs: 256 full waves), so a turn costs
// one wave's latency, and a lane-per-answer token loop makes that latency the length of the
// longest answer's token chain (~17 iterations of ~250 instructions).  Here the 16 lanes of one
// DPP row own one answer, one TOKEN per lane, and everything but the arithmetic runs across
// the tokens at once:
//  * classify: lane j builds the digit / space nibbles of answer bytes 4j..4j+3; the row
//    assembles the 64-bit masks through LDS; lane k finds the k-th token start (popcount
//    search), reads its bytes (two 8-B LDS reads) and parses its digit run (SWAR);
//  * syntax: py_eval's checks are local to neighbouring tokens (an operand where an operator
//    is expected, ')' '*' '/' where an operand is expected, the end) plus the parenthesis
//    depth (a DPP row scan), so each lane checks its own token against the previous one;
//    unary + / - signs fold into the digit run they precede;
//  * tree: a binary operator's key is 2 * depth + (1 for * /).  Python's parse tree
//    (left-associative) is the Cartesian tree of the keys with the rightmost of equal keys
//    on top: the parent of operator i is the tighter (larger key; the left one on a tie) of
//    L = the nearest operator left of i with a smaller key and R = the nearest one right of
//    i with a key <= key_i (ballot masks per key), and i is R's left / L's right operand;
//  * evaluate: each operator computes once both operands are ready (tree height rounds, LDS
//    value slots), with exactly the node's f64 operation of the per-lane path, so every value
//    is bit-identical (an operator's value depends only on its two operands);
//  * check_format: for each of the instance's numbers, the count of equal digit runs (ballot)
//    against its count among the numbers.
// Whatever leaves this envelope (more than 16 tokens or 64 bytes, nesting deeper than 3, a
// sign before '(' or a run of more than 3 signs, and everything the per-lane path itself
// leaves: other bytes, '**', '//', long or 0-led literals, ints past 2**53) is evaluated by
// the row's lane 0 with the per-lane path (countdown_reward) and broadcast.
// Diagnostic build only (tools/prof_countdown_stamps.py compiles with RMI_CD_STAMPS): per-wave
// s_memtime at the turn's phase boundaries (row 0 of each wave), written by lane 0 at the end.
#ifdef RMI_CD_STAMPS
__device__ unsigned long long* g_cd_stamps;
constexpr int kCdStamps = 6;
__device__ unsigned long long* g_cd_pstamps;  // [waves][8] inside par_reward (row 0, lane 0)
#define CD_STAMP(arr, i) ((arr)[i] = __builtin_amdgcn_s_memtime())
#define CD_PSTAMP(i, dep)                                                                          \
  do {                                                                                              \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime() + (unsigned long long)((dep) == -7); \
    if ((threadIdx.x & 63) == 0) g_cd_pstamps[(int64_t)blockIdx.x * 8 + (i)] = t_;                 \
  } while (0)
#else
#define CD_STAMP(arr, i) ((void)0)
#define CD_PSTAMP(i, dep) ((void)0)
#endif
constexpr int kRow = 16;
constexpr int kParDepth = 3;
constexpr int kParBytes = 16 * kRow + 2 * kRow + kRow + kRow;  // value slots, children, keys, mask bytes
// par: the cooperative path's scratch, or (the fallback, after it) the result broadcast in its
// first kParHead bytes and the big-int pool behind them
constexpr int kParHead = 16;
constexpr int kParRegion = kParBytes > kParHead + kBigPoolBytes ? kParBytes : kParHead + kBigPoolBytes;
enum : int { C_NONE = 0, C_NUM, C_LP, C_RP, C_ADD, C_SUB, C_MUL, C_DIV };

template <int CTRL>
__device__ __forceinline__ int dpp(int old, int x) {  // row_shr:n = 0x110 + n, row_shl:n = 0x100 + n
  return __builtin_amdgcn_update_dpp(old, x, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t row_bits(uint64_t ballot, int rowbase) {
  return (uint32_t)(ballot >> rowbase) & 0xFFFFu;
}
__device__ __forceinline__ int hi_bit(uint32_t x) { return x ? 31 - __builtin_clz(x) : -1; }
__device__ __forceinline__ int lo_bit(uint32_t x) { return x ? __builtin_ctz(x) : -1; }
__device__ __forceinline__ int nth_bit(uint64_t t, int k) {  // position of set bit k (k < popcount)
  int pos = 0;
  int c = __popc((uint32_t)t);
  if (k >= c) { k -= c; pos = 32; t >>= 32; }
  c = __popc((uint32_t)t & 0xFFFFu);
  if (k >= c) { k -= c; pos += 16; t >>= 16; }
  c = __popc((uint32_t)t & 0xFFu);
  if (k >= c) { k -= c; pos += 8; t >>= 8; }
  c = __popc((uint32_t)t & 0xFu);
  if (k >= c) { k -= c; pos += 4; t >>= 4; }
  c = __popc((uint32_t)t & 0x3u);
  if (k >= c) { k -= c; pos += 2; t >>= 2; }
  c = (int)(t & 1u);
  if (k >= c) pos += 1;
  return pos;
}

__device__ __forceinline__ int ok_dep(int x) { return x; }
struct ParOut {
  int fb;  // leave to the per-lane path
  int fmt, correct;
};

// Called by the 16 lanes of a row together (j = lane in the row), the answer staged at row
// (16-B aligned, 80 bytes readable), n <= 64.  par: the row's kParBytes of LDS scratch.
__device__ ParOut par_reward(const uint8_t* row, int n, int j, int rowbase, uint8_t* par,
                             const int32_t (&nums)[kMaxNums], int n_nums, int32_t target) {
  ParOut o;
  o.fb = 0;
  o.fmt = 0;
  o.correct = 0;
  volatile double* slot_v = reinterpret_cast<volatile double*>(par);             // [16] value (stride 16 B)
  volatile uint32_t* slot_f = reinterpret_cast<volatile uint32_t*>(par + 8);     // [16] 1 ready | 2 float
  volatile uint8_t* child = par + 16 * kRow;                                      // [16][2]
  volatile uint8_t* mbytes = par + 16 * kRow + 3 * kRow;                          // [16]
  // ---- masks: lane j classifies bytes 4j..4j+3
  {
    const uint32_t x = reinterpret_cast<const uint32_t*>(row)[j];
    mbytes[j] = (uint8_t)(digit4(x) | space4(x) << 4);
  }
  asm volatile("" ::: "memory");  // the row's mask bytes (same wave: LDS keeps program order)
  const uint4 mb = *reinterpret_cast<const uint4*>(const_cast<uint8_t*>(mbytes));
  CD_PSTAMP(0, (int)mb.x);
  uint64_t D = 0, SP = 0;
  {
    const uint32_t w4[4] = {mb.x, mb.y, mb.z, mb.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // 4 mask bytes -> 16 bits of each mask
      uint32_t d = w4[q] & 0x0F0F0F0Fu, s = (w4[q] >> 4) & 0x0F0F0F0Fu;
      d = (d | d >> 4) & 0x00FF00FFu;
      d = (d | d >> 8) & 0xFFFFu;
      s = (s | s >> 4) & 0x00FF00FFu;
      s = (s | s >> 8) & 0xFFFFu;
      D |= (uint64_t)d << (16 * q);
      SP |= (uint64_t)s << (16 * q);
    }
  }
  const uint64_t lm = n >= 64 ? ~0ull : ((1ull << n) - 1);
  D &= lm;
  const uint64_t TS = lm & ~SP & ~(D & (D << 1));
  const int ntok = __popcll(TS);
  if (ntok > kRow) {
    o.fb = 1;
    return o;
  }
  // ---- lane k = token k
  const int k = j;
  const int valid = k < ntok;
  const int p = valid ? nth_bit(TS, k) : 0;
  const uint64_t cw = load8(row, p);
  const int b0 = (int)(cw & 0xFF), b1 = p + 1 < n ? (int)((cw >> 8) & 0xFF) : 0;
  const int isdig = (unsigned)(b0 - '0') < 10u;
  const unsigned kc = (unsigned)(b0 - '(');
  const int kind = kc < 8u ? (int)((0x70504632u >> (4 * kc)) & 15u) : 0;  // ( ) * + , - . /  -> C_*
  const int cls = valid ? (isdig ? C_NUM : kind) : C_NONE;
  const int L = cls == C_NUM ? ctz64(~(D >> p)) : 0;
  const int Lc = L < 1 ? 1 : L > 8 ? 8 : L;
  uint64_t x8 = (cw & (~0ull >> (64 - 8 * Lc))) << (8 * (8 - Lc));
  x8 &= 0x0F0F0F0F0F0F0F0Full;
  x8 = (x8 * 10 + (x8 >> 8)) & 0x00FF00FF00FF00FFull;
  x8 = (x8 * 100 + (x8 >> 16)) & 0x0000FFFF0000FFFFull;
  x8 = (x8 * 10000 + (x8 >> 32)) & 0xFFFFFFFFull;
  const uint32_t u = (uint32_t)x8;
  CD_PSTAMP(1, (int)u);
  int fb = valid & (cls == C_NONE);                                           // a byte outside the subset
  fb |= (cls == C_NUM) & (((b0 == '0') & (L > 1)) | (L > 8));                 // 0-led or > 8 digits
  fb |= ((cls == C_MUL) | (cls == C_DIV)) & (b1 == b0);                      // ** or //
  // ---- syntax against the previous token, parenthesis depth
  const int prev = dpp<0x111>(C_NONE, cls), next = dpp<0x101>(C_NONE, cls);
  const int ends_prev = (prev == C_NUM) | (prev == C_RP);
  const int expect = ends_prev ^ 1;
  int err = valid & ((((cls == C_NUM) | (cls == C_LP)) & (expect ^ 1)) |
                     (((cls == C_RP) | (cls == C_MUL) | (cls == C_DIV)) & expect));
  err |= (k == ntok - 1) & (cls != C_NUM) & (cls != C_RP);  // the end where an operand is expected
  const int delta = (cls == C_LP) - (cls == C_RP);
  int incl = delta;
  incl += dpp<0x111>(0, incl);
  incl += dpp<0x112>(0, incl);
  incl += dpp<0x114>(0, incl);
  incl += dpp<0x118>(0, incl);
  err |= valid & (incl < 0);
  err |= (k == ntok - 1) & (incl != 0);
  fb |= incl > kParDepth;
  const int depth = incl - delta;
  const int un = valid & ((cls == C_ADD) | (cls == C_SUB)) & expect;
  fb |= un & (next == C_LP);  // a sign before a group
  const int uw = un | ((un & (cls == C_SUB)) << 1);
  const int p1 = dpp<0x111>(0, uw), p2 = dpp<0x112>(0, uw), p3 = dpp<0x113>(0, uw), p4 = dpp<0x114>(0, uw);
  int c = p1 & 1, neg = c & (p1 >> 1);
  c &= p2 & 1;
  neg ^= c & (p2 >> 1);
  c &= p3 & 1;
  neg ^= c & (p3 >> 1);
  fb |= (cls == C_NUM) & c & (p4 & 1);  // a run of more than 3 signs
  const int bin = valid & (cls >= C_ADD) & (expect ^ 1);
  const int key = 2 * depth + ((cls == C_MUL) | (cls == C_DIV));
  const uint32_t rerr = row_bits(__ballot(err), rowbase), rfb = row_bits(__ballot(fb), rowbase);
  CD_PSTAMP(2, (int)(rerr + rfb + key));
  if (rfb) {  // first: check_format needs every digit run exactly (> 8 digits, other Unicode digits)
    o.fb = 1;
    return o;
  }
  // check_format: every digit run is a C_NUM token (<= 8 digits here).  For each of the numbers
  // q, the count of equal runs must equal its count among the numbers: every run lane and every
  // number lane j < n_nums add 1 << 4q per matching q (<= 8 per nibble when nf == n_nums), two
  // DPP row sums, compared in lane 15
  const uint32_t nummask = row_bits(__ballot(cls == C_NUM), rowbase);
  {
    int32_t mine = -1;
#pragma unroll
    for (int q = 0; q < kMaxNums; ++q) mine = q == j ? nums[q] : mine;
    uint32_t cl = 0, cn = 0;
#pragma unroll
    for (int q = 0; q < kMaxNums; ++q) {
      const int live = q < n_nums;
      cl += (uint32_t)(live & (cls == C_NUM) & ((int64_t)u == (int64_t)nums[q])) << (4 * q);
      cn += (uint32_t)(live & (j < n_nums) & (mine == nums[q])) << (4 * q);
    }
    cl += (uint32_t)dpp<0x111>(0, (int)cl);
    cn += (uint32_t)dpp<0x111>(0, (int)cn);
    cl += (uint32_t)dpp<0x112>(0, (int)cl);
    cn += (uint32_t)dpp<0x112>(0, (int)cn);
    cl += (uint32_t)dpp<0x114>(0, (int)cl);
    cn += (uint32_t)dpp<0x114>(0, (int)cn);
    cl += (uint32_t)dpp<0x118>(0, (int)cl);
    cn += (uint32_t)dpp<0x118>(0, (int)cn);
    o.fmt = (__popc(nummask) == n_nums) & (row_bits(__ballot((j == kRow - 1) & (cl == cn)), rowbase) != 0);
  }
  CD_PSTAMP(3, ok_dep(o.fmt));
  if (ntok == 0 || rerr) return o;  // a syntax error: not correct
  // ---- the parse tree: per key value (up to the OR of the wave's keys, an upper bound of the
  // largest) a ballot of the row's operators; L / R and their keys from the same masks
  const uint32_t below = (1u << k) - 1, above = 0xFFFFu & ~((2u << k) - 1);
  int kmax = 0;
#pragma unroll
  for (int bit = 0; bit < 3; ++bit) kmax |= __ballot(bin & ((key >> bit) & 1)) ? 1 << bit : 0;
  int Lp = -1, Rp = -1, kL = -1, kR = -1;
  for (int kk = 0; kk <= kmax; ++kk) {
    const uint32_t m = row_bits(__ballot(bin & (key == kk)), rowbase);
    const int cl = hi_bit(m & below), cr = lo_bit(m & above);
    const int takeL = (kk < key) & (cl > Lp);
    Lp = takeL ? cl : Lp;
    kL = takeL ? kk : kL;
    const int takeR = (kk <= key) & (cr >= 0) & ((Rp < 0) | (cr < Rp));
    Rp = takeR ? cr : Rp;
    kR = takeR ? kk : kR;
  }
  child[2 * k] = 0xFF;
  child[2 * k + 1] = 0xFF;
  const int toR = Rp >= 0 && (Lp < 0 || kR > kL);
  const int parent = toR ? Rp : Lp;
  if (bin && parent >= 0) child[2 * parent + (toR ? 0 : 1)] = (uint8_t)k;
  const int cl = child[2 * k], cr = child[2 * k + 1];
  const int lo = cl != 0xFF ? cl : hi_bit(nummask & below), ro = cr != 0xFF ? cr : lo_bit(nummask & above);
  if (row_bits(__ballot(bin & ((lo < 0) | (ro < 0))), rowbase)) {  // not reached for valid syntax
    o.fb = 1;
    return o;
  }
  const uint32_t rootm = row_bits(__ballot(bin & (parent < 0)), rowbase);
  const int root = rootm ? lo_bit(rootm) : lo_bit(nummask);
  CD_PSTAMP(4, root + lo + ro);
  // ---- evaluate: literals are ready, each operator fires once both operands are
  {
    const double uv = (double)u;
    slot_v[2 * k] = neg ? 0.0 - uv : uv;  // an int -0 is 0
    slot_f[4 * k] = cls == C_NUM ? 1u : 0u;
  }
  int ready = cls == C_NUM, zdiv = 0, big = 0;
  for (int round = 0; round < kRow; ++round) {
    if (!__ballot(bin & (ready ^ 1))) break;  // every operator of the wave has fired
    if (bin && !ready) {
      asm volatile("" ::: "memory");  // value + flags of both operands: two 16-B reads, one round trip
      const uint4 sx = *reinterpret_cast<const uint4*>(par + 16 * lo);
      const uint4 sy = *reinterpret_cast<const uint4*>(par + 16 * ro);
      const uint32_t fx = sx.z, fy = sy.z;
      if (fx & fy & 1u) {
        const double x = __hiloint2double((int)sx.y, (int)sx.x), y = __hiloint2double((int)sy.y, (int)sy.x);
        const int dv = cls == C_DIV;
        const double sm = x + (cls == C_SUB ? -y : y), pr = x * y, qt = x / y;
        double r = cls == C_MUL ? pr : dv ? qt : sm;
        const int rf = (int)((fx | fy) >> 1 & 1u) | dv;
        r = rf ? r : r + 0.0;  // an int -0 is 0
        zdiv |= dv & (y == 0.0);
        big |= (rf ^ 1) & (fabs(r) >= 9007199254740992.0);
        slot_v[2 * k] = r;
        slot_f[4 * k] = 1u | (uint32_t)rf << 1;
        ready = 1;
      }
    }
  }
  CD_PSTAMP(5, ready);
  if (row_bits(__ballot(big), rowbase)) {
    o.fb = 1;
    return o;
  }
  const int zd = row_bits(__ballot(zdiv), rowbase) != 0;
  const double rv = slot_v[2 * root];
  const uint32_t rfl = slot_f[4 * root];
  o.correct = !zd && ((rfl & 2u) ? fabs(rv - (double)target) < 1e-5 : rv == (double)target);
  CD_PSTAMP(6, o.correct);
  return o;
}

// The row's reward: the 16 lanes call this together; every lane gets the same result.
// fallback: lane 0 runs the per-lane path and broadcasts through par.
__device__ double row_reward(const uint8_t* stage, const uint8_t* src_global, int n, int j, int rowbase,
                             uint8_t* par, uint8_t* work, const int32_t (&nums)[kMaxNums], int n_nums,
                             int32_t target, double score, double format_score, uint8_t& flags, uint8_t& err) {
  int fb = !stage || n > kFastMax;
  int fmt = 0, correct = 0;
  if (!fb) {
    const ParOut o = par_reward(stage, n, j, rowbase, par, nums, n_nums, target);
    fb = o.fb;
    correct = o.correct;
    fmt = o.fmt;
  }
  if (fb) {
    double* bv = reinterpret_cast<double*>(par);  // LDS: the row's lanes read lane 0's result
    uint32_t* bf = reinterpret_cast<uint32_t*>(par + 8);
    if (j == 0) {
      uint8_t fl = 0, e = 0;
      const double r = countdown_reward(stage ? stage : src_global, n, stage != nullptr, nums, n_nums, target,
                                        score, format_score, fl, e, work, par + kParHead);
      *bv = r;
      *bf = (uint32_t)fl | (uint32_t)e << 8;
    }
    wave_sync();
    const double r = *bv;
    const uint32_t w = *bf;
    flags = (uint8_t)(w & 0xFF);
    err |= (uint8_t)(w >> 8);
    return r;
  }
  flags = (uint8_t)(fmt ? (correct ? 3 : 1) : 0);
  return fmt ? (correct ? score : format_score) : 0.0;
}

// An answer string is staged into its row's LDS with 16-B loads, one per lane of the row
// (a 256-B answer in one round trip); answer 0's first 64 B are loaded with the kernel's other
// loads (prestage), so only longer answers pay a round trip of their own.
constexpr int kStageMax = 256;  // answers up to this many bytes are staged (Lmax above: parsed in place)
constexpr int kPre = 64;        // bytes of answer 0 prestaged
__device__ __forceinline__ bool stage16(const uint8_t* g, int Lmax) {  // 16-B loads stay inside the slot
  return (Lmax & 15) == 0 && (reinterpret_cast<uintptr_t>(g) & 15u) == 0;
}
// bytes [from, n) of the answer at g into lds_row (from a multiple of 16 when stage16); lane j of the row
__device__ __forceinline__ void stage_answer(const uint8_t* g, int from, int n, int Lmax, uint8_t* lds_row, int j) {
  if (stage16(g, Lmax)) {
    const int c = j;
    if (16 * c >= from && 16 * c < n) *reinterpret_cast<uint4*>(lds_row + 16 * c) = reinterpret_cast<const uint4*>(g)[c];
  } else {
    for (int i = from + j; i < n; i += kRow) lds_row[i] = g[i];
  }
}

// Per row (16 lanes, one env or answer) of LDS: the staged answer, lane 0's per-lane evaluator
// stacks, the cooperative scratch.  64-thread blocks = 4 rows.
constexpr int kCdBlock = 64;
#ifndef RMI_CD_WPE
#define RMI_CD_WPE 4
#endif
// 16 readable bytes for the clamped answer-head loads of rows without one
__device__ __attribute__((aligned(16))) const uint32_t kZero16[4] = {0, 0, 0, 0};
// a staged row is 16-B aligned and readable 80 bytes past its start (the token reads)
__host__ __device__ constexpr int stage_stride(int Lmax) { return Lmax <= kStageMax ? ((Lmax + 15) & ~15) + 16 : 0; }
__host__ __device__ constexpr int cd_slice(int Lmax) { return stage_stride(Lmax) + kMachineBytes + kParRegion; }

__device__ __forceinline__ void load_nums(const rmi_countdown_t& env, int64_t b, int32_t (&nums)[kMaxNums]) {
#pragma unroll
  for (int k = 0; k < kMaxNums; ++k) nums[k] = k < env.max_nums ? env.nums[b * env.max_nums + k] : -1;
}

// One env per DPP row: all 16 lanes load the env's words (one broadcast per word) and run the
// turn's bookkeeping redundantly, so the answer evaluation is convergent across the row; lane
// 0 stores.  The turn is EnvStateManager.step's loop (run_turn, common.hpp) specialised to
// Countdown: every parsed answer is a valid action (no action_lookup, es_manager.py:234-235)
// and step() always ends the episode (env.py:58-62), so a turn steps at most once, on answer
// slot 0, when it has a parsed answer and the cap leaves room; the format penalty applies iff
// it has none.  Straight-line, so the wave carries no loop state (the generic loop's hoisted
// per-slot predicates spilled SGPRs and put ≈2 k cycles between the loads and the evaluator).
__global__ __launch_bounds__(kCdBlock) __attribute__((amdgpu_waves_per_eu(RMI_CD_WPE))) void countdown_step_turn_kernel(rmi_countdown_t env, rmi_episode_t ep,
                                                                       rmi_turn_t in,
                                                                       const uint8_t* __restrict__ answers,
                                                                       const int32_t* __restrict__ answer_len,
                                                                       int Lmax, uint8_t* __restrict__ err_out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t cd_lds[];  // [kCdBlock / kRow][cd_slice(Lmax)]
  const int j = threadIdx.x & (kRow - 1), rowbase = threadIdx.x & 63 & ~(kRow - 1);
  const int64_t b = ((int64_t)blockIdx.x * kCdBlock + threadIdx.x) / kRow;
  const int B = ep.B;
  if (b >= B) return;
#ifdef RMI_CD_STAMPS
  unsigned long long st[kCdStamps];
  st[0] = __builtin_amdgcn_s_memtime();
#endif
  // every load of this env is issued before the first use (one memory round trip): no load
  // sits behind a branch or a store that needs an earlier load's data (either makes the
  // compiler wait there and split the loads into serial round trips); the has_input byte,
  // lens[0], the answer head and the numbers come through pointers that are always valid
  // (clamped), selected afterwards
  uint8_t flags = ep.flags[b];
  const uint8_t has_in = *(in.has_input ? in.has_input + b : ep.flags + b);
  uint8_t* slice = cd_lds + (threadIdx.x / kRow) * cd_slice(Lmax);
  const uint8_t* ans = answers + b * (int64_t)in.K * Lmax;  // answer slot 0 of this env
  uint8_t* stage = Lmax <= kStageMax ? slice : nullptr;
  uint8_t* work = slice + stage_stride(Lmax);
  uint8_t* par = work + kMachineBytes;
  const bool pre_ok = in.K > 0 && stage && stage16(ans, Lmax);  // answer 0's head, with the other loads
  const int nc = (Lmax < kPre ? Lmax : kPre) >> 4;
  const uint4 head = *(pre_ok && j < nc ? reinterpret_cast<const uint4*>(ans) + j
                                        : reinterpret_cast<const uint4*>(kZero16));
  const int32_t len0 = *(in.K > 0 ? answer_len + b * (int64_t)in.K : env.n_nums + b);
  const int mn = env.max_nums;
  int32_t raw[kMaxNums];
#pragma unroll
  for (int k = 0; k < kMaxNums; ++k) raw[k] = env.nums[b * mn + (k < mn ? k : mn - 1)];
  const int n_nums = env.n_nums[b];
  const int32_t target = env.target[b];
  const int n_act = in.n_actions[b];
  int32_t num_actions = ep.num_actions[b], n_turns = ep.n_turns[b];
  double penalty = ep.penalty[b];
  // uses
  int32_t nums[kMaxNums];
#pragma unroll
  for (int k = 0; k < kMaxNums; ++k) nums[k] = k < mn ? raw[k] : -1;
  const int pre_n = pre_ok ? 16 * nc : 0;
  if (pre_ok && j < nc) *reinterpret_cast<uint4*>(stage + 16 * j) = head;
  const bool act = in.has_input ? has_in != 0 : !(flags & RMI_FLAG_DONE);
  if (!act) return;
#ifdef RMI_CD_STAMPS
  st[1] = __builtin_amdgcn_s_memtime() + (unsigned long long)(penalty == -12345.0);  // loads landed
  st[2] = st[3] = st[1];
#endif
  uint8_t err = 0;
  flags &= (uint8_t)~RMI_FLAG_DONE;  // done-ness is decided per stepped turn (es_manager.py:168)
  const int nact = n_act < in.K ? n_act : in.K;
  const bool stp = nact >= 1 && in.max_actions_per_traj - num_actions > 0;  // row-uniform
  double acc = 0.0;
  uint8_t info = 0, exec = 0;
  if (stp) {
    const int n = len0 > Lmax ? Lmax : (len0 < 0 ? 0 : len0);
    if (stage && n > 0) stage_answer(ans, pre_n, n, Lmax, stage, j);
    CD_STAMP(st, 2);  // the staging stores wait for their loads
    uint8_t fl;
    const double r = row_reward(stage, ans, n, j, rowbase, par, work, nums, n_nums, target, env.score,
                                env.format_score, fl, err);
#ifdef RMI_CD_STAMPS
    st[3] = (unsigned long long)(r != -12345.0) * __builtin_amdgcn_s_memtime();
#endif
    const bool eff = r > 0, succ = r == env.score;
    acc += r;
    exec = 1;
    info = (uint8_t)(RMI_INFO_PRESENT | (eff ? RMI_INFO_EFFECTIVE : 0) | RMI_INFO_VALID | (succ ? RMI_INFO_SUCCESS : 0));
    flags |= RMI_FLAG_TERMINATED | RMI_FLAG_DONE;  // done: terminated, truncated = not success
    flags = succ ? (uint8_t)(flags & ~RMI_FLAG_TRUNCATED) : (uint8_t)(flags | RMI_FLAG_TRUNCATED);
  }
  if (nact == 0) penalty += in.format_penalty;  // every parsed answer is valid: penalty iff none
  num_actions += exec;
  n_turns += 1;
  if (!stp && num_actions >= in.max_actions_per_traj) flags |= RMI_FLAG_TERMINATED | RMI_FLAG_TRUNCATED | RMI_FLAG_DONE;
#ifdef RMI_CD_STAMPS
  st[4] = __builtin_amdgcn_s_memtime();
#endif
  if (j) return;
  ep.num_actions[b] = num_actions;
  ep.flags[b] = flags;
  ep.n_turns[b] = n_turns;
  ep.penalty[b] = penalty;
  const int64_t tb = (int64_t)in.turn * B + b;
  ep.turn_reward[tb] = acc;
  ep.turn_info[tb] = info;
  ep.turn_exec[tb] = exec;
  if (err_out && err) err_out[b] |= err;
#ifdef RMI_CD_STAMPS
  if ((threadIdx.x & 63) == 0) {
    st[5] = __builtin_amdgcn_s_memtime();
    for (int q = 0; q < kCdStamps; ++q) g_cd_stamps[(int64_t)blockIdx.x * kCdStamps + q] = st[q];
  }
#endif
}

__global__ __launch_bounds__(kCdBlock) __attribute__((amdgpu_waves_per_eu(RMI_CD_WPE))) void countdown_reward_kernel(rmi_countdown_t env,
                                                                    const uint8_t* __restrict__ answers,
                                                                    const int32_t* __restrict__ answer_len, int Lmax,
                                                                    int n, double* __restrict__ reward,
                                                                    uint8_t* __restrict__ flags_out,
                                                                    uint8_t* __restrict__ err_out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t cd_lds[];
  const int j = threadIdx.x & (kRow - 1), rowbase = threadIdx.x & 63 & ~(kRow - 1);
  const int64_t i = ((int64_t)blockIdx.x * kCdBlock + threadIdx.x) / kRow;
  if (i >= n) return;
  uint8_t* slice = cd_lds + (threadIdx.x / kRow) * cd_slice(Lmax);
  uint8_t* stage = Lmax <= kStageMax ? slice : nullptr;
  uint8_t* work = slice + stage_stride(Lmax);
  uint8_t fl = 0, err = 0;
  int len = answer_len[i];
  if (len > Lmax) len = Lmax;
  if (len < 0) len = 0;
  int32_t nums[kMaxNums];
  load_nums(env, i, nums);
  const uint8_t* src = answers + i * (int64_t)Lmax;
  if (stage && len > 0) stage_answer(src, 0, len, Lmax, stage, j);
  const double r = row_reward(stage, src, len, j, rowbase, work + kMachineBytes, work, nums, env.n_nums[i],
                              env.target[i], env.score, env.format_score, fl, err);
  if (j) return;
  reward[i] = r;
  if (flags_out) flags_out[i] = fl;
  if (err_out) err_out[i] = err;
}

}  // namespace
}  // namespace rmi

#ifdef RMI_CD_STAMPS
RMI_API int rmi_countdown_set_stamps(unsigned long long* buf, unsigned long long* pbuf) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(rmi::g_cd_stamps), &buf, sizeof(buf)) != hipSuccess) return -2;
  return hipMemcpyToSymbol(HIP_SYMBOL(rmi::g_cd_pstamps), &pbuf, sizeof(pbuf)) == hipSuccess ? 0 : -2;
}
#endif

RMI_API int rmi_countdown_step_turn(const rmi_countdown_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                    const uint8_t* answers, const int32_t* answer_len, int32_t Lmax, uint8_t* err,
                                    rmi_stream_t stream) {
  using namespace rmi;
  if (!env || Lmax <= 0 || env->max_nums <= 0 || env->max_nums > 8) return RMI_EINVAL;
  if (!ep || !in || in->K < 0 || in->K > kMaxK || ep->B < 0 || in->turn < 0 || in->turn >= ep->T) return RMI_EINVAL;
  if (ep->T > 255 || in->max_actions_per_traj > 255) return RMI_EUNSUP;  // u8 counters
  if (ep->B == 0) return RMI_OK;
  if (!answers || !answer_len || !env->nums || !env->n_nums || !env->target || !in->n_actions || !ep->num_actions ||
      !ep->flags || !ep->n_turns || !ep->penalty || !ep->turn_reward || !ep->turn_info || !ep->turn_exec)
    return RMI_EINVAL;
  const int64_t lanes = (int64_t)ep->B * kRow;
  const dim3 grid((unsigned)((lanes + kCdBlock - 1) / kCdBlock));
  const size_t lds = (size_t)(kCdBlock / kRow) * cd_slice(Lmax);
  hipLaunchKernelGGL(countdown_step_turn_kernel, grid, dim3(kCdBlock), lds, as_stream(stream), *env, *ep, *in,
                     answers, answer_len, Lmax, err);
  return launch_status();
}

RMI_API int rmi_countdown_reward(const rmi_countdown_t* env, const uint8_t* answers, const int32_t* answer_len,
                                 int32_t Lmax, int32_t n, double* reward, uint8_t* flags, uint8_t* err,
                                 rmi_stream_t stream) {
  using namespace rmi;
  if (!env || Lmax <= 0 || n < 0 || env->max_nums <= 0 || env->max_nums > 8) return RMI_EINVAL;
  if (n == 0) return RMI_OK;
  if (!answers || !answer_len || !reward || !env->nums || !env->n_nums || !env->target) return RMI_EINVAL;
  const dim3 grid((unsigned)(((int64_t)n * kRow + kCdBlock - 1) / kCdBlock));
  const size_t lds = (size_t)(kCdBlock / kRow) * cd_slice(Lmax);
  hipLaunchKernelGGL(countdown_reward_kernel, grid, dim3(kCdBlock), lds, as_stream(stream), *env, answers, answer_len,
                     Lmax, n, reward, flags, err);
  return launch_status();
}
