// Host build of ragen_amd/csrc/bigint.hpp (TEST INFRASTRUCTURE): reads lines
//   <op> <a> <b>
// (a, b signed hex integers; b decimal for pow / shl / shr; a decimal digits for dec) from
// argv[1] and writes one result line per input to argv[2]: a signed hex integer, the IEEE bits
// of a double as 16 hex digits (todbl, tdiv), or RANGE / OVERFLOW / ZERODIV.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../ragen_amd/csrc/bigint.hpp"

using namespace rmi;

static bool parse_hex(const char* s, uint32_t* w) {
  bool neg = false;
  if (*s == '-') {
    neg = true;
    ++s;
  }
  const int len = (int)std::strlen(s);
  int n = 0;
  for (int i = len; i > 0; i -= 8) {
    const int st = i - 8 > 0 ? i - 8 : 0;
    std::string chunk(s + st, s + i);
    if (n >= kBigCap) return false;
    w[2 + n++] = (uint32_t)std::strtoul(chunk.c_str(), nullptr, 16);
  }
  w[1] = neg ? 1u : 0u;
  big_norm(w, n);
  return true;
}

static void print_big(std::FILE* o, const uint32_t* w) {
  const int n = big_n(w);
  if (n == 0) {
    std::fputs("0\n", o);
    return;
  }
  if (big_neg(w)) std::fputc('-', o);
  std::fprintf(o, "%x", big_d(w)[n - 1]);
  for (int i = n - 2; i >= 0; --i) std::fprintf(o, "%08x", big_d(w)[i]);
  std::fputc('\n', o);
}

static void print_status(std::FILE* o, int st) {
  std::fputs(st == BIG_RANGE ? "RANGE\n" : st == BIG_OVERFLOW ? "OVERFLOW\n" : "ZERODIV\n", o);
}

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  std::FILE* f = std::fopen(argv[1], "r");
  std::FILE* o = std::fopen(argv[2], "w");
  if (!f || !o) return 2;
  uint32_t a[kBigWords * 2], b[kBigWords * 2], r[kBigWords], q[kBigWords], t1[kBigWords], t2[kBigWords];
  uint32_t un[kDivU + 2], vn[2 * kBigCap], qs[kDivQ], xs[kDivU + 2];
  char op[16], sa[4096], sb[4096];
  while (std::fscanf(f, "%15s %4095s %4095s", op, sa, sb) == 3) {
    const std::string k(op);
    if (k == "dec") {
      const int st = big_from_dec(reinterpret_cast<const uint8_t*>(sa), (int)std::strlen(sa), r);
      if (st) print_status(o, st);
      else print_big(o, r);
      continue;
    }
    if (!parse_hex(sa, a)) {
      std::fputs("BADA\n", o);
      continue;
    }
    if (k == "todbl") {
      double d;
      const int st = big_to_double(a, d);
      if (st) print_status(o, st);
      else {
        unsigned long long bits;
        std::memcpy(&bits, &d, 8);
        std::fprintf(o, "%016llx\n", bits);
      }
      continue;
    }
    if (k == "pow" || k == "shl" || k == "shr") {
      const unsigned long long e = std::strtoull(sb, nullptr, 10);
      int st = BIG_OK;
      if (k == "pow") st = big_pow(a, e, r, t1, t2);
      else if (k == "shl") st = big_shl(a, e, r);
      else big_shr_floor(a, e, r);
      if (st) print_status(o, st);
      else print_big(o, r);
      continue;
    }
    if (!parse_hex(sb, b)) {
      std::fputs("BADB\n", o);
      continue;
    }
    int st = BIG_OK;
    if (k == "add") st = big_add(a, b, false, r);
    else if (k == "sub") st = big_add(a, b, true, r);
    else if (k == "mul") st = big_mul(a, b, r);
    else if (k == "fdiv") st = big_floordiv(a, b, r, nullptr, un, vn);
    else if (k == "mod") st = big_floordiv(a, b, nullptr, r, un, vn);
    else if (k == "divmod") {
      st = big_floordiv(a, b, q, r, un, vn);
      if (!st) {  // the quotient then the remainder on one line: "q r"
        const int n = big_n(q);
        if (n == 0) std::fputs("0 ", o);
        else {
          if (big_neg(q)) std::fputc('-', o);
          std::fprintf(o, "%x", big_d(q)[n - 1]);
          for (int i = n - 2; i >= 0; --i) std::fprintf(o, "%08x", big_d(q)[i]);
          std::fputc(' ', o);
        }
      }
    } else if (k == "and") st = big_bitop(0, a, b, r);
    else if (k == "or") st = big_bitop(1, a, b, r);
    else if (k == "xor") st = big_bitop(2, a, b, r);
    else if (k == "tdiv") {
      double d;
      st = big_true_div(a, b, d, un, vn, qs, xs);
      if (!st) {
        unsigned long long bits;
        std::memcpy(&bits, &d, 8);
        std::fprintf(o, "%016llx\n", bits);
        continue;
      }
    } else {
      std::fputs("BADOP\n", o);
      continue;
    }
    if (st) print_status(o, st);
    else print_big(o, r);
  }
  std::fclose(f);
  std::fclose(o);
  return 0;
}
