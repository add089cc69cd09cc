// parse_core.hpp — the one-response-per-wave decode and parse of parse.hip (detok_row, parse_row and
// their helpers), shared with the Sokoban token turn (sokoban.hip: rmi_sokoban_token_turn), which runs
// them in front of the turn and the render in one launch.  See parse.hip for the design notes.
#pragma once
#include "common.hpp"
#include "text.hpp"

#include <stdlib.h>

namespace rmi {
namespace {

// Diagnostic build only (tools/prof_parse_stamps.py compiles this file with RMI_PARSE_STAMPS):
// per-wave s_memtime at phase boundaries, kept in SGPRs and written once at the end.
#ifdef RMI_PARSE_STAMPS
__device__ unsigned long long* g_parse_stamps;
__device__ unsigned long long* g_detok_stamps;
#define PSTAMP_DECL unsigned long long pst_[10] = {0}, prt0_ = __builtin_amdgcn_s_memrealtime()
#define PSTAMP(i) (pst_[i] = __builtin_amdgcn_s_memtime())
#define PSTAMP_FLUSH()                                                                 \
  do {                                                                                 \
    const unsigned long long rt_ = __builtin_amdgcn_s_memrealtime();                   \
    if ((threadIdx.x & 63) == 0) {                                                     \
      for (int s_ = 0; s_ < 10; ++s_) g_parse_stamps[b * 12 + s_] = pst_[s_];          \
      g_parse_stamps[b * 12 + 10] = prt0_;                                             \
      g_parse_stamps[b * 12 + 11] = rt_;                                               \
    }                                                                                  \
  } while (0)
// detok: 0 entry | 1 ids landed | 2 offsets landed | 3 bytes placed | 4 validity | 5 stored;
// 6 / 7 s_memrealtime at entry / end
#define DSTAMP_DECL unsigned long long dst_[6] = {0}, drt0_ = __builtin_amdgcn_s_memrealtime()
#define DSTAMP(i) (dst_[i] = __builtin_amdgcn_s_memtime())
#define DSTAMP_WAIT(i) (__builtin_amdgcn_s_waitcnt(0), dst_[i] = __builtin_amdgcn_s_memtime())
#define DSTAMP_FLUSH()                                                                 \
  do {                                                                                 \
    const unsigned long long rt_ = __builtin_amdgcn_s_memrealtime();                   \
    if ((threadIdx.x & 63) == 0) {                                                     \
      for (int s_ = 0; s_ < 6; ++s_) g_detok_stamps[b * 8 + s_] = dst_[s_];            \
      g_detok_stamps[b * 8 + 6] = drt0_;                                               \
      g_detok_stamps[b * 8 + 7] = rt_;                                                 \
    }                                                                                  \
  } while (0)
#else
#define PSTAMP_DECL \
  do {              \
  } while (0)
#define PSTAMP(i) \
  do {            \
  } while (0)
#define PSTAMP_FLUSH() \
  do {                 \
  } while (0)
#define DSTAMP_DECL \
  do {              \
  } while (0)
#define DSTAMP(i) \
  do {            \
  } while (0)
#define DSTAMP_WAIT(i) \
  do {                 \
  } while (0)
#define DSTAMP_FLUSH() \
  do {                 \
  } while (0)
#endif

constexpr int kPre = 8;                 // room for the implicit prefix tag in front of the text
constexpr int kTail = 24;               // zero bytes after a row (16-byte compares read 20 past)
constexpr int kMaxStride = 16384;       // detokenize rows (2 LDS rows per wave)
constexpr int kMaxParseStride = 8192;   // parse rows (rows + event lists: < 64 KB of LDS per wave)
constexpr int kRowWaves = 4;            // at most this many rows (one wave each) per workgroup
constexpr size_t kWgLds = 65536;        // LDS one workgroup may take; fewer rows per group on long rows
inline int row_waves(size_t lds_per_wave) {
  const size_t n = kWgLds / lds_per_wave;
  return n >= (size_t)kRowWaves ? kRowWaves : (n < 1 ? 1 : (int)n);
}

// A string of <= 16 bytes packed little-endian into two words (compile-time tags, the
// runtime separator and names alike), so that no byte table needs dynamic indexing.
struct Tag {
  uint64_t lo, hi;
  int n;
};
constexpr Tag make_tag(const char* s) {
  Tag t{0, 0, 0};
  while (s[t.n]) {
    const uint64_t c = (uint8_t)s[t.n];
    if (t.n < 8)
      t.lo |= c << (8 * t.n);
    else
      t.hi |= c << (8 * (t.n - 8));
    ++t.n;
  }
  return t;
}
__host__ __device__ constexpr uint64_t low_mask(int nbytes) {
  return nbytes <= 0 ? 0ull : (nbytes >= 8 ? ~0ull : ((1ull << (8 * nbytes)) - 1ull));
}
__device__ __forceinline__ uint8_t tag_byte(const Tag& t, int k) {
  return (uint8_t)(k < 8 ? t.lo >> (8 * k) : t.hi >> (8 * (k - 8)));
}

constexpr Tag kThinkOpen = make_tag("<think>");
constexpr Tag kThinkClose = make_tag("</think>");
constexpr Tag kAnsOpen = make_tag("<answer>");
constexpr Tag kAnsClose = make_tag("</answer>");
constexpr Tag kImStart = make_tag("<|im_start|>");
constexpr Tag kImEnd = make_tag("<|im_end|>");
// event ids (the special-token order of ctx_manager.py:94, 1-based; 0 = no tag)
enum : int { E_NONE = 0, E_THINK_O = 1, E_THINK_C = 2, E_ANS_O = 3, E_ANS_C = 4, E_IM_S = 5, E_IM_E = 6 };

// bytes [s, s + 16) of an LDS row (dword-aligned base, >= 20 readable bytes past s)
__device__ __forceinline__ void load16(const uint8_t* B, int s, uint64_t& lo, uint64_t& hi) {
  const uint32_t* B4 = reinterpret_cast<const uint32_t*>(B);
  const int q = s >> 2, r = s & 3;
  uint32_t w[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) w[k] = B4[q + k];
  const uint64_t a = (uint64_t)w[0] | ((uint64_t)w[1] << 32), c = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  const uint64_t e = w[4];
  lo = r == 0 ? a : (a >> (8 * r)) | (c << (64 - 8 * r));
  hi = r == 0 ? c : (c >> (8 * r)) | (e << (64 - 8 * r));
}
__device__ __forceinline__ bool tag_eq(uint64_t lo, uint64_t hi, const Tag& t) {
  return ((lo & low_mask(t.n)) == t.lo) && ((hi & low_mask(t.n - 8)) == t.hi);
}
// which of the six tags starts at B[x] (a '<'); tags never run into a row's zero tail
__device__ __forceinline__ int classify_tag(const uint8_t* B, int x) {
  uint64_t lo, hi;
  load16(B, x, lo, hi);
  return tag_eq(lo, hi, kThinkOpen)    ? E_THINK_O
         : tag_eq(lo, hi, kThinkClose) ? E_THINK_C
         : tag_eq(lo, hi, kAnsOpen)    ? E_ANS_O
         : tag_eq(lo, hi, kAnsClose)   ? E_ANS_C
         : tag_eq(lo, hi, kImStart)    ? E_IM_S
         : tag_eq(lo, hi, kImEnd)      ? E_IM_E
                                       : E_NONE;
}

// Positions x in [from, to) with B[x] == ch, ascending, into list; -> count (wave-uniform).
// One dword per lane per 256 bytes, SWAR byte test, wave prefix sum for the slots.
__device__ int collect(const uint8_t* B, int from, int to, uint32_t ch, uint16_t* list, int lane) {
  int cnt = 0;
  const uint32_t rep = ch * 0x01010101u;
  for (int c = from & ~3; c < to; c += 256) {
    const int i0 = c + 4 * lane;
    uint32_t m4 = 0;
    if (i0 < to) {
      const uint32_t x = *reinterpret_cast<const uint32_t*>(B + i0) ^ rep;  // zero byte where B == ch
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = i0 + j;
        const bool hit = ((x >> (8 * j)) & 0xFFu) == 0;
        if (hit && p >= from && p < to) m4 |= 1u << j;
      }
    }
    const int k = __builtin_popcount(m4);
    const int incl = wave_inclusive_scan(k);
    int o = cnt + incl - k;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (m4 & (1u << j)) list[o++] = (uint16_t)(i0 + j);
    cnt += __builtin_amdgcn_readlane(incl, 63);
  }
  return cnt;
}

// The classified '<' events: positions EL[i], tag ids EI[i] (i < n, position order); the
// first 64 also in registers (lane i holds event i), so typical rows never re-read LDS.
struct EvList {
  const uint16_t* EL;
  const uint8_t* EI;
  int n, p0, id0;
};
// First event with id == want (want < 0: any tag) at position in [from, lim) -> its
// position, else -1 (wave-uniform).
__device__ int next_event(const EvList& E, int want, int from, int lim, int lane) {
  for (int c = 0; c < E.n; c += 64) {
    const int i = c + lane;
    bool hit = false;
    int p = 0;
    if (i < E.n) {
      p = c == 0 ? E.p0 : (int)E.EL[i];
      const int id = c == 0 ? E.id0 : (int)E.EI[i];
      hit = p >= from && p < lim && (want < 0 ? id != E_NONE : id == want);
    }
    const uint64_t m = __ballot(hit);
    if (m) return __builtin_amdgcn_readlane(p, __builtin_ctzll(m));
  }
  return -1;
}

// Name ids of one piece against every name (lowercased ASCII, <= 16 bytes): 0 = no name.
struct Names {
  int n;
  uint64_t lo[RMI_PARSE_MAX_NAMES], hi[RMI_PARSE_MAX_NAMES];
  int len[RMI_PARSE_MAX_NAMES], id[RMI_PARSE_MAX_NAMES];
};
__device__ __forceinline__ uint64_t swar_lower(uint64_t x) {  // ASCII bytes: 'A'..'Z' += 0x20
  constexpr uint64_t k80 = 0x8080808080808080ull;
  const uint64_t ge_a = (x + 0x3F3F3F3F3F3F3F3Full) & k80;  // byte >= 'A'
  const uint64_t gt_z = (x + 0x2525252525252525ull) & k80;  // byte > 'Z'
  return x + ((ge_a & ~gt_z) >> 2);
}
__device__ int piece_id(const uint8_t* B, int s, int e, const Names& nm) {
  const int L = e - s;
  if (L <= 16) {
    uint64_t lo, hi;
    load16(B, s, lo, hi);
    lo &= low_mask(L);
    hi &= low_mask(L - 8);
    if (((lo | hi) & 0x8080808080808080ull) == 0) {
      lo = swar_lower(lo);  // zero bytes past L stay zero
      hi = swar_lower(hi);
      int id = 0;
#pragma unroll
      for (int j = 0; j < RMI_PARSE_MAX_NAMES; ++j)  // unrolled: the name table stays in registers
        if (j < nm.n && L == nm.len[j] && lo == nm.lo[j] && hi == nm.hi[j]) id = nm.id[j];
      return id;
    }
  }
  // non-ASCII (only U+212A KELVIN SIGN lowercases to ASCII) or long: per character
  int id = 0;
#pragma unroll
  for (int j = 0; j < RMI_PARSE_MAX_NAMES; ++j) {
    bool ok = j < nm.n && id == 0;
    int q = 0;
    for (int i = s; ok && i < e;) {
      uint32_t c = B[i];
      if (c < 0x80) {
        c += (c >= 'A' && c <= 'Z') ? 32u : 0u;
        ++i;
      } else if (c == 0xE2 && i + 2 < e && B[i + 1] == 0x84 && B[i + 2] == 0xAA) {
        c = 'k';
        i += 3;
      } else {
        ok = false;
        break;
      }
      const uint64_t w = q < 8 ? nm.lo[j] >> (8 * q) : nm.hi[j] >> (8 * (q - 8));
      ok = q < nm.len[j] && (uint32_t)(w & 0xFFu) == c;
      ++q;
    }
    if (ok && q == nm.len[j]) id = nm.id[j];
  }
  return id;
}

// s = s.replace(tok, "").strip() on src[a, z) -> the returned buffer's [a, z'): wave-parallel.
// The six tokens cannot overlap themselves ('<' only first, '>' only last), so Python's
// left-to-right non-overlapping replace removes exactly every occurrence present in src.
// A pass whose token is absent copies nothing.
__device__ uint8_t* replace_strip_wave(uint8_t* src, uint8_t* dst, uint16_t* lst, uint8_t* cov, int a, int& z,
                                       const Tag& t, int lane) {
  const int n = collect(src, a, z, '<', lst, lane);
  wave_sync();
  for (int x = a + lane; x < z; x += 64) cov[x] = 0;
  wave_sync();
  bool any = false;
  for (int c = 0; c < n; c += 64) {
    const int i = c + lane;
    bool occ = false;
    int x = 0;
    if (i < n) {
      x = lst[i];
      uint64_t lo, hi;
      load16(src, x, lo, hi);
      occ = x + t.n <= z && tag_eq(lo, hi, t);
    }
    if (occ)
      for (int d = 0; d < t.n; ++d) cov[x + d] = 1;
    any |= __ballot(occ) != 0;
  }
  uint8_t* out = src;
  if (any) {
    wave_sync();
    int o = a;
    for (int c = a; c < z; c += 64) {
      const int x = c + lane;
      const bool keep = x < z && !cov[x];
      const int incl = wave_inclusive_scan(keep ? 1 : 0);
      if (keep) dst[o + incl - 1] = src[x];
      o += __builtin_amdgcn_readlane(incl, 63);
    }
    z = o;
    out = dst;
    if (lane < kTail) dst[z + lane] = 0;
    wave_sync();
  }
  return out;
}

struct ParseArgs {
  rmi_parse_cfg_t cfg;
  const uint8_t* text;
  const int32_t* text_len;
  int64_t B;
  int stride;
  const uint8_t* sel;
  int8_t* actions;
  uint8_t* n_actions;
  int32_t* spans;
  uint8_t* action_text;
  int32_t* action_len;
  int Lact;
  uint8_t* err;
};

__host__ __device__ constexpr int row_bytes(int stride) { return (4 + kPre + stride + kTail + 7) & ~7; }
__host__ __device__ constexpr int list_cap(int stride) { return (kPre + stride + 8) & ~7; }
// T row | W row | EL u16[cap] | ES u16[cap] | EI u8[cap]
__host__ __device__ constexpr size_t parse_lds(int stride) {  // per wave, a multiple of 8
  return (2 * (size_t)row_bytes(stride) + 5 * (size_t)list_cap(stride) + 7) & ~(size_t)7;
}

// The lookup names of one row's id column (kernel arguments, so no memory round trip of its own)
__device__ __forceinline__ Names load_names(const rmi_parse_cfg_t& cfg, int col) {
  Names nm;
  nm.n = cfg.n_names;
#pragma unroll
  for (int j = 0; j < RMI_PARSE_MAX_NAMES; ++j) {
    nm.lo[j] = cfg.name_lo[j];
    nm.hi[j] = cfg.name_hi[j];
    nm.len[j] = cfg.name_len[j];
    nm.id[j] = cfg.name_id[col][j];
  }
  return nm;
}

#ifdef RMI_PARSE_STAMPS
#define PSTAMP_PARAM , unsigned long long* pst_
#define PSTAMP_ARG , pst_
#else
#define PSTAMP_PARAM
#define PSTAMP_ARG
#endif

// One response, staged: its len bytes at T + kPre of the wave's LDS (T, Wb, EL, ES, EI: the
// regions of parse_lds).  Adds the implicit "<think>" / "<answer>" prefix and the zero tail,
// then the regex, the special-token cascade, the split and the name lookup, and writes row b's
// outputs.  err: bits already set for this row (with the parse's own: a.err[b] = them).
__device__ __forceinline__ void parse_row(const ParseArgs& a, uint8_t* T, uint8_t* Wb, uint16_t* EL, uint16_t* ES,
                                          uint8_t* EI, int64_t b, int len, uint8_t err, const Names& nm,
                                          int lane PSTAMP_PARAM) {
  const rmi_parse_cfg_t& cfg = a.cfg;
  const int K = cfg.K;
  const Tag pre = cfg.enable_think ? kThinkOpen : kAnsOpen;
  const int plen = cfg.prepend ? pre.n : 0;
  const int base = kPre - plen, n_end = kPre + len;  // the prefixed response is T[base, n_end)
  wave_sync();
  if (lane < kTail) T[n_end + lane] = 0;
  if (lane < 4 + kPre) T[lane - 4] = (lane - 4 >= base) ? tag_byte(pre, lane - 4 - base) : 0;
  wave_sync();
  PSTAMP(1);

  // ---- 1. '<' events, classified (64 per step)
  EvList E{EL, EI, collect(T, base, n_end, '<', EL, lane), 0, E_NONE};
  wave_sync();
  for (int i = lane; i < E.n; i += 64) {
    const int p = EL[i], id = classify_tag(T, p);
    if (i < 64) {
      E.p0 = p;
      E.id0 = id;
    } else {
      EI[i] = (uint8_t)id;
    }
  }
  wave_sync();
  PSTAMP(2);

  // ---- 2. re.search(pattern, response, re.DOTALL)  (ctx_manager.py:149-150)
  int ts = -1, te = -1, as = -1, ae = -1;
  if (cfg.enable_think) {
    // <think>(.*?)</think>\s*<answer>(.*?)</answer>: the leftmost <think> decides (a later
    // start only sees a subset of the </think> candidates); group 1 grows over the
    // </think> candidates in order until \s*<answer> follows; group 2 ends at the first
    // </answer> after it (if there is none, no later candidate can have one either)
    const int i = next_event(E, E_THINK_O, base, n_end, lane);
    if (i >= 0) {
      int j = i + kThinkOpen.n, k = -1;
      for (;;) {
        j = next_event(E, E_THINK_C, j, n_end, lane);
        if (j < 0) break;
        k = j + kThinkClose.n;
        for (int l; (l = ws_fwd(T, k, n_end)) != 0;) k += l;  // \s* is greedy and '<' is no space
        if (T[k] == '<' && next_event(E, E_ANS_O, k, k + 1, lane) == k) break;
        ++j;
      }
      if (j >= 0) {
        const int e = next_event(E, E_ANS_C, k + kAnsOpen.n, n_end, lane);
        if (e >= 0) {
          ts = i + kThinkOpen.n;
          te = j;
          as = k + kAnsOpen.n;
          ae = e;
        }
      }
    }
  } else {
    const int i = next_event(E, E_ANS_O, base, n_end, lane);
    if (i >= 0) {
      const int e = next_event(E, E_ANS_C, i + kAnsOpen.n, n_end, lane);
      if (e >= 0) {
        as = i + kAnsOpen.n;
        ae = e;
      }
    }
  }
  PSTAMP(3);

  // ---- 3. special-token replace cascade + strip of the action content (:161-163).  A token
  //         starting inside [as, ae) ends inside it (every token ends in '>', and the only '>'
  //         of </answer> is its last byte), so the event test over [as, ae) is exact.
  uint8_t* C = T;
  int ca = 0, cz = 0;
  if (as >= 0) {
    ca = as;
    cz = ae;
    if (next_event(E, -1, ca, cz, lane) < 0) {
      // every replace is a no-op, and strip() six times is strip() once.  An all-ASCII content of
      // <= 64 bytes strips on a mask (one byte per lane), anything else byte by byte
      const int Lr = cz - ca;
      const uint32_t cr = lane < Lr ? (uint32_t)T[ca + lane] : 0u;
      if (Lr <= 64 && __ballot(cr >= 0x80u) == 0) {
        const uint64_t text = __ballot(lane < Lr && !ascii_space(cr));
        if (text) {
          cz = ca + 64 - __builtin_clzll(text);
          ca += __builtin_ctzll(text);
        } else {
          ca = cz;
        }
      } else {
        strip(T, ca, cz);
      }
    } else {
      for (int q = 0; q < 6; ++q) {  // ctx_manager.py:94 order
        const Tag tok = q == 0 ? kThinkOpen
                        : q == 1 ? kThinkClose
                        : q == 2 ? kAnsOpen
                        : q == 3 ? kAnsClose
                        : q == 4 ? kImStart
                                 : kImEnd;
        uint8_t* other = C == T ? Wb : T;
        C = replace_strip_wave(C, other, EL, EI, ca, cz, tok, lane);
        strip(C, ca, cz);
      }
    }
  }
  PSTAMP(4);

  // ---- 4. split(action_sep), strip, drop empties, cap at K (:165-169); name -> id (es :230-240)
  const Tag sep{cfg.sep_lo, cfg.sep_hi, cfg.sep_len};
  int count = 0;
  // one step of up to 64 pieces, lane i's stripped [s, e) (in: lane i holds a piece): the
  // non-empty ones take the next slots in order, up to K
  auto put_pieces = [&](bool in, int s, int e) {
    const bool keep = in && e > s;
    const uint64_t km = __ballot(keep);
    const int slot = count + __builtin_popcountll(km & ((1ull << lane) - 1ull));
    if (keep && slot < K) {
      a.actions[b * K + slot] = (int8_t)(nm.n > 0 ? piece_id(C, s, e, nm) : 1);
      if (a.action_text) {
        const int L = e - s, Lc = L < a.Lact ? L : a.Lact;
        uint8_t* dst = a.action_text + (b * K + slot) * (int64_t)a.Lact;
        for (int q = 0; q < Lc; ++q) dst[q] = C[s + q];
        a.action_len[b * K + slot] = Lc;
        if (L > a.Lact) err |= RMI_ERR_UNSUP;
      }
    }
    count += __builtin_popcountll(km);
  };
  if (as >= 0) {
    // An all-ASCII answer shorter than 64 bytes (the usual one) is split on bit masks, one byte
    // per lane: the separator's occurrences are the AND of one ballot per separator byte, the
    // greedy left-to-right selection (str.split) walks their bits, the pieces' bounds go to
    // their lanes by a select per piece, and each strip is the first / last non-whitespace bit of the
    // piece's span — no LDS lists and no per-byte loops.  Anything else takes the lists below.
    const int La = cz - ca;
    const uint32_t ch = lane < La ? (uint32_t)C[ca + lane] : 0u;
    if (La < 64 && __ballot(ch >= 0x80u) == 0) {
      const uint64_t live = (1ull << La) - 1ull;
      uint64_t m = La >= sep.n ? live >> (sep.n - 1) : 0ull;  // occurrence starts i, i + sep.n <= La
      for (int k = 0; k < sep.n; ++k) m &= (__ballot(ch == tag_byte(sep, k)) & live) >> k;
      PSTAMP(7);
      uint64_t sel = 0;
      for (int last = 0; m;) {  // left to right, non-overlapping
        const int i = __builtin_ctzll(m);
        m &= m - 1;
        if (i >= last) {
          sel |= 1ull << i;
          last = i + sep.n;
        }
      }
      int ps = 0, pe = 0, np = 0;  // piece np = [ps, pe) on lane np (answer offsets)
      for (int start = 0;; ++np) {
        const int end = sel ? __builtin_ctzll(sel) : La;
        ps = lane == np ? start : ps;
        pe = lane == np ? end : pe;
        if (!sel) break;
        start = end + sep.n;
        sel &= sel - 1;
      }
      ++np;
      const uint64_t text = live & ~__ballot(ascii_space(ch));
      PSTAMP(8);
      int s = 0, e = 0;
      if (lane < np) {
        const uint64_t in = text & ((1ull << pe) - 1ull) & ~((1ull << ps) - 1ull);  // ps <= pe <= La < 64
        if (in) {
          s = ca + __builtin_ctzll(in);
          e = ca + 64 - __builtin_clzll(in);
        }
      }
      put_pieces(lane < np, s, e);
    } else {
      // separator candidates: positions of its first byte, full compare, greedy selection
      const int nc = collect(C, ca, cz, (uint32_t)(sep.lo & 0xFFu), ES, lane);
      wave_sync();
      PSTAMP(7);
      int ns = 0, last = ca;  // selected separators -> EL (the '<' list is no longer needed)
      for (int c = 0; c < nc; c += 64) {
        const int i = c + lane;
        bool m = false;
        int p = 0;
        if (i < nc) {
          p = ES[i];
          uint64_t lo, hi;
          load16(C, p, lo, hi);
          m = p + sep.n <= cz && tag_eq(lo, hi, sep);
        }
        uint64_t bits = __ballot(m);
        while (bits) {  // left to right, non-overlapping (str.split)
          const int L = __builtin_ctzll(bits);
          bits &= bits - 1;
          const int q = __builtin_amdgcn_readlane(p, L);
          if (q >= last) {
            if (lane == 0) EL[ns] = (uint16_t)q;
            ++ns;
            last = q + sep.n;
          }
        }
      }
      wave_sync();
      PSTAMP(8);
      // pieces: piece i = [i ? sel[i-1] + sep.n : ca, i < ns ? sel[i] : cz); one per lane
      for (int c = 0; c <= ns && count < K; c += 64) {
        const int i = c + lane;
        int s = 0, e = 0;
        if (i <= ns) {
          s = i ? EL[i - 1] + sep.n : ca;
          e = i < ns ? EL[i] : cz;
          strip(C, s, e);
        }
        put_pieces(i <= ns, s, e);
      }
    }
    if (count > K) count = K;
  }
  PSTAMP(5);
  if (lane >= count && lane < K) {
    a.actions[b * K + lane] = 0;
    if (a.action_text) a.action_len[b * K + lane] = 0;
  }
  const uint64_t any_err = __ballot(err != 0);
  uint8_t err_all = err;
  if (any_err) {  // OR over lanes (UNSUP may come from any piece lane)
    for (int off = 32; off > 0; off >>= 1) err_all |= (uint8_t)__shfl_xor((int)err_all, off);
  }
  if (lane == 0) {
    a.n_actions[b] = (uint8_t)count;
    if (a.spans) {  // offsets in the prefixed response
      a.spans[4 * b + 0] = ts < 0 ? -1 : ts - base;
      a.spans[4 * b + 1] = te < 0 ? -1 : te - base;
      a.spans[4 * b + 2] = as < 0 ? -1 : as - base;
      a.spans[4 * b + 3] = ae < 0 ? -1 : ae - base;
    }
    if (a.err) a.err[b] = err_all;  // every row's byte written: no pre-zeroed buffer
  }
  PSTAMP(6);
}

// ------------------------------------------------------------------ detokenize
// Lossy UTF-8 (Unicode Table 3-7 well-formed sequences; each maximal invalid subpart ->
// U+FFFD, as CPython's errors="replace" and Rust's from_utf8_lossy).  One lane.
__device__ int utf8_lossy(const uint8_t* src, int n, uint8_t* dst, int cap, bool& over) {
  int o = 0;
  auto put = [&](uint8_t c) {
    if (o < cap)
      dst[o++] = c;
    else
      over = true;
  };
  for (int i = 0; i < n;) {
    const uint32_t c = src[i];
    if (c < 0x80) {
      put((uint8_t)c);
      ++i;
      continue;
    }
    int need = 0;
    uint32_t lo1 = 0x80, hi1 = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) {
      need = 1;
    } else if (c >= 0xE0 && c <= 0xEF) {
      need = 2;
      if (c == 0xE0) lo1 = 0xA0;
      if (c == 0xED) hi1 = 0x9F;
    } else if (c >= 0xF0 && c <= 0xF4) {
      need = 3;
      if (c == 0xF0) lo1 = 0x90;
      if (c == 0xF4) hi1 = 0x8F;
    }
    int k = 1;
    bool ok = need > 0;
    for (; ok && k <= need; ++k) {
      if (i + k >= n) {
        ok = false;
        break;
      }
      const uint32_t d = src[i + k];
      const uint32_t lo = k == 1 ? lo1 : 0x80u, hi = k == 1 ? hi1 : 0xBFu;
      if (d < lo || d > hi) {
        ok = false;
        break;
      }
    }
    if (ok) {
      for (int j = 0; j <= need; ++j) put(src[i + j]);
      i += need + 1;
    } else {
      put(0xEF);  // U+FFFD over the maximal subpart src[i, i + k)
      put(0xBF);
      put(0xBD);
      i += need > 0 ? k : 1;
    }
  }
  return o;
}

// Ids are processed 256 per step (4 per lane): their loads, then the (offset, end, skip)
// gathers of all of them, then the byte gathers, each stage issued together so a step costs
// three memory round trips however long its tokens are.  Token bytes come as the aligned
// dwords covering them (tokens <= 9 bytes: 3 dwords; longer ones loop), clamped inside the
// vocabulary blob.
constexpr int kDetokG = 4;  // 64-id chunks per step
// the low n bytes of a dword set (n clamped to [0, 4])
__device__ __forceinline__ uint32_t byte_mask_n(int n) {
  return n >= 4 ? 0xFFFFFFFFu : (n <= 0 ? 0u : (1u << (8 * n)) - 1u);
}
// UTF-8 well-formedness (Unicode Table 3-7, what CPython's strict decode accepts) of the 4 bytes
// of dword w, with the 4 bytes before them in wp; -> bit 7 of each bad byte.  SWAR, no branches:
// a byte is a continuation byte (10xxxxxx) exactly when a lead 1-3 bytes back expects one (the
// byte before >= C0, two before >= E0, three before >= F0); C0, C1 and F5..FF never occur; and
// the second byte after E0 / ED / F0 / F4 is limited to A0-BF / 80-9F / 90-BF / 80-8F.  Bytewise
// compares use only bit 7 of each byte (shifted-in bits from the byte below never reach it).
__device__ __forceinline__ uint32_t swar_zero_bytes(uint32_t z) {  // bit 7 of each zero byte
  return ~((((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u) & 0x80808080u;
}
__device__ __forceinline__ uint32_t utf8_dword_bad(uint32_t w, uint32_t wp) {
  constexpr uint32_t H = 0x80808080u, L = 0x01010101u;
  const uint32_t c = w;
  const uint32_t p1 = __builtin_amdgcn_alignbyte(w, wp, 3);  // the byte before each byte of w
  const uint32_t p2 = __builtin_amdgcn_alignbyte(w, wp, 2);
  const uint32_t p3 = __builtin_amdgcn_alignbyte(w, wp, 1);
  const uint32_t cont = c & ~(c << 1) & H;
  const uint32_t expect = (p1 & (p1 << 1)) | (p2 & (p2 << 1) & (p2 << 2)) | (p3 & (p3 << 1) & (p3 << 2) & (p3 << 3));
  uint32_t err = (cont ^ expect) & H;
  err |= swar_zero_bytes((c & 0xFEFEFEFEu) ^ 0xC0C0C0C0u);                                   // C0, C1
  err |= c & (c << 1) & (c << 2) & (c << 3) & (c << 4);                                       // F8..FF
  err |= swar_zero_bytes((c & 0xF8F8F8F8u) ^ 0xF0F0F0F0u) & (c << 5) & ((c << 6) | (c << 7));  // F5..F7
  const uint32_t b5 = c << 2, b4 = c << 3;  // bits 5 and 4 of each byte, at bit 7
  err |= swar_zero_bytes(p1 ^ (0xE0u * L)) & ~b5;
  err |= swar_zero_bytes(p1 ^ (0xEDu * L)) & b5;
  err |= swar_zero_bytes(p1 ^ (0xF0u * L)) & ~(b5 | b4);
  err |= swar_zero_bytes(p1 ^ (0xF4u * L)) & (b5 | b4);
  return err & H;
}
__host__ __device__ constexpr size_t detok_lds(int stride) { return 2 * ((size_t)stride + 4) + 16; }  // per wave

struct DetokArgs {
  const int64_t* ids;
  int64_t R;
  const int32_t* n_ids;
  const uint4* vpk;
  const uint8_t* vbytes;
  int64_t n_bytes, V;
  uint8_t* out;
  int stride;
  int32_t* out_len;
  uint8_t* err_out;
  int64_t B;
};

#ifdef RMI_PARSE_STAMPS
#define DSTAMP_PARAM , unsigned long long* dst_
#define DSTAMP_ARG , dst_
#else
#define DSTAMP_PARAM
#define DSTAMP_ARG
#endif

// Row b decoded into buf (dword aligned; 4 writable bytes before it and stride + 8 after; fix:
// a second such buffer for the rare lossy rewrite, copied back), then written to out / out_len
// / err_out (and *derr, wave-uniform, when given).  -> the decoded length (the row stays in buf).
__device__ __forceinline__ int detok_row(const DetokArgs& d, uint8_t* buf, uint8_t* fix, int64_t b,
                                         int lane DSTAMP_PARAM, uint8_t* derr = nullptr) {
  const int stride = d.stride;
  int64_t rn = d.n_ids ? (int64_t)d.n_ids[b] : d.R;
  rn = rn < 0 ? 0 : (rn > d.R ? d.R : rn);
  const int64_t* row = d.ids + b * d.R;
  int pos = 0;
  bool bad = false, over = false;
  uint32_t high = 0;
  // the row buffer starts zeroed: token bytes are OR-ed into its dwords
  for (int i = lane; i < (stride + 8) / 4; i += 64) reinterpret_cast<uint32_t*>(buf)[i] = 0u;
  wave_sync();
  for (int64_t c0 = 0; c0 < rn; c0 += 64 * kDetokG) {
    int64_t id[kDetokG];
#pragma unroll
    for (int g = 0; g < kDetokG; ++g) {  // (c0 + 64 * g < rn: wave-uniform; empty chunks issue nothing)
      const int64_t i = c0 + 64 * g + lane;
      id[g] = c0 + 64 * g < rn && i < rn ? row[i] : -1;
    }
    DSTAMP_WAIT(1);
    // one 16-B gather per id: the token's bytes inline (<= 12) or its blob offset, and its
    // length / skip bit (rmi_vocab_pack)
    uint4 ent[kDetokG];
#pragma unroll
    for (int g = 0; g < kDetokG; ++g) {
      ent[g] = make_uint4(0u, 0u, 0u, 0x80000000u);  // an empty chunk: skipped
      if (c0 + 64 * g >= rn) continue;
      const bool in = c0 + 64 * g + lane < rn;
      const bool valid = id[g] >= 0 && id[g] < d.V;
      bad |= in && !valid;
      ent[g] = d.vpk[valid ? id[g] : 0];  // clamped, branch-free gather
      if (!valid) ent[g].w = 0x80000000u;
    }
    DSTAMP_WAIT(2);
    int len[kDetokG], start[kDetokG];
#pragma unroll
    for (int g = 0; g < kDetokG; ++g) {
      len[g] = (ent[g].w >> 31) ? 0 : (int)(ent[g].w & 0xFFFFFFu);
      start[g] = pos;
      if (c0 + 64 * g >= rn) continue;
      const int incl = wave_inclusive_scan(len[g]);
      start[g] = pos + incl - len[g];
      pos += __builtin_amdgcn_readlane(incl, 63);
    }
#pragma unroll
    for (int g = 0; g < kDetokG; ++g) {
      if (c0 + 64 * g >= rn) continue;
      const int sl = start[g], ln = len[g];
      if (ln <= 12 && sl + ln <= stride) {
        // the token's bytes, masked to ln, shifted to the destination's byte offset and OR-ed
        // into <= 4 zeroed dwords (no loop over the bytes, no divergence)
        const uint32_t x0 = ent[g].x & byte_mask_n(ln);
        const uint32_t x1 = ent[g].y & byte_mask_n(ln - 4);
        const uint32_t x2 = ent[g].z & byte_mask_n(ln - 8);
        high |= x0 | x1 | x2;
        const int sh = sl & 3;
        const uint32_t y0 = x0 << (8 * sh);
        const uint32_t y1 = sh ? __builtin_amdgcn_alignbyte(x1, x0, 4 - sh) : x1;
        const uint32_t y2 = sh ? __builtin_amdgcn_alignbyte(x2, x1, 4 - sh) : x2;
        const uint32_t y3 = sh ? x2 >> (8 * (4 - sh)) : 0u;
        uint32_t* q = reinterpret_cast<uint32_t*>(buf) + (sl >> 2);
        if (y0) atomicOr(q, y0);
        if (y1) atomicOr(q + 1, y1);
        if (y2) atomicOr(q + 2, y2);
        if (y3) atomicOr(q + 3, y3);
      } else {
        // tokens longer than 12 bytes (their bytes in the blob at offset .x), or running past
        // the row: byte by byte
        for (int k = 0; k < ln; ++k) {
          const int p = sl + k;
          uint32_t c;
          if (ln <= 12)
            c = ((k < 4 ? ent[g].x : k < 8 ? ent[g].y : ent[g].z) >> (8 * (k & 3))) & 0xFFu;
          else
            c = (int64_t)ent[g].x + k < d.n_bytes ? d.vbytes[(int64_t)ent[g].x + k] : 0u;
          if (p < stride) {
            atomicOr(reinterpret_cast<uint32_t*>(buf) + (p >> 2), c << (8 * (p & 3)));
            high |= c;
          } else {
            over = true;
          }
        }
      }
    }
  }
  DSTAMP(3);
  int n = pos < stride ? pos : stride;
  if (lane < 8) buf[n + lane] = 0;  // the validity windows read up to 8 bytes past the end
  if (lane < 4) buf[lane - 4] = 0;  // ... and 4 before the start
  wave_sync();
  // Non-ASCII bytes: a wave-parallel validity test first, branch-free over 4 bytes per lane
  // (utf8_dword_bad).  Positions n .. n + 2 are tested too: the zero bytes after the row are no
  // continuation bytes, so a sequence cut off by the row's end is an error there.  Only an invalid
  // row takes the serial replacement pass.
  bool invalid = false;
  if (__ballot((high & 0x80808080u) != 0)) {  // high: the OR of the row's bytes, 4 per dword
    for (int c0 = 0; c0 < n + 3; c0 += 256) {
      const int i0 = c0 + 4 * lane;
      if (i0 >= n + 3) continue;
      const uint32_t* b4 = reinterpret_cast<const uint32_t*>(buf + i0);  // buf[-4, 0), buf[n, n + 8): zero
      invalid |= utf8_dword_bad(b4[0], b4[-1]) != 0u;
    }
  }
  DSTAMP(4);
  if (__ballot(invalid)) {  // some invalid sequence: the lossy rewrite (one lane), copied back
    int n0 = 0;
    bool ov = false;
    if (lane == 0) n0 = utf8_lossy(buf, n, fix, stride, ov);
    n = __builtin_amdgcn_readlane(n0, 0);
    over |= __builtin_amdgcn_readlane((int)ov, 0) != 0;
    wave_sync();
    for (int i = lane; i < (n + 3) >> 2; i += 64)
      reinterpret_cast<uint32_t*>(buf)[i] = reinterpret_cast<const uint32_t*>(fix)[i];
    wave_sync();
  }
  const int nw = (n + 3) >> 2;
  if (lane < 4 && (n & 3)) buf[n + lane] = 0;  // deterministic tail bytes
  wave_sync();
  uint32_t* o4 = reinterpret_cast<uint32_t*>(d.out + b * (int64_t)stride);
  const uint32_t* r4 = reinterpret_cast<const uint32_t*>(buf);
  for (int i = lane; i < nw; i += 64) o4[i] = r4[i];
  const uint64_t any_bad = __ballot(bad), any_over = __ballot(over);
  const uint8_t de = (uint8_t)((any_bad ? RMI_ERR_INDEX : 0) | (any_over ? RMI_ERR_UNSUP : 0));
  if (derr) *derr = de;
  if (lane == 0) {
    d.out_len[b] = n;
    if (d.err_out) d.err_out[b] = de;
  }
  DSTAMP(5);
  return n;
}


// rmi_detok_parse's argument checks (also those of rmi_sokoban_token_turn's decode + parse): ->
// RMI_OK with d / a filled, 1 for an empty batch (nothing to launch), or the error.
inline int detok_parse_args(const int64_t* ids, int64_t B, int64_t R, const int32_t* n_ids,
                            const uint32_t* vocab_packed, const uint8_t* vocab_bytes, int64_t n_bytes, int64_t V,
                            uint8_t* text, int32_t stride, int32_t* text_len, uint8_t* decode_err,
                            const rmi_parse_cfg_t* cfg, const uint8_t* sel, int8_t* actions, uint8_t* n_actions,
                            int32_t* spans, uint8_t* action_text, int32_t* action_len, int32_t Lact,
                            uint8_t* parse_err, DetokArgs& d, ParseArgs& a) {
  if (!cfg || B < 0 || R < 0 || V < 1 || stride <= 0) return RMI_EINVAL;
  if (cfg->K < 1 || cfg->sep_len < 1 || cfg->sep_len > 16 || cfg->n_names < 0) return RMI_EINVAL;
  if (cfg->K > kMaxK || cfg->n_names > RMI_PARSE_MAX_NAMES || stride % 4 != 0 || stride > kMaxParseStride ||
      B > 0x7FFFFFFF)
    return RMI_EUNSUP;
  for (int j = 0; j < cfg->n_names; ++j)
    if (cfg->name_len[j] < 1 || cfg->name_len[j] > 16) return RMI_EINVAL;
  if (B == 0) return 1;
  if (!text || !text_len || !vocab_packed || (R > 0 && !ids) || n_bytes < 0 || (n_bytes > 0 && !vocab_bytes) ||
      !actions || !n_actions)
    return RMI_EINVAL;
  if (action_text && (!action_len || Lact < 1)) return RMI_EINVAL;
  if ((reinterpret_cast<uintptr_t>(text) & 3u) || (reinterpret_cast<uintptr_t>(vocab_packed) & 15u)) return RMI_EUNSUP;
  d = DetokArgs{ids, R, n_ids, reinterpret_cast<const uint4*>(vocab_packed), vocab_bytes, n_bytes, V, text,
                (int)stride, text_len, decode_err, B};
  a = ParseArgs{*cfg, text, text_len, B, (int)stride, sel, actions, n_actions, spans, action_text, action_len,
                (int)Lact, parse_err};
  return RMI_OK;
}

}  // namespace
}  // namespace rmi
