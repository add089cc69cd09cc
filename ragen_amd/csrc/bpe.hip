// bpe.hip — byte-level BPE encoding of prompt text on the device (gfx950).
//
//  rmi_bpe_encode   the tokenizer call of ContextManager.get_lm_inputs (ctx_manager.py:265-278)
//                   for a HF `tokenizers` byte-level BPE (the Qwen2 model family's tokenizer)
//
// One wave per row, the row staged in LDS.  The phases follow the tokenizer's pipeline:
//  1. UTF-8 decode + code-point classes (one lane per byte position, table lookups), written
//     over every byte of a character so that runs can be counted in bytes;
//  2. added tokens (<|im_start|> ...): candidate positions by a first-byte bitmap, the longest
//     match per position, then the leftmost-longest non-overlapping selection (a short serial
//     walk over the matches — the text holds a handful);
//  3. the pre-tokenizer regex: the match length at EVERY position, computed lane-parallel from
//     128-byte category bitmasks (wave ballots): the seven alternatives of the Qwen2 pattern are
//     runs and last-bit queries on those masks; a run that outgrows the window takes a serial
//     scan of the same rules;
//  4. the leftmost match chain (pre-token starts) by one wave-uniform walk: the window's match
//     lengths sit in a VGPR and each step is a v_readlane at the walk position;
//  5. BPE per pre-token, one lane per pre-token: symbols start as byte ids, the rank of every
//     adjacent pair is looked up once (all pairs of the row in parallel), then the lowest
//     (rank, position) pair is merged until none is left — the tokenizers crate's merge order
//     (word.rs merge_all: lowest rank first, leftmost on ties) — re-looking up only the two
//     pairs a merge changes;
//  6. token counts per pre-token, a wave scan for the row offsets, the ids written.
// Merges are an open-addressed hash of (left, right) -> (rank, merged id) in HBM (L2 / MALL
// resident for the hot pairs).
#include "common.hpp"

namespace rmi {
namespace {

// per-byte category bits in LDS (the code point's class spread over all its bytes)
enum : uint32_t {
  B_L = 1, B_N = 2, B_W = 4, B_NL = 8,  // = RMI_CP_L / N / W / NL
  B_START = 16,                         // first byte of a character
  B_SP = 32,                            // U+0020
  B_ADD = 64,                           // first byte of a selected added token
  B_IN = 128                            // any byte of a selected added token
};
constexpr uint32_t kNoRank = 0xFFFFFFFFu;
// Stamp points (diagnostic builds): stage | phases 1-4 | word cache + symbols | merges, or with
// RMI_BPE_FINE phase 1 | 2 | 3 | 4 (tools/prof_prompt_stamps.py prints four spans either way).
#ifdef RMI_BPE_FINE
#define BST_N(i) do {} while (0)
#define BST_F(i) RMI_STAMP(i)
#else
#define BST_N(i) RMI_STAMP(i)
#define BST_F(i) do {} while (0)
#endif
constexpr uint16_t kEnd = 0xFFFF;
constexpr int kKHit = 0x8000, kKMerge = 0x4000;  // K[j] flags of phase 5 (counts stay < 0x4000)
constexpr int kMaxStride = 3072;

// The added tokens and the ASCII code points' classes are staged in the wave's LDS when the
// table is small (Qwen2: 22 added tokens, ~300 bytes): phases 1 and 2 then read no global
// memory per byte.  (They used to: a class lookup was two dependent global loads per byte, and
// each added-token comparison a chain of global byte loads — ≈64 k cycles of a wave's 161 k.)
constexpr int kStageAdded = 64;
constexpr int kPairBatch = 4;     // a merge step's pair lookups in flight together
// 16 bytes per text byte (T, C 1; M, P, K 2; Y, R 4) and the staged tables (≈1.5 KB for the
// Qwen2 tokenizer with the prompt expansions): the wave's LDS, which sets how many rows are
// in flight per CU.  (R held the merged id too, as a u64: 20 bytes per text byte and ≈4.5 KB of
// tables, with the byte ids, the added tokens' bytes and 64 token slots always staged.)
struct Lds {  // carved from dynamic LDS, n = stride, na = the staged added tokens (0 or n_added)
  uint64_t* AW;  // each staged added token's first 32 bytes, zero padded [na][4]
  int32_t* Y;    // symbol id at a symbol start
  int32_t* AO;   // added_off [na + 1] (staged tables only)
  int32_t* AI;   // added_id [na]
  uint32_t* AF;  // added tokens' first-byte bitmap [8]
  uint16_t* M;   // match length at a position; then the symbol chain (next symbol start)
  uint16_t* P;   // pre-token starts
  uint16_t* K;   // tokens per pre-token, then the row offsets
  uint8_t* T;    // text, n + 16 (zero tail)
  uint8_t* C;    // category bits, n + 128
  uint8_t* AC;   // classes of the code points 0..127 [128]
  int32_t* EO;   // exp_off [ne + 1] (staged expansions only)
  int32_t* EI;   // exp_ids [nei]
};
__host__ __device__ constexpr int staged_added(int n_added) {
  return n_added > 0 && n_added <= kStageAdded ? n_added : 0;
}
// the staged tokens' 32-byte words: the plain tokens only when expansions follow them (an
// expansion is matched by its index byte, never by a word compare)
__host__ __device__ constexpr int staged_words(int n_added, int n_exp) {
  return staged_added(n_added) > 0 && n_exp > 0 && n_exp <= n_added ? n_added - n_exp : staged_added(n_added);
}
// the expansion tables are staged with the row when small (their ids are copied to every row
// that holds one; from HBM that was one dependent load per id)
constexpr int kStageExpIds = 512;
__host__ __device__ constexpr bool staged_exp(int n_exp, int n_exp_ids) {
#ifdef RMI_BPE_NO_EXP_LDS  // (A/B variant)
  return false;
#else
  return n_exp > 0 && n_exp_ids > 0 && n_exp_ids <= kStageExpIds;
#endif
}
// kernel modes: the one-kernel algorithm, its pre-tokenizer pass alone (two-pass form: no
// symbol ids, no counts, no expansion tables in LDS), the one-kernel algorithm over the rows the
// word pass flagged
enum { kModeFull = 0, kModePretok = 1, kModeRetry = 2 };
__host__ __device__ constexpr size_t bpe_lds(int stride, int na, int nw, int ne, int nei, int mode = kModeFull) {
  return 32 * (size_t)nw + (mode == kModePretok ? 0 : 4 * (size_t)stride) + 4 * (size_t)(na + 1) + 4 +
         4 * (size_t)na + 32 + 4 * (size_t)stride + (mode == kModePretok ? 0 : 2 * (size_t)stride + 128) +
         (size_t)stride + 16 + (size_t)stride + 128 + 128 +
         (mode != kModePretok && staged_exp(ne, nei) ? 4 * (size_t)(ne + 1) + 4 * (size_t)nei : 0);
}

// dst[0, n) = src[0, n) by one wave, 8 loads a lane in flight before the stores (a plain
// load-store loop waited on each load: one memory round trip per 64 entries)
__device__ __forceinline__ void stage_i32(int32_t* dst, const int32_t* __restrict__ src, int n, int lane) {
  constexpr int kU = 8;
  for (int i0 = 0; i0 < n; i0 += 64 * kU) {
    int32_t v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) v[u] = i0 + 64 * u + lane < n ? src[i0 + 64 * u + lane] : 0;
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (i0 + 64 * u + lane < n) dst[i0 + 64 * u + lane] = v[u];
  }
}

__device__ __forceinline__ uint64_t merge_lookup(const rmi_bpe_t& t, uint32_t a, uint32_t b) {
  const uint64_t key = ((uint64_t)a << 32) | b;
  uint64_t h = (key * 0x9E3779B97F4A7C15ull) >> t.merge_shift;
  for (;;) {
    const uint64_t k = t.merges[2 * h];
    if (k == key) return t.merges[2 * h + 1];
    if (k == ~0ull) return ~0ull;
    h = (h + 1) & t.merge_mask;
  }
}

// ---- the word cache (rmi_bpe_t.word_cache): 16 u32 per entry — the word's bytes (4 u32,
// zero padded), meta = ready | claimed | count << 8 | length, up to 9 ids stored as id + 1.
// Linear probing over kWcProbe slots; a slot is claimed by compare-and-swap on meta
// (0 -> claimed) and written once.  No acquire / release: the 8 XCDs' L2s are not coherent with
// each other inside a launch, and agent-scope ordering would write back / invalidate L2 on every
// probe.  A reader may therefore see an older state of a slot — empty, claimed, or a partly
// written entry — and the entry is laid out so that any such state is a miss, exactly: every
// dword of a slot goes 0 -> its final value once (dword stores and loads are single-copy
// atomic); meta is ready only in its final value; only words whose every key dword below the
// length is nonzero are inserted, and ids are stored plus one, so a dword still invisible (0)
// never equals the reader's key dword and never passes as an id.  Such a miss merges the word
// as before (and maybe inserts it again one slot on).  Launch boundaries make every XCD's
// entries visible to the next call.
constexpr int kWcWordMax = 16, kWcIdsMax = 9, kWcProbe = 8;
constexpr uint32_t kWcReady = 1u << 31, kWcClaimed = 1u << 30;

// the word T[a, a + len) as the key's four little-endian words, zero padded: five aligned dword
// reads of the row and a byte shift (T is 4-aligned with a zero tail; the fifth dword may reach
// into the next LDS array, whose bytes are masked off)
__device__ __forceinline__ void wc_key(const uint8_t* T, int a, int len, uint32_t k[4]) {
  const uint32_t* t4 = reinterpret_cast<const uint32_t*>(T + (a & ~3));
  uint32_t d[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) d[i] = t4[i];
  const int sh = a & 3;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t v = sh ? __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh) : d[i];
    const int r = len - 4 * i;  // bytes of the word in this key word
    k[i] = v & (r >= 4 ? ~0u : (r <= 0 ? 0u : (1u << (8 * r)) - 1u));
  }
}

__device__ __forceinline__ uint32_t wc_slot(const uint32_t k[4], int len, uint32_t mask) {
  uint64_t x = (((uint64_t)k[1] << 32) | k[0]) * 0x9E3779B97F4A7C15ull;
  x ^= ((((uint64_t)k[3] << 32) | k[2]) + (uint64_t)len) * 0xC2B2AE3D27D4EB4Full;
  x ^= x >> 29;
  return (uint32_t)(x >> 32) & mask;
}

// One probed entry, loaded whole (the ids come with the key: no second round trip for a hit):
// -> the word's id count (ids written to Y[0..)) if it holds the word, else 0; empty: the slot
// is empty (the probe sequence ends there).
__device__ __forceinline__ int wc_take(const uint4 (&w)[4], const uint32_t k[4], int len, int32_t* Y, bool& empty) {
  const uint32_t m = w[1].x;
  empty = m == 0;
  if (!(m & kWcReady) || (int)(m & 0xFF) != len || w[0].x != k[0] || w[0].y != k[1] || w[0].z != k[2] ||
      w[0].w != k[3])
    return 0;
  const int cnt = (int)((m >> 8) & 0xFF);
  if (cnt < 1 || cnt > kWcIdsMax) return 0;
  const uint32_t ids[kWcIdsMax] = {w[1].y, w[1].z, w[1].w, w[2].x, w[2].y, w[2].z, w[2].w, w[3].x, w[3].y};
  bool vis = true;  // every id written (stored + 1: 0 = not visible here yet)
#pragma unroll
  for (int q = 0; q < kWcIdsMax; ++q)
    if (q < cnt) vis &= ids[q] != 0u;
  if (!vis) return 0;
#pragma unroll
  for (int q = 0; q < kWcIdsMax; ++q)
    if (q < cnt) Y[q] = (int32_t)(ids[q] - 1u);
  return cnt;
}

__device__ __forceinline__ void wc_load(const rmi_bpe_t& t, uint32_t h, uint4 (&w)[4]) {
  const uint4* s = reinterpret_cast<const uint4*>(t.word_cache + 16 * (size_t)h);
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = s[i];
}

// the probe sequence from its (i0)th slot h on: -> the word's id count, or 0 on a miss
__device__ __forceinline__ int wc_find_from(const rmi_bpe_t& t, const uint32_t k[4], int len, int32_t* Y, uint32_t h,
                                            int i0) {
  for (int i = i0; i < kWcProbe; ++i, h = (h + 1) & t.word_cache_mask) {
    uint4 w[4];
    wc_load(t, h, w);
    bool empty;
    const int cnt = wc_take(w, k, len, Y, empty);
    if (cnt || empty) return cnt;
  }
  return 0;
}

// the ids: the symbol chain from a (Y at each symbol start, M the next start)
__device__ void wc_insert(const rmi_bpe_t& t, const uint32_t k[4], int len, const int32_t* Y, const uint16_t* M,
                          int a, int cnt) {
  // a key dword below the length that is zero could not tell "not visible yet" from the word
  // (four NUL bytes): such words are not cached
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (4 * i < len && k[i] == 0u) return;
  uint32_t h = wc_slot(k, len, t.word_cache_mask);
  for (int i = 0; i < kWcProbe; ++i, h = (h + 1) & t.word_cache_mask) {
    uint32_t* s = t.word_cache + 16 * (size_t)h;
    // a plain read first: on a cold cache thousands of waves insert the same few words, and a
    // compare-and-swap per wave per probed slot serialises them on a handful of lines (the
    // reset's encode spent 530 k cycles per wave here).  A slot being written, or a lost race,
    // is most likely this same word: give up (a missed insert only costs a later merge).
    const uint32_t m0 = *reinterpret_cast<volatile const uint32_t*>(s + 4);
    if (m0 != 0u) {
      if (!(m0 & kWcReady)) return;
      const uint4 w0 = *reinterpret_cast<const uint4*>(s);
      if ((int)(m0 & 0xFF) == len && w0.x == k[0] && w0.y == k[1] && w0.z == k[2] && w0.w == k[3]) return;
      continue;
    }
    if (atomicCAS(s + 4, 0u, kWcClaimed) != 0u) return;
    const uint32_t m = kWcReady | ((uint32_t)cnt << 8) | (uint32_t)len;
    *reinterpret_cast<uint4*>(s) = make_uint4(k[0], k[1], k[2], k[3]);
    for (int q = 0, p = a; q < cnt; ++q, p = M[p]) s[5 + q] = (uint32_t)Y[p] + 1u;
    s[4] = m;
    return;
  }
}

__device__ __forceinline__ int utf8_len(uint32_t b) {
  return b < 0x80 ? 1 : (b >= 0xC2 && b <= 0xDF) ? 2 : (b >= 0xE0 && b <= 0xEF) ? 3 : (b >= 0xF0 && b <= 0xF4) ? 4 : 0;
}

// the 64 bits of a 128-bit window (lo = [base, base+64), hi = [base+64, base+128)) from bit i
__device__ __forceinline__ uint64_t view(uint64_t lo, uint64_t hi, int i) {
  return i == 0 ? lo : (lo >> i) | (hi << (64 - i));
}
// end of the run of set bits of v starting at bit k (k <= 64): the first clear bit >= k
__device__ __forceinline__ int run_end(uint64_t v, int k) {
  if (k >= 64) return 64;
  const uint64_t r = ~(v >> k);
  return r == 0 ? 64 : k + __builtin_ctzll(r);
}
__device__ __forceinline__ uint64_t low_bits(int e) { return e >= 64 ? ~0ull : ((1ull << e) - 1); }

// case-insensitive match of the contraction letters after an apostrophe at p (the regex's
// (?i:'s|'t|'re|'ve|'m|'ll|'d)); -> match length in bytes or 0.  s also folds U+017F.
__device__ __forceinline__ int contraction(const uint8_t* T, int p, int lim) {
  if (p + 1 >= lim) return 0;
  const uint32_t a = T[p + 1] | 0x20, a_is = ((T[p + 1] & 0xDF) >= 'A' && (T[p + 1] & 0xDF) <= 'Z');
  if (a_is && (a == 's' || a == 't' || a == 'm' || a == 'd')) return 2;
  if (T[p + 1] == 0xC5 && p + 2 < lim && T[p + 2] == 0xBF) return 3;  // U+017F, folds to 's'
  if (p + 2 >= lim) return 0;
  const uint32_t b = T[p + 2] | 0x20, b_is = ((T[p + 2] & 0xDF) >= 'A' && (T[p + 2] & 0xDF) <= 'Z');
  if (!a_is || !b_is) return 0;
  if ((a == 'r' && b == 'e') || (a == 'v' && b == 'e') || (a == 'l' && b == 'l')) return 3;
  return 0;
}

// The Qwen2 pre-tokenizer match at char start p by a serial scan of the category bytes (the
// path for runs longer than the bitmask window, and the definition the fast path follows):
//   1 (?i:'s|'t|'re|'ve|'m|'ll|'d)   2 [^\r\n\p{L}\p{N}]?\p{L}+   3 \p{N}
//   4  ?[^\s\p{L}\p{N}]+[\r\n]*      5 \s*[\r\n]+   6 \s+(?!\S)   7 \s+
// s1 = segment end (the next selected added token, or the text end): the regex engine sees
// the segment as the whole input.
__device__ int match_serial(const uint8_t* T, const uint8_t* C, int p, int s1) {
  auto cat = [&](int q) -> uint32_t { return q < s1 ? C[q] : 0u; };
  auto is_o = [&](int q) { return q < s1 && !(C[q] & (B_L | B_N | B_W)); };
  auto run = [&](int q, uint32_t bit) {
    while (q < s1 && (C[q] & bit)) ++q;
    return q;
  };
  auto run_o = [&](int q) {
    while (is_o(q)) ++q;
    return q;
  };
  auto next_start = [&](int q) {
    ++q;
    while (q < s1 && !(C[q] & B_START)) ++q;
    return q;
  };
  const uint32_t c = cat(p);
  if (T[p] == '\'') {
    const int l = contraction(T, p, s1);
    if (l) return l;
  }
  const int n0 = next_start(p);
  if (c & B_L) return run(p, B_L) - p;
  if (!(c & (B_NL | B_N)) && (cat(n0) & B_L)) return run(n0, B_L) - p;
  if (c & B_N) return n0 - p;
  if ((c & B_SP) && is_o(n0)) return run(run_o(n0), B_NL) - p;
  if (!(c & B_W)) return run(run_o(p), B_NL) - p;  // c is [^\s\p{L}\p{N}]
  const int e = run(p, B_W);
  int last_nl = -1, last_start = p;
  for (int q = p; q < e; ++q) {
    if (C[q] & B_NL) last_nl = q;
    if (C[q] & B_START) last_start = q;
  }
  if (last_nl >= 0) return last_nl + 1 - p;
  if (e == s1) return e - p;
  if (last_start > p) return last_start - p;
  return e - p;
}

// The merges of one word whose symbols are the chain Y / M from a (the tokenizers crate's
// word.rs merge_all order: lowest rank first, leftmost on ties) -> its symbol count.
__device__ int merge_word(const rmi_bpe_t& tok, int32_t* Y, uint16_t* M, int a) {
  // each step: the ranks of the word's current pairs (kPairBatch first probes in flight
  // together; the entry carries the merged id with the rank), then the lowest rank merged
  // (leftmost on ties: the scan keeps the first of equal ranks)
  for (;;) {
    uint64_t best = ~0ull;
    int bq = -1;
    for (int q = a; q != kEnd;) {
      int qs[kPairBatch];
      uint64_t key[kPairBatch];
      uint4 ent[kPairBatch];
#pragma unroll
      for (int g = 0; g < kPairBatch; ++g) {
        qs[g] = q;
        const int nq = q != kEnd ? M[q] : kEnd;
        key[g] = (q != kEnd && nq != kEnd) ? ((uint64_t)(uint32_t)Y[q] << 32) | (uint32_t)Y[nq] : ~0ull;
        q = q != kEnd ? nq : kEnd;
      }
#pragma unroll
      for (int g = 0; g < kPairBatch; ++g) {
        const uint64_t h = (key[g] * 0x9E3779B97F4A7C15ull) >> tok.merge_shift;
        ent[g] = key[g] != ~0ull ? *reinterpret_cast<const uint4*>(tok.merges + 2 * h) : make_uint4(~0u, ~0u, ~0u, ~0u);
      }
#pragma unroll
      for (int g = 0; g < kPairBatch; ++g) {
        if (key[g] == ~0ull) continue;
        const uint64_t k0 = ((uint64_t)ent[g].y << 32) | ent[g].x, v0 = ((uint64_t)ent[g].w << 32) | ent[g].z;
        const uint64_t v = k0 == key[g] ? v0 : (k0 == ~0ull ? ~0ull : merge_lookup(tok, (uint32_t)(key[g] >> 32),
                                                                                     (uint32_t)key[g]));
        if ((v >> 32) < (best >> 32)) {
          best = v;
          bq = qs[g];
        }
      }
    }
    if (bq < 0) break;
    const int rq = M[bq];
    Y[bq] = (int32_t)(uint32_t)best;
    M[bq] = M[rq];
  }
  int cnt = 0;
  for (int q = a; q != kEnd; q = M[q]) ++cnt;
  return cnt;
}

template <int kMode>
__global__ __launch_bounds__(64) void bpe_encode_kernel(rmi_bpe_t tok, const uint8_t* __restrict__ text, int64_t pitch,
                                                        int stride,
                                                        const int32_t* __restrict__ text_len, int64_t* __restrict__ out,
                                                        int64_t out_stride, int32_t* __restrict__ out_len,
                                                        int32_t* __restrict__ n_tok,
                                                        const int32_t* __restrict__ mark_byte,
                                                        int32_t* __restrict__ mark_tok, uint8_t* __restrict__ err) {
  extern __shared__ __align__(16) uint8_t smem[];
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int S = stride;
  if (kMode == kModeRetry && !tok.pre_retry[b]) return;  // finished by the word pass
  if (kMode == kModePretok && threadIdx.x == 0) tok.pre_retry[b] = 0;
  const int na = staged_added(tok.n_added), nw = staged_words(tok.n_added, tok.n_exp);
  Lds L;
  {  // (the order of bpe_lds: the 8-byte words first, then 4-, 2- and 1-byte arrays)
    uint8_t* p = smem;
    L.AW = reinterpret_cast<uint64_t*>(p);
    p += 32 * (size_t)nw;
    L.Y = nullptr;
    if (kMode != kModePretok) {
      L.Y = reinterpret_cast<int32_t*>(p);
      p += 4 * (size_t)S;
    }
    L.AO = reinterpret_cast<int32_t*>(p);
    p += 4 * (size_t)(na + 1) + 4;
    L.AI = reinterpret_cast<int32_t*>(p);
    p += 4 * (size_t)na;
    L.AF = reinterpret_cast<uint32_t*>(p);
    p += 32;
    L.M = reinterpret_cast<uint16_t*>(p);
    p += 2 * (size_t)S;
    L.P = reinterpret_cast<uint16_t*>(p);
    p += 2 * (size_t)S;
    L.K = nullptr;
    if (kMode != kModePretok) {
      L.K = reinterpret_cast<uint16_t*>(p);
      p += 2 * (size_t)S + 128;
    }
    L.T = p;
    p += S + 16;
    L.C = p;
    p += S + 128;
    L.AC = p;
    p += 128;
    L.EO = reinterpret_cast<int32_t*>(p);  // (4-aligned: every array above is a multiple of 4 bytes)
    L.EI = L.EO + (tok.n_exp + 1);
  }
  const bool exp_lds = kMode != kModePretok && staged_exp(tok.n_exp, tok.n_exp_ids);
  const int32_t* EO = exp_lds ? L.EO : tok.exp_off;
  const int32_t* EI = exp_lds ? L.EI : tok.exp_ids;
  RMI_STAMP_DECL;
  RMI_STAMP(0);
  // the row's first 1 KB is loaded with its length (one round trip, not two: every row has
  // min(stride, pitch) readable bytes)
  const uint32_t* src = reinterpret_cast<const uint32_t*>(text + b * pitch);
  const int readable = (S < pitch ? S : (int)pitch) / 4;
  constexpr int kPre = 4;
  uint32_t pre[kPre];
#pragma unroll
  for (int i = 0; i < kPre; ++i) pre[i] = lane + 64 * i < readable ? src[lane + 64 * i] : 0u;
  const int n = text_len[b];
  const int base_len = out_len ? out_len[b] : 0;
  if (n < 0 || n > S) {
    if (lane == 0) {
      err[b] = RMI_ERR_STATE;
      if (n_tok) n_tok[b] = 0;
      if (mark_tok) mark_tok[b] = base_len;
    }
    return;
  }
  // ---- stage the row (dwords, the bytes past n zeroed), the byte ids, the first-byte bitmap
  const auto tail_mask = [n](int w, uint32_t v) {
    if (4 * w >= n) return 0u;
    return 4 * w + 4 > n ? v & (0xFFFFFFFFu >> (8 * (4 * w + 4 - n))) : v;
  };
#pragma unroll
  for (int i = 0; i < kPre; ++i) {
    const int w = lane + 64 * i;
    if (w < (n + 3) / 4 + 4) reinterpret_cast<uint32_t*>(L.T)[w] = tail_mask(w, pre[i]);
  }
  for (int w = lane + 64 * kPre; w < (n + 3) / 4 + 4; w += 64)
    reinterpret_cast<uint32_t*>(L.T)[w] = tail_mask(w, 4 * w < n ? src[w] : 0u);
  if (lane < 8) L.AF[lane] = tok.added_first[lane];
  const bool stage_added = na > 0;
  if (stage_added) {
    for (int i = lane; i <= tok.n_added; i += 64) L.AO[i] = tok.added_off[i];
    for (int i = lane; i < tok.n_added; i += 64) L.AI[i] = tok.added_id[i];
  }
  // the host's staging tables when given: every load below is independent of the others
  const bool words_given = stage_added && tok.added_words != nullptr;
  if (words_given)
    for (int i = lane; i < 4 * nw; i += 64) L.AW[i] = tok.added_words[i];
  if (tok.ascii_class && lane < 32)
    reinterpret_cast<uint32_t*>(L.AC)[lane] = reinterpret_cast<const uint32_t*>(tok.ascii_class)[lane];
  if (exp_lds) {
    stage_i32(L.EO, tok.exp_off, tok.n_exp + 1, lane);
    stage_i32(L.EI, tok.exp_ids, tok.n_exp_ids, lane);
  }
  // an expansion's first two bytes (lane e: expansion e), for the layout check below
  const int n_plain0 = tok.n_added - tok.n_exp;
  const uint64_t xw = (words_given && tok.n_exp > 0 && n_plain0 >= 0 && lane < tok.n_exp)
                          ? tok.added_words[4 * (n_plain0 + lane)] : 0ull;
  const uint32_t blk0 = tok.ascii_class ? 0u : tok.cp_block[0];  // the block of U+0000..U+00FF
  for (int w = lane; w < (n + 128 + 3) / 4; w += 64) reinterpret_cast<uint32_t*>(L.C)[w] = 0u;  // (C is 4-aligned)
  wave_sync();
  // second batch (without the host's tables): the ASCII classes from block 0, the token words
  if (!tok.ascii_class) {
    L.AC[lane] = tok.cp_class[blk0 * 256u + (uint32_t)lane];
    L.AC[lane + 64] = tok.cp_class[blk0 * 256u + 64u + (uint32_t)lane];
  }
  // the staged tokens as 32-byte words (lane a: token a), compared 8 bytes at a time below; a
  // token longer than 32 bytes sends the row to the global-table compare
  bool added_words = words_given;
  if (stage_added && !words_given) {
    bool longer = false;
    for (int a = lane; a < nw; a += 64) longer |= L.AO[a + 1] - L.AO[a] > 32;
    added_words = !__any(longer);
    for (int a = lane; added_words && a < nw; a += 64) {
      const int o0 = L.AO[a], len = L.AO[a + 1] - o0;
      uint64_t w[4] = {0, 0, 0, 0};
      for (int k = 0; k < len; ++k) w[k >> 3] |= (uint64_t)tok.added_bytes[o0 + k] << (8 * (k & 7));
#pragma unroll
      for (int q = 0; q < 4; ++q) L.AW[4 * a + q] = w[q];
    }
  }
  wave_sync();
  // the expansion placeholders are the last n_exp added tokens, e at n_plain + e with bytes
  // (0xFF, 0x80 + e) and id -(e + 1) (tokenizer.py builds them so): phase 2 then matches a 0xFF
  // candidate by its index byte and compares the others with the plain tokens only
  const int n_plain = tok.n_added - tok.n_exp;
  bool exp_tail = words_given && added_words && tok.n_exp > 0 && tok.n_exp <= 64 && n_plain >= 0;
  if (exp_tail) {  // (the expansions' first bytes came with the staging batch: xw, lane e)
    bool ok = true;
    if (lane < tok.n_exp) {
      const int e = lane, a = n_plain + e;
      ok = L.AI[a] == -(e + 1) && L.AO[a + 1] - L.AO[a] == 2 &&
           (uint32_t)(xw & 0xFFFFu) == (0xFFu | ((0x80u + (uint32_t)e) << 8));
    }
    exp_tail = !__any(!ok);
  }
  // without that layout every token is compared, and only nw of them are staged as words
  if (!exp_tail && nw < tok.n_added) added_words = false;
#ifndef RMI_BPE_FINE
  RMI_STAMP_WAIT(1);
#endif
  // ---- 1. UTF-8 decode and classes: a dword (4 text bytes) per lane; an all-ASCII dword (the
  //         bulk of a prompt) takes four class lookups and one dword store, any other goes
  //         byte by byte (a lead byte writes its continuation bytes, which their own lanes skip)
  bool bad = false, unsafe = false;
  for (int w = lane; 4 * w < n; w += 64) {
    const uint32_t v = reinterpret_cast<const uint32_t*>(L.T)[w];
    if ((v & 0x80808080u) == 0 && 4 * w + 4 <= n) {
      uint32_t cw = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t bk = (v >> (8 * k)) & 0xFFu;
        const uint32_t cat = (uint32_t)L.AC[bk] & (B_L | B_N | B_W | B_NL);
        cw |= (cat | B_START | (bk == 0x20 ? B_SP : 0u)) << (8 * k);
      }
      reinterpret_cast<uint32_t*>(L.C)[w] = cw;
      continue;
    }
    for (int p = 4 * w; p < 4 * w + 4 && p < n; ++p) {
    const uint32_t b0 = L.T[p];
    if ((b0 & 0xC0) == 0x80) continue;  // continuation: written by its lead byte's lane
    if (b0 == 0xFF && tok.n_exp > 0) {  // an expansion placeholder (0xFF, 0x80 + e): an added token
      if (p + 2 > n || (L.T[p + 1] & 0xC0) != 0x80) bad = true;
      else L.C[p] = (uint8_t)B_START;  // class "other"; the index byte keeps 0
      continue;
    }
    const int l = utf8_len(b0);
    uint32_t cp = 0;
    if (l == 0 || p + l > n) {
      bad = true;
      continue;
    }
    if (l == 1) {
      cp = b0;
    } else {
      cp = b0 & (0x7F >> l);
      for (int k = 1; k < l; ++k) {
        const uint32_t bk = L.T[p + k];
        if ((bk & 0xC0) != 0x80) bad = true;
        cp = (cp << 6) | (bk & 0x3F);
      }
    }
    if (cp > 0x10FFFF) {
      bad = true;
      continue;
    }
    const uint32_t cls = cp < 128 ? (uint32_t)L.AC[cp] : tok.cp_class[(uint32_t)tok.cp_block[cp >> 8] * 256u + (cp & 255u)];
    if (tok.nfc && (cls & RMI_CP_UNSAFE)) unsafe = true;
    const uint32_t cat = cls & (B_L | B_N | B_W | B_NL);
    L.C[p] = (uint8_t)(cat | B_START | (b0 == 0x20 ? B_SP : 0u));
    for (int k = 1; k < l; ++k) L.C[p + k] = (uint8_t)cat;
    }
  }
  const bool row_bad = __any(bad), row_unsafe = __any(unsafe);
  auto fail = [&](uint8_t code) {
    if (lane == 0) {
      err[b] = code;
      if (n_tok) n_tok[b] = 0;
      if (mark_tok) mark_tok[b] = base_len;
    }
  };
  if (row_bad) return fail(RMI_ERR_STATE);
  if (row_unsafe) return fail(RMI_ERR_UNSUP);
  wave_sync();
  BST_F(1);
  // ---- 2. added tokens: the candidate positions (character starts whose first byte starts
  //         some added token) listed first, then one candidate per lane: its longest match;
  //         then the leftmost-longest selection.  (Matching inside the 64-byte chunk loop ran
  //         the token loop once per chunk holding a candidate.)
  int n_cand = 0;
  if (tok.n_added > 0) {
    for (int w0 = 0; w0 < n; w0 += 64) {  // candidates -> P (ascending)
      const int p = w0 + lane;
      const bool c = p < n && (L.C[p] & B_START) && ((L.AF[L.T[p] >> 5] >> (L.T[p] & 31)) & 1u);
      const uint64_t m = __ballot(c);
      if (c) L.P[n_cand + __builtin_popcountll(m & ((1ull << lane) - 1))] = (uint16_t)p;
      n_cand += __builtin_popcountll(m);
    }
    wave_sync();
    // the longest match of each candidate (one per lane, id -> Y), then the leftmost-longest
    // selection over the chunk's candidates in ascending order: a scalar walk over the lanes'
    // (position, length) by readlane, and each selected token's bytes marked by the whole wave.
    // (A serial walk of lane 0 over the LDS lists, marking byte by byte, took ≈8 k cycles.)
    int cur = 0;
    for (int c0 = 0; c0 < n_cand; c0 += 64) {
      const int ci = c0 + lane;
      const bool has_c = ci < n_cand;
      const int p = has_c ? L.P[ci] : 0;
      int best_len = 0, best_id = 0;
      if (has_c) {
        if (added_words) {  // the text's next 32 bytes against each token, 8 bytes per compare
          const uint32_t* t4 = reinterpret_cast<const uint32_t*>(L.T + (p & ~3));
          uint32_t d[9];
#pragma unroll
          for (int q = 0; q < 9; ++q) d[q] = t4[q];
          const int sh = p & 3;
          uint64_t x[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t lo = sh ? __builtin_amdgcn_alignbyte(d[2 * q + 1], d[2 * q], sh) : d[2 * q];
            const uint32_t hi = sh ? __builtin_amdgcn_alignbyte(d[2 * q + 2], d[2 * q + 1], sh) : d[2 * q + 1];
            x[q] = ((uint64_t)hi << 32) | lo;
          }
          if (exp_tail && L.T[p] == 0xFFu) {  // an expansion placeholder: its index byte names it
            const int e = (int)L.T[p + 1] - 0x80;
            if (p + 2 <= n && e >= 0 && e < tok.n_exp) {
              best_len = 2;
              best_id = L.AI[n_plain + e];
            }
          } else {
            const int n_cmp = exp_tail ? n_plain : tok.n_added;
            for (int a = 0; a < n_cmp; ++a) {
              const int len = L.AO[a + 1] - L.AO[a];
              // the first word first: most tokens differ there (the rest only for a match)
              const uint64_t m0 = len >= 8 ? ~0ull : (1ull << (8 * len)) - 1;
              if (((x[0] ^ L.AW[4 * a]) & m0) != 0 || len <= best_len || p + len > n) continue;
              uint64_t diff = 0;
#pragma unroll
              for (int q = 1; q < 4; ++q) {
                const int r = len - 8 * q;  // bytes of this word inside the token
                const uint64_t m = r >= 8 ? ~0ull : (r <= 0 ? 0ull : (1ull << (8 * r)) - 1);
                diff |= (x[q] ^ L.AW[4 * a + q]) & m;
              }
              if (diff == 0) {
                best_len = len;
                best_id = L.AI[a];
              }
            }
          }
        } else {
          for (int a = 0; a < tok.n_added; ++a) {
            const int o0 = tok.added_off[a], len = tok.added_off[a + 1] - o0;
            if (len <= best_len || p + len > n) continue;
            int k = 0;
            while (k < len && tok.added_bytes[o0 + k] == L.T[p + k]) ++k;
            if (k == len) {
              best_len = len;
              best_id = tok.added_id[a];
            }
          }
        }
        if (best_len > 0) {
          if (kMode == kModePretok) tok.pre_gid[b * (int64_t)S + p] = best_id;  // (read by the word pass)
          else L.Y[p] = best_id;
        }
      }
      const int nc = n_cand - c0 < 64 ? n_cand - c0 : 64;
      uint64_t sel = 0;
      for (int i = 0; i < nc; ++i) {
        const int pi = __builtin_amdgcn_readlane(p, i), li = __builtin_amdgcn_readlane(best_len, i);
        if (li > 0 && pi >= cur) {
          sel |= 1ull << i;
          cur = pi + li;
        }
      }
      if ((sel >> lane) & 1) L.M[p] = (uint16_t)best_len;
      while (sel) {
        const int i = __builtin_ctzll(sel);
        sel &= sel - 1;
        const int pi = __builtin_amdgcn_readlane(p, i), li = __builtin_amdgcn_readlane(best_len, i);
        for (int q = lane; q < li; q += 64) L.C[pi + q] |= (uint8_t)(q == 0 ? (B_ADD | B_IN) : B_IN);
      }
    }
    wave_sync();
  }
  BST_F(2);
  // ---- 3. match length at every character start (outside added tokens)
  for (int w0 = 0; w0 < n; w0 += 64) {
    const int p = w0 + lane;
    const bool v0 = p < n, v1 = p + 64 < n;
    const uint32_t c0 = v0 ? L.C[p] : 0u, c1 = v1 ? L.C[p + 64] : 0u;
    // segment ends: the start of a selected added token, and every position from n on
    const uint64_t E0 = __ballot(!v0 || (c0 & B_ADD)), E1 = __ballot(!v1 || (c1 & B_ADD));
    const uint64_t Lm0 = __ballot(c0 & B_L), Lm1 = __ballot(c1 & B_L);
    const uint64_t N0 = __ballot(c0 & B_N), N1 = __ballot(c1 & B_N);
    const uint64_t W0 = __ballot(c0 & B_W), W1 = __ballot(c1 & B_W);
    const uint64_t NL0 = __ballot(c0 & B_NL), NL1 = __ballot(c1 & B_NL);
    const uint64_t S0 = __ballot(c0 & B_START), S1 = __ballot(c1 & B_START);
    if (!v0 || !(c0 & B_START) || (c0 & B_IN)) continue;
    const int l0 = utf8_len(L.T[p]);
    int len = 0;
    if (tok.pretok == RMI_PRETOK_CHARS) {
      len = l0;
    } else {
      const int i = lane;
      const uint64_t vE = view(E0, E1, i);
      const int es = vE ? __builtin_ctzll(vE) : 64;  // segment end (64: beyond the view)
      const uint64_t keep = low_bits(es);
      const uint64_t vL = view(Lm0, Lm1, i) & keep, vN = view(N0, N1, i) & keep, vW = view(W0, W1, i) & keep;
      const uint64_t vNL = view(NL0, NL1, i) & keep, vS = view(S0, S1, i);
      const uint64_t vO = keep & ~(vL | vN | vW);
      bool slow = false;
      if (L.T[p] == '\'') len = contraction(L.T, p, p + es);
      if (!len) {
        if (c0 & B_L) {
          len = run_end(vL, 0);
          slow = len == 64;
        } else if (!(c0 & (B_NL | B_N)) && ((vL >> l0) & 1)) {
          len = run_end(vL, l0);
          slow = len == 64;
        } else if (c0 & B_N) {
          len = l0;
        } else if ((c0 & B_SP) && ((vO >> 1) & 1)) {
          const int k = run_end(vO, 1);
          len = run_end(vNL, k);
          slow = k == 64 || len == 64;
        } else if (!(c0 & B_W)) {
          const int k = run_end(vO, 0);
          len = run_end(vNL, k);
          slow = k == 64 || len == 64;
        } else {
          const int e = run_end(vW, 0);
          if (e == 64) {
            slow = true;
          } else {
            const uint64_t nl = vNL & low_bits(e);
            if (nl) {
              len = 64 - __builtin_clzll(nl);
            } else if (e == es) {
              len = e;
            } else {
              const int ls = 63 - __builtin_clzll(vS & low_bits(e));
              len = ls > 0 ? ls : e;
            }
          }
        }
      }
#ifdef RMI_BPE_SERIAL_MATCH
      slow = true;  // diagnostic build: every match by the serial scan
#endif
      if (slow) {
        int s1 = p;
        while (s1 < n && !(L.C[s1] & B_ADD)) ++s1;
        len = match_serial(L.T, L.C, p, s1);
      }
    }
    L.M[p] = (uint16_t)(len > 0 ? len : l0);
  }
  wave_sync();
  BST_F(3);
  // ---- 4. the leftmost match chain: pre-token starts (added tokens are pre-tokens too)
  int np = 0;
  for (int p = 0; p < n;) {
    const int base = p;
    const uint32_t mw = base + lane < n ? L.M[base + lane] : 1u;
    uint64_t starts = 0;
    while (p < n && p - base < 64) {
      starts |= 1ull << (p - base);
      p += (int)__builtin_amdgcn_readlane((int)mw, p - base);
    }
    const int j = np + __builtin_popcountll(starts & ((1ull << lane) - 1));
    if ((starts >> lane) & 1) L.P[j] = (uint16_t)(base + lane);
    np += __builtin_popcountll(starts);
  }
  wave_sync();
  BST_N(2);
  BST_F(4);
  if constexpr (kMode == kModePretok) {  // the row's pre-token list, then the word pass
    uint32_t* pe = tok.pre + b * (int64_t)S;
    for (int j = lane; j < np; j += 64) {
      const int a = L.P[j], e = j + 1 < np ? L.P[j + 1] : n;
      pe[j] = (uint32_t)a | ((uint32_t)(e - a) << 12) | ((L.C[a] & B_ADD) ? (1u << 24) : 0u);
    }
    if (lane == 0) {
      tok.pre_np[b] = np;
      err[b] = 0;
    }
    return;
  }
  // ---- 5. BPE: symbols, pair ranks, merges (one lane per pre-token)
  // piece bounds: P[j] .. P[j+1] (or n); the symbol chain in M: next symbol start or kEnd.
  // K[j] after this loop: an added token's or a word-cache hit's id count (a hit flagged
  // kKHit: its ids sit at Y[a ..)), or kKMerge for a word the merge loop below takes.  A row
  // without such a word (a warm cache) skips the symbol set-up, the pair lookups and the merges.
  // Two pre-tokens per lane per trip, every global load of both (the word-cache entry at the
  // first probe, a single byte's id) issued before any is waited on.
  struct Probe {
    int j, a, len, kind;  // kind: 0 none, 1 added token, 2 one byte, 3 word cache, 4 merge
    uint32_t k[4];
    uint32_t h;
    uint4 w[4];
    int32_t bid;
  };
  const auto issue = [&](int j, Probe& q) {
    q.j = j;
    q.kind = 0;
    q.a = 0;
    q.len = 0;
    if (j < np) {
      q.a = L.P[j];
      q.len = (j + 1 < np ? L.P[j + 1] : n) - q.a;
      q.kind = (L.C[q.a] & B_ADD) ? 1 : q.len == 1 ? 2 : (tok.word_cache && q.len <= kWcWordMax) ? 3 : 4;
    }
    q.bid = tok.byte_id[q.kind == 2 ? L.T[q.a] : 0];
    if (tok.word_cache) {
      if (q.kind == 3) wc_key(L.T, q.a, q.len, q.k);
      q.h = q.kind == 3 ? wc_slot(q.k, q.len, tok.word_cache_mask) : 0u;
      wc_load(tok, q.h, q.w);
    }
  };
  bool miss = false;
  const auto finish = [&](Probe& q) {
    const int j = q.j, a = q.a;
    if (q.kind == 0) return;
    if (q.kind == 1) {  // an added token: one symbol (id set in phase 2), or an expansion's ids
      L.M[a] = kEnd;
      const int32_t y = L.Y[a];
      L.K[j] = (uint16_t)(y < 0 ? EO[-y] - EO[-y - 1] : 1);
      return;
    }
    if (q.kind == 2) {  // one byte: its byte id (no pair)
      L.Y[a] = q.bid;
      L.K[j] = (uint16_t)(kKHit | 1);
      return;
    }
    if (q.kind == 3) {
      bool empty;
      int cnt = wc_take(q.w, q.k, q.len, L.Y + a, empty);
      if (!cnt && !empty) cnt = wc_find_from(tok, q.k, q.len, L.Y + a, (q.h + 1) & tok.word_cache_mask, 1);
      if (cnt > 0) {
        L.K[j] = (uint16_t)(kKHit | cnt);
        return;
      }
    }
    miss = true;
    L.K[j] = kKMerge;
    for (int p = a; p < a + q.len; ++p) {
      L.Y[p] = tok.byte_id[L.T[p]];  // 1 KB, cache resident (a word-cache miss only)
      L.M[p] = p + 1 < a + q.len ? (uint16_t)(p + 1) : kEnd;
    }
  };
#ifdef RMI_BPE_ONE_PROBE  // (A/B variant: one pre-token per lane per trip)
  for (int j0 = 0; j0 < np; j0 += 64) {
    Probe q0;
    issue(j0 + lane, q0);
    finish(q0);
  }
#else
  for (int j0 = 0; j0 < np; j0 += 128) {
    Probe q0, q1;
    issue(j0 + lane, q0);
    issue(j0 + 64 + lane, q1);
    finish(q0);
    finish(q1);
  }
#endif
  const bool row_merges = __any(miss);
  wave_sync();
  BST_N(3);
  // The merges, one lane per word-cache miss.  (Interleaving several words per lane, with their
  // pair probes in flight together and a bit mask of live symbols instead of the chain walk,
  // measured slower in round 3: 78-95 k cycles per wave against 75 k.)  A row without a miss
  // skips this block.
  if (row_merges) {
  for (int j = lane; j < np; j += 64) {
    const int a = L.P[j];
    if (L.K[j] != kKMerge) continue;  // an added token or a word-cache hit
    int cnt = 1;
    {
      cnt = merge_word(tok, L.Y, L.M, a);
      const int len = (j + 1 < np ? L.P[j + 1] : n) - a;
      if (tok.word_cache && len >= 2 && len <= kWcWordMax && cnt <= kWcIdsMax) {
        uint32_t k[4];
        wc_key(L.T, a, len, k);
        wc_insert(tok, k, len, L.Y, L.M, a, cnt);
      }
    }
    L.K[j] = (uint16_t)cnt;
  }
  wave_sync();
  }  // row_merges
  BST_N(4);
  // ---- 6. row offsets (wave scan over pre-tokens), mark, capacity, the ids
  const int mk = mark_byte ? mark_byte[b] : -1;
  int total = 0, before_mark = 0;
  for (int j0 = 0; j0 < np; j0 += 64) {
    const int j = j0 + lane;
    const int kj = j < np ? L.K[j] : 0;
    const int c = kj & ~kKHit;
    const int incl = wave_inclusive_scan(c);
    const bool pre = j < np && (int)L.P[j] < mk;
    const int pre_sum = wave_inclusive_scan(pre ? c : 0);
    before_mark += __builtin_amdgcn_readlane(pre_sum, 63);
    // the exclusive offset (< 4096: n <= 3072), the hit flag kept
    if (j < np) L.K[j] = (uint16_t)((total + incl - c) | (kj & kKHit));
    total += __builtin_amdgcn_readlane(incl, 63);
  }
  if (base_len + total > out_stride) return fail(RMI_ERR_UNSUP);
  wave_sync();
  int64_t* orow = out + b * out_stride + base_len;
  for (int j0 = 0; j0 < np; j0 += 64) {
    const int j = j0 + lane;
    const int kj = j < np ? L.K[j] : 0;
    int o = kj & ~kKHit;
    const int a = j < np ? L.P[j] : 0;
    const bool is_exp = j < np && !(kj & kKHit) && (L.C[a] & B_ADD) && L.Y[a] < 0;
    // expansions: the wave copies each one's ids together (a lane's own copy loop waited on a
    // table read per id, tens of ids per expansion)
    for (uint64_t em = __ballot(is_exp); em; em &= em - 1) {
      const int src_l = __builtin_ctzll(em);
      const int e = -L.Y[__builtin_amdgcn_readlane(a, src_l)] - 1, eo = __builtin_amdgcn_readlane(o, src_l);
      const int e0 = EO[e], ec = EO[e + 1] - e0;
      for (int i = lane; i < ec; i += 64) orow[eo + i] = (int64_t)EI[e0 + i];
    }
    if (j >= np || is_exp) continue;
    if (kj & kKHit) {  // a word-cache hit (<= kWcIdsMax ids at Y[a ..)): every read, then every store
      const int c = (j + 1 < np ? (L.K[j + 1] & ~kKHit) : total) - o;
      int32_t v[kWcIdsMax];
#pragma unroll
      for (int i = 0; i < kWcIdsMax; ++i) v[i] = i < c ? L.Y[a + i] : 0;
#pragma unroll
      for (int i = 0; i < kWcIdsMax; ++i)
        if (i < c) orow[o + i] = (int64_t)v[i];
      continue;
    }
    for (int q = a; q != kEnd; q = L.M[q]) orow[o++] = (int64_t)L.Y[q];
  }
  if (lane == 0) {
    err[b] = 0;
    if (out_len) out_len[b] = base_len + total;
    if (n_tok) n_tok[b] = total;
    if (mark_tok) mark_tok[b] = base_len + before_mark;
  }
}

// ---- the word pass of the two-pass form: one wave per row over the pre-token list the
// pre-tokenizer pass wrote, 64 pre-tokens per trip, one per lane: an added token's id (or an
// expansion's ids), a byte's id, or the word cache's ids, all loads of a trip issued together;
// the misses merged lane by lane in a per-wave scratch (kScr symbols for the trip's misses
// together), the trip's counts scanned into the row's offsets and its ids stored.  LDS: the row's
// text (keys, merges), the scratch and the expansion tables -- a few KB, so the pass runs at full
// occupancy.  A row whose trip needs more scratch is flagged for the one-kernel pass.
constexpr int kScr = 256;
__host__ __device__ constexpr size_t words_lds(int stride, int ne, int nei) {
  return (size_t)stride + 16 + 4 * (size_t)kScr + 2 * (size_t)kScr +
         (staged_exp(ne, nei) ? 4 * (size_t)(ne + 1) + 4 * (size_t)nei : 0);
}

__global__ __launch_bounds__(64) void bpe_words_kernel(rmi_bpe_t tok, const uint8_t* __restrict__ text, int64_t pitch,
                                                       int stride, const int32_t* __restrict__ text_len,
                                                       int64_t* __restrict__ out, int64_t out_stride,
                                                       int32_t* __restrict__ out_len, int32_t* __restrict__ n_tok,
                                                       const int32_t* __restrict__ mark_byte,
                                                       int32_t* __restrict__ mark_tok, uint8_t* __restrict__ err) {
  extern __shared__ __align__(16) uint8_t smem[];
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int S = stride;
  uint8_t* T = smem;                                                  // S + 16 (4-aligned: S % 4 == 0)
  int32_t* Ys = reinterpret_cast<int32_t*>(smem + S + 16);            // [kScr] symbol ids of the trip's misses
  int32_t* EOl = Ys + kScr;                                            // [n_exp + 1], [n_exp_ids] (staged)
  int32_t* EIl = EOl + (tok.n_exp + 1);
  const bool exp_lds = staged_exp(tok.n_exp, tok.n_exp_ids);
  uint16_t* Ms = reinterpret_cast<uint16_t*>(exp_lds ? EIl + tok.n_exp_ids : EOl);  // [kScr] their chain
  const int32_t* EO = exp_lds ? EOl : tok.exp_off;
  const int32_t* EI = exp_lds ? EIl : tok.exp_ids;
  // one batch of loads: the row's state, its first 128 pre-token entries and first 1 KB of text
  // (none depends on another: entries past the row's count and bytes past its length are masked)
  const uint32_t* pe = tok.pre + b * (int64_t)S;
  const int32_t* gid = tok.pre_gid + b * (int64_t)S;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(text + b * pitch);
  const int readable = (S < pitch ? S : (int)pitch) / 4;
  constexpr int kPre = 4;
  uint32_t tpre[kPre];
#pragma unroll
  for (int i = 0; i < kPre; ++i) tpre[i] = lane + 64 * i < readable ? src[lane + 64 * i] : 0u;
  uint32_t ent0 = lane < S ? pe[lane] : 0u, ent1 = lane + 64 < S ? pe[lane + 64] : 0u;
  const uint8_t row_err = err[b];
  const int n = text_len[b], np = tok.pre_np[b];
  const int base_len = out_len ? out_len[b] : 0;
  const int mk = mark_byte ? mark_byte[b] : -1;
  if (row_err != 0) return;  // the pre-tokenizer pass failed the row (its outputs are written)
  const auto tail_mask = [n](int w, uint32_t v) {
    if (4 * w >= n) return 0u;
    return 4 * w + 4 > n ? v & (0xFFFFFFFFu >> (8 * (4 * w + 4 - n))) : v;
  };
#pragma unroll
  for (int i = 0; i < kPre; ++i) {
    const int w = lane + 64 * i;
    if (w < (n + 3) / 4 + 4) reinterpret_cast<uint32_t*>(T)[w] = tail_mask(w, tpre[i]);
  }
  for (int w = lane + 64 * kPre; w < (n + 3) / 4 + 4; w += 64)
    reinterpret_cast<uint32_t*>(T)[w] = tail_mask(w, 4 * w < n ? src[w] : 0u);
  if (exp_lds) {
    stage_i32(EOl, tok.exp_off, tok.n_exp + 1, lane);
    stage_i32(EIl, tok.exp_ids, tok.n_exp_ids, lane);
  }
  wave_sync();
  int64_t* orow = out + b * out_stride + base_len;
  int total = 0, before_mark = 0;
  bool retry = false, over = false;
  struct Q {
    int j, a, len, kind;  // kind: 0 none, 1 added token, 2 one byte, 3 word cache, 4 merge
    uint32_t k[4];
    uint32_t h;
    uint4 w[4];
    int32_t bid, aid;
  };
  // every load of a pre-token (the byte id, the added id, the word-cache entry), issued for two
  // pre-tokens per lane before either is waited on
  const auto issue = [&](int j, uint32_t ent, Q& q) {
    const bool act = j < np;
    q.j = j;
    q.a = (int)(ent & 0xFFFu);
    q.len = (int)((ent >> 12) & 0xFFFu);
    q.kind = !act ? 0 : ((ent >> 24) & 1u) ? 1 : q.len == 1 ? 2 : (tok.word_cache && q.len <= kWcWordMax) ? 3 : 4;
    q.bid = tok.byte_id[q.kind == 2 ? T[q.a] : 0];
    q.aid = gid[q.kind == 1 ? q.a : 0];
    q.k[0] = q.k[1] = q.k[2] = q.k[3] = 0u;
    q.h = 0;
    if (tok.word_cache) {
      if (q.kind == 3) {
        wc_key(T, q.a, q.len, q.k);
        q.h = wc_slot(q.k, q.len, tok.word_cache_mask);
      }
      wc_load(tok, q.h, q.w);
    }
  };
  // one trip of 64 pre-tokens (every lane together): ids, the misses merged in the scratch, the
  // counts scanned into the row's offsets, the ids stored; false: the row goes to the retry pass
  const auto finish = [&](Q& q) -> bool {
    const bool act = q.kind != 0;
    const int a = q.a, len = q.len;
    int cnt = 0;
    int32_t ids[kWcIdsMax];
    bool miss = q.kind == 4;
    if (q.kind == 1) {
      cnt = q.aid < 0 ? EO[-q.aid] - EO[-q.aid - 1] : 1;
    } else if (q.kind == 2) {
      cnt = 1;
    } else if (q.kind == 3) {
      bool empty;
      cnt = wc_take(q.w, q.k, len, ids, empty);
      if (!cnt && !empty) cnt = wc_find_from(tok, q.k, len, ids, (q.h + 1) & tok.word_cache_mask, 1);
      miss = cnt == 0;
    }
    const int need = miss ? len : 0;
    const int need_incl = wave_inclusive_scan(need);
    if (__builtin_amdgcn_readlane(need_incl, 63) > kScr) return false;
    const int off = need_incl - need;
    if (miss) {
      for (int i = 0; i < len; ++i) {
        Ys[off + i] = tok.byte_id[T[a + i]];  // 1 KB, cache resident (a word-cache miss only)
        Ms[off + i] = i + 1 < len ? (uint16_t)(off + i + 1) : kEnd;
      }
      cnt = merge_word(tok, Ys, Ms, off);
      if (q.kind == 3 && cnt <= kWcIdsMax) wc_insert(tok, q.k, len, Ys, Ms, off, cnt);
    }
    const int incl = wave_inclusive_scan(cnt);
    const int trip = __builtin_amdgcn_readlane(incl, 63);
    const int pre_sum = wave_inclusive_scan(act && a < mk ? cnt : 0);
    before_mark += __builtin_amdgcn_readlane(pre_sum, 63);
    if (base_len + total + trip > out_stride) {
      over = true;
      return true;
    }
    int o = total + incl - cnt;
    // expansions: the wave copies each one's ids together (a lane's own copy loop waited on an
    // LDS read per id, tens of ids per expansion)
    const bool is_exp = q.kind == 1 && q.aid < 0;
    for (uint64_t em = __ballot(is_exp); em; em &= em - 1) {
      const int src_l = __builtin_ctzll(em);
      const int e = -__builtin_amdgcn_readlane(q.aid, src_l) - 1, eo = __builtin_amdgcn_readlane(o, src_l);
      const int e0 = EO[e], ec = EO[e + 1] - e0;
      for (int i = lane; i < ec; i += 64) orow[eo + i] = (int64_t)EI[e0 + i];
    }
    if (q.kind == 1) {
      if (q.aid >= 0) orow[o] = (int64_t)q.aid;
    } else if (q.kind == 2) {
      orow[o] = (int64_t)q.bid;
    } else if (miss) {
      for (int i = off; i != kEnd; i = Ms[i]) orow[o++] = (int64_t)Ys[i];
    } else if (q.kind == 3) {
#pragma unroll
      for (int i = 0; i < kWcIdsMax; ++i)
        if (i < cnt) orow[o + i] = (int64_t)ids[i];
    }
    total += trip;
    wave_sync();  // (the scratch is the next trip's)
    return true;
  };
  for (int j0 = 0; j0 < np && !retry && !over; j0 += 128) {
    if (j0) {  // entries past the first 128
      ent0 = j0 + lane < np ? pe[j0 + lane] : 0u;
      ent1 = j0 + 64 + lane < np ? pe[j0 + 64 + lane] : 0u;
    }
    if (j0 + lane >= np) ent0 = 0u;
    if (j0 + 64 + lane >= np) ent1 = 0u;
    Q q0, q1;
    issue(j0 + lane, ent0, q0);
    issue(j0 + 64 + lane, ent1, q1);
    retry = !finish(q0);
    if (!retry && !over && j0 + 64 < np) retry = !finish(q1);
  }
  if (retry) {  // the one-kernel pass takes the row (its outputs from out_len[b] on, as here)
    if (lane == 0) tok.pre_retry[b] = 1;
    return;
  }
  if (lane == 0) {
    if (over) {
      err[b] = RMI_ERR_UNSUP;
      if (n_tok) n_tok[b] = 0;
      if (mark_tok) mark_tok[b] = base_len;
    } else {
      if (out_len) out_len[b] = base_len + total;
      if (n_tok) n_tok[b] = total;
      if (mark_tok) mark_tok[b] = base_len + before_mark;
    }
  }
}

}  // namespace
}  // namespace rmi

#ifdef RMI_STAMPS
RMI_API int rmi_bpe_set_stamps(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(rmi::g_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -2;
}
#endif

RMI_API int rmi_bpe_encode(const rmi_bpe_t* tok, const uint8_t* text, int64_t pitch, int32_t stride,
                           const int32_t* text_len, int64_t B, int64_t* out, int64_t out_stride, int32_t* out_len,
                           int32_t* n_tok, const int32_t* mark_byte, int32_t* mark_tok, uint8_t* err,
                           rmi_stream_t stream) {
  using namespace rmi;
  if (!tok || B < 0 || stride <= 0 || stride % 4 || pitch % 4 || out_stride <= 0) return RMI_EINVAL;
  if (stride > kMaxStride || B > 0x7FFFFFFF || tok->n_added < 0 || tok->n_added > 4096) return RMI_EUNSUP;
  if (tok->pretok != RMI_PRETOK_QWEN2 && tok->pretok != RMI_PRETOK_CHARS) return RMI_EUNSUP;
  if (B == 0) return RMI_OK;
  if (!text || !text_len || !out || !err || !tok->cp_block || !tok->cp_class || !tok->byte_id || !tok->merges ||
      (tok->n_added > 0 && (!tok->added_bytes || !tok->added_off || !tok->added_id)) || tok->n_exp < 0 ||
      tok->n_exp > 64 || (tok->n_exp > 0 && (!tok->exp_off || !tok->exp_ids)))
    return RMI_EINVAL;
  if (tok->n_exp_ids < 0) return RMI_EINVAL;
  const int na = staged_added(tok->n_added), nw = staged_words(tok->n_added, tok->n_exp);
  const size_t lds = bpe_lds(stride, na, nw, tok->n_exp, tok->n_exp_ids);
  const bool two_pass = tok->pre && tok->pre_gid && tok->pre_np && tok->pre_retry && tok->pre_cap >= B * (int64_t)stride &&
                        tok->pretok == RMI_PRETOK_QWEN2;
  if (!two_pass) {
    hipLaunchKernelGGL(bpe_encode_kernel<kModeFull>, dim3((unsigned)B), dim3(64), lds, as_stream(stream), *tok, text,
                       pitch, (int)stride, text_len, out, out_stride, out_len, n_tok, mark_byte, mark_tok, err);
    return launch_status();
  }
  // the pre-tokenizer pass, the word pass, the one-kernel pass over the rows the word pass flagged
  hipLaunchKernelGGL(bpe_encode_kernel<kModePretok>, dim3((unsigned)B), dim3(64),
                     bpe_lds(stride, na, nw, tok->n_exp, tok->n_exp_ids, kModePretok), as_stream(stream), *tok, text,
                     pitch, (int)stride, text_len, out, out_stride, out_len, n_tok, mark_byte, mark_tok, err);
  hipLaunchKernelGGL(bpe_words_kernel, dim3((unsigned)B), dim3(64), words_lds(stride, tok->n_exp, tok->n_exp_ids),
                     as_stream(stream), *tok, text, pitch, (int)stride, text_len, out, out_stride, out_len, n_tok,
                     mark_byte, mark_tok, err);
  hipLaunchKernelGGL(bpe_encode_kernel<kModeRetry>, dim3((unsigned)B), dim3(64), lds, as_stream(stream), *tok, text,
                     pitch, (int)stride, text_len, out, out_stride, out_len, n_tok, mark_byte, mark_tok, err);
  return launch_status();
}
