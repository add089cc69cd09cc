// parse.hip — the LLM response -> action-id boundary on the device (gfx950), SURVEY §8(f) rank 2.
//
//  rmi_detokenize      tokenizer.batch_decode(responses, skip_special_tokens=True)
//                      (ctx_manager.py:334-337) for byte-level BPE vocabularies
//  rmi_parse_actions   ContextManager._parse_response (ctx_manager.py:148-173) on the
//                      "<think>"/"<answer>"-prefixed response (:338-339), then
//                      EnvStateManager._extract_map_valid_actions (es_manager.py:230-240)
//
// One wave per response, the row staged in LDS.  The parse is driven by EVENTS instead of
// byte scans: one SWAR pass (a dword per lane) compacts the positions of every '<' into an
// LDS list; all six tags begin with '<', so the lanes then classify 64 events per step with
// one 16-byte compare each, and the regex (its backtracking over </think> candidates
// included) runs as ballots over the classified list.  The separator is handled the same
// way (positions of its first byte -> full compare -> greedy left-to-right selection), and
// the pieces between separators are stripped and name-matched one piece per lane.  Only the
// rare answer that contains a special token takes the replace cascade (wave-parallel
// stream compaction, one pass per token present).
//
// Exactness argument for working on UTF-8 bytes instead of Python str: every tag, the
// separator and the action names are ASCII; UTF-8 is self-synchronising, so an ASCII byte is
// always a whole character and a multi-byte whitespace sequence (U+0085, U+00A0, U+1680,
// U+2000-U+200A, U+2028/9, U+202F, U+205F, U+3000) found at a character boundary (forward)
// or ending at one (backward: its lead byte can never be a continuation byte) is that
// character.  str.lower() maps exactly one non-ASCII character to an ASCII string: U+212A
// KELVIN SIGN -> 'k' (U+0130 -> "i" + U+0307 is never all-ASCII); it is handled below.
#include "common.hpp"
#include "parse_core.hpp"

namespace rmi {
namespace {

__global__ __launch_bounds__(64 * kRowWaves) __attribute__((amdgpu_waves_per_eu(8))) void parse_kernel(ParseArgs a) {
  extern __shared__ uint64_t lds_q[];
  const int wv = threadIdx.x >> 6;
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds_q) + wv * parse_lds(a.stride);
  const int cap = list_cap(a.stride);
  uint8_t* T = lds + 4;                                                   // the prefixed row
  uint8_t* Wb = lds + row_bytes(a.stride) + 4;                            // replace-cascade row
  uint16_t* EL = reinterpret_cast<uint16_t*>(lds + 2 * row_bytes(a.stride));  // '<' positions
  uint16_t* ES = EL + cap;                                                // separator candidates
  uint8_t* EI = reinterpret_cast<uint8_t*>(ES + cap);                     // event ids
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (b >= a.B) return;  // the whole wave: no cross-wave barrier follows
  PSTAMP_DECL;
  PSTAMP(0);
  // ---- 0. stage.  The first 256 bytes are loaded together with the length (one round trip
  //         for typical responses); the rest, if any, after it.
  const uint32_t* s4 = reinterpret_cast<const uint32_t*>(a.text + b * a.stride);
  uint32_t* d4 = reinterpret_cast<uint32_t*>(T + kPre);
  const int rw = a.stride >> 2;
  const uint32_t first = lane < rw ? s4[lane] : 0u;
  int len = a.text_len[b];
  uint8_t err = 0;
  if (len < 0 || len > a.stride) {
    err |= RMI_ERR_STATE;
    len = 0;
  }
  const Names nm = load_names(a.cfg, (a.sel && a.sel[b]) ? 1 : 0);
  const int nw = (len + 3) >> 2;
  if (lane < nw) d4[lane] = first;
  for (int i = 64 + lane; i < nw; i += 64) d4[i] = s4[i];
  parse_row(a, T, Wb, EL, ES, EI, b, len, err, nm, lane PSTAMP_ARG);
  PSTAMP_FLUSH();
}

__global__ __launch_bounds__(64 * kRowWaves) __attribute__((amdgpu_waves_per_eu(8))) void detok_kernel(DetokArgs d) {
  extern __shared__ uint32_t lds_words[];
  const int wv = threadIdx.x >> 6;
  uint8_t* buf = reinterpret_cast<uint8_t*>(lds_words) + wv * detok_lds(d.stride) + 4;  // raw row [stride + 8]
  uint8_t* fix = buf + d.stride + 8;                                                      // lossy row [stride + 4]
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (b >= d.B) return;  // the whole wave
  DSTAMP_DECL;
  DSTAMP(0);
  detok_row(d, buf, fix, b, lane DSTAMP_ARG);
  DSTAMP_FLUSH();
}

// The fused per-turn boundary: decode row b straight into the parse's LDS row (T + kPre), write
// the decoded text out (the prompts and the history read it), then parse it in place: the
// parse's stage (a global read of the text just written) and one launch disappear, and the
// decode's memory-bound waves overlap other waves' parse work.
__global__ __launch_bounds__(64 * kRowWaves) __attribute__((amdgpu_waves_per_eu(8))) void detok_parse_kernel(
    DetokArgs d, ParseArgs a) {
  extern __shared__ uint64_t lds_q[];
  const int wv = threadIdx.x >> 6;
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds_q) + wv * parse_lds(a.stride);
  const int cap = list_cap(a.stride);
  uint8_t* T = lds + 4;
  uint8_t* Wb = lds + row_bytes(a.stride) + 4;
  uint16_t* EL = reinterpret_cast<uint16_t*>(lds + 2 * row_bytes(a.stride));
  uint16_t* ES = EL + cap;
  uint8_t* EI = reinterpret_cast<uint8_t*>(ES + cap);
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (b >= a.B) return;  // the whole wave: no cross-wave barrier follows
  PSTAMP_DECL;
  PSTAMP(0);
#ifdef RMI_PARSE_STAMPS
  unsigned long long dst_[6];
#endif
  const Names nm = load_names(a.cfg, (a.sel && a.sel[b]) ? 1 : 0);
  const int n = detok_row(d, T + kPre, Wb + kPre, b, lane DSTAMP_ARG);
  parse_row(a, T, Wb, EL, ES, EI, b, n, 0, nm, lane PSTAMP_ARG);
  PSTAMP_FLUSH();
}

// ============================================================ four responses per wave
// The one-response-per-wave parse is VALU-issue-bound at full occupancy (≈750 VALU + 460 SALU
// per response; tools/parse_pmc.sh), and most of its steps keep a few lanes busy: a handful of
// '<' events, four or five action pieces, ballots whose answer one lane reads.  Here a wave
// parses FOUR responses, one per 16-lane DPP row ("segment"): the byte passes cover 64 bytes
// per step instead of 256, and every other step serves four responses per instruction.  The
// control flow of each step is per segment; cross-lane operations (ballots, row scans,
// bpermute reads) run with every lane active, each segment reading its own 16-bit field.  The
// rare special-token replace cascade runs the wave-wide code on one row at a time.  Results
// are those of parse_row, bit for bit (the same steps on the same bytes).
constexpr int kSegRows = 4;  // responses per wave

__device__ __forceinline__ int seg_scan(int x) {  // inclusive prefix sum inside each 16-lane row
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);  // row_shr:8
  return x;
}
// the value of lane 15 of this lane's row (ds_swizzle bitmask mode: and 0x10, or 0x0F)
__device__ __forceinline__ int seg_last(int x) { return __builtin_amdgcn_ds_swizzle(x, 0x1F0); }
__device__ __forceinline__ uint32_t seg_field(uint64_t m, int r) { return (uint32_t)(m >> (16 * r)) & 0xFFFFu; }
// lane j of this lane's row (every lane must execute it)
__device__ __forceinline__ int seg_read(int v, int r, int j) { return __shfl(v, (r << 4) | j, 64); }

// collect() per segment: positions x in [from, to) with B[x] == ch, ascending, into list
// (16 lanes x 4 bytes per step); -> the row's count (on each of its lanes)
__device__ int seg_collect(const uint8_t* B, int from, int to, uint32_t ch, uint16_t* list, int l) {
  int cnt = 0;
  const uint32_t rep = ch * 0x01010101u;
  for (int c = from & ~3;; c += 64) {
    if (!__any(c < to)) break;
    const int i0 = c + 4 * l;
    uint32_t m4 = 0;
    if (c < to && i0 < to) {
      const uint32_t x = *reinterpret_cast<const uint32_t*>(B + i0) ^ rep;  // zero byte where B == ch
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = i0 + j;
        const bool hit = ((x >> (8 * j)) & 0xFFu) == 0;
        if (hit && p >= from && p < to) m4 |= 1u << j;
      }
    }
    const int k = __builtin_popcount(m4);
    const int incl = seg_scan(k);
    int o = cnt + incl - k;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (m4 & (1u << j)) list[o++] = (uint16_t)(i0 + j);
    cnt += seg_last(incl);
  }
  return cnt;
}

// next_event() per segment: the first classified event with id == want (< 0: any tag) at a
// position in [from, lim) of the rows that ask (act), else -1
__device__ int seg_next_event(const uint16_t* EL, int n, int want, int from, int lim, bool act, int r, int l) {
  int res = -1;
  bool open = act;
  for (int c = 0;; c += 16) {
    if (c >= n) open = false;
    if (!__any(open)) break;
    const int i = c + l;
    bool hit = false;
    int p = 0;
    if (open && i < n) {  // packed: position | tag id << 12
      const int ev = EL[i];
      p = ev & 0xFFF;
      const int id = ev >> 12;
      hit = p >= from && p < lim && (want < 0 ? id != E_NONE : id == want);
    }
    const uint32_t f = seg_field(__ballot(hit), r);
    const int q = seg_read(p, r, f ? __builtin_ctz(f) : 0);
    if (open && f) {
      res = q;
      open = false;
    }
  }
  return res;
}

// piece_id with the lookup column chosen per lane (Bandit's per-env ids): the names are
// wave-uniform, only the id differs between the columns
__device__ int piece_id_col(const uint8_t* B, int s, int e, const Names& nm0, const Names& nm1, bool col) {
  return col ? piece_id(B, s, e, nm1) : piece_id(B, s, e, nm0);
}

struct SegLds {  // one row's LDS: the prefixed text and its list (events, then separators)
  uint8_t* T;
  uint16_t* EL;
};
// per row: T row | EL u16[cap]; per wave: 4 rows, then the shared cascade row and the cascade's
// position list and coverage bytes (the cascade runs on one row at a time)
__host__ __device__ constexpr size_t seg_row_lds(int stride) {
  return ((size_t)row_bytes(stride) + 2 * (size_t)list_cap(stride) + 7) & ~(size_t)7;
}
__host__ __device__ constexpr size_t seg_wave_lds(int stride) {
  return (kSegRows * seg_row_lds(stride) + (size_t)row_bytes(stride) + 3 * (size_t)list_cap(stride) + 7) &
         ~(size_t)7;
}
constexpr int kSegMaxStride = 4000;  // event positions packed in 12 bits (kPre + stride < 4096)
__device__ __forceinline__ SegLds seg_row(uint8_t* wave_lds, int stride, int r) {
  uint8_t* base = wave_lds + r * seg_row_lds(stride);
  SegLds L;
  L.T = base + 4;
  L.EL = reinterpret_cast<uint16_t*>(base + row_bytes(stride));
  return L;
}
struct SegShared {  // the wave's cascade buffers
  uint8_t* Wb;
  uint16_t* lst;
  uint8_t* cov;
};
__device__ __forceinline__ SegShared seg_shared(uint8_t* wave_lds, int stride) {
  uint8_t* base = wave_lds + kSegRows * seg_row_lds(stride);
  SegShared S;
  S.Wb = base + 4;
  S.lst = reinterpret_cast<uint16_t*>(base + row_bytes(stride));
  S.cov = reinterpret_cast<uint8_t*>(S.lst + list_cap(stride));
  return S;
}

// The four responses of a wave, staged (row r's len bytes at seg_row(r).T + kPre): parse_row's
// steps per segment.  live: the row exists; err: bits already set for the row.
__device__ void parse_rows4(const ParseArgs& a, uint8_t* wave_lds, int64_t b, bool live, int len, uint8_t err,
                            const Names& nm0, const Names& nm1, bool col, int lane) {
  const rmi_parse_cfg_t& cfg = a.cfg;
  const int K = cfg.K;
  const int r = lane >> 4, l = lane & 15;
  const SegLds L = seg_row(wave_lds, a.stride, r);
  uint8_t* T = L.T;
  const SegShared S = seg_shared(wave_lds, a.stride);
  const Tag pre = cfg.enable_think ? kThinkOpen : kAnsOpen;
  const int plen = cfg.prepend ? pre.n : 0;
  const int base = kPre - plen, n_end = kPre + len;
  wave_sync();
  for (int i = l; i < kTail; i += 16) T[n_end + i] = 0;
  if (l < 4 + kPre) T[l - 4] = (l - 4 >= base) ? tag_byte(pre, l - 4 - base) : 0;
  wave_sync();

  // ---- 1. '<' events, classified
  const int n_ev = seg_collect(T, base, n_end, '<', L.EL, l);
  wave_sync();
  for (int i = l; i < n_ev; i += 16) {
    const int p = L.EL[i];
    L.EL[i] = (uint16_t)(p | (classify_tag(T, p) << 12));
  }
  wave_sync();

  // ---- 2. the regex (see parse_row)
  int ts = -1, te = -1, as = -1, ae = -1;
  if (cfg.enable_think) {
    const int i = seg_next_event(L.EL, n_ev, E_THINK_O, base, n_end, live, r, l);
    bool go = live && i >= 0, found = false;
    int j = i + kThinkOpen.n, k = -1;
    while (__any(go)) {
      const int jj = seg_next_event(L.EL, n_ev, E_THINK_C, j, n_end, go, r, l);
      if (go && jj < 0) go = false;
      if (go) {
        j = jj;
        k = j + kThinkClose.n;
        for (int w; (w = ws_fwd(T, k, n_end)) != 0;) k += w;  // \s* is greedy and '<' is no space
      }
      const bool lt = go && T[k] == '<';
      const int ao = seg_next_event(L.EL, n_ev, E_ANS_O, k, k + 1, lt, r, l);
      if (lt && ao == k) {
        found = true;
        go = false;
      } else if (go) {
        ++j;
      }
    }
    const int e = seg_next_event(L.EL, n_ev, E_ANS_C, k + kAnsOpen.n, n_end, found, r, l);
    if (found && e >= 0) {
      ts = i + kThinkOpen.n;
      te = j;
      as = k + kAnsOpen.n;
      ae = e;
    }
  } else {
    const int i = seg_next_event(L.EL, n_ev, E_ANS_O, base, n_end, live, r, l);
    const int e = seg_next_event(L.EL, n_ev, E_ANS_C, i + kAnsOpen.n, n_end, live && i >= 0, r, l);
    if (live && i >= 0 && e >= 0) {
      as = i + kAnsOpen.n;
      ae = e;
    }
  }

  // ---- 3. the replace cascade + strip of the action content
  int ca = 0, cz = 0;
  const bool has = as >= 0;
  if (has) {
    ca = as;
    cz = ae;
  }
  const bool need = seg_next_event(L.EL, n_ev, -1, ca, cz, has, r, l) >= 0;
  if (has && !need) strip(T, ca, cz);  // every replace is a no-op, and strip() six times is strip() once
  const uint64_t needm = __ballot(need && l == 0);
  for (int rr = 0; rr < kSegRows; ++rr) {
    if (!((needm >> (16 * rr)) & 1ull)) continue;  // wave-uniform: the whole wave on row rr
    const SegLds R = seg_row(wave_lds, a.stride, rr);
    int a0 = __builtin_amdgcn_readlane(ca, 16 * rr), z0 = __builtin_amdgcn_readlane(cz, 16 * rr);
    uint8_t* C = R.T;
    for (int q = 0; q < 6; ++q) {  // ctx_manager.py:94 order
      const Tag tok = q == 0 ? kThinkOpen : q == 1 ? kThinkClose : q == 2 ? kAnsOpen
                    : q == 3 ? kAnsClose : q == 4 ? kImStart : kImEnd;
      uint8_t* other = C == R.T ? S.Wb : R.T;
      C = replace_strip_wave(C, other, S.lst, S.cov, a0, z0, tok, lane);
      strip(C, a0, z0);
    }
    if (C != R.T) {  // back into the row (the shared cascade row serves the next one)
      wave_sync();
      for (int x = a0 + lane; x < z0; x += 64) R.T[x] = C[x];
      if (lane < kTail) R.T[z0 + lane] = 0;
    }
    wave_sync();
    if (r == rr) {
      ca = a0;
      cz = z0;
    }
  }

  // ---- 4. split(action_sep), strip, drop empties, cap at K; name -> id
  const Tag sep{cfg.sep_lo, cfg.sep_hi, cfg.sep_len};
  int count = 0;
  // candidates -> EL (the events are no longer needed), then the selected ones compacted in
  // place: a chunk's candidates are read before any of its selections is written, and the
  // selections so far never outnumber the candidates read
  const int nc = seg_collect(T, has ? ca : 0, has ? cz : 0, (uint32_t)(sep.lo & 0xFFu), L.EL, l);
  wave_sync();
  int ns = 0, last = ca;
  for (int c = 0;; c += 16) {
    const bool more = c < nc;
    if (!__any(more)) break;
    const int i = c + l;
    bool m = false;
    int p = 0;
    if (more && i < nc) {
      p = L.EL[i];
      uint64_t lo, hi;
      load16(T, p, lo, hi);
      m = p + sep.n <= cz && tag_eq(lo, hi, sep);
    }
    uint32_t bits = seg_field(__ballot(m), r);
    while (__any(bits != 0)) {  // left to right, non-overlapping (str.split); rows in step
      const int q = seg_read(p, r, bits ? __builtin_ctz(bits) : 0);
      if (bits) {
        bits &= bits - 1;
        if (q >= last) {
          if (l == 0) L.EL[ns] = (uint16_t)q;
          ++ns;
          last = q + sep.n;
        }
      }
    }
  }
  wave_sync();
  uint8_t perr = 0;
  for (int c = 0;; c += 16) {
    const bool more = has && c <= ns && count < K;
    if (!__any(more)) break;
    const int i = c + l;
    int s0 = 0, e0 = 0;
    if (more && i <= ns) {
      s0 = i ? L.EL[i - 1] + sep.n : ca;
      e0 = i < ns ? L.EL[i] : cz;
      strip(T, s0, e0);
    }
    const bool keep = more && e0 > s0;
    const uint32_t km = seg_field(__ballot(keep), r);
    const int slot = count + __builtin_popcount(km & ((1u << l) - 1u));
    if (keep && slot < K) {
      a.actions[b * K + slot] = (int8_t)(nm0.n > 0 ? piece_id_col(T, s0, e0, nm0, nm1, col) : 1);
      if (a.action_text) {
        const int Ln = e0 - s0, Lc = Ln < a.Lact ? Ln : a.Lact;
        uint8_t* dst = a.action_text + (b * K + slot) * (int64_t)a.Lact;
        for (int q = 0; q < Lc; ++q) dst[q] = T[s0 + q];
        a.action_len[b * K + slot] = Lc;
        if (Ln > a.Lact) perr |= RMI_ERR_UNSUP;
      }
    }
    if (more) count += __builtin_popcount(km);
  }
  if (count > K) count = K;
  if (live && l >= count && l < K) {
    a.actions[b * K + l] = 0;
    if (a.action_text) a.action_len[b * K + l] = 0;
  }
  const uint8_t err_all = err | (seg_field(__ballot(perr != 0), r) ? (uint8_t)RMI_ERR_UNSUP : (uint8_t)0);
  if (live && l == 0) {
    a.n_actions[b] = (uint8_t)count;
    if (a.spans) {
      a.spans[4 * b + 0] = ts < 0 ? -1 : ts - base;
      a.spans[4 * b + 1] = te < 0 ? -1 : te - base;
      a.spans[4 * b + 2] = as < 0 ? -1 : as - base;
      a.spans[4 * b + 3] = ae < 0 ? -1 : ae - base;
    }
    if (a.err) a.err[b] = err_all;
  }
}

__device__ __forceinline__ void load_names2(const rmi_parse_cfg_t& cfg, Names& nm0, Names& nm1) {
  nm0 = load_names(cfg, 0);
  nm1 = load_names(cfg, 1);
}

__global__ __launch_bounds__(64 * kRowWaves) __attribute__((amdgpu_waves_per_eu(8))) void parse4_kernel(ParseArgs a) {
  extern __shared__ uint64_t lds_q[];
  const int wv = threadIdx.x >> 6;
  uint8_t* wl = reinterpret_cast<uint8_t*>(lds_q) + wv * seg_wave_lds(a.stride);
  const int lane = threadIdx.x & 63, r = lane >> 4, l = lane & 15;
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (w * kSegRows >= a.B) return;  // the whole wave
  const int64_t b = w * kSegRows + r;
  const bool live = b < a.B;
  const int64_t bc = live ? b : a.B - 1;
  const SegLds L = seg_row(wl, a.stride, r);
  int len = a.text_len[bc];
  uint8_t err = 0;
  if (len < 0 || len > a.stride) {
    err |= RMI_ERR_STATE;
    len = 0;
  }
  if (!live) len = 0;
  Names nm0, nm1;
  load_names2(a.cfg, nm0, nm1);
  const bool col = live && a.sel && a.sel[b];
  const uint32_t* s4 = reinterpret_cast<const uint32_t*>(a.text + bc * a.stride);
  uint32_t* d4 = reinterpret_cast<uint32_t*>(L.T + kPre);
  for (int i = l; i < (len + 3) >> 2; i += 16) d4[i] = s4[i];
  parse_rows4(a, wl, b, live, len, err, nm0, nm1, col, lane);
}

}  // namespace
}  // namespace rmi

namespace rmi {
namespace {
// rmi_parse_actions takes the four-responses-per-wave kernel for rows whose LDS (4 rows + the
// cascade row) fits 48 KB per wave; RAGEN_AMD_PARSE1=1 forces the one-response-per-wave kernel
// (A/B, tests).  The fused decode + parse keeps one response per wave: four decodes per wave
// one after another measured 32.7 us against 24.7 us.
bool use_seg(int stride) {
  const char* e = getenv("RAGEN_AMD_PARSE1");
  if (e && e[0] == '1') return false;
  return stride <= kSegMaxStride && seg_wave_lds(stride) <= 48 * 1024;
}
int seg_waves_per_group(int stride) {
  const size_t n = kWgLds / seg_wave_lds(stride);
  return n >= (size_t)kRowWaves ? kRowWaves : (n < 1 ? 1 : (int)n);
}
// ---- the turn's generations onto the env batch (rmi_gen_rows): one wave per env row.  The
// rows' longest raw byte count is reduced per wave (scan), then per 16-wave block (LDS), and
// reaches raw_max with ONE atomic per block: every wave's atomicMax on the same word (8192 at the
// bench size) serialised at the memory side and made this an 80-us launch.
constexpr int kGenWaves = 16;
__global__ __launch_bounds__(64 * kGenWaves) void gen_rows_kernel(const int64_t* __restrict__ resp, int64_t R,
                                                                  const int64_t* __restrict__ src, int64_t n_envs,
                                                                  const uint32_t* __restrict__ packed, int64_t V,
                                                                  int64_t* __restrict__ ids, int32_t* __restrict__ n_ids,
                                                                  uint8_t* __restrict__ has, int32_t* __restrict__ raw_max,
                                                                  int32_t* __restrict__ raw_next) {
  __shared__ int wave_max[kGenWaves];
  if (raw_next && blockIdx.x == 0 && threadIdx.x == 0) *raw_next = 0;  // the next call's raw_max
  const int wv = threadIdx.x / 64;
  const int64_t e = (int64_t)blockIdx.x * kGenWaves + wv;
  const int lane = threadIdx.x & 63;
  int best = -1;  // this wave's row: its raw bytes, -1 = none
  if (e < n_envs) {
    const int64_t r = src ? src[e] : e;
    int64_t* orow = ids ? ids + e * R : nullptr;
    int raw = 0;
    if (r >= 0) {
      const int64_t* row = resp + r * R;
      for (int64_t k = lane; k < R; k += 64) {
        const int64_t t = row[k];
        if (orow) orow[k] = t;
        const int64_t c = t < 0 ? 0 : (t >= V ? V - 1 : t);  // the clamp of the sizing (ids outside
        const uint32_t meta = packed[4 * c + 3];              // [0, V) are flagged by the decode)
        raw += (meta >> 31) ? 0 : (int)(meta & 0xFFFFFFu);
      }
    } else if (orow) {
      for (int64_t k = lane; k < R; k += 64) orow[k] = 0;
    }
    if (lane == 0) {
      if (n_ids) n_ids[e] = r >= 0 ? (int32_t)R : 0;
      if (has) has[e] = r >= 0 ? 1 : 0;
    }
    const int tot = __builtin_amdgcn_readlane(wave_inclusive_scan(raw), 63);
    best = r >= 0 ? tot : -1;
  }
  if (lane == 0) wave_max[wv] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    int m = -1;
#pragma unroll
    for (int w = 0; w < kGenWaves; ++w) m = wave_max[w] > m ? wave_max[w] : m;
    if (m >= 0) atomicMax(raw_max, m);
  }
}

}  // namespace
}  // namespace rmi

RMI_API int rmi_detokenize(const int64_t* ids, int64_t B, int64_t R, const int32_t* n_ids, const uint32_t* vocab_packed,
                           const uint8_t* vocab_bytes, int64_t n_bytes, int64_t V, uint8_t* out, int32_t stride,
                           int32_t* out_len, uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || R < 0 || V < 1 || stride <= 0) return RMI_EINVAL;
  if (stride % 4 != 0 || stride > kMaxStride || B > 0x7FFFFFFF) return RMI_EUNSUP;
  if (B == 0) return RMI_OK;
  if (!out || !out_len || !vocab_packed || (R > 0 && !ids) || n_bytes < 0 || (n_bytes > 0 && !vocab_bytes))
    return RMI_EINVAL;
  if ((reinterpret_cast<uintptr_t>(out) & 3u) || (reinterpret_cast<uintptr_t>(vocab_packed) & 15u)) return RMI_EUNSUP;
  const int nw = row_waves(detok_lds(stride));
  const size_t shm = detok_lds(stride) * nw;
  DetokArgs d{ids, R, n_ids, reinterpret_cast<const uint4*>(vocab_packed), vocab_bytes, n_bytes, V, out, (int)stride,
              out_len, err, B};
  hipLaunchKernelGGL(detok_kernel, dim3((unsigned)((B + nw - 1) / nw)), dim3(64 * nw), shm, as_stream(stream), d);
  return launch_status();
}

RMI_API int rmi_detok_parse(const int64_t* ids, int64_t B, int64_t R, const int32_t* n_ids,
                            const uint32_t* vocab_packed, const uint8_t* vocab_bytes, int64_t n_bytes, int64_t V,
                            uint8_t* text, int32_t stride, int32_t* text_len, uint8_t* decode_err,
                            const rmi_parse_cfg_t* cfg, const uint8_t* sel, int8_t* actions, uint8_t* n_actions,
                            int32_t* spans, uint8_t* action_text, int32_t* action_len, int32_t Lact,
                            uint8_t* parse_err, rmi_stream_t stream) {
  using namespace rmi;
  DetokArgs d;
  ParseArgs a;
  const int rc = detok_parse_args(ids, B, R, n_ids, vocab_packed, vocab_bytes, n_bytes, V, text, stride, text_len,
                                  decode_err, cfg, sel, actions, n_actions, spans, action_text, action_len, Lact,
                                  parse_err, d, a);
  if (rc != RMI_OK) return rc > 0 ? RMI_OK : rc;
  const int nw = row_waves(parse_lds(stride));
  const size_t shm = parse_lds(stride) * nw;
  hipLaunchKernelGGL(detok_parse_kernel, dim3((unsigned)((B + nw - 1) / nw)), dim3(64 * nw), shm,
                     as_stream(stream), d, a);
  return launch_status();
}

#ifdef RMI_PARSE_STAMPS
RMI_API int rmi_parse_set_stamps(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(rmi::g_parse_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -2;
}
RMI_API int rmi_detok_set_stamps(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(rmi::g_detok_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -2;
}
#endif

RMI_API int rmi_parse_actions(const rmi_parse_cfg_t* cfg, const uint8_t* text, const int32_t* text_len, int64_t B,
                              int32_t stride, const uint8_t* sel, int8_t* actions, uint8_t* n_actions,
                              int32_t* spans, uint8_t* action_text, int32_t* action_len, int32_t Lact, uint8_t* err,
                              rmi_stream_t stream) {
  using namespace rmi;
  if (!cfg || B < 0 || stride <= 0) return RMI_EINVAL;
  if (cfg->K < 1 || cfg->sep_len < 1 || cfg->sep_len > 16 || cfg->n_names < 0) return RMI_EINVAL;
  if (cfg->K > kMaxK || cfg->n_names > RMI_PARSE_MAX_NAMES || stride % 4 != 0 || stride > kMaxParseStride ||
      B > 0x7FFFFFFF)
    return RMI_EUNSUP;
  for (int j = 0; j < cfg->n_names; ++j)
    if (cfg->name_len[j] < 1 || cfg->name_len[j] > 16) return RMI_EINVAL;
  if (B == 0) return RMI_OK;
  if (!text || !text_len || !actions || !n_actions) return RMI_EINVAL;
  if (action_text && (!action_len || Lact < 1)) return RMI_EINVAL;
  if (reinterpret_cast<uintptr_t>(text) & 3u) return RMI_EUNSUP;
  ParseArgs a{*cfg, text, text_len, B, (int)stride, sel, actions, n_actions, spans, action_text, action_len,
              (int)Lact, err};
  if (use_seg(stride)) {
    const int nw = seg_waves_per_group(stride);
    const int64_t rows = (int64_t)nw * kSegRows;
    hipLaunchKernelGGL(parse4_kernel, dim3((unsigned)((B + rows - 1) / rows)), dim3(64 * nw),
                       seg_wave_lds(stride) * nw, as_stream(stream), a);
    return launch_status();
  }
  const int nw = row_waves(parse_lds(stride));
  const size_t shm = parse_lds(stride) * nw;
  hipLaunchKernelGGL(parse_kernel, dim3((unsigned)((B + nw - 1) / nw)), dim3(64 * nw), shm,
                     as_stream(stream), a);
  return launch_status();
}

RMI_API int rmi_gen_rows(const int64_t* resp, int64_t n_resp, int64_t R, const int64_t* src, int64_t n_envs,
                         const uint32_t* vocab_packed, int64_t V, int64_t* ids, int32_t* n_ids, uint8_t* has,
                         int32_t* raw_max, rmi_stream_t stream) {
  using namespace rmi;
  if (n_resp < 0 || R < 0 || n_envs < 0 || V < 1 || !raw_max || !vocab_packed) return RMI_EINVAL;
  if ((src == nullptr) != (ids == nullptr) || (src == nullptr && n_resp != n_envs)) return RMI_EINVAL;
  if (!resp && n_resp > 0 && R > 0) return RMI_EINVAL;
  hipStream_t st = as_stream(stream);
  if (hipMemsetAsync(raw_max, 0, sizeof(int32_t), st) != hipSuccess) return RMI_EDEVICE;
  if (n_envs == 0) return RMI_OK;
  hipLaunchKernelGGL(gen_rows_kernel, dim3((unsigned)((n_envs + kGenWaves - 1) / kGenWaves)), dim3(64 * kGenWaves), 0,
                     st, resp, R, src, n_envs, vocab_packed, V, ids, n_ids, has, raw_max, nullptr);
  return launch_status();
}

RMI_API int rmi_gen_rows_chained(const int64_t* resp, int64_t n_resp, int64_t R, const int64_t* src, int64_t n_envs,
                                 const uint32_t* vocab_packed, int64_t V, int64_t* ids, int32_t* n_ids, uint8_t* has,
                                 int32_t* raw_max, int32_t* raw_next, rmi_stream_t stream) {
  using namespace rmi;
  if (n_resp < 0 || R < 0 || n_envs < 0 || V < 1 || !raw_max || !vocab_packed || raw_next == raw_max) return RMI_EINVAL;
  if ((src == nullptr) != (ids == nullptr) || (src == nullptr && n_resp != n_envs)) return RMI_EINVAL;
  if (!resp && n_resp > 0 && R > 0) return RMI_EINVAL;
  if (n_envs == 0) {  // nothing to reduce: raw_max stays 0; raw_next still zeroed
    return raw_next && hipMemsetAsync(raw_next, 0, sizeof(int32_t), as_stream(stream)) != hipSuccess ? RMI_EDEVICE
                                                                                                   : RMI_OK;
  }
  hipLaunchKernelGGL(gen_rows_kernel, dim3((unsigned)((n_envs + kGenWaves - 1) / kGenWaves)), dim3(64 * kGenWaves), 0,
                     as_stream(stream), resp, R, src, n_envs, vocab_packed, V, ids, n_ids, has, raw_max, raw_next);
  return launch_status();
}
