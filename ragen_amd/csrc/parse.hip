// parse.hip — the LLM response -> action-id boundary on the device (gfx950), SURVEY §8(f) rank 2.
//
//  rmi_detokenize      tokenizer.batch_decode(responses, skip_special_tokens=True)
//                      (ctx_manager.py:334-337) for byte-level BPE vocabularies
//  rmi_parse_actions   ContextManager._parse_response (ctx_manager.py:148-173) on the
//                      "<think>"/"<answer>"-prefixed response (:338-339), then
//                      EnvStateManager._extract_map_valid_actions (es_manager.py:230-240)
//
// One wave per response.  The row is staged in LDS with coalesced dword loads; every scan
// over it (tag search, special-token test, separator search) is wave-parallel: 64 candidate
// positions per step, the first hit found by ballot.  What the reference does with Python
// string methods between the scans (regex backtracking over </think> candidates, \s* and
// str.strip over Unicode whitespace, the special-token replace cascade) runs wave-uniformly
// on the few bytes involved.  Only the rare row whose answer contains a special token takes
// the serial replace cascade (lane 0).
//
// Exactness argument for working on UTF-8 bytes instead of Python str: every tag, the
// separator and the action names are ASCII; UTF-8 is self-synchronising, so an ASCII byte is
// always a whole character and a multi-byte whitespace sequence (U+0085, U+00A0, U+1680,
// U+2000-U+200A, U+2028/9, U+202F, U+205F, U+3000) found at a character boundary (forward)
// or ending at one (backward: its lead byte can never be a continuation byte) is that
// character.  str.lower() maps exactly one non-ASCII character to an ASCII string: U+212A
// KELVIN SIGN -> 'k' (U+0130 -> "i" + U+0307 is never all-ASCII); it is handled below.
#include "common.hpp"

namespace rmi {
namespace {

constexpr int kPre = 8;             // room for the implicit prefix tag in front of the text
constexpr int kPad = 16;            // zero bytes after the text
constexpr int kMaxStride = 16384;

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
__device__ __forceinline__ uint8_t tag_byte(const Tag& t, int k) {
  return (uint8_t)(k < 8 ? t.lo >> (8 * k) : t.hi >> (8 * (k - 8)));
}
__device__ __forceinline__ bool match_at(const uint8_t* V, int p, int lim, const Tag& t) {
  if (p < 0 || p + t.n > lim) return false;
  bool ok = true;
  for (int k = 0; k < t.n; ++k) ok = ok && V[p + k] == tag_byte(t, k);
  return ok;
}

constexpr Tag kThinkOpen = make_tag("<think>");
constexpr Tag kThinkClose = make_tag("</think>");
constexpr Tag kAnsOpen = make_tag("<answer>");
constexpr Tag kAnsClose = make_tag("</answer>");
constexpr Tag kImStart = make_tag("<|im_start|>");
constexpr Tag kImEnd = make_tag("<|im_end|>");

// smallest p >= from with V[p, p + n) == tag inside [.., lim), else -1 (wave-uniform)
__device__ int find_tag(const uint8_t* V, int from, int lim, const Tag& t, int lane) {
  for (int base = from; base + t.n <= lim; base += 64) {
    const int p = base + lane;
    bool hit = p + t.n <= lim && V[p] == (uint8_t)t.lo;
    if (hit)
      for (int k = 1; k < t.n; ++k) hit = hit && V[p + k] == tag_byte(t, k);
    const uint64_t m = __ballot(hit);
    if (m) return base + __builtin_ctzll(m);
  }
  return -1;
}

// Length of the Unicode whitespace character (str.isspace / re \s) starting at p, or 0.
__device__ __forceinline__ int ws_fwd(const uint8_t* V, int p, int lim) {
  if (p >= lim) return 0;
  const uint32_t c = V[p];
  if (c < 0x80) return ((c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x20)) ? 1 : 0;
  if (c == 0xC2) return (p + 1 < lim && (V[p + 1] == 0x85 || V[p + 1] == 0xA0)) ? 2 : 0;
  if (p + 2 >= lim) return 0;
  const uint32_t c1 = V[p + 1], c2 = V[p + 2];
  if (c == 0xE1) return (c1 == 0x9A && c2 == 0x80) ? 3 : 0;
  if (c == 0xE2) {
    if (c1 == 0x80) return ((c2 >= 0x80 && c2 <= 0x8A) || c2 == 0xA8 || c2 == 0xA9 || c2 == 0xAF) ? 3 : 0;
    return (c1 == 0x81 && c2 == 0x9F) ? 3 : 0;
  }
  if (c == 0xE3) return (c1 == 0x80 && c2 == 0x80) ? 3 : 0;
  return 0;
}
// Length of the whitespace character ending at e (within [s, e)), or 0.
__device__ __forceinline__ int ws_back(const uint8_t* V, int s, int e) {
  if (e <= s) return 0;
  const uint32_t c = V[e - 1];
  if (c < 0x80) return ((c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x20)) ? 1 : 0;
  if (e - 2 >= s && V[e - 2] == 0xC2 && (c == 0x85 || c == 0xA0)) return 2;
  if (e - 3 < s) return 0;
  return ws_fwd(V, e - 3, e) == 3 ? 3 : 0;
}
__device__ __forceinline__ void strip(const uint8_t* V, int& a, int& z) {
  for (int l; (l = ws_fwd(V, a, z)) != 0;) a += l;
  for (int l; (l = ws_back(V, a, z)) != 0;) z -= l;
}

// any of the six special tokens (ctx_manager.py:94) inside [a, z)  (wave-uniform)
__device__ bool has_special(const uint8_t* V, int a, int z, int lane) {
  for (int base = a; base < z; base += 64) {
    const int p = base + lane;
    bool hit = false;
    if (p < z && V[p] == '<')
      hit = match_at(V, p, z, kThinkOpen) || match_at(V, p, z, kThinkClose) || match_at(V, p, z, kAnsOpen) ||
            match_at(V, p, z, kAnsClose) || match_at(V, p, z, kImStart) || match_at(V, p, z, kImEnd);
    if (__ballot(hit)) return true;
  }
  return false;
}

// s = s.replace(tok, "").strip() in place on w[a, z)  (one lane)
__device__ void replace_strip(uint8_t* w, int& a, int& z, const Tag& t) {
  int o = a;
  for (int i = a; i < z;) {
    if (match_at(w, i, z, t)) {
      i += t.n;
    } else {
      w[o++] = w[i++];
    }
  }
  z = o;
  strip(w, a, z);
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

// dword-staged row copy global -> LDS (row start 4-B aligned, stride % 4 == 0)
__device__ __forceinline__ void stage_row(uint8_t* dst, const uint8_t* src, int len, int lane) {
  const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
  uint32_t* d4 = reinterpret_cast<uint32_t*>(dst);
  const int nw = (len + 3) >> 2;
  for (int i = lane; i < nw; i += 64) d4[i] = s4[i];
}

__global__ __launch_bounds__(64) void parse_kernel(ParseArgs a) {
  extern __shared__ uint32_t lds_words[];
  uint8_t* t = reinterpret_cast<uint8_t*>(lds_words);  // [kPre + stride + kPad]
  uint8_t* w = t + kPre + a.stride + kPad;              // replace-cascade work row [stride + kPre + kPad]
  __shared__ int sh_a, sh_z;
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  const rmi_parse_cfg_t& cfg = a.cfg;
  const int K = cfg.K;
  int len = a.text_len[b];
  uint8_t err = 0;
  if (len < 0 || len > a.stride) {
    err |= RMI_ERR_STATE;
    len = 0;
  }
  stage_row(t + kPre, a.text + b * a.stride, len, lane);
  __syncthreads();
  if (lane < kPad) t[kPre + len + lane] = 0;  // over-read bytes of the last dword -> 0
  const Tag pre = cfg.enable_think ? kThinkOpen : kAnsOpen;
  const int plen = cfg.prepend ? pre.n : 0;
  if (lane < plen) t[kPre - plen + lane] = tag_byte(pre, lane);
  __syncthreads();
  const uint8_t* V = t + kPre - plen;  // the prefixed response (get_env_inputs :338-339)
  const int n = plen + len;

  // ---- 1. re.search(pattern, response, re.DOTALL)  (ctx_manager.py:149-150)
  int ts = -1, te = -1, as = -1, ae = -1;
  if (cfg.enable_think) {
    // <think>(.*?)</think>\s*<answer>(.*?)</answer>: the leftmost <think> decides (a later
    // start only sees a subset of the </think> candidates); group 1 grows over the
    // </think> candidates in order until \s*<answer> follows; group 2 ends at the first
    // </answer> after it (if there is none, no later candidate can have one either)
    const int i = find_tag(V, 0, n, kThinkOpen, lane);
    if (i >= 0) {
      int j = i + kThinkOpen.n, k = -1;
      for (;;) {
        j = find_tag(V, j, n, kThinkClose, lane);
        if (j < 0) break;
        k = j + kThinkClose.n;
        for (int l; (l = ws_fwd(V, k, n)) != 0;) k += l;  // \s* is greedy and '<' is no space
        if (match_at(V, k, n, kAnsOpen)) break;
        ++j;
      }
      if (j >= 0) {
        const int e = find_tag(V, k + kAnsOpen.n, n, kAnsClose, lane);
        if (e >= 0) {
          ts = i + kThinkOpen.n;
          te = j;
          as = k + kAnsOpen.n;
          ae = e;
        }
      }
    }
  } else {
    const int i = find_tag(V, 0, n, kAnsOpen, lane);
    if (i >= 0) {
      const int e = find_tag(V, i + kAnsOpen.n, n, kAnsClose, lane);
      if (e >= 0) {
        as = i + kAnsOpen.n;
        ae = e;
      }
    }
  }

  // ---- 2. special-token replace cascade + strip of the action content (:161-163)
  const uint8_t* C = V;
  int ca = 0, cz = 0;
  if (as >= 0) {
    ca = as;
    cz = ae;
    if (!has_special(V, ca, cz, lane)) {
      strip(V, ca, cz);  // every replace is a no-op, and strip() six times is strip() once
    } else {
      for (int i = ca + lane; i < cz; i += 64) w[i] = V[i];
      __syncthreads();
      if (lane == 0) {
        int x = ca, y = cz;
        replace_strip(w, x, y, kThinkOpen);
        replace_strip(w, x, y, kThinkClose);
        replace_strip(w, x, y, kAnsOpen);
        replace_strip(w, x, y, kAnsClose);
        replace_strip(w, x, y, kImStart);
        replace_strip(w, x, y, kImEnd);
        sh_a = x;
        sh_z = y;
      }
      __syncthreads();
      ca = sh_a;
      cz = sh_z;
      C = w;
    }
  }

  // ---- 3. split(action_sep), strip, drop empties, cap at K (:165-169); name -> id (es :230-240)
  const Tag sep{cfg.sep_lo, cfg.sep_hi, cfg.sep_len};
  const int col = (a.sel && a.sel[b]) ? 1 : 0;
  const bool lane_name = lane < cfg.n_names;
  const Tag name{lane_name ? cfg.name_lo[lane] : 0ull, lane_name ? cfg.name_hi[lane] : 0ull,
                 lane_name ? (int)cfg.name_len[lane] : 0};
  const int my_id = lane_name ? cfg.name_id[col][lane] : 0;
  int count = 0, my_act = 0;
  if (as >= 0) {
    int pos = ca;
    while (count < K) {
      const int q = find_tag(C, pos, cz, sep, lane);
      int s = pos, e = q < 0 ? cz : q;
      strip(C, s, e);
      if (e > s) {
        int id = 0;
        if (cfg.n_names > 0) {
          // action.lower() == name (names are lowercased ASCII): lane j tests name j
          bool ok = lane_name;
          int qn = 0;
          for (int i = s; ok && i < e;) {
            uint32_t c = C[i];
            if (c < 0x80) {
              c += (c >= 'A' && c <= 'Z') ? 32u : 0u;
              ++i;
            } else if (c == 0xE2 && i + 2 < e && C[i + 1] == 0x84 && C[i + 2] == 0xAA) {
              c = 'k';  // U+212A KELVIN SIGN
              i += 3;
            } else {
              ok = false;
              break;
            }
            ok = qn < name.n && tag_byte(name, qn) == c;
            ++qn;
          }
          ok = ok && qn == name.n;
          const uint64_t m = __ballot(ok);
          if (m) id = __builtin_amdgcn_readlane(my_id, __builtin_ctzll(m));
        } else {
          id = 1;  // no lookup: the strings themselves are the actions
        }
        if (lane == count) my_act = id;
        if (a.action_text) {
          const int L = e - s, Lc = L < a.Lact ? L : a.Lact;
          uint8_t* dst = a.action_text + (b * K + count) * (int64_t)a.Lact;
          for (int i = lane; i < Lc; i += 64) dst[i] = C[s + i];
          if (lane == 0) a.action_len[b * K + count] = Lc;
          if (L > a.Lact) err |= RMI_ERR_UNSUP;
        }
        ++count;
      }
      if (q < 0) break;
      pos = q + sep.n;
    }
  }
  if (lane < K) {
    a.actions[b * K + lane] = (int8_t)(lane < count ? my_act : 0);
    if (a.action_text && lane >= count) a.action_len[b * K + lane] = 0;
  }
  if (lane == 0) {
    a.n_actions[b] = (uint8_t)count;
    if (a.spans) {
      a.spans[4 * b + 0] = ts;
      a.spans[4 * b + 1] = te;
      a.spans[4 * b + 2] = as;
      a.spans[4 * b + 3] = ae;
    }
    if (err && a.err) a.err[b] |= err;
  }
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

__global__ __launch_bounds__(64) void detok_kernel(const int64_t* __restrict__ ids, int64_t R,
                                                   const int32_t* __restrict__ n_ids,
                                                   const int64_t* __restrict__ voff,
                                                   const uint8_t* __restrict__ vbytes, int64_t V,
                                                   const uint8_t* __restrict__ skip, uint8_t* __restrict__ out,
                                                   int stride, int32_t* __restrict__ out_len,
                                                   uint8_t* __restrict__ err_out) {
  extern __shared__ uint32_t lds_words[];
  uint8_t* buf = reinterpret_cast<uint8_t*>(lds_words);  // raw concatenation [stride + 4]
  uint8_t* fix = buf + stride + 4;                          // lossy-decoded row  [stride + 4]
  __shared__ int sh_len, sh_over;
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  int64_t rn = n_ids ? (int64_t)n_ids[b] : R;
  rn = rn < 0 ? 0 : (rn > R ? R : rn);
  const int64_t* row = ids + b * R;
  int pos = 0;
  bool bad = false, over = false;
  uint32_t high = 0;
  for (int64_t c0 = 0; c0 < rn; c0 += 64) {
    const int64_t i = c0 + lane;
    const int64_t id = i < rn ? row[i] : -1;
    const bool in = i < rn;
    const bool valid = id >= 0 && id < V;
    bad |= in && !valid;
    int64_t off = 0;
    int len = 0;
    if (valid && !skip[id]) {
      off = voff[id];
      len = (int)(voff[id + 1] - off);
    }
    const int incl = wave_inclusive_scan(len);
    const int start = pos + incl - len;
    pos += __builtin_amdgcn_readlane(incl, 63);
    for (int k = 0; k < len; ++k) {
      const int p = start + k;
      if (p < stride) {
        const uint8_t c = vbytes[off + k];
        buf[p] = c;
        high |= c;
      } else {
        over = true;
      }
    }
  }
  int n = pos < stride ? pos : stride;
  __syncthreads();
  const uint8_t* res = buf;
  if (__ballot((high & 0x80u) != 0)) {  // some non-ASCII byte: validate (one lane)
    if (lane == 0) {
      bool ov = false;
      sh_len = utf8_lossy(buf, n, fix, stride, ov);
      sh_over = ov;
    }
    __syncthreads();
    n = sh_len;
    over |= sh_over != 0;
    res = fix;
  }
  const int nw = (n + 3) >> 2;
  if (lane < 4 && (n & 3)) const_cast<uint8_t*>(res)[n + lane] = 0;  // deterministic tail bytes
  __syncthreads();
  uint32_t* o4 = reinterpret_cast<uint32_t*>(out + b * (int64_t)stride);
  const uint32_t* r4 = reinterpret_cast<const uint32_t*>(res);
  for (int i = lane; i < nw; i += 64) o4[i] = r4[i];
  const uint64_t any_bad = __ballot(bad), any_over = __ballot(over);
  if (lane == 0) {
    out_len[b] = n;
    if (err_out) err_out[b] |= (any_bad ? RMI_ERR_INDEX : 0) | (any_over ? RMI_ERR_UNSUP : 0);
  }
}

}  // namespace
}  // namespace rmi

RMI_API int rmi_detokenize(const int64_t* ids, int64_t B, int64_t R, const int32_t* n_ids, const int64_t* vocab_off,
                           const uint8_t* vocab_bytes, int64_t V, const uint8_t* skip, uint8_t* out, int32_t stride,
                           int32_t* out_len, uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || R < 0 || V < 0 || stride <= 0) return RMI_EINVAL;
  if (stride % 4 != 0 || stride > kMaxStride || B > 0x7FFFFFFF) return RMI_EUNSUP;
  if (B == 0) return RMI_OK;
  if (!out || !out_len || !vocab_off || !skip || (R > 0 && !ids) || (V > 0 && !vocab_bytes)) return RMI_EINVAL;
  if (reinterpret_cast<uintptr_t>(out) & 3u) return RMI_EUNSUP;
  const size_t shm = 2 * ((size_t)stride + 4);
  hipLaunchKernelGGL(detok_kernel, dim3((unsigned)B), dim3(64), shm, as_stream(stream), ids, R, n_ids, vocab_off,
                     vocab_bytes, V, skip, out, (int)stride, out_len, err);
  return launch_status();
}

RMI_API int rmi_parse_actions(const rmi_parse_cfg_t* cfg, const uint8_t* text, const int32_t* text_len, int64_t B,
                              int32_t stride, const uint8_t* sel, int8_t* actions, uint8_t* n_actions,
                              int32_t* spans, uint8_t* action_text, int32_t* action_len, int32_t Lact, uint8_t* err,
                              rmi_stream_t stream) {
  using namespace rmi;
  if (!cfg || B < 0 || stride <= 0) return RMI_EINVAL;
  if (cfg->K < 1 || cfg->sep_len < 1 || cfg->sep_len > 16 || cfg->n_names < 0) return RMI_EINVAL;
  if (cfg->K > kMaxK || cfg->n_names > RMI_PARSE_MAX_NAMES || stride % 4 != 0 || stride > kMaxStride ||
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
  const size_t shm = (size_t)(kPre + stride + kPad) * 2;
  hipLaunchKernelGGL(parse_kernel, dim3((unsigned)B), dim3(64), shm, as_stream(stream), a);
  return launch_status();
}
