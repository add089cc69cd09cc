// prompt.hip — the prompt text one turn adds, built on the device (gfx950), SURVEY §8(f) rank 2.
//
//  rmi_prompt_text   ContextManager.get_lm_inputs' messages (ctx_manager.py:248-263) under the
//                    tokenizer's chat template, for the block a turn appends: the assistant
//                    message (_parse_response's llm_response, ctx_manager.py:148-173) and the
//                    next user message (Reward, Turn, State, actions left, the format line)
//
// One wave per row.  The row is a fixed program of pieces (constant bytes per launch or per
// env tag, the env's rendered state, integers, the reward, the response); the wave assembles
// it in LDS — constant and state bytes copied lane-parallel, numbers formatted by one lane
// (pyrepr.hpp: CPython's str of an int / float) — and stores it as dwords.  The response
// piece rebuilds _parse_response's normalised string from the parse kernel's regex spans:
// each content is stripped (Python str.strip whitespace); a content holding '<' takes the
// special-token replace / strip cascade on one lane; the separators of the answer are found
// lane-parallel and, when the answer holds more than K non-empty actions, it is re-joined
// from its first K stripped actions.
#include "common.hpp"
#include "pyrepr.hpp"
#include "text.hpp"

namespace rmi {
namespace {

constexpr int kMaxStride = 3072;

// ---- the reward text cache (rmi_prompt_t.num_cache): 16 u32 per entry — the claimed key
// (the float's bits xor kNumKeyMix, 2 u32; 0 = empty), meta = ready | length, the text (6 u32,
// zero padded).  Written once per slot (include/ragen_amd.h): the writer that wins the key's
// compare-and-swap stores the text, then the meta word; nothing rewrites a claimed slot.  So
// every dword goes 0 -> final value once (dword stores and loads are single-copy atomic), and
// a reader that sees the key, the ready bit and a nonzero byte at every text position below the
// length holds exactly the writer's text — whatever order the words became visible in, and
// with no fence on either side (a word still invisible reads 0: a miss, the row computes).
constexpr uint32_t kNumReady = 1u << 31;
constexpr uint64_t kNumKeyMix = 0x7FF4C0FFEE15BAD1ull;  // a NaN payload: no finite reward maps to 0
__device__ __forceinline__ uint32_t num_slot(uint64_t key, uint32_t mask) {
  return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 40) & mask;
}
// the cached text of key into out -> its length, or -1
__device__ __forceinline__ int num_take(const uint4 (&e)[4], uint64_t key, char* out) {
  const uint64_t kk = key ^ kNumKeyMix;
  const uint32_t meta = e[0].z;
  if (kk == 0 || !(meta & kNumReady) || (((uint64_t)e[0].y << 32) | e[0].x) != kk) return -1;
  const int len = (int)(meta & 0xFFu);
  if (len < 1 || len > 24) return -1;
  const uint32_t t[6] = {e[0].w, e[1].x, e[1].y, e[1].z, e[1].w, e[2].x};
  for (int i = 0; i < len; ++i) {
    const uint32_t ch = (t[i >> 2] >> (8 * (i & 3))) & 0xFFu;
    if (ch == 0) return -1;  // that word is not visible here yet
    out[i] = (char)ch;
  }
  return len;
}
__device__ __forceinline__ void num_put(uint32_t* s, uint64_t key, const char* txt, int len) {
  const uint64_t kk = key ^ kNumKeyMix;
  if (kk == 0) return;
  // claim the empty slot; a slot another key (or another writer of this key) holds is left alone
  if (atomicCAS(reinterpret_cast<unsigned long long*>(s), 0ull, (unsigned long long)kk) != 0ull) return;
  uint32_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < len; ++i) t[i >> 2] |= (uint32_t)(uint8_t)txt[i] << (8 * (i & 3));
#pragma unroll
  for (int i = 0; i < 6; ++i) s[3 + i] = t[i];
  s[2] = kNumReady | (uint32_t)len;
}

struct Tok6 {
  const char* s;
  int n;
};
__device__ const char kThinkO[] = "<think>", kThinkC[] = "</think>", kAnsO[] = "<answer>", kAnsC[] = "</answer>",
                      kImS[] = "<|im_start|>", kImE[] = "<|im_end|>";

// lane-parallel copy of n bytes (global or LDS source) into the LDS row at pos
__device__ __forceinline__ void put(uint8_t* row, int pos, const uint8_t* src, int n, int lane) {
  for (int i = lane; i < n; i += 64) row[pos + i] = src[i];
}

// one lane: content <- content.replace(tok, "") for tok in SPECIAL_TOKENS, .strip() after each
// (ctx_manager.py:163-165); in place on buf[a, z)
__device__ void cascade(uint8_t* buf, int& a, int& z) {
  const Tok6 toks[6] = {{kThinkO, 7}, {kThinkC, 8}, {kAnsO, 8}, {kAnsC, 9}, {kImS, 12}, {kImE, 10}};
  for (int t = 0; t < 6; ++t) {
    const char* s = toks[t].s;
    const int n = toks[t].n;
    int j = a;
    for (int i = a; i < z;) {
      bool m = i + n <= z;
      for (int k = 0; m && k < n; ++k) m = buf[i + k] == (uint8_t)s[k];
      if (m) {
        i += n;
      } else {
        buf[j++] = buf[i++];
      }
    }
    z = j;
    strip(buf, a, z);
  }
}

// The wave's staging of its row's inputs (kernel prologue): the constant pool, the rendered
// observation and the response, copied into LDS by loads that all go out before the first
// wait, so the piece loop below runs on LDS alone (it used to issue each piece's global reads
// when it reached the piece: one memory round trip per piece).
constexpr int kStagePool = 1024;  // pool bytes staged (4 dwords a lane); a longer pool is read in place
constexpr int kStageResp = 512;   // response bytes in the first batch (2 dwords a lane); the rest after
struct StageDims {
  int pool, obs, resp;  // staged region sizes (bytes, multiples of 4; 0 = not staged)
};
__host__ __device__ inline StageDims stage_dims(const rmi_prompt_t& P, int stride, bool need_obs, bool need_resp) {
  StageDims d;
  // dword loads: the pool and the response rows staged only when 4-B aligned and whole dwords
  const bool pool4 = P.pool && P.pool_len > 0 && P.pool_len % 4 == 0 && (reinterpret_cast<uintptr_t>(P.pool) & 3u) == 0;
  const bool resp4 = P.resp && P.resp_stride > 0 && P.resp_stride % 4 == 0 && (reinterpret_cast<uintptr_t>(P.resp) & 3u) == 0;
  d.pool = pool4 && P.pool_len <= kStagePool ? P.pool_len : 0;
  d.obs = need_obs && P.obs_stride > 0 && P.obs_stride <= kMaxStride ? (P.obs_stride + 3) & ~3 : 0;
  d.resp = need_resp && resp4 ? (P.resp_stride < stride ? P.resp_stride : stride) : 0;
  return d;
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(6))) void prompt_text_kernel(rmi_prompt_t P, int64_t B, uint8_t* __restrict__ out,
                                                         int stride, int32_t* __restrict__ out_len,
                                                         int32_t* __restrict__ mark, uint8_t* __restrict__ err,
                                                         StageDims sd) {
  extern __shared__ __align__(16) uint8_t smem[];
  uint8_t* row = smem;                         // the assembled row, stride + 64
  uint8_t* th = row + stride + 64;             // think content, stride
  uint8_t* an = th + stride;                   // answer content + its re-joined form, 2 * stride + 64
  uint8_t* num = an + 2 * stride + 64;         // formatted number, 64
  int* sh = reinterpret_cast<int*>(num + 64);  // lane 0 -> wave hand-off, 16 ints; the split's
                                               // piece bounds at sh + 16 / sh + 32 (K + 1 each)
  char* scr = reinterpret_cast<char*>(sh + 48);  // the number formatter's digit scratch, 64
  uint8_t* pl = reinterpret_cast<uint8_t*>(scr + 64);  // staged pool, sd.pool
  uint8_t* ob = pl + sd.pool;                          // staged observation row, sd.obs
  uint8_t* rs = ob + sd.obs;                           // staged response row, sd.resp (+ 8)
  int* pre_iv = reinterpret_cast<int*>(smem + ((rs - smem + sd.resp + 8 + 7) & ~7));  // INT values by piece [64]
  int2* pre_tc = reinterpret_cast<int2*>(pre_iv + 64);      // TAG_CONST (offset, length) [64]
  int* pre_s = reinterpret_cast<int*>(pre_tc + 64);         // tag, cond, reward_int
  double* pre_d = reinterpret_cast<double*>(pre_s + 4);     // reward
  // (lane 0's formatting and split work in LDS, not in per-lane register arrays: the wave
  // keeps a register budget that lets 8 waves share a SIMD)
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  if (P.active && !P.active[b]) {
    if (lane == 0) {
      out_len[b] = 0;
      if (mark) mark[b] = 0;
      err[b] = 0;
    }
    return;
  }
  RMI_STAMP_DECL;
  RMI_STAMP(0);
  // ---- stage: every load of the row first (pool, observation, response head, length), then
  //      the LDS stores; a response longer than kStageResp takes a second batch
  {
    const uint32_t* pool4 = reinterpret_cast<const uint32_t*>(P.pool);
    const uint32_t* resp4 = sd.resp ? reinterpret_cast<const uint32_t*>(P.resp + b * (int64_t)P.resp_stride) : nullptr;
    const uint8_t* obsr = sd.obs ? P.obs + b * (int64_t)P.obs_stride : nullptr;
    uint32_t pv[4], rv[2];
    uint8_t ov[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int w = lane + 64 * k;
      pv[k] = 4 * w < sd.pool ? pool4[w] : 0u;
      ov[k] = lane + 64 * k < sd.obs && lane + 64 * k < P.obs_stride ? obsr[lane + 64 * k] : (uint8_t)0;
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int w = lane + 64 * k;
      rv[k] = 4 * w < sd.resp && 4 * w < kStageResp ? resp4[w] : 0u;
    }
    const int rl = sd.resp ? P.resp_len[b] : 0;
    // the row's scalars with the same batch: tag, condition, reward, the INT pieces' values
    // (lane i: piece i), and the TAG_CONST pieces' (offset, length) for every tag (lane
    // i * n_tags + t, when the pieces and tags fit the wave)
    const int tg_l = P.tag ? P.tag[b] : 0;
    const double rew_l = P.reward ? P.reward[b] : 0.0;
    int cond_l, rint_l;
    if (P.turn_exec) {  // the turn form: both from the turn record
      rint_l = P.turn_exec[b] == 0 || (((P.int_reward_tags >> (tg_l & 31)) & 1u) && tg_l < 32 &&
                                       (rew_l == 0.0 || rew_l == 1.0));
      cond_l = !(P.flags[b] & RMI_FLAG_DONE) && !P.last_turn;
    } else {
      cond_l = P.cond ? P.cond[b] : 1;
      rint_l = P.reward_int ? P.reward_int[b] : 0;
    }
    int iv = 0;
    if (lane < P.n_pieces && P.pieces[lane].kind == RMI_PT_INT) iv = P.ints[(int64_t)P.pieces[lane].a * B + b];
    const bool tc_pre = P.tag_const && P.n_tags > 0 && P.n_pieces * P.n_tags <= 64;
    int2 tcv = make_int2(0, 0);
    if (tc_pre && lane < P.n_pieces * P.n_tags) {
      const int pi = lane / P.n_tags, t = lane - pi * P.n_tags;
      if (P.pieces[pi].kind == RMI_PT_TAG_CONST) {
        const int k = 2 * (P.pieces[pi].a * P.n_tags + t);
        tcv = make_int2(P.tag_const[k], P.tag_const[k + 1]);
      }
    }
    pre_iv[lane] = iv;
    pre_tc[lane] = tcv;
    if (lane == 0) {
      pre_s[0] = tg_l;
      pre_s[1] = cond_l;
      pre_s[2] = rint_l;
      pre_d[0] = rew_l;
    }
    uint32_t* pl4 = reinterpret_cast<uint32_t*>(pl);
    uint32_t* rs4 = reinterpret_cast<uint32_t*>(rs);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int w = lane + 64 * k;
      if (4 * w < sd.pool) pl4[w] = pv[k];
      if (lane + 64 * k < sd.obs) ob[lane + 64 * k] = ov[k];
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int w = lane + 64 * k;
      if (4 * w < sd.resp && 4 * w < kStageResp) rs4[w] = rv[k];
    }
    for (int i = 256 + lane; i < sd.obs && i < P.obs_stride; i += 64) ob[i] = obsr[i];  // rows past 256 B
    const int rw = ((rl < sd.resp ? rl : sd.resp) + 3) >> 2;
    for (int w = kStageResp / 4 + lane; w < rw; w += 64) rs4[w] = resp4[w];
  }
  wave_sync();
  RMI_STAMP_WAIT(1);
  // the reward's cached text: its entry's load goes out now (lane 0), waited on at the reward
  // piece, behind the pieces before it
  bool has_rew = false;
  for (int i = 0; i < P.n_pieces; ++i) has_rew |= P.pieces[i].kind == RMI_PT_REWARD;
  const bool nc = P.num_cache != nullptr && has_rew;
  uint64_t nkey = 0;
  uint4 ne[4] = {};
  if (nc && lane == 0 && !pre_s[2]) {
    nkey = __builtin_bit_cast(uint64_t, pre_d[0]);
    const uint4* e = reinterpret_cast<const uint4*>(P.num_cache + 16 * (size_t)num_slot(nkey, P.num_cache_mask));
#pragma unroll
    for (int i = 0; i < 4; ++i) ne[i] = e[i];
  }
  const uint8_t* pool = sd.pool ? pl : P.pool;
  const int tg = pre_s[0];
  const bool tc_pre = P.tag_const && P.n_tags > 0 && P.n_pieces * P.n_tags <= 64;
  int pos = 0, mk = 0;
  bool over = false, unsup = false;
  for (int pi = 0; pi < P.n_pieces && !over && !unsup; ++pi) {
    const rmi_piece_t pc = P.pieces[pi];
    switch (pc.kind) {
      case RMI_PT_CONST:
        if (pos + pc.b > stride) {
          over = true;
          break;
        }
        put(row, pos, pool + pc.a, pc.b, lane);
        pos += pc.b;
        break;
      case RMI_PT_TAG_CONST: {
        const int2 ol = tc_pre ? pre_tc[pi * P.n_tags + tg]
                               : make_int2(P.tag_const[2 * (pc.a * P.n_tags + tg)], P.tag_const[2 * (pc.a * P.n_tags + tg) + 1]);
        const int o = ol.x, l = ol.y;
        if (pos + l > stride) {
          over = true;
          break;
        }
        put(row, pos, pool + o, l, lane);
        pos += l;
        break;
      }
      case RMI_PT_OBS: {
        const int l = P.obs_len[b];
        if (pos + l > stride) {
          over = true;
          break;
        }
        put(row, pos, sd.obs ? ob : P.obs + b * (int64_t)P.obs_stride, l, lane);
        pos += l;
        break;
      }
      case RMI_PT_INT:
      case RMI_PT_REWARD: {
        if (pc.kind == RMI_PT_REWARD) RMI_STAMP(2);
        if (lane == 0) {
          char* o = reinterpret_cast<char*>(num);
          int l;
          if (pc.kind == RMI_PT_INT) {
            l = py_int_repr(pi < 64 ? pre_iv[pi] : P.ints[(int64_t)pc.a * B + b], o);
          } else {
            const double r = pre_d[0];
#ifdef RMI_PROMPT_NO_REPR  // (timing variant only: the reward's text replaced by "0.0")
            (void)r;
            o[0] = '0', o[1] = '.', o[2] = '0';
            l = 3;
#else
            if (pre_s[2]) {
              l = py_int_repr((int64_t)r, o);
            } else {
              l = nc ? num_take(ne, nkey, o) : -1;
              if (l < 0) {
                l = py_float_repr(r, o, scr);
                // inserted from the rows whose early-loaded entry was empty, and from one row in 16:
                // thousands of rows of one launch miss on the same new value, and a compare-and-swap
                // from each would serialise them on one line (ragen_amd/csrc/bpe.hip wc_insert)
                if (nc && l > 0 && l <= 24 && (ne[0].x | ne[0].y) == 0u && (b & 15) == 0)
                  num_put(P.num_cache + 16 * (size_t)num_slot(nkey, P.num_cache_mask), nkey, o, l);
              }
            }
#endif
          }
          sh[0] = l;
        }
        wave_sync();
        const int l = sh[0];
        if (l < 0) {
          unsup = true;
          break;
        }
        if (pos + l > stride) {
          over = true;
          break;
        }
        put(row, pos, num, l, lane);
        pos += l;
        if (pc.kind == RMI_PT_REWARD) RMI_STAMP_WAIT(3);
        break;
      }
      case RMI_PT_RESPONSE: {
        const int tl = P.resp_len[b];
        const uint8_t* txt = tl <= sd.resp ? rs : P.resp + b * (int64_t)P.resp_stride;  // staged unless too long
        const int plen = P.enable_think ? 7 : 8;
        const uint8_t* pre = reinterpret_cast<const uint8_t*>(P.enable_think ? kThinkO : kAnsO);
        auto raw = [&](int i) -> uint8_t { return i < plen ? pre[i] : txt[i - plen]; };
        const int32_t* sp = P.spans + 4 * b;
        const int ts = sp[0], te = sp[1], as = sp[2], ae = sp[3];
        if (as < 0) {  // no match: llm_response is the raw (prefixed) response
          if (pos + plen + tl > stride) {
            over = true;
            break;
          }
          for (int i = lane; i < plen + tl; i += 64) row[pos + i] = raw(i);
          pos += plen + tl;
          break;
        }
        const int nt = P.enable_think ? te - ts : 0, na = ae - as;
        if (nt > stride || na > stride) {
          over = true;
          break;
        }
        for (int i = lane; i < nt; i += 64) th[i] = raw(ts + i);
        for (int i = lane; i < na; i += 64) an[i] = raw(as + i);
        wave_sync();
        bool lt = false;
        for (int i = lane; i < nt; i += 64) lt |= th[i] == '<';
        for (int i = lane; i < na; i += 64) lt |= an[i] == '<';
        const bool any_lt = __any(lt);
        // separator candidates of the answer (its first byte, then the full compare)
        int ncand = 0;
        for (int i0 = 0; i0 < na; i0 += 64) {
          const int i = i0 + lane;
          bool m = i + P.sep_len <= na;
          for (int k = 0; m && k < P.sep_len; ++k) m = an[i + k] == P.sep[k];
          ncand += __builtin_popcountll(__ballot(m));
        }
        wave_sync();
        if (lane == 0) {
          int t0 = 0, t1 = nt, a0 = 0, a1 = na;
          if (any_lt) {
            cascade(th, t0, t1);
            cascade(an, a0, a1);
          } else {
            strip(th, t0, t1);
            strip(an, a0, a1);
          }
          // actions = [a.strip() for a in action_content.split(sep) if a.strip()]; > K: re-join
          // (a cascade can make new separators: then always counted)
          bool rejoin = false;
          if (any_lt || ncand + 1 > P.K) {
            int n_act = 0, *ps = sh + 16, *pe = sh + 32;
            int seg = a0, i = a0;
            while (n_act <= P.K) {
              bool m = i + P.sep_len <= a1;
              for (int k = 0; m && k < P.sep_len; ++k) m = an[i + k] == P.sep[k];
              if (m || i >= a1) {
                int x = seg, y = m ? i : a1;
                strip(an, x, y);
                if (y > x) {
                  ps[n_act] = x, pe[n_act] = y;
                  ++n_act;
                }
                if (!m) break;
                i += P.sep_len;
                seg = i;
              } else {
                ++i;
              }
            }
            if (n_act > P.K) {  // the first K actions joined by " sep ", after the contents
              rejoin = true;
              int w = a1;
              for (int k = 0; k < P.K; ++k) {
                if (k) {
                  an[w++] = ' ';
                  for (int q = 0; q < P.sep_len; ++q) an[w++] = P.sep[q];
                  an[w++] = ' ';
                }
                for (int q = ps[k]; q < pe[k]; ++q) an[w++] = an[q];
              }
              a0 = a1;
              a1 = w;
            }
          }
          sh[0] = t0, sh[1] = t1, sh[2] = a0, sh[3] = a1, sh[4] = rejoin;
        }
        wave_sync();
        const int t0 = sh[0], t1 = sh[1], a0 = sh[2], a1 = sh[3];
        const int len = P.enable_think ? 7 + (t1 - t0) + 8 + 8 + (a1 - a0) + 9 : 8 + (a1 - a0) + 9;
        if (pos + len > stride) {
          over = true;
          break;
        }
        if (P.enable_think) {
          put(row, pos, reinterpret_cast<const uint8_t*>(kThinkO), 7, lane);
          pos += 7;
          put(row, pos, th + t0, t1 - t0, lane);
          pos += t1 - t0;
          put(row, pos, reinterpret_cast<const uint8_t*>(kThinkC), 8, lane);
          pos += 8;
        }
        put(row, pos, reinterpret_cast<const uint8_t*>(kAnsO), 8, lane);
        pos += 8;
        put(row, pos, an + a0, a1 - a0, lane);
        pos += a1 - a0;
        put(row, pos, reinterpret_cast<const uint8_t*>(kAnsC), 9, lane);
        pos += 9;
        break;
      }
      case RMI_PT_MARK:
        mk = pos;
        break;
      case RMI_PT_IF:
        if (!pre_s[1]) pi = P.n_pieces;
        break;
      default:
        unsup = true;
    }
    wave_sync();
  }
  if (over || unsup) {
    if (lane == 0) {
      out_len[b] = 0;
      if (mark) mark[b] = 0;
      err[b] = RMI_ERR_UNSUP;
    }
    return;
  }
  uint32_t* o4 = reinterpret_cast<uint32_t*>(out + b * (int64_t)stride);
  const uint32_t* r4 = reinterpret_cast<const uint32_t*>(row);
  for (int w = lane; w < (pos + 3) / 4; w += 64) {
    uint32_t v = r4[w];
    if (4 * w + 4 > pos) v &= 0xFFFFFFFFu >> (8 * (4 * w + 4 - pos));
    o4[w] = v;
  }
  if (lane == 0) {
    out_len[b] = pos;
    if (mark) mark[b] = mk;
    err[b] = 0;
  }
  RMI_STAMP(4);
}

// one wave per output row, kPadRows rows per workgroup: the row's arena slice and the tail,
// left-padded (element-wise 8-B loads and stores; consecutive lanes take consecutive columns;
// the loop unrolled so a wave has several loads in flight).  NT: nontemporal stores (a batch
// far past the caches, read by a later kernel).
#ifndef RMI_PAD_ROWS_PER_BLOCK
#define RMI_PAD_ROWS_PER_BLOCK 4
#endif
constexpr int kPadRows = RMI_PAD_ROWS_PER_BLOCK;

template <bool NT>
__device__ __forceinline__ void st_i64(int64_t* p, int64_t v) {
  if (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}
typedef long long i64x2 __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ void st_i64x2(int64_t* p, int64_t a, int64_t b) {  // p 16-B aligned
  const i64x2 v = {a, b};
  if (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<i64x2*>(p));
  else
    *reinterpret_cast<i64x2*>(p) = v;
}

// The one-column form (8-B stores), for outputs whose bases differ mod 16 B.
template <bool NT>
__global__ __launch_bounds__(64 * kPadRows) void pad_rows1_kernel(const int64_t* __restrict__ arena,
                                                                 int64_t arena_stride,
                                                                 const int32_t* __restrict__ arena_len,
                                                                 const int64_t* __restrict__ rows,
                                                                 const int64_t* __restrict__ tail, int n_tail,
                                                                 int64_t n_rows, int64_t S, int64_t pad_id,
                                                                 int64_t* __restrict__ ids, int64_t* __restrict__ am,
                                                                 int64_t* __restrict__ pos, uint8_t* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kPadRows + (threadIdx.x >> 6);
  if (i >= n_rows) return;
  const int64_t r = rows[i];
  const int64_t na = arena_len[r], n = na + n_tail;
  const int64_t cut = n > S ? n - S : 0;  // an overlong row keeps its last S tokens
  const int64_t pad = n > S ? 0 : S - n;
  const int64_t* src = arena + r * arena_stride;
  int64_t* io = ids + i * S;
  int64_t* ao = am + i * S;
  int64_t* po = pos + i * S;
#pragma unroll 4
  for (int64_t c = lane; c < S; c += 64) {
    const int64_t k = c - pad + cut;  // index into the row's n tokens
    const bool on = c >= pad;
    st_i64<NT>(io + c, !on ? pad_id : (k < na ? src[k] : tail[k - na]));
    st_i64<NT>(ao + c, on ? 1 : 0);
    st_i64<NT>(po + c, on ? c - pad + 1 : 0);
  }
  if (lane == 0) err[i] = n > S ? RMI_ERR_UNSUP : 0;
}

// Two columns per lane with 16-B stores (the store instructions are what bound the one-column
// form at 3.4-4.4 TB/s); a row starting at 8 mod 16 B stores its first column alone, an odd
// remainder its last.  The three outputs share the row's alignment (the launcher takes this form
// when their bases agree mod 16 B).
template <bool NT>
__global__ __launch_bounds__(64 * kPadRows) void pad_rows_kernel(const int64_t* __restrict__ arena,
                                                                 int64_t arena_stride,
                                                                 const int32_t* __restrict__ arena_len,
                                                                 const int64_t* __restrict__ rows,
                                                                 const int64_t* __restrict__ tail, int n_tail,
                                                                 int64_t n_rows, int64_t S, int64_t pad_id,
                                                                 int64_t* __restrict__ ids, int64_t* __restrict__ am,
                                                                 int64_t* __restrict__ pos, uint8_t* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kPadRows + (threadIdx.x >> 6);
  if (i >= n_rows) return;
  const int64_t r = rows[i];
  const int64_t na = arena_len[r], n = na + n_tail;
  const int64_t cut = n > S ? n - S : 0;  // an overlong row keeps its last S tokens
  const int64_t pad = n > S ? 0 : S - n;
  const int64_t* src = arena + r * arena_stride;
  int64_t* io = ids + i * S;
  int64_t* ao = am + i * S;
  int64_t* po = pos + i * S;
  auto id_at = [&](int64_t c) -> int64_t {
    const int64_t k = c - pad + cut;  // index into the row's n tokens
    return c < pad ? pad_id : (k < na ? src[k] : tail[k - na]);
  };
  const int64_t h = (reinterpret_cast<uintptr_t>(io) & 15u) ? 1 : 0;  // a lone first column
  const int64_t end = S - ((S - h) & 1);                               // [h, end): column pairs
  if (lane == 0 && h) {
    st_i64<NT>(io, id_at(0));
    st_i64<NT>(ao, 0 >= pad ? 1 : 0);
    st_i64<NT>(po, 0 >= pad ? 1 - pad : 0);
  }
  if (lane == 0 && end < S) {
    const int64_t c = S - 1;
    st_i64<NT>(io + c, id_at(c));
    st_i64<NT>(ao + c, c >= pad ? 1 : 0);
    st_i64<NT>(po + c, c >= pad ? c - pad + 1 : 0);
  }
#pragma unroll 2
  for (int64_t c = h + 2 * lane; c < end; c += 128) {
    const bool on0 = c >= pad, on1 = c + 1 >= pad;
    st_i64x2<NT>(io + c, id_at(c), id_at(c + 1));
    st_i64x2<NT>(ao + c, on0 ? 1 : 0, on1 ? 1 : 0);
    st_i64x2<NT>(po + c, on0 ? c - pad + 1 : 0, on1 ? c - pad + 2 : 0);
  }
  if (lane == 0) err[i] = n > S ? RMI_ERR_UNSUP : 0;
}

}  // namespace
}  // namespace rmi

#ifdef RMI_STAMPS
RMI_API int rmi_prompt_set_stamps(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(rmi::g_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -2;
}
#endif

RMI_API int rmi_pad_rows(const int64_t* arena, int64_t arena_stride, const int32_t* arena_len, const int64_t* rows,
                         int64_t n_rows, const int64_t* tail, int32_t n_tail, int64_t S, int64_t pad_id,
                         int64_t* input_ids, int64_t* attention_mask, int64_t* position_ids, uint8_t* err,
                         rmi_stream_t stream) {
  using namespace rmi;
  if (n_rows < 0 || S < 1 || n_tail < 0 || arena_stride < 1) return RMI_EINVAL;
  if (n_rows > 0x7FFFFFFF) return RMI_EUNSUP;
  if (n_rows == 0) return RMI_OK;
  if (!arena || !arena_len || !rows || (n_tail && !tail) || !input_ids || !attention_mask || !position_ids || !err)
    return RMI_EINVAL;
#ifndef RMI_PAD_NT_BYTES
#define RMI_PAD_NT_BYTES (256ll << 20)  // outputs past the Infinity Cache: streamed stores
#endif
  const dim3 grid((unsigned)((n_rows + kPadRows - 1) / kPadRows)), block(64 * kPadRows);
  const bool nt = n_rows * S * 24 > RMI_PAD_NT_BYTES;
  const uintptr_t a16 = reinterpret_cast<uintptr_t>(input_ids) & 15u;
  const bool pairs = (reinterpret_cast<uintptr_t>(attention_mask) & 15u) == a16 &&
                     (reinterpret_cast<uintptr_t>(position_ids) & 15u) == a16 && (a16 & 7u) == 0;
#define RMI_PAD_LAUNCH(K_)                                                                                        \
  hipLaunchKernelGGL(K_, grid, block, 0, as_stream(stream), arena, arena_stride, arena_len, rows, tail, (int)n_tail, \
                     n_rows, S, pad_id, input_ids, attention_mask, position_ids, err)
  if (pairs && nt)
    RMI_PAD_LAUNCH(pad_rows_kernel<true>);
  else if (pairs)
    RMI_PAD_LAUNCH(pad_rows_kernel<false>);
  else if (nt)
    RMI_PAD_LAUNCH(pad_rows1_kernel<true>);
  else
    RMI_PAD_LAUNCH(pad_rows1_kernel<false>);
#undef RMI_PAD_LAUNCH
  return launch_status();
}

RMI_API int rmi_prompt_text(const rmi_prompt_t* prog, int64_t B, uint8_t* out, int32_t stride, int32_t* out_len,
                            int32_t* mark, uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (!prog || B < 0 || stride <= 0 || stride % 4 || prog->n_pieces < 0) return RMI_EINVAL;
  if (stride > kMaxStride || prog->n_pieces > RMI_PROMPT_MAX_PIECES || B > 0x7FFFFFFF || prog->sep_len > 16 ||
      prog->K > RMI_PARSE_MAX_NAMES)
    return RMI_EUNSUP;
  if (B == 0) return RMI_OK;
  if (!out || !out_len || !err) return RMI_EINVAL;
  bool need_resp = false, need_obs = false, need_int = false, need_rew = false, need_if = false, need_tag = false;
  for (int i = 0; i < prog->n_pieces; ++i) {
    const int k = prog->pieces[i].kind;
    need_resp |= k == RMI_PT_RESPONSE;
    need_obs |= k == RMI_PT_OBS;
    need_int |= k == RMI_PT_INT;
    need_rew |= k == RMI_PT_REWARD;
    need_if |= k == RMI_PT_IF;
    need_tag |= k == RMI_PT_TAG_CONST;
    if (k == RMI_PT_CONST && (prog->pieces[i].b < 0 || (prog->pieces[i].b > 0 && !prog->pool))) return RMI_EINVAL;
  }
  if ((need_resp && (!prog->resp || !prog->resp_len || !prog->spans || prog->sep_len < 1 || prog->K < 0)) ||
      (need_obs && (!prog->obs || !prog->obs_len)) || (need_int && !prog->ints) || (need_rew && !prog->reward) ||
      (need_if && !prog->cond && !prog->turn_exec) || (prog->turn_exec && !prog->flags) || (need_tag && (!prog->tag_const || !prog->pool || prog->n_tags < 1)))
    return RMI_EINVAL;
  // row (stride + 64) + think (stride) + answer and its re-joined form (2 * stride + 64) + number
  // (64) + hand-off and piece bounds (48 ints) + digit scratch (64) + the staged pool,
  // observation and response
  const StageDims sd = stage_dims(*prog, (int)stride, need_obs, need_resp);
  const size_t lds = (size_t)stride + 64 + (size_t)stride + 2 * (size_t)stride + 64 + 64 + 48 * 4 + 64 +
                     (size_t)sd.pool + (size_t)sd.obs + (size_t)sd.resp + 8 + 8 + 64 * 4 + 64 * 8 + 16 + 8;
  hipLaunchKernelGGL(prompt_text_kernel, dim3((unsigned)B), dim3(64), lds, as_stream(stream), *prog, B, out,
                     (int)stride, out_len, mark, err, sd);
  return launch_status();
}
