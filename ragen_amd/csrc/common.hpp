// common.hpp — shared device helpers for the gfx950 rollout kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ragen_amd.h"

#define RMI_API extern "C" __attribute__((visibility("default")))

namespace rmi {

// Diagnostic builds only (tools/stampbench.hip, tools/prof_fl_stamps.py define RMI_STAMPS): per-wave s_memtime /
// s_memrealtime stamps at phase boundaries.  Compiled out of the library.
// The stamps stay in SGPRs until the wave's last one, so the instrumentation adds no memory
// round trip inside the phases it measures (one s_memtime each; s_memrealtime at 0 and 4).
#ifdef RMI_STAMPS
__device__ unsigned long long* g_stamps;
#define RMI_STAMP_DECL unsigned long long rmi_st_[5], rmi_rt0_ = __builtin_amdgcn_s_memrealtime()
#define RMI_STAMP(i)                                 \
  do {                                               \
    rmi_st_[i] = __builtin_amdgcn_s_memtime();       \
    if ((i) == 4) {                                  \
      const unsigned long long rt4 = __builtin_amdgcn_s_memrealtime(); \
      if ((threadIdx.x & 63) == 0) {                 \
        unsigned long long* g = g_stamps + (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 16; \
        for (int s_ = 0; s_ < 5; ++s_) g[2 * s_] = rmi_st_[s_]; \
        g[1] = rmi_rt0_;                             \
        g[9] = rt4;                                  \
      }                                              \
    }                                                \
  } while (0)
#define RMI_STAMP_WAIT(i)          \
  do {                             \
    __builtin_amdgcn_s_waitcnt(0); \
    RMI_STAMP(i);                  \
  } while (0)
#else
#define RMI_STAMP_DECL \
  do {                 \
  } while (0)
#define RMI_STAMP(i) \
  do {               \
  } while (0)
#define RMI_STAMP_WAIT(i) RMI_STAMP(i)
#endif


constexpr int kBlock = 256;  // 4 waves of 64 lanes
constexpr int kMaxK = 8;     // max actions per turn handled by the step kernels

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? RMI_OK : RMI_EDEVICE;
}

inline hipStream_t as_stream(rmi_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
// A device -> pinned-host copy enqueued on s (capi.hip): a kernel storing into the host buffer's
// device mapping when the runtime reports one (and both ends are 4-B aligned, bytes % 4 == 0),
// else hipMemcpyAsync (whose blit started ~11 us after the stream's last kernel here).
int readback_async(void* host, const void* dev, size_t bytes, hipStream_t s);

// 64-lane inclusive prefix sum on DPP (no LDS): row_shr 1/2/4/8 inside each 16-lane row,
// then row_bcast:15 / row_bcast:31 carry the row totals across rows (gfx9 DPP).
__device__ __forceinline__ int wave_inclusive_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// LDS hand-off between the lanes of ONE wave.  The wave-per-row kernels put several waves in a
// workgroup (a one-wave workgroup per row caps how many rows a CU holds at once); the waves
// work on separate rows and never share LDS, so a wavefront-scope release / acquire around a
// wave barrier replaces __syncthreads().
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// --------------------------------------------------------------- PCG64 (numpy)
// numpy PCG64 = pcg_setseq_128_xsl_rr_64: step state = state*M + inc (mod 2^128),
// then output XSL-RR of the NEW state; Generator.random() = (out >> 11) * 2^-53.
// (verified bit-exact against numpy in tests/test_oracle.py.)
struct Pcg64 {
  uint64_t s_hi, s_lo, i_hi, i_lo;

  __device__ __forceinline__ uint64_t next64() {
    const uint64_t m_hi = 0x2360ED051FC65DA4ull, m_lo = 0x4385DF649FCCF645ull;
    uint64_t lo = s_lo * m_lo;
    uint64_t hi = __umul64hi(s_lo, m_lo) + s_lo * m_hi + s_hi * m_lo;
    uint64_t nlo = lo + i_lo;
    hi += i_hi + (nlo < lo ? 1ull : 0ull);
    s_lo = nlo;
    s_hi = hi;
    uint64_t x = s_hi ^ s_lo;
    unsigned rot = (unsigned)(s_hi >> 58);
    return (x >> rot) | (x << ((64u - rot) & 63u));
  }
  __device__ __forceinline__ double next_double() {
    return (double)(next64() >> 11) * (1.0 / 9007199254740992.0);
  }
};

__device__ __forceinline__ Pcg64 load_pcg(const uint64_t* rng, int64_t B, int64_t b) {
  Pcg64 p;
  p.s_hi = rng[b];
  p.s_lo = rng[B + b];
  p.i_hi = rng[2 * B + b];
  p.i_lo = rng[3 * B + b];
  return p;
}
__device__ __forceinline__ void store_pcg(uint64_t* rng, int64_t B, int64_t b, const Pcg64& p) {
  rng[b] = p.s_hi;
  rng[B + b] = p.s_lo;
}

// ------------------------------------------------------------ the turn driver (A3)
// EnvStateManager.step for one env (es_manager.py:149-169):
//   valid = [ids of known names]           (_extract_map_valid_actions :230-240)
//   execute valid[:max - num_actions] one by one, stop at the first done (:116-128)
//   penalty if len(valid) != len(actions) or not valid                    (:158-159)
//   num_actions += executed; rewards.append(acc); done => terminated, truncated = !success
//   cap: num_actions >= max and not done => truncated = terminated = True    (:163-166)
// Env::step(a, reward&, done&, effective&, success&) -> false on an invalid action id.
struct TurnOut {
  double acc;
  uint8_t info;
  uint8_t exec;
  bool stepped_any_state;  // the env's state may have changed
};

// Per-env element addressing: a wave-uniform base pointer plus this env's element index.  With
// Ix = uint32_t the byte offset is formed in 32 bits, so the access compiles to
// global_load/store v_offset, s[base] (no 64-bit address arithmetic per access, which on a
// latency-bound wave sits ahead of its loads); the caller guarantees the offset fits
// (kOff32MaxB envs of at most kOff32MaxRow bytes each).  Ix = int64_t is plain pointer
// arithmetic.
#ifndef RMI_OFF32_MAX_B  // (a diagnostic variant sets 0: every launch takes the 64-bit form)
#define RMI_OFF32_MAX_B ((int64_t)1 << 26)
#endif
constexpr int64_t kOff32MaxB = RMI_OFF32_MAX_B;
constexpr int kOff32MaxRow = 64;
template <class Ix, class T>
__device__ __forceinline__ T* elem(T* base, int64_t i
#ifdef RMI_ELEM_CHECK  // (diagnostic variant: an index outside the offset form's range is reported and clamped)
                                   , int line = __builtin_LINE()
#endif
) {
#ifdef RMI_ELEM_CHECK
  if (i < 0 || (sizeof(Ix) == 4 && (uint64_t)i * sizeof(T) > 0xFFFFFFFFull)) {
    printf("RMI_ELEM_CHECK line %d index %lld block %d thread %d\n", line, (long long)i, (int)blockIdx.x,
           (int)threadIdx.x);
    i = 0;
  }
#endif
  if constexpr (sizeof(Ix) == 4) {
    uint32_t off = (uint32_t)i * (uint32_t)sizeof(T);
    // (a byte array's offset would otherwise fold back into 64-bit "i & 0xffffffff")
    if constexpr (sizeof(T) == 1) asm("" : "+v"(off));
    return (T*)((const char*)base + off);
  } else
    return base + i;
}

// Actions of one env packed into a u64 (K <= 8 bytes), loaded once per turn: the at most three
// aligned dwords that hold the row's K bytes, issued back to back with clamped addresses (never
// a dword past the one holding the row's last byte, so never outside the row's page) and
// funnel-shifted afterwards -- 3 load instructions instead of one per action slot (8), which
// shortened the Sokoban turn's load phase.
// With K == 0 (no action slots; `acts` may then be null) the loads read `alt`, any valid byte,
// and the result is 0.  No branch around the loads: a branch here makes the compiler fetch the
// actions pointer from the kernel arguments only inside it, after the turn's other loads (a
// second scalar round trip ahead of the action loads).
__device__ __forceinline__ uint64_t load_actions(const int8_t* acts, int K, const uint8_t* alt) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(K > 0 ? reinterpret_cast<const void*>(acts)
                                                         : reinterpret_cast<const void*>(alt));
  const int Kc = K > 0 ? K : 1;
  const uint32_t* base = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const int sh = (int)(a & 3u);
  const int last = (sh + Kc - 1) >> 2;  // the dword holding the row's last byte (0..2)
  const uint32_t d0 = base[0], d1 = base[last >= 1 ? 1 : 0], d2 = base[last >= 2 ? 2 : last];
  const uint64_t lo = ((uint64_t)d1 << 32) | d0;
  // bytes sh .. sh + 7 of d0 | d1 | d2
  const uint64_t v = sh ? (lo >> (8 * sh)) | ((uint64_t)d2 << (64 - 8 * sh)) : lo;
  return K >= 8 ? v : (K <= 0 ? 0ull : v & ((1ull << (8 * K)) - 1ull));
}

// The same for env b of a [B, K] action array at `acts` (K > 0) or, with K == 0, the byte `alt`
// [b]: the clamped dword loads address base + 32-bit offsets under Ix = uint32_t.
template <class Ix>
__device__ __forceinline__ uint64_t load_actions_at(const int8_t* acts, int64_t b, int K, const uint8_t* alt) {
  if constexpr (sizeof(Ix) != 4) {
    return load_actions(acts + b * (int64_t)K, K, alt + b);
  } else {
    const char* base = K > 0 ? (const char*)acts : (const char*)alt;  // uniform
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(base) & 3u);
    const char* abase = base - mis;                                   // 4-aligned, uniform
    const int Kc = K > 0 ? K : 1;
    const uint32_t o = (uint32_t)b * (uint32_t)(K > 0 ? K : 1) + mis;  // the row's first byte from abase
    const uint32_t o4 = o & ~3u;
    const int sh = (int)(o & 3u);
    const int last = (sh + Kc - 1) >> 2;
    const uint32_t d0 = *(const uint32_t*)(abase + o4), d1 = *(const uint32_t*)(abase + (o4 + (last >= 1 ? 4u : 0u)));
    const uint32_t d2 = *(const uint32_t*)(abase + (o4 + 4u * (uint32_t)(last >= 2 ? 2 : last)));
    const uint64_t lo = ((uint64_t)d1 << 32) | d0;
    const uint64_t v = sh ? (lo >> (8 * sh)) | ((uint64_t)d2 << (64 - 8 * sh)) : lo;
    return K >= 8 ? v : (K <= 0 ? 0ull : v & ((1ull << (8 * K)) - 1ull));
  }
}

template <class Env>
__device__ __forceinline__ TurnOut run_turn(Env& e, uint64_t packed_acts, int n_act, int K, int32_t& num_actions,
                                            uint8_t& flags, int32_t& n_turns, double& penalty, int max_actions,
                                            double format_penalty, uint8_t& err) {
  TurnOut o;
  o.acc = 0.0;
  o.info = 0;
  o.exec = 0;
  o.stepped_any_state = false;
  flags &= (uint8_t)~RMI_FLAG_DONE;  // done-ness is decided per stepped turn (:168)
  const int left = max_actions - num_actions;
  int nv = 0;
  bool stop = false, succ_last = false, turn_done = false;
  if (n_act > K) n_act = K;
#pragma unroll 1
  for (int k = 0; k < n_act; ++k) {
    const int a = (int)(int8_t)(uint8_t)(packed_acts >> (8 * k));
    if (a == 0) continue;  // name not in action_lookup: dropped (es_manager.py:239)
    if (!stop && nv < left) {
      double r;
      bool done, eff, succ;
      if (!e.step(a, r, done, eff, succ)) {
        err |= RMI_ERR_ACTION;
        stop = true;  // the reference raises here; the rest of the turn is not executed
      } else {
        o.acc += r;
        o.exec++;
        o.stepped_any_state = true;
        o.info = (uint8_t)(RMI_INFO_PRESENT | (eff ? RMI_INFO_EFFECTIVE : 0) | RMI_INFO_VALID |
                           (succ ? RMI_INFO_SUCCESS : 0));
        succ_last = succ;
        if (done) {
          stop = true;
          turn_done = true;
        }
      }
    }
    nv++;
  }
  if (nv != n_act || nv == 0) penalty += format_penalty;
  num_actions += o.exec;
  n_turns += 1;
  if (turn_done) {
    flags |= RMI_FLAG_TERMINATED | RMI_FLAG_DONE;
    flags = succ_last ? (uint8_t)(flags & ~RMI_FLAG_TRUNCATED) : (uint8_t)(flags | RMI_FLAG_TRUNCATED);
  } else if (num_actions >= max_actions) {
    flags |= RMI_FLAG_TERMINATED | RMI_FLAG_TRUNCATED | RMI_FLAG_DONE;
  }
  return o;
}

// Validation shared by every *_step_turn entry point (an empty batch is always fine).
// ------------------------------------------------------- fused end of rollout (kFin)
// A rollout's last turn launch (Sokoban, FrozenLake) also does rmi_rollout_finalize's work (episode.hip): per env
// get_rollout_states metrics (es_manager.py:173-207), the trajectory score sum(turn rewards)
// + penalty, and _normalize_score_tensor (ctx_manager.py:175-226) over uniform contiguous
// groups of fin.group_size envs, which the launcher only accepts when every group lies in one
// wave.  The episode record of the first 8 turns is loaded with the turn's other loads (no
// extra round trip); the group sums are the same xor butterflies as finalize_kernel's
// wave_sum restricted to the group's lanes (the lanes outside a group only ever add exact
// zeros there), so every output is bit-identical to the separate launch.
constexpr int kFinT = 8;  // turns of the record loaded up front
struct FinRecord {
  double r[kFinT];
  uint8_t info[kFinT];
  template <class Ix = int64_t>
  __device__ __forceinline__ void load(const rmi_episode_t& ep, int64_t bc) {
    const int64_t B = ep.B;
#pragma unroll
    for (int k = 0; k < kFinT; ++k) {
      const int64_t t = k < ep.T ? k : ep.T - 1;  // clamped, always valid
      r[k] = *elem<Ix>(ep.turn_reward + t * B, bc);
      info[k] = *elem<Ix>(ep.turn_info + t * B, bc);
    }
  }
  __device__ __forceinline__ void set(int turn, double acc, uint8_t inf) {
#pragma unroll
    for (int k = 0; k < kFinT; ++k)
      if (k == turn) {
        r[k] = acc;
        info[k] = inf;
      }
  }
};

template <int LPE>
__device__ __forceinline__ double group_sum(double x, int gs) {  // xor butterfly over gs envs
  for (int o = gs >> 1; o >= 1; o >>= 1) x += __shfl_xor(x, o * LPE, 64);
  return x;
}

template <int LPE, class Ix = int64_t>
__device__ __forceinline__ void finalize_envs(const rmi_episode_t& ep, const rmi_finalize_t& fin, const FinRecord& rec,
                                              int64_t b, bool writer, uint8_t flags, int32_t n_turns,
                                              int32_t num_actions, double penalty, int acted_turn, double acc,
                                              uint8_t acc_info) {
  const int64_t B = ep.B;
  double score = 0.0;  // python sum over the turns, in turn order
  int eff = 0, val = 0, present = 0;
#pragma unroll
  for (int k = 0; k < kFinT; ++k)
    if (k < ep.T) {
      score += rec.r[k];
      present |= rec.info[k] & RMI_INFO_PRESENT;
      eff += (rec.info[k] >> 1) & 1;
      val += (rec.info[k] >> 2) & 1;
    }
  for (int t = kFinT; t < ep.T; ++t) {  // long episodes only
    const int64_t bc = b < B ? b : B - 1;
    const bool mine = t == acted_turn;  // written by this launch: use the registers
    const uint8_t inf = mine ? acc_info : *elem<Ix>(ep.turn_info + (int64_t)t * B, bc);
    score += mine ? acc : *elem<Ix>(ep.turn_reward + (int64_t)t * B, bc);
    present |= inf & RMI_INFO_PRESENT;
    eff += (inf >> 1) & 1;
    val += (inf >> 2) & 1;
  }
  const float scf = (float)score, pf = (float)penalty, x = scf + pf;
  if (writer) {
    if (fin.score) *elem<Ix>(fin.score, b) = scf;
    if (fin.pen) *elem<Ix>(fin.pen, b) = pf;
    if (fin.metrics) {
      const double nt = (double)n_turns;
      double* m = elem<Ix>(fin.metrics, 4 * b);
      m[0] = ((flags & RMI_FLAG_TERMINATED) && !(flags & RMI_FLAG_TRUNCATED)) ? 1.0 : 0.0;
      m[1] = (double)num_actions;
      m[2] = present ? (double)eff / nt : __builtin_nan("");
      m[3] = present ? (double)val / nt : __builtin_nan("");
    }
  }
  if (!fin.norm) return;
  const int gs = fin.group_size, method = fin.method;  // uniform; all lanes reach the shuffles
  const double md = group_sum<LPE>(0.0 + (double)x, gs) / (double)gs;
  const float mean = (float)md;
  float sd = 0.0f;
  if (method == RMI_NORM_MEAN_STD || method == RMI_NORM_ASYM_CLIP) {
    const double d = (double)x - md;
    const double q = group_sum<LPE>(0.0 + d * d, gs);
    sd = gs > 1 ? (float)sqrt(q / (double)(gs - 1)) : __builtin_nanf("");
  }
  const bool use = sd > 1e-6f;
  float y;
  if (method == RMI_NORM_IDENTITY) y = x;
  else if (method == RMI_NORM_MEAN) y = x - mean;
  else {
    y = use ? (x - mean) / (sd + 1e-6f) : 0.0f;
    if (method == RMI_NORM_ASYM_CLIP) y = fminf(fmaxf(y, -1.0f), 3.0f);
  }
  if (writer) *elem<Ix>(fin.norm, b) = y;
}

inline int check_turn_args(const rmi_episode_t* ep, const rmi_turn_t* in) {
  if (!ep || !in || ep->B < 0 || ep->T <= 0) return RMI_EINVAL;
  if (in->K < 0 || in->K > kMaxK || in->turn < 0 || in->turn >= ep->T) return RMI_EINVAL;
  // the record's counters are u8: num_actions <= cap, n_turns <= T
  if (ep->T > 255 || in->max_actions_per_traj > 255) return RMI_EUNSUP;
  if (ep->B == 0) return 1;
  if (!ep->num_actions || !ep->flags || !ep->n_turns || !ep->penalty || !ep->turn_reward || !ep->turn_info ||
      !ep->turn_exec || (in->K > 0 && !in->actions) || !in->n_actions)
    return RMI_EINVAL;
  return RMI_OK;
}

}  // namespace rmi
