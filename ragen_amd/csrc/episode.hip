// episode.hip — per-trajectory reductions after the turn loop (gfx950).
//
//  rmi_rollout_metrics   EnvStateManager.get_rollout_states   (es_manager.py:173-207)
//  rmi_trajectory_scores ctx_manager scores/penalty tensors    (ctx_manager.py:64-65, :217, :282)
//  rmi_group_normalize   ContextManager._normalize_score_tensor (ctx_manager.py:175-226)
//  rmi_filter_groups     _filter_rollout                        (agent_trainer.py:461-500)
//  rmi_row_sum           rm_scores.sum(-1)                      (agent_trainer.py:467)
//
// Segmented reductions: one 64-lane wave per segment / row, DPP-free __shfl_xor trees in
// fp64 (fixed order => bit-reproducible run to run and independent of the launch grid).
#include <math.h>

#include "common.hpp"

namespace rmi {
namespace {

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}
struct EnvTotals {
  double score;
  int eff, val, present;
};
// Trajectory score sum(turn rewards) (python sum, turn order) and the turn-info counts of env
// i.  The loads of a chunk of 8 turns are issued together (clamped, always-valid addresses),
// so an env costs one memory round trip per 8 turns instead of one per turn.
template <bool kInfo>
__device__ __forceinline__ EnvTotals env_totals(const rmi_episode_t& ep, int64_t i) {
  const int64_t B = ep.B;
  EnvTotals e;
  e.score = 0.0;
  e.eff = e.val = e.present = 0;
  for (int t0 = 0; t0 < ep.T; t0 += 8) {
    double r[8];
    uint8_t inf[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t t = min(t0 + k, ep.T - 1);
      r[k] = ep.turn_reward[t * B + i];
      if (kInfo) inf[k] = ep.turn_info[t * B + i];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (t0 + k < ep.T) {
        e.score += r[k];
        if (kInfo) {
          e.present |= inf[k] & RMI_INFO_PRESENT;
          e.eff += (inf[k] >> 1) & 1;
          e.val += (inf[k] >> 2) & 1;
        }
      }
    }
  }
  return e;
}

// get_rollout_states (es_manager.py:173-207): success, num_actions, and the per-info-key means
// over turns (turns without an executed action count in the denominator, NaN if none had one)
__device__ __forceinline__ void env_metrics(const rmi_episode_t& ep, int64_t i, const EnvTotals& e,
                                            double* __restrict__ out) {
  const uint8_t f = ep.flags[i];
  const double nt = (double)ep.n_turns[i];
  out[4 * i + 0] = ((f & RMI_FLAG_TERMINATED) && !(f & RMI_FLAG_TRUNCATED)) ? 1.0 : 0.0;
  out[4 * i + 1] = (double)ep.num_actions[i];
  out[4 * i + 2] = e.present ? (double)e.eff / nt : __builtin_nan("");
  out[4 * i + 3] = e.present ? (double)e.val / nt : __builtin_nan("");
}

__global__ __launch_bounds__(kBlock) void rollout_metrics_kernel(rmi_episode_t ep, double* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (b >= ep.B) return;
  env_metrics(ep, b, env_totals<true>(ep, b), out);
}

__global__ __launch_bounds__(kBlock) void trajectory_scores_kernel(rmi_episode_t ep, float* __restrict__ score,
                                                                   float* __restrict__ pen) {
  const int64_t b = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (b >= ep.B) return;
  score[b] = (float)env_totals<false>(ep, b).score;
  if (pen) pen[b] = (float)ep.penalty[b];
}

// one wave per segment; 4 segments per 256-thread workgroup
__global__ __launch_bounds__(kBlock) void group_normalize_kernel(const float* __restrict__ score,
                                                                 const float* __restrict__ pen,
                                                                 const int32_t* __restrict__ seg, int G, int B,
                                                                 int method, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (g >= G) return;
  const int lo = seg[g], hi = seg[g + 1], n = hi - lo;
  if (n <= 0 || lo < 0 || hi > B) return;  // malformed segments are never read past [0, B)
  double s = 0.0;
  for (int i = lo + lane; i < hi; i += 64) s += (double)(score[i] + (pen ? pen[i] : 0.0f));
  s = wave_sum(s);
  const float mean = (float)(s / (double)n);
  float sd = 0.0f;
  if (method == RMI_NORM_MEAN_STD || method == RMI_NORM_ASYM_CLIP) {
    const double md = s / (double)n;
    double q = 0.0;
    for (int i = lo + lane; i < hi; i += 64) {
      const double d = (double)(score[i] + (pen ? pen[i] : 0.0f)) - md;
      q += d * d;
    }
    q = wave_sum(q);
    sd = n > 1 ? (float)sqrt(q / (double)(n - 1)) : __builtin_nanf("");  // torch.std: unbiased
  }
  const bool use = sd > 1e-6f;  // std.abs().max() > 1e-6 (NaN compares false)
  for (int i = lo + lane; i < hi; i += 64) {
    const float x = score[i] + (pen ? pen[i] : 0.0f);
    float y;
    if (method == RMI_NORM_IDENTITY) y = x;
    else if (method == RMI_NORM_MEAN) y = x - mean;
    else {
      y = use ? (x - mean) / (sd + 1e-6f) : 0.0f;
      if (method == RMI_NORM_ASYM_CLIP) y = fminf(fmaxf(y, -1.0f), 3.0f);
    }
    out[i] = y;
  }
}

__global__ __launch_bounds__(kBlock) void row_sum_kernel(const float* __restrict__ x, int64_t B, int64_t L,
                                                         float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (r >= B) return;
  double s = 0.0;
  for (int64_t i = lane; i < L; i += 64) s += (double)x[r * L + i];
  s = wave_sum(s);
  if (lane == 0) out[r] = (float)s;
}

// ---- rollout filter: per-group stats, then a deterministic top-k by a bitonic sort in LDS
constexpr int kFilterThreads = 1024;
constexpr int kFilterMaxG = 8192;

__device__ __forceinline__ uint32_t orderable(float f) {  // monotone float -> u32 (NaN = largest)
  if (f != f) return 0xffffffffu;
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// per-group statistics of _filter_rollout (agent_trainer.py:466-469): unbiased std (NaN for a
// group of one, as torch), max and mean of the group's row scores; fp64 accumulation.
__device__ __forceinline__ void group_stats(const float* __restrict__ x, int gs, float& sd, float& mx, float& mean) {
  double s = 0.0;
  mx = -INFINITY;
  for (int i = 0; i < gs; ++i) {
    s += (double)x[i];
    mx = fmaxf(mx, x[i]);
  }
  const double m = s / gs;
  double q = 0.0;
  for (int i = 0; i < gs; ++i) q += ((double)x[i] - m) * ((double)x[i] - m);
  sd = gs > 1 ? (float)sqrt(q / (gs - 1)) : __builtin_nanf("");
  mean = (float)m;
}

__global__ __launch_bounds__(kFilterThreads) void filter_kernel(const float* __restrict__ scores, int G, int gs,
                                                                int k, int type, float* __restrict__ g_std,
                                                                float* __restrict__ g_max, float* __restrict__ g_mean,
                                                                uint8_t* __restrict__ keep,
                                                                double* __restrict__ metrics) {
  __shared__ uint64_t key[kFilterMaxG];
  __shared__ double red[6][kFilterThreads / 64];
  int P = 1;
  while (P < G) P <<= 1;
  double a_std = 0, a_max = 0, a_mean = 0;
  for (int g = threadIdx.x; g < P; g += kFilterThreads) {
    if (g < G) {
      float sd, mx, m;
      group_stats(scores + (int64_t)g * gs, gs, sd, mx, m);
      g_std[g] = sd;
      g_max[g] = mx;
      g_mean[g] = m;
      a_std += sd;
      a_max += mx;
      a_mean += m;
      const float kf = type == 1 ? -sd : sd;
      key[g] = ((uint64_t)orderable(kf) << 32) | (uint64_t)(0xffffffffu - (uint32_t)g);
    } else {
      key[g] = 0;  // padding sorts last
    }
  }
  __syncthreads();
  // bitonic sort, descending
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < P; i += kFilterThreads) {
        const int j = i ^ stride;
        if (j > i) {
          const bool desc = (i & size) == 0;
          const uint64_t a = key[i], bb = key[j];
          if ((a < bb) == desc) {
            key[i] = bb;
            key[j] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int g = threadIdx.x; g < G; g += kFilterThreads) keep[g] = 0;
  __syncthreads();
  double c_std = 0, c_max = 0, c_mean = 0;
  for (int i = threadIdx.x; i < k; i += kFilterThreads) {
    const int g = (int)(0xffffffffu - (uint32_t)(key[i] & 0xffffffffu));
    keep[g] = 1;
    c_std += g_std[g];
    c_max += g_max[g];
    c_mean += g_mean[g];
  }
  double v[6] = {a_std, a_max, a_mean, c_std, c_max, c_mean};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const double t = wave_sum(v[j]);
    if (lane == 0) red[j][w] = t;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    double t = 0;
    for (int i = 0; i < kFilterThreads / 64; ++i) t += red[threadIdx.x][i];
    const double d = threadIdx.x < 3 ? (double)G : (double)k;
    metrics[threadIdx.x] = (float)(t / d);  // torch f32 .mean()
  }
}

// G > kFilterMaxG (no LDS sort): the group statistics in parallel, then one workgroup selects
// the same set the sort would — the k largest (key, -index) pairs — by a 4-pass radix select
// of the threshold key over LDS histograms, and takes the tied groups at the threshold in
// ascending index order with a block-wide prefix count.  The reductions are fp64 as above.
__global__ __launch_bounds__(kBlock) void filter_stats_kernel(const float* __restrict__ scores, int G, int gs,
                                                              float* __restrict__ g_std, float* __restrict__ g_max,
                                                              float* __restrict__ g_mean) {
  const int g = blockIdx.x * kBlock + threadIdx.x;
  if (g >= G) return;
  float sd, mx, m;
  group_stats(scores + (int64_t)g * gs, gs, sd, mx, m);
  g_std[g] = sd;
  g_max[g] = mx;
  g_mean[g] = m;
}

__device__ __forceinline__ uint32_t filter_key(const float* g_std, int g, int type) {
  const float sd = g_std[g];
  return orderable(type == 1 ? -sd : sd);
}

__global__ __launch_bounds__(kFilterThreads) void filter_select_kernel(int G, int k, int type,
                                                                       const float* __restrict__ g_std,
                                                                       const float* __restrict__ g_max,
                                                                       const float* __restrict__ g_mean,
                                                                       uint8_t* __restrict__ keep,
                                                                       double* __restrict__ metrics) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t sel[2];  // chosen bin, keys still to take below it
  __shared__ uint32_t wcount[kFilterThreads / 64];
  __shared__ double red[6][kFilterThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // radix select of the threshold T: #(key > T) < k <= #(key >= T)
  uint32_t prefix = 0, pmask = 0, need = (uint32_t)k;
  for (int shift = 24; shift >= 0 && k > 0; shift -= 8) {
    for (int i = tid; i < 256; i += kFilterThreads) hist[i] = 0;
    __syncthreads();
    for (int g = tid; g < G; g += kFilterThreads) {
      const uint32_t key = filter_key(g_std, g, type);
      if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t cum = 0;
      int b = 255;
      for (; b > 0; --b) {
        if (cum + hist[b] >= need) break;
        cum += hist[b];
      }
      sel[0] = (uint32_t)b;
      sel[1] = need - cum;
    }
    __syncthreads();
    prefix |= sel[0] << shift;
    pmask |= 255u << shift;
    need = sel[1];
    __syncthreads();
  }
  // keep = key > T, or key == T among the first `need` such groups in index order
  double c_std = 0, c_max = 0, c_mean = 0, a_std = 0, a_max = 0, a_mean = 0;
  uint32_t base = 0;
  for (int g0 = 0; g0 < G; g0 += kFilterThreads) {
    const int g = g0 + tid;
    uint32_t key = 0;
    bool eq = false;
    if (g < G) {
      key = filter_key(g_std, g, type);
      eq = k > 0 && key == prefix;
      a_std += g_std[g];
      a_max += g_max[g];
      a_mean += g_mean[g];
    }
    const uint64_t bal = __ballot(eq);
    const uint32_t below = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wcount[w] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t before = base, total = 0;
    for (int i = 0; i < kFilterThreads / 64; ++i) {
      if (i < w) before += wcount[i];
      total += wcount[i];
    }
    if (g < G) {
      const bool kp = k > 0 && (key > prefix || (eq && before + below < need));
      keep[g] = kp ? 1 : 0;
      if (kp) {
        c_std += g_std[g];
        c_max += g_max[g];
        c_mean += g_mean[g];
      }
    }
    base += total;
    __syncthreads();
  }
  double v[6] = {a_std, a_max, a_mean, c_std, c_max, c_mean};
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const double t = wave_sum(v[j]);
    if (lane == 0) red[j][w] = t;
  }
  __syncthreads();
  if (tid < 6) {
    double t = 0;
    for (int i = 0; i < kFilterThreads / 64; ++i) t += red[tid][i];
    const double d = tid < 3 ? (double)G : (double)k;
    metrics[tid] = (float)(t / d);  // torch f32 .mean()
  }
}

// score_tensor[:, -1] + penalty in f32 (ctx_manager.py:194-217)
__device__ __forceinline__ float env_x(const rmi_episode_t& ep, int64_t i) {
  return (float)env_totals<false>(ep, i).score + (float)ep.penalty[i];
}

// Fused end-of-rollout pass: per env metrics + trajectory score + penalty, then the group
// normalisation, one wave per segment (get_rollout_states + get_masks_and_scores score
// placement + _normalize_score_tensor in one launch).  A segment's first 64 envs keep their
// x in a register across the mean / variance / output passes.
__global__ __launch_bounds__(kBlock) void finalize_kernel(rmi_episode_t ep, const int32_t* __restrict__ seg, int G,
                                                          int method, double* __restrict__ metrics,
                                                          float* __restrict__ score_out, float* __restrict__ pen_out,
                                                          float* __restrict__ norm_out) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (g >= G) return;
  const int lo = seg[g], hi = seg[g + 1], n = hi - lo;
  if (n <= 0 || lo < 0 || hi > ep.B) return;  // malformed segments are never read past [0, B)
  double s = 0.0;
  float x0 = 0.0f;
  for (int i = lo + lane; i < hi; i += 64) {
    const float pf = (float)ep.penalty[i];
    const EnvTotals e = env_totals<true>(ep, i);
    const float scf = (float)e.score;
    if (score_out) score_out[i] = scf;
    if (pen_out) pen_out[i] = pf;
    if (metrics) env_metrics(ep, i, e, metrics);
    const float x = scf + pf;
    if (i < lo + 64) x0 = x;
    s += (double)x;
  }
  if (!norm_out || n <= 0) return;
  s = wave_sum(s);
  const double md = s / (double)n;
  const float mean = (float)md;
  float sd = 0.0f;
  if (method == RMI_NORM_MEAN_STD || method == RMI_NORM_ASYM_CLIP) {
    double q = 0.0;
    for (int i = lo + lane; i < hi; i += 64) {
      const double d = (double)(i < lo + 64 ? x0 : env_x(ep, i)) - md;
      q += d * d;
    }
    q = wave_sum(q);
    sd = n > 1 ? (float)sqrt(q / (double)(n - 1)) : __builtin_nanf("");
  }
  const bool use = sd > 1e-6f;
  for (int i = lo + lane; i < hi; i += 64) {
    const float x = i < lo + 64 ? x0 : env_x(ep, i);
    float y;
    if (method == RMI_NORM_IDENTITY) y = x;
    else if (method == RMI_NORM_MEAN) y = x - mean;
    else {
      y = use ? (x - mean) / (sd + 1e-6f) : 0.0f;
      if (method == RMI_NORM_ASYM_CLIP) y = fminf(fmaxf(y, -1.0f), 3.0f);
    }
    norm_out[i] = y;
  }
}

}  // namespace
}  // namespace rmi

RMI_API int rmi_rollout_metrics(const rmi_episode_t* ep, double* out, rmi_stream_t stream) {
  using namespace rmi;
  if (!ep || ep->B < 0) return RMI_EINVAL;
  if (ep->B == 0) return RMI_OK;
  if (!out || !ep->flags || !ep->turn_info || !ep->n_turns || !ep->num_actions) return RMI_EINVAL;
  hipLaunchKernelGGL(rollout_metrics_kernel, dim3((ep->B + kBlock - 1) / kBlock), dim3(kBlock), 0,
                     as_stream(stream), *ep, out);
  return launch_status();
}

RMI_API int rmi_trajectory_scores(const rmi_episode_t* ep, float* score, float* pen, rmi_stream_t stream) {
  using namespace rmi;
  if (!ep || ep->B < 0) return RMI_EINVAL;
  if (ep->B == 0) return RMI_OK;
  if (!score || !ep->turn_reward || (pen && !ep->penalty)) return RMI_EINVAL;
  hipLaunchKernelGGL(trajectory_scores_kernel, dim3((ep->B + kBlock - 1) / kBlock), dim3(kBlock), 0,
                     as_stream(stream), *ep, score, pen);
  return launch_status();
}

RMI_API int rmi_group_normalize(const float* score, const float* pen, const int32_t* seg, int32_t G, int32_t B,
                                int32_t method, float* out, rmi_stream_t stream) {
  using namespace rmi;
  if (G < 0 || B < 0 || method < 0 || method > 3) return RMI_EINVAL;
  if (B == 0 || G == 0) return RMI_OK;
  if (!score || !seg || !out) return RMI_EINVAL;
  // the reference normalises only when some group has more than one member (ctx_manager.py:220)
  if (G >= B) method = RMI_NORM_IDENTITY;
  const int per = kBlock / 64;
  hipLaunchKernelGGL(group_normalize_kernel, dim3((G + per - 1) / per), dim3(kBlock), 0, as_stream(stream), score,
                     pen, seg, G, B, method, out);
  return launch_status();
}

RMI_API int rmi_row_sum(const float* x, int64_t B, int64_t L, float* out, rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || L < 0) return RMI_EINVAL;
  if (B == 0) return RMI_OK;
  if (!x || !out) return RMI_EINVAL;
  const int per = kBlock / 64;
  hipLaunchKernelGGL(row_sum_kernel, dim3((unsigned)((B + per - 1) / per)), dim3(kBlock), 0, as_stream(stream), x,
                     B, L, out);
  return launch_status();
}

RMI_API int rmi_filter_groups(const float* scores, int64_t n, int32_t G, int32_t gs, double ratio, int32_t type,
                              float* g_std, float* g_max, float* g_mean, uint8_t* keep, double* metrics,
                              rmi_stream_t stream) {
  using namespace rmi;
  if (!scores || !g_std || !g_max || !g_mean || !keep || !metrics || G <= 0 || gs <= 0) return RMI_EINVAL;
  if (n != (int64_t)G * gs) return RMI_EINVAL;  // rm_scores.view(num_groups, group_size) raises
  if (type != 0 && type != 1) return RMI_EINVAL;
  int k = (ratio == 1.0) ? G : (int)(ratio * (double)G);  // int(rollout_filter_ratio * num_groups)
  if (k < 0) k = 0;
  if (k > G) k = G;
  hipStream_t s = as_stream(stream);
  if (G <= kFilterMaxG) {
    hipLaunchKernelGGL(filter_kernel, dim3(1), dim3(kFilterThreads), 0, s, scores, G, gs, k, type, g_std, g_max,
                       g_mean, keep, metrics);
  } else {
    hipLaunchKernelGGL(filter_stats_kernel, dim3((unsigned)((G + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, scores,
                       G, gs, g_std, g_max, g_mean);
    hipLaunchKernelGGL(filter_select_kernel, dim3(1), dim3(kFilterThreads), 0, s, G, k, type, g_std, g_max, g_mean,
                       keep, metrics);
  }
  return launch_status();
}

RMI_API int rmi_rollout_finalize(const rmi_episode_t* ep, const int32_t* seg, int32_t G, int32_t method,
                                 double* metrics, float* score, float* pen, float* norm, rmi_stream_t stream) {
  using namespace rmi;
  if (!ep || ep->B < 0 || G < 0 || method < 0 || method > 3) return RMI_EINVAL;
  if (ep->B == 0 || G == 0) return RMI_OK;
  if (!seg || !ep->turn_reward || !ep->turn_info || !ep->penalty || !ep->flags || !ep->n_turns || !ep->num_actions)
    return RMI_EINVAL;
  if (G >= ep->B) method = RMI_NORM_IDENTITY;  // ctx_manager.py:220: only if some group has > 1 member
  const int per = kBlock / 64;
  hipLaunchKernelGGL(finalize_kernel, dim3((G + per - 1) / per), dim3(kBlock), 0, as_stream(stream), *ep, seg, G,
                     method, metrics, score, pen, norm);
  return launch_status();
}
