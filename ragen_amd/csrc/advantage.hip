// advantage.hip — GAE family, GRPO broadcast and masked whitening (gfx950).
//
//  rmi_gae           verl compute_gae_advantage_return (legacy + masked), App. A.4;
//                    called by compute_advantage (agent_trainer.py:77-83)
//  rmi_bilevel_gae   compute_bi_level_gae_advantage_return (core_algos.py:4-92)
//  rmi_masked_whiten verl masked_whiten (core_algos.py:90)
//  rmi_grpo_outcome  verl compute_grpo_outcome_advantage (agent_trainer.py:94-99)
//
// Exactness: the GAE recurrence runs sequentially per row in the reference's f32 op order
// ((r + g*nv) - v, then delta + (g*lam)*last, g*lam formed in double as Python does) and
// the build compiles with -ffp-contract=off, so advantages/returns before whitening are
// bit-identical to the torch CPU loop.  Whitening statistics are fp64 with a fixed
// reduction tree (run-to-run reproducible; within ~1 ulp of torch's f32 sums).
//
// Memory: one 64-lane wave owns 32 rows.  Column chunks of 64 are streamed right-to-left
// through LDS with coalesced 256-B row segments (r, v, mask in; adv, ret out), the LDS
// tiles padded to 65 floats per row so the per-row (per-lane) column walk is conflict-free.
#include <math.h>

#include "common.hpp"

namespace rmi {
namespace {

constexpr int kRows = 32;   // rows per wave (256 workgroups at B = 8192)
constexpr int kCols = 64;   // columns per LDS chunk
constexpr int kPad = kCols + 1;

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

template <int VARIANT>
__global__ __launch_bounds__(64) void gae_kernel(const float* __restrict__ r, const float* __restrict__ v,
                                                 const uint8_t* __restrict__ mask, int64_t B, int64_t L, float g,
                                                 float gl, float* __restrict__ adv, float* __restrict__ ret,
                                                 double* __restrict__ row_stats) {
  __shared__ float sr[kRows * kPad];
  __shared__ float sv[kRows * kPad];
  __shared__ float sm[kRows * kPad];
  const int lane = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kRows;
  const int nrows = (int)min<int64_t>(kRows, B - row0);
  // per-row carried state (lane < nrows owns row row0 + lane)
  float last = 0.0f, nv = 0.0f;
  double s1 = 0.0, s2 = 0.0, cnt = 0.0;
  const int64_t nchunks = (L + kCols - 1) / kCols;
  for (int64_t ch = nchunks - 1; ch >= 0; --ch) {
    const int64_t c0 = ch * kCols;
    const int ncols = (int)min<int64_t>(kCols, L - c0);
    // coalesced load: lane = column
    for (int rr = 0; rr < nrows; ++rr) {
      const int64_t base = (row0 + rr) * L + c0;
      if (lane < ncols) {
        sr[rr * kPad + lane] = r[base + lane];
        sv[rr * kPad + lane] = v[base + lane];
        sm[rr * kPad + lane] = mask ? (float)mask[base + lane] : 1.0f;
      }
    }
    __syncthreads();
    if (lane < nrows) {
      float* pr = sr + lane * kPad;
      float* pv = sv + lane * kPad;
      const float* pm = sm + lane * kPad;
      for (int c = ncols - 1; c >= 0; --c) {
        const float rt = pr[c], vt = pv[c], mt = pm[c];
        const float delta = (rt + g * nv) - vt;
        float a;
        if (VARIANT == 0) {  // legacy: nextvalues = values[:, t+1]
          last = delta + gl * last;
          a = last;
          nv = vt;
        } else {  // masked: carry next in-mask value / advantage
          const float l2 = delta + gl * last;
          nv = vt * mt + (1.0f - mt) * nv;
          last = l2 * mt + (1.0f - mt) * last;
          a = last;
        }
        pr[c] = a;           // adv (overwrite r tile)
        pv[c] = a + vt;      // ret = adv + values (overwrite v tile)
        if (mt != 0.0f) {
          s1 += (double)a;
          s2 += (double)a * (double)a;
          cnt += 1.0;
        }
      }
    }
    __syncthreads();
    for (int rr = 0; rr < nrows; ++rr) {
      const int64_t base = (row0 + rr) * L + c0;
      if (lane < ncols) {
        adv[base + lane] = sr[rr * kPad + lane];
        ret[base + lane] = sv[rr * kPad + lane];
      }
    }
    __syncthreads();
  }
  if (row_stats && lane < nrows) {
    row_stats[3 * (row0 + lane) + 0] = s1;
    row_stats[3 * (row0 + lane) + 1] = s2;
    row_stats[3 * (row0 + lane) + 2] = cnt;
  }
}

// One thread per row, one reverse sweep doing both levels of core_algos.py:44-88.
__global__ __launch_bounds__(kBlock) void bilevel_kernel(const float* __restrict__ r, const float* __restrict__ v,
                                                         const uint8_t* __restrict__ mask, int64_t B, int64_t L,
                                                         float g, float gl, float hg, float hgl,
                                                         float* __restrict__ adv, float* __restrict__ ret,
                                                         double* __restrict__ row_stats, uint8_t* __restrict__ err) {
  const int64_t b = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (b >= B) return;
  const float* rr = r + b * L;
  const float* vv = v + b * L;
  const uint8_t* mm = mask + b * L;
  float* aa = adv + b * L;
  float* qq = ret + b * L;
  float hl = 0.0f, ll = 0.0f, v_next_eos = 0.0f, v_next_valid = 0.0f;
  bool has_eos = false, has_valid = false, bad = false;
  double s1 = 0.0, s2 = 0.0, cnt = 0.0;
  for (int64_t t = L - 1; t >= 0; --t) {
    const float rt = rr[t], vt = vv[t];
    const bool m = mm[t] != 0;
    const bool eos = rt != 0.0f || rt != rt;  // token_level_rewards.bool()
    float a = 0.0f, q = 0.0f, upd = rt;
    if (eos) {
      const float delta = (rt + (has_eos ? hg * v_next_eos : 0.0f)) - vt;
      hl = delta + hgl * hl;
      a = hl;
      upd = hl + vt;  // updated_reward = advantages + values
      q = upd;        // returns = advantages + values
      v_next_eos = vt;
      has_eos = true;
    }
    if (m) {
      float nvv;
      if (eos) {
        nvv = 0.0f;
        ll = 0.0f;
      } else {
        if (!has_valid) bad = true;  // valid_positions[i + 1] -> IndexError
        nvv = v_next_valid;
      }
      const float delta = (upd + g * nvv) - vt;
      ll = delta + gl * ll;
      a = ll;
      q = ll + vt;
      v_next_valid = vt;
      has_valid = true;
      s1 += (double)a;
      s2 += (double)a * (double)a;
      cnt += 1.0;
    }
    aa[t] = a;
    qq[t] = q;
  }
  if (row_stats) {
    row_stats[3 * b + 0] = s1;
    row_stats[3 * b + 1] = s2;
    row_stats[3 * b + 2] = cnt;
  }
  if (err) err[b] = bad ? RMI_ERR_INDEX : 0;
}

__global__ __launch_bounds__(kBlock) void row_stats_kernel(const float* __restrict__ x,
                                                           const uint8_t* __restrict__ mask, int64_t B, int64_t L,
                                                           double* __restrict__ stats) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (row >= B) return;
  double s1 = 0, s2 = 0, c = 0;
  for (int64_t i = lane; i < L; i += 64) {
    if (mask[row * L + i]) {
      const double a = x[row * L + i];
      s1 += a;
      s2 += a * a;
      c += 1.0;
    }
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  c = wave_sum(c);
  if (lane == 0) {
    stats[3 * row + 0] = s1;
    stats[3 * row + 1] = s2;
    stats[3 * row + 2] = c;
  }
}

struct WhitenParams {
  float mean;
  float scale;
  int32_t status;  // 0 ok, 1: mask sum == 0, 2: mask sum == 1 (verl raises ValueError)
  int32_t pad;
};

__global__ __launch_bounds__(1024) void whiten_finalize_kernel(const double* __restrict__ stats, int64_t B,
                                                               WhitenParams* __restrict__ out) {
  __shared__ double red[3][16];
  double s1 = 0, s2 = 0, c = 0;
  for (int64_t i = threadIdx.x; i < B; i += 1024) {
    s1 += stats[3 * i];
    s2 += stats[3 * i + 1];
    c += stats[3 * i + 2];
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  c = wave_sum(c);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][w] = s1;
    red[1][w] = s2;
    red[2][w] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t1 = 0, t2 = 0, tc = 0;
    for (int i = 0; i < 16; ++i) {
      t1 += red[0][i];
      t2 += red[1][i];
      tc += red[2][i];
    }
    WhitenParams p;
    p.pad = 0;
    p.status = tc == 0.0 ? 1 : (tc == 1.0 ? 2 : 0);
    const double mean = tc > 0 ? t1 / tc : 0.0;
    // masked_var: mean((x-mean)^2) * n/(n-1)  ==  (sum x^2 - n mean^2) / (n - 1)
    double var = tc > 1 ? (t2 - tc * mean * mean) / (tc - 1.0) : 0.0;
    if (var < 0) var = 0;
    p.mean = (float)mean;
    const float vf = (float)var + 1e-8f;
    p.scale = 1.0f / sqrtf(vf);  // torch.rsqrt(var + 1e-8)
    *out = p;
  }
}

__global__ __launch_bounds__(kBlock) void whiten_apply_kernel(float* __restrict__ x, int64_t n,
                                                              const WhitenParams* __restrict__ p) {
  const float mean = p->mean, scale = p->scale;
  const int64_t n4 = (reinterpret_cast<uintptr_t>(x) & 15) ? 0 : (n >> 2);
  float4* x4 = reinterpret_cast<float4*>(x);
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kBlock) {
    float4 a = x4[i];
    a.x = (a.x - mean) * scale;
    a.y = (a.y - mean) * scale;
    a.z = (a.z - mean) * scale;
    a.w = (a.w - mean) * scale;
    x4[i] = a;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    x[i] = (x[i] - mean) * scale;
}

// GRPO: one wave per group segment; rows of the group are summed (fp64 -> f32) per row,
// group mean/std in fp64, then the per-row score is broadcast over the row's mask.
__global__ __launch_bounds__(kBlock) void grpo_kernel(const float* __restrict__ r, const uint8_t* __restrict__ mask,
                                                      int64_t L, const int32_t* __restrict__ seg, int G, float eps,
                                                      int norm_by_std, float* __restrict__ adv,
                                                      float* __restrict__ ret) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (g >= G) return;
  const int lo = seg[g], hi = seg[g + 1], n = hi - lo;
  // pass 1: group sums of row scores
  double gs = 0.0, gq = 0.0;
  for (int row = lo; row < hi; ++row) {
    double s = 0.0;
    for (int64_t i = lane; i < L; i += 64) s += (double)r[row * L + i];
    s = wave_sum(s);
    const float sf = (float)s;
    gs += sf;
    gq += (double)sf * (double)sf;
  }
  float mean = 0.0f, sd = 1.0f;
  if (n > 1) {
    const double m = gs / n;
    mean = (float)m;
    double var = (gq - n * m * m) / (n - 1);
    if (var < 0) var = 0;
    sd = (float)sqrt(var);
  }
  for (int row = lo; row < hi; ++row) {
    double s = 0.0;
    for (int64_t i = lane; i < L; i += 64) s += (double)r[row * L + i];
    s = wave_sum(s);
    float sc = (float)s - mean;
    if (norm_by_std) sc = sc / (sd + eps);
    for (int64_t i = lane; i < L; i += 64) {
      const float y = sc * (float)(mask[row * L + i] != 0);
      adv[row * L + i] = y;
      ret[row * L + i] = y;
    }
  }
}

}  // namespace
}  // namespace rmi

RMI_API int rmi_gae(const float* r, const float* v, const uint8_t* mask, int64_t B, int64_t L, double gamma,
                    double lam, int32_t variant, float* adv, float* ret, double* row_stats, rmi_stream_t stream) {
  using namespace rmi;
  if (!r || !v || !adv || !ret || B < 0 || L < 0 || (variant != 0 && variant != 1)) return RMI_EINVAL;
  if ((row_stats || variant == 1) && !mask) return RMI_EINVAL;
  if (B == 0 || L == 0) return RMI_OK;
  const float g = (float)gamma;
  const float gl = (float)(gamma * lam);  // python: gamma * lam * lastgaelam
  const unsigned grid = (unsigned)((B + kRows - 1) / kRows);
  if (variant == 0)
    hipLaunchKernelGGL(gae_kernel<0>, dim3(grid), dim3(64), 0, as_stream(stream), r, v, mask, B, L, g, gl, adv, ret,
                       row_stats);
  else
    hipLaunchKernelGGL(gae_kernel<1>, dim3(grid), dim3(64), 0, as_stream(stream), r, v, mask, B, L, g, gl, adv, ret,
                       row_stats);
  return launch_status();
}

RMI_API int rmi_bilevel_gae(const float* r, const float* v, const uint8_t* mask, int64_t B, int64_t L, double gamma,
                            double lam, double high_level_gamma, float* adv, float* ret, double* row_stats,
                            uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (!r || !v || !mask || !adv || !ret || B < 0 || L < 0) return RMI_EINVAL;
  if (B == 0 || L == 0) return RMI_OK;
  hipLaunchKernelGGL(bilevel_kernel, dim3((unsigned)((B + kBlock - 1) / kBlock)), dim3(kBlock), 0, as_stream(stream),
                     r, v, mask, B, L, (float)gamma, (float)(gamma * lam), (float)high_level_gamma,
                     (float)(high_level_gamma * lam), adv, ret, row_stats, err);
  return launch_status();
}

RMI_API size_t rmi_whiten_scratch_bytes(int64_t B) {
  return (size_t)(B > 0 ? B : 1) * 3 * sizeof(double) + 64;
}

RMI_API int rmi_masked_whiten(float* x, const uint8_t* mask, int64_t B, int64_t L, const double* row_stats,
                              void* scratch, rmi_stream_t stream) {
  using namespace rmi;
  if (!x || !mask || !scratch || B < 0 || L < 0) return RMI_EINVAL;
  if (B == 0 || L == 0) return RMI_OK;
  hipStream_t s = as_stream(stream);
  WhitenParams* params = reinterpret_cast<WhitenParams*>(scratch);
  double* stats = reinterpret_cast<double*>(reinterpret_cast<char*>(scratch) + 64);
  if (!row_stats) {
    const int per = kBlock / 64;
    hipLaunchKernelGGL(row_stats_kernel, dim3((unsigned)((B + per - 1) / per)), dim3(kBlock), 0, s, x, mask, B, L,
                       stats);
    row_stats = stats;
  }
  hipLaunchKernelGGL(whiten_finalize_kernel, dim3(1), dim3(1024), 0, s, row_stats, B, params);
  const int64_t n = B * L;
  int64_t blocks = (n / 4 + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(whiten_apply_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, x, n, params);
  return launch_status();
}

RMI_API int rmi_grpo_outcome(const float* r, const uint8_t* mask, int64_t B, int64_t L, const int32_t* seg, int32_t G,
                             double eps, int32_t norm_by_std, float* adv, float* ret, rmi_stream_t stream) {
  using namespace rmi;
  if (!r || !mask || !seg || !adv || !ret || B < 0 || L < 0 || G < 0) return RMI_EINVAL;
  if (B == 0 || G == 0) return RMI_OK;
  const int per = kBlock / 64;
  hipLaunchKernelGGL(grpo_kernel, dim3((G + per - 1) / per), dim3(kBlock), 0, as_stream(stream), r, mask, L, seg, G,
                     (float)eps, norm_by_std, adv, ret);
  return launch_status();
}
