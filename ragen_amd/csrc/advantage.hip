// advantage.hip — GAE family, GRPO broadcast and masked whitening (gfx950).
//
//  rmi_gae           verl compute_gae_advantage_return (legacy + masked), App. A.4;
//                    called by compute_advantage (agent_trainer.py:77-83)
//  rmi_bilevel_gae   compute_bi_level_gae_advantage_return (core_algos.py:4-92)
//  rmi_masked_whiten verl masked_whiten (core_algos.py:90)
//  rmi_grpo_outcome  verl compute_grpo_outcome_advantage (agent_trainer.py:94-99)
//  rmi_reinforce_pp_returns  verl compute_reinforce_plus_plus_outcome_advantage before its
//                    whitening (agent_trainer.py:110-117)
//  rmi_remax         verl compute_remax_outcome_advantage (agent_trainer.py:118-126)
//  rmi_rloo_outcome  verl compute_rloo_outcome_advantage (agent_trainer.py:127-134)
//  rmi_mask_mul      the trailing `* response_mask` of verl's REINFORCE++ estimators
//
// Exactness: the GAE recurrence runs sequentially per row in the reference's f32 op order
// ((r + g*nv) - v, then delta + (g*lam)*last, g*lam formed in double as Python does) and
// the build compiles with -ffp-contract=off, so advantages/returns before whitening are
// bit-identical to the torch CPU loop.  Whitening statistics are fp64 with a fixed
// reduction tree (run-to-run reproducible; within ~1 ulp of torch's f32 sums).
//
// Memory (GAE): one 64-lane wave owns kGRows = 4 rows and streams them right to left in
// 4 x 64 tiles: every lane moves 4-column groups (16-B loads/stores, 256-B coalesced row
// segments) into a 3-deep register pipeline (two tiles in flight behind the one being
// worked on).  The column-parallel work (delta, ret = adv + v, fp64 whitening partials)
// runs on all 64 lanes; the tile is staged in LDS for the serial recurrence, walked by one
// lane per row (16-B LDS reads, row stride 272 B: conflict-free).  Few rows per wave keeps
// the serial walk the only long per-wave chain and puts 2 waves on every SIMD; at 8192 x
// 1093 tokens the kernel streams ~4.8 TB/s (HBM-bound).  Algorithmic traffic 17 B/token.
#include <math.h>
#include <stdlib.h>

#include "common.hpp"

namespace rmi {
namespace {


__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

constexpr int kGRows = 4;             // rows per wave: lane < 4 walks its row (2048 waves at B = 8192, 2 per SIMD)
constexpr int kGCols = 64;            // columns per tile
constexpr int kGStr = kGCols + 4;     // LDS row stride in floats (272 B): conflict-free 16-B row walks
constexpr int kGMStr = kGCols + 4;    // LDS mask row stride in bytes
constexpr int kGLoads = kGRows * kGCols / 4 / 64;  // 4-column groups per lane per array per tile (8)

struct __attribute__((packed, aligned(4))) F4 {
  float x, y, z, w;
};
struct __attribute__((packed, aligned(1))) U8x4 {
  uint32_t x;
};

// Streamed tile loads and output stores.  NT (a launch whose rows are far past the 256 MiB
// Infinity Cache): nontemporal, the copy probe's faster form there (profiles/r04_copy_probe.json);
// in-cache launches keep the cached form (nontemporal loads measured 31 -> 55 us at 8192 x 1093).
typedef float rmi_f4u __attribute__((ext_vector_type(4), aligned(4)));
template <bool NT>
__device__ __forceinline__ F4 ld_f4(const float* p) {
  if constexpr (NT) {
    const rmi_f4u x = __builtin_nontemporal_load(reinterpret_cast<const rmi_f4u*>(p));
    return F4{x.x, x.y, x.z, x.w};
  } else {
    return *reinterpret_cast<const F4*>(p);
  }
}
template <bool NT>
__device__ __forceinline__ void st_f4(float* p, const F4& v) {
#ifdef RMI_NT_LOADS_ONLY  // (A/B build: streamed loads, cached stores)
  if constexpr (false) {
#else
  if constexpr (NT) {
#endif
    const rmi_f4u x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<rmi_f4u*>(p));
  } else {
    *reinterpret_cast<F4*>(p) = v;
  }
}
constexpr double kStreamBytes = 256.0 * 1024 * 1024;  // a launch's traffic from which NT is used


// Mask bytes -> 0x01 per nonzero byte: a mask is a boolean (RAGEN passes a bool loss_mask,
// ctx_manager.py:46-49), so any nonzero byte counts as 1 in the recurrence, the whitening
// count and the sums alike.
__device__ __forceinline__ uint32_t nz8(uint32_t x) {
  x |= x >> 4;
  x |= x >> 2;
  x |= x >> 1;
  return x & 0x01010101u;
}

// One tile = rows [row0, row0+32) x columns [c0, c0+64) of r, v, mask, as 4-column groups:
// lane l, slot j -> row 4j + l/16, columns c0 + 4*(l%16) .. +3 (256-B coalesced row segments).
// Columns >= L and rows >= B read as zeros (a zero tail is an exact no-op for the recurrence:
// it starts the walk at column L-1 with last = nv = 0).
// m holds the raw mask words: they are normalised (nz8(m | mor)) where they are used, not
// where they are loaded — consuming a load right after issuing it would make the compiler wait
// for every load in flight (s_waitcnt vmcnt(0)) and drain the tile pipeline.  mor = 0x01010101
// without a mask (every column counts), else 0.
struct GaeTile {
  F4 r[kGLoads], v[kGLoads];
  uint32_t m[kGLoads];
  uint32_t mor;
  __device__ __forceinline__ uint32_t mask(int j) const { return nz8(m[j] | mor); }
};

template <bool NT = false>
__device__ __forceinline__ void gae_load_tile(GaeTile& t, const float* __restrict__ r, const float* __restrict__ v,
                                              const uint8_t* __restrict__ mask, int64_t B, int64_t L, int64_t row0,
                                              int64_t c0, int lane) {
  const int g = lane & 15;
  const int64_t col = c0 + 4 * g;
  const bool dummy = c0 < 0;  // a pipeline slot past column 0: every lane reads one shared line
  const bool full_col = col + 4 <= L && !dummy;
  t.mor = mask ? 0u : 0x01010101u;
  // 1. every full 4-column group, branch-free from clamped (always valid) addresses, so all
  //    loads of the tile are in flight together; invalid groups are zeroed when staged
#pragma unroll
  for (int j = 0; j < kGLoads; ++j) {
    const int64_t row = min<int64_t>(row0 + 4 * j + (lane >> 4), B - 1);
    const int64_t o = dummy ? min<int64_t>(row0, B - 1) * L : (full_col ? row * L + col : row * L);
    t.r[j] = ld_f4<NT>(r + o);
    t.v[j] = ld_f4<NT>(v + o);
    t.m[j] = reinterpret_cast<const U8x4*>((mask ? mask : reinterpret_cast<const uint8_t*>(r)) + o)->x;
  }
  // 2. the ragged group at a row end (L % 4 != 0: one group per row, in one tile) and rows
  //    past B, element by element, never past the row
  if (__any(!full_col || row0 + kGRows > B)) {
#pragma unroll
    for (int j = 0; j < kGLoads; ++j) {
      const int64_t row = row0 + 4 * j + (lane >> 4);
      if (row >= B || col >= L || dummy) {
        t.r[j] = F4{0.f, 0.f, 0.f, 0.f};
        t.v[j] = F4{0.f, 0.f, 0.f, 0.f};
        t.m[j] = 0;
      } else if (!full_col) {
        const int64_t o = row * L + col;
        float rr[4] = {0.f, 0.f, 0.f, 0.f}, vv[4] = {0.f, 0.f, 0.f, 0.f};
        uint32_t mm = 0;
        for (int e = 0; e < 4; ++e) {
          if (col + e < L) {
            rr[e] = r[o + e];
            vv[e] = v[o + e];
            mm |= (uint32_t)(mask ? mask[o + e] != 0 : 1) << (8 * e);
          }
        }
        t.r[j] = F4{rr[0], rr[1], rr[2], rr[3]};
        t.v[j] = F4{vv[0], vv[1], vv[2], vv[3]};
        t.m[j] = mm;
      }
    }
  }
}

// verl compute_gae_advantage_return, reverse recurrence in the reference's f32 op order:
//   delta = (r_t + g * nv) - v_t ;  last = delta + gl * last ;  adv = last ; ret = adv + v_t
// legacy (VARIANT 0): nv = v_{t+1}; masked (1): nv / last carried through mask-0 positions.
// VARIANT 2, REINFORCE++ returns (verl, torch CPU loop): running = r_t + g * running;
//   ret_t = running; running = running * m_t  (adv_t = ret_t: whitened afterwards).
// VARIANT 3, REMAX: ret = flip(cumsum(flip(r * m))) with torch's CPU cumsum accumulator
//   (double, each output rounded to f32); adv_t = ret_t - base * m_t  (base: the row's baseline).
template <int VARIANT>
__device__ __forceinline__ void gae_col(float rt, float vt, float mt, float g, float gl, float& nv, float& last,
                                        float& a_out, float& ret_out, double& dacc, float base) {
  if (VARIANT == 2) {
    const float run = rt + g * last;
    a_out = run;
    ret_out = run;
    last = run * mt;
    return;
  }
  if (VARIANT == 3) {
    dacc += (double)(rt * mt);
    ret_out = (float)dacc;
    a_out = ret_out - base * mt;
    return;
  }
  const float delta = (rt + g * nv) - vt;
  if (VARIANT == 0) {
    last = delta + gl * last;
    nv = vt;
  } else {
    const float l2 = delta + gl * last;
    nv = vt * mt + (1.0f - mt) * nv;
    last = l2 * mt + (1.0f - mt) * last;
  }
  a_out = last;
  ret_out = last + vt;
}

template <int VARIANT, bool NT = false>
__global__ __launch_bounds__(64) void gae_kernel(const float* __restrict__ r, const float* __restrict__ v,
                                                 const uint8_t* __restrict__ mask, int64_t B, int64_t L, float g,
                                                 float gl, float* __restrict__ adv, float* __restrict__ ret,
                                                 double* __restrict__ row_stats,
                                                 const float* __restrict__ row_base = nullptr) {
  __shared__ __attribute__((aligned(16))) float sr[kGRows * kGStr];  // r in, adv out
  __shared__ __attribute__((aligned(16))) float sv[kGRows * kGStr];  // v in, ret out
  __shared__ __attribute__((aligned(16))) uint8_t sm[kGRows * kGMStr];
  const int lane = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kGRows;
  const int64_t ntiles = (L + kGCols - 1) / kGCols;
  const bool walker = lane < kGRows && row0 + lane < B;
  float last = 0.0f, nv = 0.0f;
  double dacc = 0.0;  // REMAX: torch CPU cumsum's double accumulator
  const float base = (VARIANT == 3 && walker) ? row_base[row0 + lane] : 0.0f;
  double s1a = 0.0, s1b = 0.0, s2a = 0.0, s2b = 0.0, cnt = 0.0;  // row stats, two chains each

  GaeTile t;
  gae_load_tile<NT>(t, r, v, mask, B, L, row0, (ntiles - 1) * kGCols, lane);
  for (int64_t k = ntiles - 1; k >= 0; --k) {
    const int64_t c0 = k * kGCols;
    // registers -> LDS (the tile's 4-column groups), then prefetch the next tile to the left
#pragma unroll
    for (int j = 0; j < kGLoads; ++j) {
      const int row = 4 * j + (lane >> 4), grp = lane & 15;
      *reinterpret_cast<F4*>(sr + row * kGStr + 4 * grp) = t.r[j];
      *reinterpret_cast<F4*>(sv + row * kGStr + 4 * grp) = t.v[j];
      *reinterpret_cast<uint32_t*>(sm + row * kGMStr + 4 * grp) = t.mask(j);
    }
    __syncthreads();
    if (k > 0) gae_load_tile<NT>(t, r, v, mask, B, L, row0, c0 - kGCols, lane);
    // the walk: lane = row, columns right to left, 4 at a time
    if (walker) {
      float* pr = sr + lane * kGStr;
      float* pv = sv + lane * kGStr;
      const uint8_t* pm = sm + lane * kGMStr;
#pragma unroll 4
      for (int q = kGCols / 4 - 1; q >= 0; --q) {
        const F4 r4 = *reinterpret_cast<const F4*>(pr + 4 * q);
        const F4 v4 = *reinterpret_cast<const F4*>(pv + 4 * q);
        const uint32_t m4 = *reinterpret_cast<const uint32_t*>(pm + 4 * q);
        F4 a4, t4;
        gae_col<VARIANT>(r4.w, v4.w, (float)((m4 >> 24) & 0xFF), g, gl, nv, last, a4.w, t4.w, dacc, base);
        gae_col<VARIANT>(r4.z, v4.z, (float)((m4 >> 16) & 0xFF), g, gl, nv, last, a4.z, t4.z, dacc, base);
        gae_col<VARIANT>(r4.y, v4.y, (float)((m4 >> 8) & 0xFF), g, gl, nv, last, a4.y, t4.y, dacc, base);
        gae_col<VARIANT>(r4.x, v4.x, (float)(m4 & 0xFF), g, gl, nv, last, a4.x, t4.x, dacc, base);
        *reinterpret_cast<F4*>(pr + 4 * q) = a4;
        *reinterpret_cast<F4*>(pv + 4 * q) = t4;
        // whitening partials over in-mask positions (mask bytes are 0/1)
        const double dw = (double)a4.w, dz = (double)a4.z, dy = (double)a4.y, dx = (double)a4.x;
        const bool mw = (m4 >> 24) & 0xFF, mz = (m4 >> 16) & 0xFF, my = (m4 >> 8) & 0xFF, mx = m4 & 0xFF;
        s1a += (mw ? dw : 0.0) + (mz ? dz : 0.0);
        s1b += (my ? dy : 0.0) + (mx ? dx : 0.0);
        s2a += (mw ? dw * dw : 0.0) + (mz ? dz * dz : 0.0);
        s2b += (my ? dy * dy : 0.0) + (mx ? dx * dx : 0.0);
        cnt += (double)((int)mw + (int)mz + (int)my + (int)mx);
      }
    }
    __syncthreads();
    // LDS -> global (same 4-column group mapping), never past a row's end
    const int grp = lane & 15;
    const int64_t col = c0 + 4 * grp;
#pragma unroll
    for (int j = 0; j < kGLoads; ++j) {
      const int row = 4 * j + (lane >> 4);
      const int64_t grow = row0 + row;
      if (grow < B && col < L) {
        const F4 a4 = *reinterpret_cast<const F4*>(sr + row * kGStr + 4 * grp);
        const F4 t4 = *reinterpret_cast<const F4*>(sv + row * kGStr + 4 * grp);
        const int64_t o = grow * L + col;
        if (col + 4 <= L) {
          st_f4<NT>(adv + o, a4);
          st_f4<NT>(ret + o, t4);
        } else {
          const float aa[4] = {a4.x, a4.y, a4.z, a4.w}, tt[4] = {t4.x, t4.y, t4.z, t4.w};
          for (int e = 0; e < 4; ++e)
            if (col + e < L) {
              adv[o + e] = aa[e];
              ret[o + e] = tt[e];
            }
        }
      }
    }
    __syncthreads();
  }
  if (row_stats && walker) {
    const int64_t row = row0 + lane;
    row_stats[3 * row + 0] = s1a + s1b;
    row_stats[3 * row + 1] = s2a + s2b;
    row_stats[3 * row + 2] = cnt;
  }
}

// Legacy GAE (the StarPO default) with the column-parallel work lifted out of the serial walk.
// In legacy verl nv_t = v_{t+1} whatever the mask, so delta_t = (r_t + g*v_{t+1}) - v_t is
// independent across columns: every lane computes it for its 4-column groups (the next
// column's value comes from the neighbouring lane by a DPP row rotate, or from the tile to
// the right), the tile is staged in LDS, and the serial walk (lane = row) is reduced to the
// recurrence last = delta + gl*last — two dependent f32 ops per column.  ret = adv + v and
// the fp64 whitening partials are again column-parallel, on the staging lanes.  Same f32
// op order as the reference (bit-exact adv / ret).
__device__ __forceinline__ float ror15(float x) {  // lane l of each 16-lane row <- lane (l+1) % 16
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x12F, 0xF, 0xF, false));  // row_ror:15
}
__device__ __forceinline__ double xor_sum16(double x) {  // sum over the 16 lanes of a DPP row
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) x += __shfl_xor(x, o, 16);
  return x;
}

// Per-lane walk state of the legacy kernel.
struct GaeLegacyState {
  float last;                 // walkers: the running advantage of their row
  float nv_right[kGLoads];    // lane 15 of a row: v at the first column of the tile to the right
  double s1[kGLoads], s2[kGLoads];
  int cnt[kGLoads];
};

// One 32 x 64 tile (columns [c0, c0+64)); c0 < 0 is a pipeline dummy (zero data: the walk
// continues past column 0 harmlessly, nothing is stored).
template <bool NT>
__device__ __forceinline__ void gae_legacy_tile(const GaeTile& cur, int64_t c0, GaeLegacyState& st, float* sd,
                                                int lane, bool walker, int64_t row0, int64_t B, int64_t L, float g,
                                                float gl, float* __restrict__ adv, float* __restrict__ ret) {
  const int grp = lane & 15;
  // 1. delta for this lane's groups, staged in LDS
#pragma unroll
  for (int j = 0; j < kGLoads; ++j) {
    const F4 r4 = cur.r[j], v4 = cur.v[j];
    const float rot = ror15(v4.x);
    const float nvx = grp == 15 ? st.nv_right[j] : rot;
    st.nv_right[j] = rot;  // lane 15 now holds group 0's v.x: the next tile's right neighbour
    F4 d4;
    d4.x = (r4.x + g * v4.y) - v4.x;
    d4.y = (r4.y + g * v4.z) - v4.y;
    d4.z = (r4.z + g * v4.w) - v4.z;
    d4.w = (r4.w + g * nvx) - v4.w;
    const int row = 4 * j + (lane >> 4);
    *reinterpret_cast<F4*>(sd + row * kGStr + 4 * grp) = d4;
  }
  __syncthreads();
  // 2. the serial walk: lane = row, right to left, last = delta + gl * last
  if (walker) {
    float* p = sd + lane * kGStr;
    float last = st.last;
#pragma unroll 4
    for (int q = kGCols / 4 - 1; q >= 0; --q) {
      F4 d4 = *reinterpret_cast<const F4*>(p + 4 * q);
      last = d4.w + gl * last;
      d4.w = last;
      last = d4.z + gl * last;
      d4.z = last;
      last = d4.y + gl * last;
      d4.y = last;
      last = d4.x + gl * last;
      d4.x = last;
      *reinterpret_cast<F4*>(p + 4 * q) = d4;
    }
    st.last = last;
  }
  __syncthreads();
  // 3. ret = adv + v, whitening partials, stores (column-parallel again)
  const int64_t col = c0 + 4 * grp;
#pragma unroll
  for (int j = 0; j < kGLoads; ++j) {
    const int row = 4 * j + (lane >> 4);
    const int64_t grow = row0 + row;
    const F4 a4 = *reinterpret_cast<const F4*>(sd + row * kGStr + 4 * grp);
    const F4 v4 = cur.v[j];
    const F4 t4 = F4{a4.x + v4.x, a4.y + v4.y, a4.z + v4.z, a4.w + v4.w};
    const uint32_t m4 = cur.mask(j);
    const double ax = (m4 & 0xFF) ? (double)a4.x : 0.0, ay = ((m4 >> 8) & 0xFF) ? (double)a4.y : 0.0;
    const double az = ((m4 >> 16) & 0xFF) ? (double)a4.z : 0.0, aw = (m4 >> 24) ? (double)a4.w : 0.0;
    st.s1[j] += (ax + ay) + (az + aw);
    st.s2[j] += (ax * ax + ay * ay) + (az * az + aw * aw);
    st.cnt[j] += __popc(m4 & 0x01010101u);
    if (grow < B && col >= 0 && col < L) {
      const int64_t o = grow * L + col;
      if (col + 4 <= L) {
        st_f4<NT>(adv + o, a4);
        st_f4<NT>(ret + o, t4);
      } else {
        const float aa[4] = {a4.x, a4.y, a4.z, a4.w}, tt[4] = {t4.x, t4.y, t4.z, t4.w};
        for (int e = 0; e < 4; ++e)
          if (col + e < L) {
            adv[o + e] = aa[e];
            ret[o + e] = tt[e];
          }
      }
    }
  }
  __syncthreads();
}

template <bool NT = false>
__global__ __launch_bounds__(64) void gae_legacy_kernel(const float* __restrict__ r, const float* __restrict__ v,
                                                        const uint8_t* __restrict__ mask, int64_t B, int64_t L,
                                                        float g, float gl, float* __restrict__ adv,
                                                        float* __restrict__ ret, double* __restrict__ row_stats) {
  __shared__ __attribute__((aligned(16))) float sd[kGRows * kGStr];  // delta in, adv out
  const int lane = threadIdx.x;
  const int grp = lane & 15;
  const int64_t row0 = (int64_t)blockIdx.x * kGRows;
  const int64_t ntiles = (L + kGCols - 1) / kGCols;
  const bool walker = lane < kGRows && row0 + lane < B;
  GaeLegacyState st;
  st.last = 0.0f;
#pragma unroll
  for (int j = 0; j < kGLoads; ++j) {
    st.nv_right[j] = 0.0f;
    st.s1[j] = st.s2[j] = 0.0;
    st.cnt[j] = 0;
  }
  // three register tiles, two loads in flight behind the tile being walked; the loop body
  // is straight-line (dummy tiles past column 0 keep it so) so the compiler's vmcnt
  // accounting lets the prefetches overlap the walk
  GaeTile ta, tb, tc;
  const int64_t k0 = ntiles - 1;
  gae_load_tile<NT>(ta, r, v, mask, B, L, row0, k0 * kGCols, lane);
  gae_load_tile<NT>(tb, r, v, mask, B, L, row0, (k0 - 1) * kGCols, lane);
  for (int64_t k = k0; k >= 0; k -= 3) {
    gae_load_tile<NT>(tc, r, v, mask, B, L, row0, (k - 2) * kGCols, lane);
    gae_legacy_tile<NT>(ta, k * kGCols, st, sd, lane, walker, row0, B, L, g, gl, adv, ret);
    gae_load_tile<NT>(ta, r, v, mask, B, L, row0, (k - 3) * kGCols, lane);
    gae_legacy_tile<NT>(tb, (k - 1) * kGCols, st, sd, lane, walker, row0, B, L, g, gl, adv, ret);
    gae_load_tile<NT>(tb, r, v, mask, B, L, row0, (k - 4) * kGCols, lane);
    gae_legacy_tile<NT>(tc, (k - 2) * kGCols, st, sd, lane, walker, row0, B, L, g, gl, adv, ret);
  }
  // per-row partials: the 16 lanes of a DPP row hold one row's groups
  if (row_stats) {
#pragma unroll
    for (int j = 0; j < kGLoads; ++j) {
      const double a = xor_sum16(st.s1[j]), b = xor_sum16(st.s2[j]);
      const double n = xor_sum16((double)st.cnt[j]);
      const int64_t grow = row0 + 4 * j + (lane >> 4);
      if (grp == 0 && grow < B) {
        row_stats[3 * grow + 0] = a;
        row_stats[3 * grow + 1] = b;
        row_stats[3 * grow + 2] = n;
      }
    }
  }
}

// Bi-level GAE (core_algos.py:44-88) on the same tiled stream as the legacy kernel (tiles of
// 4 rows x 64 columns, 3-deep register pipeline).  The reference's two sweeps are one reverse
// sweep (the low level at a position needs the high level only at that same position), and
// per tile it is split so that only true recurrences stay serial:
//   P1 column-parallel (every lane, its 4 columns): eos = reward != 0 (bool()), valid = mask;
//      the value at the next valid / next eos position to the right — a 16-lane DPP suffix
//      selection across the row's column groups plus the carry from the tile to the right
//      (selection only: no arithmetic, so nothing is reassociated); then each column's delta:
//      eos -> high-level delta (r + hg * v_next_eos) - v, valid non-eos -> (r + g * v_next_valid) - v.
//   P2 serial over the row's eos columns only (typically 0-2 per tile): hl = delta + hgl * hl,
//      updated reward = hl + v, and the eos column's low-level delta (upd + g * 0) - v.
//   P3 serial over the valid columns (groups with none are skipped): ll = d + gl * (eos ? 0 : ll).
//   P4 column-parallel: outputs (valid: ll, ll + v; eos only: hl, upd; else 0) and fp64 row stats.
// Every f32 operation is the reference's, in its order (-ffp-contract=off).
constexpr int kBStr = kGCols + 4;  // LDS row stride (floats / bytes)

// Diagnostic build only (tools/prof_bilevel_stamps.py compiles with RMI_BL_STAMPS): per-wave
// s_memtime sums of the tile phases (P1 incl. the tile's load wait | P2+P3 walk | P4).
#ifdef RMI_BL_STAMPS
__device__ unsigned long long* g_bl_stamps;
#define BL_T(x) const unsigned long long x = __builtin_amdgcn_s_memtime()
#define BL_ACC(i, d) (bl_acc[i] += (d))
#else
#define BL_T(x) \
  do {          \
  } while (0)
#define BL_ACC(i, d) \
  do {               \
  } while (0)
#endif

struct BilevelCarry {  // per row, replicated on the row's 16 lanes
  float v_valid, v_eos;  // value at the leftmost valid / eos position right of this tile
  uint32_t h_valid, h_eos;
};

// lane 0 of each 16-lane DPP row, broadcast to the whole row (DPP row_newbcast:0): a VALU move,
// where __shfl from the row's lead lane is a ds_bpermute and an LDS round trip per tile
__device__ __forceinline__ int row_lead(int x) { return __builtin_amdgcn_update_dpp(0, x, 0x150, 0xF, 0xF, false); }
__device__ __forceinline__ uint32_t row_lead(uint32_t x) { return (uint32_t)row_lead((int)x); }
__device__ __forceinline__ float row_lead(float x) { return __int_as_float(row_lead(__float_as_int(x))); }

// inclusive suffix selection over the 16 column groups of a DPP row: (h, v) <- first (h, v) with
// h set at or right of this group; lanes past the row end read h = 0 (bound_ctrl)
__device__ __forceinline__ void row_suffix_first(uint32_t& h, float& v) {
#define RMI_SHL(K)                                                                                        \
  {                                                                                                       \
    const uint32_t h2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)h, 0x100 + (K), 0xF, 0xF, true);    \
    const float v2 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x100 + (K), 0xF, 0xF, true)); \
    v = h ? v : v2;                                                                                       \
    h |= h2;                                                                                              \
  }
  RMI_SHL(1) RMI_SHL(2) RMI_SHL(4) RMI_SHL(8)
#undef RMI_SHL
}
__device__ __forceinline__ void row_shift_left1(uint32_t& h, float& v) {  // group g <- group g + 1
  h = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)h, 0x101, 0xF, 0xF, true);
  v = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x101, 0xF, 0xF, true));
}

struct BilevelWalk {  // the row walker's (group-0 lane's) chain state
  float hl, ll;
};

template <bool NT>
__device__ __forceinline__ void bilevel_tile(const GaeTile& cur, int64_t c0, BilevelCarry& cy, BilevelWalk& wk,
                                             double& s1, double& s2, double& cnt, uint32_t& bad, float* sv, float* sd,
                                             float* sh, float* su, uint32_t* sf, int lane, int64_t row0, int64_t B,
                                             int64_t L, float g, float gl, float hg, float hgl,
                                             float* __restrict__ adv, float* __restrict__ ret
#ifdef RMI_BL_STAMPS
                                             , unsigned long long* bl_acc
#endif
) {
  BL_T(t0);
  const int grp = lane & 15, rho = lane >> 4;
  const F4 r4 = cur.r[0], v4 = cur.v[0];
  const uint32_t m4 = cur.mask(0);
  const float rr[4] = {r4.x, r4.y, r4.z, r4.w}, vv[4] = {v4.x, v4.y, v4.z, v4.w};
  uint32_t valid[4], eos[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    valid[e] = ((m4 >> (8 * e)) & 0xFFu) != 0;
    eos[e] = rr[e] != 0.0f || rr[e] != rr[e];  // token_level_rewards.bool()
  }
  // ---- P1: next valid / next eos values, columns' deltas
  uint32_t hv = 0, he = 0;
  float fv = 0.0f, fe = 0.0f;  // leftmost valid / eos value of this group
#pragma unroll
  for (int e = 3; e >= 0; --e) {
    fv = valid[e] ? vv[e] : fv;
    hv |= valid[e];
    fe = eos[e] ? vv[e] : fe;
    he |= eos[e];
  }
  uint32_t hsv = hv, hse = he;
  float vsv = fv, vse = fe;
  row_suffix_first(hsv, vsv);
  row_suffix_first(hse, vse);
  uint32_t nhv = hsv, nhe = hse;  // groups strictly right of this one
  float nvv = vsv, nve = vse;
  row_shift_left1(nhv, nvv);
  row_shift_left1(nhe, nve);
  nvv = nhv ? nvv : cy.v_valid;
  nhv |= cy.h_valid;
  nve = nhe ? nve : cy.v_eos;
  nhe |= cy.h_eos;
  float d[4];
  uint32_t fl = 0;
#pragma unroll
  for (int e = 3; e >= 0; --e) {
    if (eos[e]) d[e] = (rr[e] + (nhe ? hg * nve : 0.0f)) - vv[e];          // high-level delta
    else d[e] = (rr[e] + g * (nhv ? nvv : 0.0f)) - vv[e];                   // low level (upd = reward)
    bad |= valid[e] & (eos[e] ^ 1u) & (nhv ^ 1u);                            // valid_positions[i + 1]
    fl |= (valid[e] | (eos[e] << 1)) << (8 * e);
    nvv = valid[e] ? vv[e] : nvv;
    nhv |= valid[e];
    nve = eos[e] ? vv[e] : nve;
    nhe |= eos[e];
  }
  // the next tile to the left continues from this tile's leftmost valid / eos position
  const uint32_t row_hv = row_lead(hsv), row_he = row_lead(hse);
  const float row_vv = row_lead(vsv), row_ve = row_lead(vse);
  cy.v_valid = row_hv ? row_vv : cy.v_valid;
  cy.h_valid |= row_hv;
  cy.v_eos = row_he ? row_ve : cy.v_eos;
  cy.h_eos |= row_he;
  const int o = rho * kBStr + 4 * grp;
  *reinterpret_cast<F4*>(sv + o) = v4;
  *reinterpret_cast<F4*>(sd + o) = F4{d[0], d[1], d[2], d[3]};
  sf[rho * (kBStr / 4) + grp] = fl;
  const uint64_t any_eos = __ballot(he), any_valid = __ballot(hv);
  __syncthreads();
  BL_T(t1);
  BL_ACC(0, t1 - t0);
  // ---- P2 / P3: the row walkers (group-0 lanes)
  if (grp == 0) {
    const float* pv = sv + rho * kBStr;
    float* pd = sd + rho * kBStr;
    float* ph = sh + rho * kBStr;
    float* pu = su + rho * kBStr;
    const uint32_t* pf = sf + rho * (kBStr / 4);
    uint32_t ge = (uint32_t)(any_eos >> (16 * rho)) & 0xFFFFu;
    while (ge) {  // eos groups, right to left
      const int q = 31 - __clz(ge);
      ge &= ~(1u << q);
      const uint32_t f4 = pf[q];
#pragma unroll
      for (int e = 3; e >= 0; --e) {
        if ((f4 >> (8 * e + 1)) & 1u) {
          const int c = 4 * q + e;
          wk.hl = pd[c] + hgl * wk.hl;
          const float vt = pv[c], upd = wk.hl + vt;  // updated_reward = returns = advantages + values
          ph[c] = wk.hl;
          pu[c] = upd;
          if (f4 >> (8 * e) & 1u) pd[c] = (upd + g * 0.0f) - vt;  // its low-level delta (nextvalue = 0)
        }
      }
    }
    uint32_t gv = (uint32_t)(any_valid >> (16 * rho)) & 0xFFFFu;
    while (gv) {  // valid groups, right to left
      const int q = 31 - __clz(gv);
      gv &= ~(1u << q);
      const uint32_t f4 = pf[q];
      F4 d4 = *reinterpret_cast<const F4*>(pd + 4 * q);
      float dd[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
      for (int e = 3; e >= 0; --e) {
        if ((f4 >> (8 * e)) & 1u) {
          wk.ll = dd[e] + gl * (((f4 >> (8 * e + 1)) & 1u) ? 0.0f : wk.ll);  // reset at an eos
          dd[e] = wk.ll;
        }
      }
      *reinterpret_cast<F4*>(pd + 4 * q) = F4{dd[0], dd[1], dd[2], dd[3]};
    }
  }
  __syncthreads();
  BL_T(t2);
  BL_ACC(1, t2 - t1);
  // ---- P4: outputs and row stats
  const F4 a4 = *reinterpret_cast<const F4*>(sd + o);
  const F4 h4 = *reinterpret_cast<const F4*>(sh + o);
  const F4 u4 = *reinterpret_cast<const F4*>(su + o);
  const float aa[4] = {a4.x, a4.y, a4.z, a4.w}, hh[4] = {h4.x, h4.y, h4.z, h4.w}, uu[4] = {u4.x, u4.y, u4.z, u4.w};
  float oa[4], oq[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (valid[e]) {
      oa[e] = aa[e];
      oq[e] = aa[e] + vv[e];
      s1 += (double)aa[e];
      s2 += (double)aa[e] * (double)aa[e];
      cnt += 1.0;
    } else if (eos[e]) {
      oa[e] = hh[e];
      oq[e] = uu[e];
    } else {
      oa[e] = 0.0f;
      oq[e] = 0.0f;
    }
  }
  const int64_t grow = row0 + rho, col = c0 + 4 * grp;
  if (grow < B && col >= 0 && col < L) {
    const int64_t go = grow * L + col;
    if (col + 4 <= L) {
      st_f4<NT>(adv + go, F4{oa[0], oa[1], oa[2], oa[3]});
      st_f4<NT>(ret + go, F4{oq[0], oq[1], oq[2], oq[3]});
    } else {
      for (int e = 0; e < 4; ++e)
        if (col + e < L) {
          adv[go + e] = oa[e];
          ret[go + e] = oq[e];
        }
    }
  }
  __syncthreads();
  BL_T(t3);
  BL_ACC(2, t3 - t2);
}

#ifdef RMI_BL_STAMPS
#define BL_ARG , bl_acc
#else
#define BL_ARG
#endif
#ifndef RMI_BL_DEPTH
#define RMI_BL_DEPTH 4
#endif
constexpr int kBlDepth = RMI_BL_DEPTH;  // tiles in the register pipeline (3 before round 4)
template <bool NT = false>
__global__ __launch_bounds__(64) void bilevel_tiled_kernel(const float* __restrict__ r, const float* __restrict__ v,
                                                           const uint8_t* __restrict__ mask, int64_t B, int64_t L,
                                                           float g, float gl, float hg, float hgl,
                                                           float* __restrict__ adv, float* __restrict__ ret,
                                                           double* __restrict__ row_stats,
                                                           uint8_t* __restrict__ err) {
  static_assert(kGLoads == 1 && kGRows * 16 == 64, "one 4-column group per lane");
  __shared__ __attribute__((aligned(16))) float sv[kGRows * kBStr];
  __shared__ __attribute__((aligned(16))) float sd[kGRows * kBStr];
  __shared__ __attribute__((aligned(16))) float sh[kGRows * kBStr];
  __shared__ __attribute__((aligned(16))) float su[kGRows * kBStr];
  __shared__ uint32_t sf[kGRows * kBStr / 4];
  const int lane = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kGRows;
  const int64_t ntiles = (L + kGCols - 1) / kGCols;
  BilevelCarry cy{0.0f, 0.0f, 0u, 0u};
  BilevelWalk wk{0.0f, 0.0f};
  double s1 = 0.0, s2 = 0.0, cnt = 0.0;
  uint32_t bad = 0;
#ifdef RMI_BL_STAMPS
  unsigned long long bl_acc[3] = {0, 0, 0};
  BL_T(tbeg);
#endif
  // a kBlDepth-deep register pipeline of tiles (right to left): tile k is walked while tiles
  // k-1 .. k-kBlDepth+1 are in flight.  Past the Infinity Cache the walks' serial chains leave
  // the loads alone in the memory system, so the bytes in flight per CU set the rate.
  const int64_t k0 = ntiles - 1;
  GaeTile t[kBlDepth];
#pragma unroll
  for (int i = 0; i < kBlDepth - 1; ++i) gae_load_tile<NT>(t[i], r, v, mask, B, L, row0, (k0 - i) * kGCols, lane);
  for (int64_t k = k0; k >= 0; k -= kBlDepth) {
#pragma unroll
    for (int j = 0; j < kBlDepth; ++j) {
      if (k - j < 0) break;
      gae_load_tile<NT>(t[(j + kBlDepth - 1) % kBlDepth], r, v, mask, B, L, row0, (k - j - (kBlDepth - 1)) * kGCols,
                    lane);
      bilevel_tile<NT>(t[j], (k - j) * kGCols, cy, wk, s1, s2, cnt, bad, sv, sd, sh, su, sf, lane, row0, B, L, g, gl, hg,
                   hgl, adv, ret BL_ARG);
    }
  }
#ifdef RMI_BL_STAMPS
  BL_T(tend);
  if (lane == 0) {
    g_bl_stamps[blockIdx.x * 4 + 0] = bl_acc[0];
    g_bl_stamps[blockIdx.x * 4 + 1] = bl_acc[1];
    g_bl_stamps[blockIdx.x * 4 + 2] = bl_acc[2];
    g_bl_stamps[blockIdx.x * 4 + 3] = tend - tbeg;
  }
#endif
  const double a = xor_sum16(s1), b2 = xor_sum16(s2), n = xor_sum16(cnt);
  const uint64_t bads = __ballot(bad);
  const int64_t row = row0 + (lane >> 4);
  if ((lane & 15) == 0 && row < B) {
    if (row_stats) {
      row_stats[3 * row + 0] = a;
      row_stats[3 * row + 1] = b2;
      row_stats[3 * row + 2] = n;
    }
    if (err) err[row] = ((bads >> (lane & ~15)) & 0xFFFFull) ? RMI_ERR_INDEX : 0;
  }
}

// ---- Bi-level GAE, segment-parallel (rows of up to kBsMaxCols columns; longer rows take
// bilevel_tiled_kernel above).  The low-level walk restarts at every valid eos column
// (core_algos.py:81-84: lastgaelam = 0.0 there), so after the high-level pass a row's
// low-level recurrence is independent per *segment* — the valid columns from one segment
// start (a valid eos column, or the rightmost valid column when it is not one) leftwards up to
// the next start.  The tiled kernel walks a row's segments one after another on one lane per
// row; here the whole row's deltas stay in LDS and every segment gets its own lane (16 per
// row), each walking its columns in the reference's order, so each element's f32 operations
// and operands are unchanged (bit-identical) while a wave's walk takes its longest segment
// instead of its longest row.
//   tile loop (right to left, the 3-deep register pipeline):  P1 column-parallel deltas and
//     flags into the row buffer, segment starts appended to a per-row list (DPP suffix count),
//     P2 the serial high-level walk over the tile's eos columns (as in the tiled kernel);
//   P3 the segment walks (a wave with more than kBsSeg starts in a row walks each row serially,
//     one lane per row, over the same buffer);
//   P4 column-parallel outputs and fp64 row stats (v re-read: an L2 hit, the row was read
//     microseconds before).
// LDS per wave: D f32[4][Lr], F u8[4][Lr/4] (valid nibble | eos nibble << 4 per 4-column
// group), S u16[4][kBsSeg], the tile's v staging, VG u16[4][tiles] (groups holding a valid
// column); at L = 1107 this is 20 KB (8 waves per CU).
constexpr int kBsSeg = 48;
#ifndef RMI_BS_PIPE
#define RMI_BS_PIPE 6
#endif
constexpr int kBsPipe = RMI_BS_PIPE;
#ifndef RMI_BS_MAX_LDS  // the segment kernel's LDS ceiling per wave (rows past it take the tiled kernel)
#define RMI_BS_MAX_LDS 65536
#endif
constexpr int64_t kBsMaxLds = RMI_BS_MAX_LDS;

__host__ __device__ inline int64_t bs_lr(int64_t L) { return (L + 3) & ~(int64_t)3; }
__host__ __device__ inline int64_t bs_foff(int64_t Lr) { return (int64_t)kGRows * Lr * 4; }
__host__ __device__ inline int64_t bs_soff(int64_t Lr) { return bs_foff(Lr) + (((int64_t)kGRows * (Lr / 4) + 15) & ~15); }
__host__ __device__ inline int64_t bs_voff(int64_t Lr) { return bs_soff(Lr) + (int64_t)kGRows * kBsSeg * 2; }
__host__ __device__ inline int64_t bs_nt(int64_t Lr) { return ((Lr + 63) / 64 + 1) & ~(int64_t)1; }  // VG words per row
__host__ __device__ inline int64_t bs_goff(int64_t Lr) { return bs_voff(Lr) + (int64_t)kGRows * kBStr * 4; }
__host__ __device__ inline int64_t bs_lds_bytes(int64_t L) {
  return bs_goff(bs_lr(L)) + (int64_t)kGRows * bs_nt(bs_lr(L)) * 2;
}

// inclusive suffix sum over the 16 groups of a DPP row (group g <- sum of groups >= g)
__device__ __forceinline__ int row_suffix_sum(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x101, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x102, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x104, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x108, 0xF, 0xF, true);
  return x;
}

__device__ __forceinline__ void bs_tile(const GaeTile& cur, int64_t c0, BilevelCarry& cy, float& hl, int& nseg,
                                        uint32_t& bad, float* __restrict__ D, uint8_t* __restrict__ F,
                                        uint16_t* __restrict__ S, float* __restrict__ sv, uint16_t* __restrict__ VG,
                                        int64_t Lr, int lane, float g, float hg, float hgl) {
  const int grp = lane & 15, rho = lane >> 4;
  const F4 r4 = cur.r[0], v4 = cur.v[0];
  const uint32_t m4 = cur.mask(0);
  const float rr[4] = {r4.x, r4.y, r4.z, r4.w}, vv[4] = {v4.x, v4.y, v4.z, v4.w};
  uint32_t valid[4], eos[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    valid[e] = ((m4 >> (8 * e)) & 0xFFu) != 0;
    eos[e] = rr[e] != 0.0f || rr[e] != rr[e];  // token_level_rewards.bool()
  }
  // ---- P1: as bilevel_tile (next valid / next eos values by DPP suffix selection + carry)
  uint32_t hv = 0, he = 0;
  float fv = 0.0f, fe = 0.0f;
#pragma unroll
  for (int e = 3; e >= 0; --e) {
    fv = valid[e] ? vv[e] : fv;
    hv |= valid[e];
    fe = eos[e] ? vv[e] : fe;
    he |= eos[e];
  }
  uint32_t hsv = hv, hse = he;
  float vsv = fv, vse = fe;
  row_suffix_first(hsv, vsv);
  row_suffix_first(hse, vse);
  uint32_t nhv = hsv, nhe = hse;
  float nvv = vsv, nve = vse;
  row_shift_left1(nhv, nvv);
  row_shift_left1(nhe, nve);
  nvv = nhv ? nvv : cy.v_valid;
  nhv |= cy.h_valid;
  nve = nhe ? nve : cy.v_eos;
  nhe |= cy.h_eos;
  float d[4];
  uint32_t fl = 0, st = 0;
#pragma unroll
  for (int e = 3; e >= 0; --e) {
    // high-level delta (r + (next eos ? hg * v_next_eos : 0)) - v, or the low level's
    // (r + g * (next valid ? v_next_valid : 0)) - v (upd = reward): each element's own f32
    // operations, with the add and the subtract shared
    const float t = eos[e] ? (nhe ? hg * nve : 0.0f) : g * (nhv ? nvv : 0.0f);
    d[e] = (rr[e] + t) - vv[e];
    bad |= valid[e] & (eos[e] ^ 1u) & (nhv ^ 1u);                    // valid_positions[i + 1]
    st |= (valid[e] & (eos[e] | (nhv ^ 1u))) << e;                   // segment start
    fl |= (valid[e] << e) | (eos[e] << (4 + e));
    nvv = valid[e] ? vv[e] : nvv;
    nhv |= valid[e];
    nve = eos[e] ? vv[e] : nve;
    nhe |= eos[e];
  }
  const uint32_t row_hv = row_lead(hsv), row_he = row_lead(hse);
  const float row_vv = row_lead(vsv), row_ve = row_lead(vse);
  cy.v_valid = row_hv ? row_vv : cy.v_valid;
  cy.h_valid |= row_hv;
  cy.v_eos = row_he ? row_ve : cy.v_eos;
  cy.h_eos |= row_he;
  const int64_t col = c0 + 4 * grp;
  float* Dr = D + rho * Lr;
  if (col < Lr) {
    *reinterpret_cast<F4*>(Dr + col) = F4{d[0], d[1], d[2], d[3]};
    F[rho * (Lr / 4) + (col >> 2)] = (uint8_t)fl;
  }
  *reinterpret_cast<F4*>(sv + rho * kBStr + 4 * grp) = v4;
  // segment starts, right to left: this group's rank = starts in the row's groups to its right
  const int ns = __popc(st);
  const int incl = row_suffix_sum(ns);
  const int tot = row_lead(incl);
  int idx = nseg + incl - ns;
#pragma unroll
  for (int e = 3; e >= 0; --e) {
    if ((st >> e) & 1u) {
      if (idx < kBsSeg) S[rho * kBsSeg + idx] = (uint16_t)(col + e);
      ++idx;
    }
  }
  nseg += tot;
  const uint64_t any_eos = __ballot(he), any_valid = __ballot(hv);
  if (grp == 0) VG[rho * bs_nt(Lr) + (c0 >> 6)] = (uint16_t)((any_valid >> (16 * rho)) & 0xFFFFu);
  __syncthreads();
  // ---- P2: the row's high-level walk over this tile's eos columns (group-0 lanes)
  if (grp == 0) {
    const uint8_t* Fr = F + rho * (Lr / 4) + (c0 >> 2);
    const float* pv = sv + rho * kBStr;
    float* pd = Dr + c0;
    uint32_t ge = (uint32_t)(any_eos >> (16 * rho)) & 0xFFFFu;
    while (ge) {
      const int q = 31 - __clz(ge);
      ge &= ~(1u << q);
      const uint32_t f = Fr[q];
#pragma unroll
      for (int e = 3; e >= 0; --e) {
        if ((f >> (4 + e)) & 1u) {
          const int c = 4 * q + e;
          hl = pd[c] + hgl * hl;
          const float vt = pv[c], upd = hl + vt;  // updated_reward = returns = advantages + values
          pd[c] = ((f >> e) & 1u) ? (upd + g * 0.0f) - vt : hl;  // valid: its low-level delta
        }
      }
    }
  }
  __syncthreads();
}

// one group of the walk: columns in vm advance the chain, the others keep their value
__device__ __forceinline__ float4 bs_group(uint32_t f, uint32_t vm, float4 d4, float gl, float& ll) {
  float dd[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
  for (int e = 3; e >= 0; --e) {
    const float nl = dd[e] + gl * (((f >> (4 + e)) & 1u) ? 0.0f : ll);
    const bool in = (vm >> e) & 1u;
    ll = in ? nl : ll;
    dd[e] = in ? nl : dd[e];
  }
  return make_float4(dd[0], dd[1], dd[2], dd[3]);
}
// a group shared with a neighbouring segment: only vm's columns are stored (the others go to
// the lane's dummy slot), so neither segment overwrites the other's results
__device__ __forceinline__ void bs_store_part(float* Dq, float4 r, uint32_t vm, float* dummy) {
  *((vm & 1u) ? Dq + 0 : dummy) = r.x;
  *((vm & 2u) ? Dq + 1 : dummy) = r.y;
  *((vm & 4u) ? Dq + 2 : dummy) = r.z;
  *((vm & 8u) ? Dq + 3 : dummy) = r.w;
}
// One segment's low-level walk: valid columns from s leftwards while > end, in the
// reference's order (ll = d + gl * (eos ? 0 : ll), the reset at a valid eos, core_algos.py:81-88).
// Branch-free over the segment's 4-column groups: every column is computed, and one outside
// the segment's valid columns keeps its value and the chain; the next group's flag byte and
// deltas are read before this one is worked on.
__device__ __forceinline__ void bs_walk(float* __restrict__ Dr, const uint8_t* __restrict__ Fr,
                                        float* __restrict__ dummy, int s, int end, float gl) {
  float ll = 0.0f;
  const int qs = s >> 2, qe = (end + 1) >> 2;
  const uint32_t ms = (2u << (s & 3)) - 1u, me = ~((1u << ((end + 1) & 3)) - 1u) & 0xFu;
  // the start group (shared with the segment to the right), then the interior groups — wholly
  // this segment's, stored as 16 B — then the end group (shared with the next segment)
  uint32_t f = Fr[qs];
  float4 d4 = *reinterpret_cast<const float4*>(Dr + 4 * qs);
  const int q1 = qs > qe ? qs - 1 : qs;
  uint32_t fn = Fr[q1];
  float4 dn = *reinterpret_cast<const float4*>(Dr + 4 * q1);
  uint32_t vm = f & ms & (qs == qe ? me : 0xFu);
  bs_store_part(Dr + 4 * qs, bs_group(f, vm, d4, gl, ll), vm, dummy);
  if (qs == qe) return;
  f = fn;
  d4 = dn;
  for (int q = qs - 1; q > qe; --q) {
    fn = Fr[q - 1];  // the next group's flags and deltas, read before this one is worked on
    dn = *reinterpret_cast<const float4*>(Dr + 4 * (q - 1));
    *reinterpret_cast<float4*>(Dr + 4 * q) = bs_group(f, f & 0xFu, d4, gl, ll);
    f = fn;
    d4 = dn;
  }
  vm = f & me;
  bs_store_part(Dr + 4 * qe, bs_group(f, vm, d4, gl, ll), vm, dummy);
}

// v groups c0, c0 + 64, ..., c0 + 7 * 64 of one row (zeros past L; the ragged group at L % 4)
template <bool NT>
__device__ __forceinline__ void bs_load_v(F4 (&vq)[8], const float* __restrict__ vrow, int64_t c0, int64_t L) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int64_t c = c0 + (int64_t)u * kGCols;
    vq[u] = F4{0.f, 0.f, 0.f, 0.f};
    if (c + 4 <= L) {
      vq[u] = ld_f4<NT>(vrow + c);
    } else if (c < L) {
      float t[4] = {0.f, 0.f, 0.f, 0.f};
      for (int e = 0; e < 4; ++e)
        if (c + e < L) t[e] = vrow[c + e];
      vq[u] = F4{t[0], t[1], t[2], t[3]};
    }
  }
}

template <bool NT = false>
__global__ __launch_bounds__(64) void bilevel_seg_kernel(const float* __restrict__ r, const float* __restrict__ v,
                                                         const uint8_t* __restrict__ mask, int64_t B, int64_t L,
                                                         float g, float gl, float hg, float hgl,
                                                         float* __restrict__ adv, float* __restrict__ ret,
                                                         double* __restrict__ row_stats, uint8_t* __restrict__ err) {
  static_assert(kGLoads == 1 && kGRows * 16 == 64, "one 4-column group per lane");
  extern __shared__ __attribute__((aligned(16))) uint8_t bs_smem[];
  const int64_t Lr = bs_lr(L);
  float* D = reinterpret_cast<float*>(bs_smem);
  uint8_t* F = bs_smem + bs_foff(Lr);
  uint16_t* S = reinterpret_cast<uint16_t*>(bs_smem + bs_soff(Lr));
  float* sv = reinterpret_cast<float*>(bs_smem + bs_voff(Lr));
  uint16_t* VG = reinterpret_cast<uint16_t*>(bs_smem + bs_goff(Lr));
  const int lane = threadIdx.x, grp = lane & 15, rho = lane >> 4;
  const int64_t row0 = (int64_t)blockIdx.x * kGRows;
  const int64_t ntiles = (L + kGCols - 1) / kGCols;
  BilevelCarry cy{0.0f, 0.0f, 0u, 0u};
  float hl = 0.0f;
  int nseg = 0;
  uint32_t bad = 0;
  BL_T(tb0);
  // kBsPipe register tiles, kBsPipe - 1 loads in flight behind the tile being worked on: the
  // tile work here is short (the walks come later), so the loads need the deeper pipeline
  GaeTile tq[kBsPipe];
  const int64_t k0 = ntiles - 1;
#pragma unroll
  for (int u = 0; u < kBsPipe - 1; ++u) gae_load_tile<NT>(tq[u], r, v, mask, B, L, row0, (k0 - u) * kGCols, lane);
  for (int64_t k = k0; k >= 0; k -= kBsPipe) {
#pragma unroll
    for (int u = 0; u < kBsPipe; ++u) {
      if (k - u < 0) break;
      gae_load_tile<NT>(tq[(u + kBsPipe - 1) % kBsPipe], r, v, mask, B, L, row0, (k - u - (kBsPipe - 1)) * kGCols, lane);
      bs_tile(tq[u], (k - u) * kGCols, cy, hl, nseg, bad, D, F, S, sv, VG, Lr, lane, g, hg, hgl);
    }
  }
  BL_T(tb1);
  const int64_t grow = row0 + rho;
  const bool live = grow < B;
  const float* vrow = v + (live ? grow : B - 1) * L;
  // ---- P3: segment walks
  float* Dr = D + rho * Lr;
  const uint8_t* Fr = F + rho * (Lr / 4);
  const uint16_t* Sr = S + rho * kBsSeg;
  const uint16_t* VGr = VG + rho * bs_nt(Lr);
  float* dummy = sv + lane;  // the tile staging is free now: one scratch slot per lane
  // the row's leftmost valid column bounds its last segment (the prompt and the left padding
  // to its left hold no valid column)
  int clo = 0;
  if (nseg > 0) {
    int tl = 0;
    while (VGr[tl] == 0) ++tl;
    const int ql = 16 * tl + __builtin_ctz((uint32_t)VGr[tl]);
    clo = 4 * ql + __builtin_ctz((uint32_t)Fr[ql] & 0xFu);
  }
  if (!__any(nseg > kBsSeg)) {
    for (int j = grp; j < nseg; j += 16)
      bs_walk(Dr, Fr, dummy, Sr[j], j + 1 < nseg ? (int)Sr[j + 1] : clo - 1, gl);
  } else if (grp == 0 && nseg > 0) {
    bs_walk(Dr, Fr, dummy, Sr[0], clo - 1, gl);  // the row's whole walk on one lane (the same element order)
  }
  __syncthreads();
  BL_T(tb2);
  // ---- P4: outputs and row stats; v re-read (an L2 hit) 8 tiles' groups at a time
  double s1 = 0.0, s2 = 0.0;
  int icnt = 0;  // the valid-column count (a sum of 1.0s is exact: counted as an integer)
  for (int64_t cb = 4 * grp; cb < L; cb += 8 * kGCols) {
    F4 cur[8];
    bs_load_v<NT>(cur, vrow, cb, L);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t c = cb + (int64_t)u * kGCols;
      if (c >= L) break;
      const F4 a4 = *reinterpret_cast<const F4*>(Dr + c);
      const uint32_t f = Fr[c >> 2];
      const float aa[4] = {a4.x, a4.y, a4.z, a4.w}, vv[4] = {cur[u].x, cur[u].y, cur[u].z, cur[u].w};
      float oa[4], oq[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // valid: the low-level walk; eos outside the mask: the high level (ret = adv + v); else 0.
        // Selects, not branches: an invalid column adds +0.0 to the row sums, which leaves them
        // unchanged (they start at +0.0, so they are never -0.0)
        const bool va = (f >> e) & 1u, out = ((f >> e) | (f >> (4 + e))) & 1u;
        oa[e] = out ? aa[e] : 0.0f;
        oq[e] = out ? aa[e] + vv[e] : 0.0f;
        const double ad = va ? (double)aa[e] : 0.0;
        s1 += ad;
        s2 += ad * ad;
        icnt += (int)va;
      }
      if (live) {
        const int64_t go = grow * L + c;
        if (c + 4 <= L) {
          st_f4<NT>(adv + go, F4{oa[0], oa[1], oa[2], oa[3]});
          st_f4<NT>(ret + go, F4{oq[0], oq[1], oq[2], oq[3]});
        } else {
          for (int e = 0; e < 4; ++e)
            if (c + e < L) {
              adv[go + e] = oa[e];
              ret[go + e] = oq[e];
            }
        }
      }
    }
  }
  const double a = xor_sum16(s1), b2 = xor_sum16(s2), n = xor_sum16((double)icnt);
  const uint64_t bads = __ballot(bad);
#ifdef RMI_BL_STAMPS
  BL_T(tb3);
  if (lane == 0) {
    g_bl_stamps[blockIdx.x * 4 + 0] = tb1 - tb0;
    g_bl_stamps[blockIdx.x * 4 + 1] = tb2 - tb1;
    g_bl_stamps[blockIdx.x * 4 + 2] = tb3 - tb2;
    g_bl_stamps[blockIdx.x * 4 + 3] = tb3 - tb0;
  }
#endif
  if (grp == 0 && live) {
    if (row_stats) {
      row_stats[3 * grow + 0] = a;
      row_stats[3 * grow + 1] = b2;
      row_stats[3 * grow + 2] = n;
    }
    if (err) err[grow] = ((bads >> (lane & ~15)) & 0xFFFFull) ? RMI_ERR_INDEX : 0;
  }
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
#pragma unroll 8  // the loads of 8 strides in flight together (the sums keep their order)
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

// x *= (mask != 0) elementwise (f32 multiply, so a negative value becomes -0.0 as in torch)
__global__ __launch_bounds__(kBlock) void mask_mul_kernel(float* __restrict__ x, const uint8_t* __restrict__ mask,
                                                          int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    x[i] = x[i] * (mask[i] ? 1.0f : 0.0f);
}

// GRPO: one wave per group segment; rows of the group are summed (fp64 -> f32) per row,
// group mean/std in fp64, then the per-row score is broadcast over the row's mask.
// mode 0: GRPO without std (also REINFORCE++-baseline's centred score), 1: GRPO, 2: RLOO
// (n > 1: s * n / (n - 1) - mean * n / (n - 1) in the reference's f32 op order; n == 1: s).
// Rows are read once: the first 64 row scores of a group stay in registers (lane i: row lo + i)
// for the broadcast pass, which reads only the mask.  Each row is split at 4-element
// boundaries of the flat index (a head and a tail of < 4 elements, one per lane, and a body
// where a lane moves 4 columns with 16-B accesses), whatever L is; `vec` = the base pointers
// allow it.
struct GrpoSpan {
  int64_t o, b0, b1, e;  // row start, body [b0, b1) (multiples of 4), row end
};
__device__ __forceinline__ GrpoSpan grpo_span(int64_t row, int64_t L, bool vec) {
  const int64_t o = row * L, e = o + L;
  int64_t b0 = vec ? (o + 3) & ~(int64_t)3 : e, b1 = vec ? e & ~(int64_t)3 : e;
  if (b0 > b1) b0 = b1 = e;
  return GrpoSpan{o, b0, b1, e};
}
__device__ __forceinline__ double grpo_row_sum(const float* __restrict__ r, const GrpoSpan& sp, int lane) {
  double s = 0.0;
  for (int64_t i = sp.o + lane; i < sp.b0; i += 64) s += (double)r[i];   // head (all of it without vec)
  for (int64_t i = sp.b0 + 4 * lane; i < sp.b1; i += 256) {
    const float4 x = *reinterpret_cast<const float4*>(r + i);
    s += ((double)x.x + (double)x.y) + ((double)x.z + (double)x.w);
  }
  for (int64_t i = sp.b1 + lane; i < sp.e; i += 64) s += (double)r[i];   // tail
  return wave_sum(s);
}

__global__ __launch_bounds__(kBlock) void grpo_kernel(const float* __restrict__ r, const uint8_t* __restrict__ mask,
                                                      int64_t B, int64_t L, const int32_t* __restrict__ seg, int G,
                                                      float eps, int norm_by_std, float* __restrict__ adv,
                                                      float* __restrict__ ret) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (g >= G) return;
  const int lo = seg[g], hi = seg[g + 1], n = hi - lo;
  if (n <= 0 || lo < 0 || hi > B) return;  // malformed segments are never read past [0, B)
  const bool vec = ((reinterpret_cast<uintptr_t>(r) | reinterpret_cast<uintptr_t>(adv) |
                     reinterpret_cast<uintptr_t>(ret)) & 15) == 0 && (reinterpret_cast<uintptr_t>(mask) & 3) == 0;
  // pass 1: group sums of row scores
  double gs = 0.0, gq = 0.0;
  float kept = 0.0f;
  for (int row = lo; row < hi; ++row) {
    const float sf = (float)grpo_row_sum(r, grpo_span(row, L, vec), lane);
    gs += sf;
    gq += (double)sf * (double)sf;
    kept = row - lo == lane ? sf : kept;
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
    const GrpoSpan sp = grpo_span(row, L, vec);
    const float sf = row - lo < 64 ? __shfl(kept, row - lo) : (float)grpo_row_sum(r, sp, lane);
    float sc;
    if (norm_by_std == 2) {
      const float fn = (float)n, fd = (float)(n - 1);
      sc = n > 1 ? (sf * fn) / fd - (mean * fn) / fd : sf;
    } else {
      sc = sf - mean;
      if (norm_by_std) sc = sc / (sd + eps);
    }
    for (int64_t i = sp.o + lane; i < sp.b0; i += 64) {
      const float y = sc * (float)(mask[i] != 0);
      adv[i] = y;
      ret[i] = y;
    }
    for (int64_t i = sp.b0 + 4 * lane; i < sp.b1; i += 256) {
      const uint32_t m4 = *reinterpret_cast<const uint32_t*>(mask + i);
      const float4 y = make_float4(sc * (float)((m4 & 0xFFu) != 0), sc * (float)((m4 & 0xFF00u) != 0),
                                   sc * (float)((m4 & 0xFF0000u) != 0), sc * (float)((m4 >> 24) != 0));
      *reinterpret_cast<float4*>(adv + i) = y;
      *reinterpret_cast<float4*>(ret + i) = y;
    }
    for (int64_t i = sp.b1 + lane; i < sp.e; i += 64) {
      const float y = sc * (float)(mask[i] != 0);
      adv[i] = y;
      ret[i] = y;
    }
  }
}

// RAGEN_AMD_BILEVEL_TILED=1 routes every row length to bilevel_tiled_kernel (parity tests run
// both kernels on the same rows; read per call so a test can flip it).
bool bilevel_force_tiled() {
  const char* s = getenv("RAGEN_AMD_BILEVEL_TILED");
  return s && s[0] == '1';
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
  const unsigned grid = (unsigned)((B + kGRows - 1) / kGRows);
  const bool nt = (double)B * (double)L * 17.0 > kStreamBytes;  // r, V, mask in; adv, ret out
  hipStream_t s = as_stream(stream);
  if (variant == 0 && nt)
    hipLaunchKernelGGL(gae_legacy_kernel<true>, dim3(grid), dim3(64), 0, s, r, v, mask, B, L, g, gl, adv, ret,
                       row_stats);
  else if (variant == 0)
    hipLaunchKernelGGL(gae_legacy_kernel<false>, dim3(grid), dim3(64), 0, s, r, v, mask, B, L, g, gl, adv, ret,
                       row_stats);
  else if (nt)
    hipLaunchKernelGGL((gae_kernel<1, true>), dim3(grid), dim3(64), 0, s, r, v, mask, B, L, g, gl, adv, ret, row_stats);
  else
    hipLaunchKernelGGL((gae_kernel<1, false>), dim3(grid), dim3(64), 0, s, r, v, mask, B, L, g, gl, adv, ret,
                       row_stats);
  return launch_status();
}

#ifdef RMI_BL_STAMPS
RMI_API int rmi_bilevel_set_stamps(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(rmi::g_bl_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -2;
}
#endif

RMI_API int rmi_bilevel_gae(const float* r, const float* v, const uint8_t* mask, int64_t B, int64_t L, double gamma,
                            double lam, double high_level_gamma, float* adv, float* ret, double* row_stats,
                            uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (!r || !v || !mask || !adv || !ret || B < 0 || L < 0) return RMI_EINVAL;
  if (B == 0 || L == 0) return RMI_OK;
  const dim3 grid((unsigned)((B + kGRows - 1) / kGRows));
  const float g = (float)gamma, gl = (float)(gamma * lam), hg = (float)high_level_gamma,
              hgl = (float)(high_level_gamma * lam);
  const int64_t lds = bs_lds_bytes(L);
  const bool nt = (double)B * (double)L * 17.0 > kStreamBytes;
  hipStream_t s = as_stream(stream);
  if (lds <= kBsMaxLds && !bilevel_force_tiled()) {
    if (lds > 65536) {  // (past 64 KB a launch declares the larger dynamic LDS first; gfx950 has 160 KB a CU)
      static const bool raised =
          hipFuncSetAttribute(reinterpret_cast<const void*>(bilevel_seg_kernel<true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBsMaxLds) == hipSuccess &&
          hipFuncSetAttribute(reinterpret_cast<const void*>(bilevel_seg_kernel<false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBsMaxLds) == hipSuccess;
      if (!raised) return RMI_EDEVICE;
    }
    if (nt)
      hipLaunchKernelGGL(bilevel_seg_kernel<true>, grid, dim3(64), (unsigned)lds, s, r, v, mask, B, L, g, gl, hg, hgl,
                         adv, ret, row_stats, err);
    else
      hipLaunchKernelGGL(bilevel_seg_kernel<false>, grid, dim3(64), (unsigned)lds, s, r, v, mask, B, L, g, gl, hg,
                         hgl, adv, ret, row_stats, err);
  } else if (nt) {
    hipLaunchKernelGGL(bilevel_tiled_kernel<true>, grid, dim3(64), 0, s, r, v, mask, B, L, g, gl, hg, hgl, adv, ret,
                       row_stats, err);
  } else {
    hipLaunchKernelGGL(bilevel_tiled_kernel<false>, grid, dim3(64), 0, s, r, v, mask, B, L, g, gl, hg, hgl, adv, ret,
                       row_stats, err);
  }
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

RMI_API int rmi_whiten_row_stats(const float* x, const uint8_t* mask, int64_t B, int64_t L, double* row_stats,
                                 rmi_stream_t stream) {
  using namespace rmi;
  if (!x || !mask || !row_stats || B < 0 || L < 0) return RMI_EINVAL;
  if (B == 0) return RMI_OK;
  const int per = kBlock / 64;
  hipLaunchKernelGGL(row_stats_kernel, dim3((unsigned)((B + per - 1) / per)), dim3(kBlock), 0, as_stream(stream), x,
                     mask, B, L, row_stats);
  return launch_status();
}

RMI_API int rmi_masked_whiten_stats(float* x, int64_t B, int64_t L, const double* stats, int64_t n_stats,
                                    void* scratch, rmi_stream_t stream) {
  using namespace rmi;
  if (!x || !stats || !scratch || B < 0 || L < 0 || n_stats < 0) return RMI_EINVAL;
  hipStream_t s = as_stream(stream);
  WhitenParams* params = reinterpret_cast<WhitenParams*>(scratch);
  hipLaunchKernelGGL(whiten_finalize_kernel, dim3(1), dim3(1024), 0, s, stats, n_stats, params);
  const int64_t n = B * L;
  if (n > 0) {
    int64_t blocks = (n / 4 + kBlock - 1) / kBlock;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(whiten_apply_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, x, n, params);
  }
  return launch_status();
}

RMI_API int rmi_grpo_outcome(const float* r, const uint8_t* mask, int64_t B, int64_t L, const int32_t* seg, int32_t G,
                             double eps, int32_t norm_by_std, float* adv, float* ret, rmi_stream_t stream) {
  using namespace rmi;
  if (!r || !mask || !seg || !adv || !ret || B < 0 || L < 0 || G < 0) return RMI_EINVAL;
  if (B == 0 || G == 0) return RMI_OK;
  const int per = kBlock / 64;
  hipLaunchKernelGGL(grpo_kernel, dim3((G + per - 1) / per), dim3(kBlock), 0, as_stream(stream), r, mask, B, L, seg, G,
                     (float)eps, norm_by_std, adv, ret);
  return launch_status();
}

RMI_API int rmi_reinforce_pp_returns(const float* r, const uint8_t* mask, int64_t B, int64_t L, double gamma,
                                     float* adv, float* ret, double* row_stats, rmi_stream_t stream) {
  using namespace rmi;
  if (!r || !mask || !adv || !ret || B < 0 || L < 0) return RMI_EINVAL;
  if (B == 0 || L == 0) return RMI_OK;
  const unsigned grid = (unsigned)((B + kGRows - 1) / kGRows);
  // v is not part of this recurrence: r stands in for it (read, never used)
  hipLaunchKernelGGL((gae_kernel<2, false>), dim3(grid), dim3(64), 0, as_stream(stream), r, r, mask, B, L, (float)gamma, 0.0f,
                     adv, ret, row_stats, nullptr);
  return launch_status();
}

RMI_API int rmi_remax(const float* r, const uint8_t* mask, const float* baseline, int64_t B, int64_t L, float* adv,
                      float* ret, rmi_stream_t stream) {
  using namespace rmi;
  if (!r || !mask || !baseline || !adv || !ret || B < 0 || L < 0) return RMI_EINVAL;
  if (B == 0 || L == 0) return RMI_OK;
  const unsigned grid = (unsigned)((B + kGRows - 1) / kGRows);
  hipLaunchKernelGGL((gae_kernel<3, false>), dim3(grid), dim3(64), 0, as_stream(stream), r, r, mask, B, L, 0.0f, 0.0f, adv,
                     ret, nullptr, baseline);
  return launch_status();
}

RMI_API int rmi_rloo_outcome(const float* r, const uint8_t* mask, int64_t B, int64_t L, const int32_t* seg, int32_t G,
                             float* adv, float* ret, rmi_stream_t stream) {
  using namespace rmi;
  if (!r || !mask || !seg || !adv || !ret || B < 0 || L < 0 || G < 0) return RMI_EINVAL;
  if (B == 0 || G == 0) return RMI_OK;
  const int per = kBlock / 64;
  hipLaunchKernelGGL(grpo_kernel, dim3((G + per - 1) / per), dim3(kBlock), 0, as_stream(stream), r, mask, B, L, seg, G,
                     0.0f, 2, adv, ret);
  return launch_status();
}

RMI_API int rmi_mask_mul(float* x, const uint8_t* mask, int64_t n, rmi_stream_t stream) {
  using namespace rmi;
  if (!x || !mask || n < 0) return RMI_EINVAL;
  if (n == 0) return RMI_OK;
  int64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(mask_mul_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, as_stream(stream), x, mask, n);
  return launch_status();
}
