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
// Memory (GAE): one 64-lane wave owns kGRows = 4 rows and streams them right to left in
// 4 x 64 tiles: every lane moves 4-column groups (16-B loads/stores, 256-B coalesced row
// segments) into a 3-deep register pipeline (two tiles in flight behind the one being
// worked on).  The column-parallel work (delta, ret = adv + v, fp64 whitening partials)
// runs on all 64 lanes; the tile is staged in LDS for the serial recurrence, walked by one
// lane per row (16-B LDS reads, row stride 272 B: conflict-free).  Few rows per wave keeps
// the serial walk the only long per-wave chain and puts 2 waves on every SIMD; at 8192 x
// 1093 tokens the kernel streams ~4.8 TB/s (HBM-bound).  Algorithmic traffic 17 B/token.
#include <math.h>

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

// One tile = rows [row0, row0+32) x columns [c0, c0+64) of r, v, mask, as 4-column groups:
// lane l, slot j -> row 4j + l/16, columns c0 + 4*(l%16) .. +3 (256-B coalesced row segments).
// Columns >= L and rows >= B read as zeros (a zero tail is an exact no-op for the recurrence:
// it starts the walk at column L-1 with last = nv = 0).
struct GaeTile {
  F4 r[kGLoads], v[kGLoads];
  uint32_t m[kGLoads];
};

__device__ __forceinline__ void gae_load_tile(GaeTile& t, const float* __restrict__ r, const float* __restrict__ v,
                                              const uint8_t* __restrict__ mask, int64_t B, int64_t L, int64_t row0,
                                              int64_t c0, int lane) {
  const int g = lane & 15;
  const int64_t col = c0 + 4 * g;
  const bool dummy = c0 < 0;  // a pipeline slot past column 0: every lane reads one shared line
  const bool full_col = col + 4 <= L && !dummy;
  // 1. every full 4-column group, branch-free from clamped (always valid) addresses, so all
  //    loads of the tile are in flight together; invalid groups are zeroed when staged
#pragma unroll
  for (int j = 0; j < kGLoads; ++j) {
    const int64_t row = min<int64_t>(row0 + 4 * j + (lane >> 4), B - 1);
    const int64_t o = dummy ? min<int64_t>(row0, B - 1) * L : (full_col ? row * L + col : row * L);
    t.r[j] = *reinterpret_cast<const F4*>(r + o);
    t.v[j] = *reinterpret_cast<const F4*>(v + o);
    t.m[j] = mask ? reinterpret_cast<const U8x4*>(mask + o)->x : 0x01010101u;
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
            mm |= (uint32_t)(mask ? mask[o + e] : 1) << (8 * e);
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
template <int VARIANT>
__device__ __forceinline__ void gae_col(float rt, float vt, float mt, float g, float gl, float& nv, float& last,
                                        float& a_out, float& ret_out) {
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

template <int VARIANT>
__global__ __launch_bounds__(64) void gae_kernel(const float* __restrict__ r, const float* __restrict__ v,
                                                 const uint8_t* __restrict__ mask, int64_t B, int64_t L, float g,
                                                 float gl, float* __restrict__ adv, float* __restrict__ ret,
                                                 double* __restrict__ row_stats) {
  __shared__ __attribute__((aligned(16))) float sr[kGRows * kGStr];  // r in, adv out
  __shared__ __attribute__((aligned(16))) float sv[kGRows * kGStr];  // v in, ret out
  __shared__ __attribute__((aligned(16))) uint8_t sm[kGRows * kGMStr];
  const int lane = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kGRows;
  const int64_t ntiles = (L + kGCols - 1) / kGCols;
  const bool walker = lane < kGRows && row0 + lane < B;
  float last = 0.0f, nv = 0.0f;
  double s1a = 0.0, s1b = 0.0, s2a = 0.0, s2b = 0.0, cnt = 0.0;  // row stats, two chains each

  GaeTile t;
  gae_load_tile(t, r, v, mask, B, L, row0, (ntiles - 1) * kGCols, lane);
  for (int64_t k = ntiles - 1; k >= 0; --k) {
    const int64_t c0 = k * kGCols;
    // registers -> LDS (the tile's 4-column groups), then prefetch the next tile to the left
#pragma unroll
    for (int j = 0; j < kGLoads; ++j) {
      const int row = 4 * j + (lane >> 4), grp = lane & 15;
      *reinterpret_cast<F4*>(sr + row * kGStr + 4 * grp) = t.r[j];
      *reinterpret_cast<F4*>(sv + row * kGStr + 4 * grp) = t.v[j];
      *reinterpret_cast<uint32_t*>(sm + row * kGMStr + 4 * grp) = t.m[j];
    }
    __syncthreads();
    if (k > 0) gae_load_tile(t, r, v, mask, B, L, row0, c0 - kGCols, lane);
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
        gae_col<VARIANT>(r4.w, v4.w, (float)((m4 >> 24) & 0xFF), g, gl, nv, last, a4.w, t4.w);
        gae_col<VARIANT>(r4.z, v4.z, (float)((m4 >> 16) & 0xFF), g, gl, nv, last, a4.z, t4.z);
        gae_col<VARIANT>(r4.y, v4.y, (float)((m4 >> 8) & 0xFF), g, gl, nv, last, a4.y, t4.y);
        gae_col<VARIANT>(r4.x, v4.x, (float)(m4 & 0xFF), g, gl, nv, last, a4.x, t4.x);
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
          *reinterpret_cast<F4*>(adv + o) = a4;
          *reinterpret_cast<F4*>(ret + o) = t4;
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
    const uint32_t m4 = cur.m[j];
    const double ax = (m4 & 0xFF) ? (double)a4.x : 0.0, ay = ((m4 >> 8) & 0xFF) ? (double)a4.y : 0.0;
    const double az = ((m4 >> 16) & 0xFF) ? (double)a4.z : 0.0, aw = (m4 >> 24) ? (double)a4.w : 0.0;
    st.s1[j] += (ax + ay) + (az + aw);
    st.s2[j] += (ax * ax + ay * ay) + (az * az + aw * aw);
    st.cnt[j] += __popc(m4 & 0x01010101u);
    if (grow < B && col >= 0 && col < L) {
      const int64_t o = grow * L + col;
      if (col + 4 <= L) {
        *reinterpret_cast<F4*>(adv + o) = a4;
        *reinterpret_cast<F4*>(ret + o) = t4;
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
  gae_load_tile(ta, r, v, mask, B, L, row0, k0 * kGCols, lane);
  gae_load_tile(tb, r, v, mask, B, L, row0, (k0 - 1) * kGCols, lane);
  for (int64_t k = k0; k >= 0; k -= 3) {
    gae_load_tile(tc, r, v, mask, B, L, row0, (k - 2) * kGCols, lane);
    gae_legacy_tile(ta, k * kGCols, st, sd, lane, walker, row0, B, L, g, gl, adv, ret);
    gae_load_tile(ta, r, v, mask, B, L, row0, (k - 3) * kGCols, lane);
    gae_legacy_tile(tb, (k - 1) * kGCols, st, sd, lane, walker, row0, B, L, g, gl, adv, ret);
    gae_load_tile(tb, r, v, mask, B, L, row0, (k - 4) * kGCols, lane);
    gae_legacy_tile(tc, (k - 2) * kGCols, st, sd, lane, walker, row0, B, L, g, gl, adv, ret);
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

// Bi-level GAE on the same tiled stream as the legacy kernel: tiles of 4 rows x 64 columns in
// a 3-deep register pipeline, staged in LDS (r, v, mask), walked right to left by one lane
// per row with the exact per-token logic of core_algos.py:44-88 (one reverse sweep doing both levels), the
// results staged back and stored as 16-B groups.
struct BilevelState {
  float hl, ll, v_next_eos, v_next_valid;
  bool has_eos, has_valid, bad;
  double s1, s2, cnt;
};

__device__ __forceinline__ void bilevel_col(float rt, float vt, bool m, float g, float gl, float hg, float hgl,
                                            BilevelState& w, float& a_out, float& q_out) {
  const bool eos = rt != 0.0f || rt != rt;  // token_level_rewards.bool()
  float a = 0.0f, q = 0.0f, upd = rt;
  if (eos) {
    const float delta = (rt + (w.has_eos ? hg * w.v_next_eos : 0.0f)) - vt;
    w.hl = delta + hgl * w.hl;
    a = w.hl;
    upd = w.hl + vt;  // updated_reward = advantages + values
    q = upd;          // returns = advantages + values
    w.v_next_eos = vt;
    w.has_eos = true;
  }
  if (m) {
    float nvv;
    if (eos) {
      nvv = 0.0f;
      w.ll = 0.0f;
    } else {
      if (!w.has_valid) w.bad = true;  // valid_positions[i + 1] -> IndexError
      nvv = w.v_next_valid;
    }
    const float delta = (upd + g * nvv) - vt;
    w.ll = delta + gl * w.ll;
    a = w.ll;
    q = w.ll + vt;
    w.v_next_valid = vt;
    w.has_valid = true;
    w.s1 += (double)a;
    w.s2 += (double)a * (double)a;
    w.cnt += 1.0;
  }
  a_out = a;
  q_out = q;
}

__device__ __forceinline__ void bilevel_tile(const GaeTile& cur, int64_t c0, BilevelState& w, float* sr, float* sv,
                                             uint8_t* sm, int lane, bool walker, int64_t row0, int64_t B, int64_t L,
                                             float g, float gl, float hg, float hgl, float* __restrict__ adv,
                                             float* __restrict__ ret) {
  const int grp = lane & 15;
#pragma unroll
  for (int j = 0; j < kGLoads; ++j) {
    const int row = 4 * j + (lane >> 4);
    *reinterpret_cast<F4*>(sr + row * kGStr + 4 * grp) = cur.r[j];
    *reinterpret_cast<F4*>(sv + row * kGStr + 4 * grp) = cur.v[j];
    *reinterpret_cast<uint32_t*>(sm + row * kGMStr + 4 * grp) = cur.m[j];
  }
  __syncthreads();
  if (walker) {
    float* pr = sr + lane * kGStr;
    float* pv = sv + lane * kGStr;
    const uint8_t* pm = sm + lane * kGMStr;
    for (int q = kGCols / 4 - 1; q >= 0; --q) {
      const F4 r4 = *reinterpret_cast<const F4*>(pr + 4 * q);
      const F4 v4 = *reinterpret_cast<const F4*>(pv + 4 * q);
      const uint32_t m4 = *reinterpret_cast<const uint32_t*>(pm + 4 * q);
      F4 a4, t4;
      bilevel_col(r4.w, v4.w, (m4 >> 24) & 0xFF, g, gl, hg, hgl, w, a4.w, t4.w);
      bilevel_col(r4.z, v4.z, (m4 >> 16) & 0xFF, g, gl, hg, hgl, w, a4.z, t4.z);
      bilevel_col(r4.y, v4.y, (m4 >> 8) & 0xFF, g, gl, hg, hgl, w, a4.y, t4.y);
      bilevel_col(r4.x, v4.x, m4 & 0xFF, g, gl, hg, hgl, w, a4.x, t4.x);
      *reinterpret_cast<F4*>(pr + 4 * q) = a4;
      *reinterpret_cast<F4*>(pv + 4 * q) = t4;
    }
  }
  __syncthreads();
  const int64_t col = c0 + 4 * grp;
#pragma unroll
  for (int j = 0; j < kGLoads; ++j) {
    const int row = 4 * j + (lane >> 4);
    const int64_t grow = row0 + row;
    if (grow < B && col >= 0 && col < L) {
      const F4 a4 = *reinterpret_cast<const F4*>(sr + row * kGStr + 4 * grp);
      const F4 t4 = *reinterpret_cast<const F4*>(sv + row * kGStr + 4 * grp);
      const int64_t o = grow * L + col;
      if (col + 4 <= L) {
        *reinterpret_cast<F4*>(adv + o) = a4;
        *reinterpret_cast<F4*>(ret + o) = t4;
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

__global__ __launch_bounds__(64) void bilevel_tiled_kernel(const float* __restrict__ r, const float* __restrict__ v,
                                                           const uint8_t* __restrict__ mask, int64_t B, int64_t L,
                                                           float g, float gl, float hg, float hgl,
                                                           float* __restrict__ adv, float* __restrict__ ret,
                                                           double* __restrict__ row_stats,
                                                           uint8_t* __restrict__ err) {
  __shared__ __attribute__((aligned(16))) float sr[kGRows * kGStr];
  __shared__ __attribute__((aligned(16))) float sv[kGRows * kGStr];
  __shared__ __attribute__((aligned(16))) uint8_t sm[kGRows * kGMStr];
  const int lane = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kGRows;
  const int64_t ntiles = (L + kGCols - 1) / kGCols;
  const bool walker = lane < kGRows && row0 + lane < B;
  BilevelState w;
  w.hl = w.ll = w.v_next_eos = w.v_next_valid = 0.0f;
  w.has_eos = w.has_valid = w.bad = false;
  w.s1 = w.s2 = w.cnt = 0.0;
  GaeTile ta, tb, tc;
  const int64_t k0 = ntiles - 1;
  gae_load_tile(ta, r, v, mask, B, L, row0, k0 * kGCols, lane);
  gae_load_tile(tb, r, v, mask, B, L, row0, (k0 - 1) * kGCols, lane);
  for (int64_t k = k0; k >= 0; k -= 3) {
    gae_load_tile(tc, r, v, mask, B, L, row0, (k - 2) * kGCols, lane);
    bilevel_tile(ta, k * kGCols, w, sr, sv, sm, lane, walker, row0, B, L, g, gl, hg, hgl, adv, ret);
    gae_load_tile(ta, r, v, mask, B, L, row0, (k - 3) * kGCols, lane);
    bilevel_tile(tb, (k - 1) * kGCols, w, sr, sv, sm, lane, walker, row0, B, L, g, gl, hg, hgl, adv, ret);
    gae_load_tile(tb, r, v, mask, B, L, row0, (k - 4) * kGCols, lane);
    bilevel_tile(tc, (k - 2) * kGCols, w, sr, sv, sm, lane, walker, row0, B, L, g, gl, hg, hgl, adv, ret);
  }
  if (walker) {
    const int64_t row = row0 + lane;
    if (row_stats) {
      row_stats[3 * row + 0] = w.s1;
      row_stats[3 * row + 1] = w.s2;
      row_stats[3 * row + 2] = w.cnt;
    }
    if (err) err[row] = w.bad ? RMI_ERR_INDEX : 0;
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
  const unsigned grid = (unsigned)((B + kGRows - 1) / kGRows);
  if (variant == 0)
    hipLaunchKernelGGL(gae_legacy_kernel, dim3(grid), dim3(64), 0, as_stream(stream), r, v, mask, B, L, g, gl, adv,
                       ret, row_stats);
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
  hipLaunchKernelGGL(bilevel_tiled_kernel, dim3((unsigned)((B + kGRows - 1) / kGRows)), dim3(64), 0,
                     as_stream(stream), r, v, mask, B, L, (float)gamma, (float)(gamma * lam), (float)high_level_gamma,
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
