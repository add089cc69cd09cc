// turnglue.hip — the per-turn glue of the device turn loop, one launch each (gfx950).
//
//  rmi_turn_inputs    EnvStateManager._step_device before the turn: which envs step (the rows
//                     with a generation that decoded) and their zeroed error bytes
//  rmi_turn_readback  _step_device after the turn + render: the turn record's flags copy and
//                     actions-left column, and ONE packed buffer the host reads back (flags,
//                     step errors, decode errors, the longest decoded response and observation)
//  rmi_prompt_commit  DevicePrompts._encode after the BPE launch: the rows the device could not
//                     build, and the update-batch marks of the rows that took part
//  rmi_rows_stats     DevicePrompts.gen_batch: the longest arena row among the batch rows and
//                     whether any row waits for the host, as two ints read back together
//  rmi_next_rows_stats  the same over the envs that go on after a turn (a generation this turn,
//                     not done), launched by the turn itself after the next prompt's encode, so
//                     the turn's one readback carries them (no readback of its own)
//
// Each replaced 3-8 torch elementwise / reduction launches; in a kernel trace of the API rollout
// (profiles/r04_api_timeline.txt) the turn loop's GPU sat idle between small launches for most
// of each turn.  The reductions (readback, rows_stats) are single 1024-thread workgroups: no
// atomics, no zero fill, a few microseconds at 8192 rows.
#include "common.hpp"

namespace rmi {
namespace {

constexpr int kGlueBlock = 256;
constexpr int kRedBlock = 1024;

__global__ __launch_bounds__(kGlueBlock) void turn_inputs_kernel(const uint8_t* __restrict__ has_t,
                                                                 const uint8_t* __restrict__ dec_err, int64_t B,
                                                                 uint8_t* __restrict__ has, uint8_t* __restrict__ err) {
  for (int64_t e = (int64_t)blockIdx.x * kGlueBlock + threadIdx.x; e < B; e += (int64_t)gridDim.x * kGlueBlock) {
    const bool in = has_t ? has_t[e] != 0 : true;
    has[e] = (in && dec_err[e] == 0) ? 1 : 0;
    err[e] = 0;
  }
}

// block-wide max of one int per thread (kRedBlock threads) -> every thread
__device__ __forceinline__ int block_max(int v, int* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  int m = red[0];
#pragma unroll
  for (int w = 1; w < kRedBlock / 64; ++w) m = max(m, red[w]);
  __syncthreads();
  return m;
}

// block-wide sum of one int per thread -> every thread
__device__ __forceinline__ int block_sum(int v, int* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  int m = 0;
#pragma unroll
  for (int w = 0; w < kRedBlock / 64; ++w) m += red[w];
  __syncthreads();
  return m;
}

// block-wide OR of one int per thread -> every thread
__device__ __forceinline__ int block_or(int v, int* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  int m = 0;
#pragma unroll
  for (int w = 0; w < kRedBlock / 64; ++w) m |= red[w];
  __syncthreads();
  return m;
}

// the OR of the eight bytes of x
__device__ __forceinline__ uint32_t fold_or(uint64_t x) {
  x |= x >> 32;
  x |= x >> 16;
  x |= x >> 8;
  return (uint32_t)(x & 0xFFu);
}

// V8: eight envs per thread with 8-B / 16-B loads and stores (B % 8 == 0, aligned arrays): at
// 8192 envs one pass of independent loads instead of eight dependent loop trips
// (NULL counts as aligned: an absent optional array)
inline bool aligned(const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }
__device__ __forceinline__ int4 ld_i4(const int32_t* p) { return *reinterpret_cast<const int4*>(p); }
__device__ __forceinline__ uint64_t ld_u8x8(const uint8_t* p) { return *reinterpret_cast<const uint64_t*>(p); }
__device__ __forceinline__ int max4(int4 v) { return max(max(v.x, v.y), max(v.z, v.w)); }

template <bool V8>
__global__ __launch_bounds__(kRedBlock) void turn_readback_kernel(
    const uint8_t* __restrict__ flags, const uint8_t* __restrict__ err, const uint8_t* __restrict__ dec_err,
    const uint8_t* __restrict__ num_actions, const int32_t* __restrict__ max_actions,
    const int32_t* __restrict__ text_len, const int32_t* __restrict__ obs_len, int64_t B,
    uint8_t* __restrict__ flags_copy, int32_t* __restrict__ left, uint8_t* __restrict__ pack,
    const uint8_t* __restrict__ pad_err = nullptr, int64_t n_pad = 0, bool summary = false) {
  __shared__ int red[kRedBlock / 64];
  int tmax = 0, omax = 0, npad = 0, ndone = 0;
  uint32_t eor = 0, dor = 0;  // (summary) OR of the step / decode error bytes
  if (pad_err)  // the generation batch's rows rmi_pad_rows flagged (left-cut): counted
    for (int64_t i = threadIdx.x; i < n_pad; i += kRedBlock) npad += pad_err[i] != 0;
  if (V8) {
    for (int64_t g = threadIdx.x; g < (B >> 3); g += kRedBlock) {
      const int64_t e = g << 3;
      const uint64_t f = ld_u8x8(flags + e), er = ld_u8x8(err + e), de = ld_u8x8(dec_err + e);
      const uint64_t na = ld_u8x8(num_actions + e);
      const int4 m0 = ld_i4(max_actions + e), m1 = ld_i4(max_actions + e + 4);
      if (text_len) tmax = max(tmax, max(max4(ld_i4(text_len + e)), max4(ld_i4(text_len + e + 4))));
      if (obs_len) omax = max(omax, max(max4(ld_i4(obs_len + e)), max4(ld_i4(obs_len + e + 4))));
      *reinterpret_cast<uint64_t*>(flags_copy + e) = f;
      const auto nb = [na](int j) { return (int32_t)((na >> (8 * j)) & 0xFFu); };
      *reinterpret_cast<int4*>(left + e) = make_int4(m0.x - nb(0), m0.y - nb(1), m0.z - nb(2), m0.w - nb(3));
      *reinterpret_cast<int4*>(left + e + 4) = make_int4(m1.x - nb(4), m1.y - nb(5), m1.z - nb(6), m1.w - nb(7));
      *reinterpret_cast<uint64_t*>(pack + e) = f;
      *reinterpret_cast<uint64_t*>(pack + B + e) = er;
      *reinterpret_cast<uint64_t*>(pack + 2 * B + e) = de;
      eor |= fold_or(er);
      dor |= fold_or(de);
      ndone += __popcll(f & (0x0101010101010101ull * RMI_FLAG_DONE));
    }
  } else {
    for (int64_t e = threadIdx.x; e < B; e += kRedBlock) {
      const uint8_t f = flags[e];
      flags_copy[e] = f;
      left[e] = max_actions[e] - (int32_t)num_actions[e];
      pack[e] = f;
      pack[B + e] = err[e];
      pack[2 * B + e] = dec_err[e];
      eor |= err[e];
      dor |= dec_err[e];
      ndone += (f & RMI_FLAG_DONE) != 0;
      if (text_len) tmax = max(tmax, text_len[e]);
      if (obs_len) omax = max(omax, obs_len[e]);
    }
  }
  tmax = block_max(tmax, red);
  omax = block_max(omax, red);
  if (summary) {
    npad = block_sum(npad, red);
    ndone = block_sum(ndone, red);
    eor = (uint32_t)block_or((int)(eor | (dor << 8)), red);
  }
  if (threadIdx.x == 0) {
    int32_t* tail = reinterpret_cast<int32_t*>(pack + ((3 * B + 3) & ~(int64_t)3));
    tail[0] = tmax;
    tail[1] = omax;
    if (summary) {
      tail[6] = npad;
      tail[7] = (int32_t)eor;
      tail[8] = ndone;
    }
  }
}

__global__ __launch_bounds__(kGlueBlock) void prompt_commit_kernel(const uint8_t* __restrict__ bpe_err,
                                                                   const uint8_t* __restrict__ text_err,
                                                                   const uint8_t* __restrict__ active,
                                                                   const int32_t* __restrict__ mark_tok,
                                                                   int32_t* __restrict__ len_upd, int64_t B,
                                                                   uint8_t* __restrict__ bad) {
  for (int64_t e = (int64_t)blockIdx.x * kGlueBlock + threadIdx.x; e < B; e += (int64_t)gridDim.x * kGlueBlock) {
    const bool on = active ? active[e] != 0 : true;
    bad[e] = (on && (bpe_err[e] != 0 || text_err[e] != 0)) ? 1 : 0;
    if (mark_tok && on) len_upd[e] = mark_tok[e];
  }
}

// rmi_prompt_commit followed by rmi_next_rows_stats over the bad rows it writes, in one
// workgroup (both on the turn's critical path after the encode): bad / len_upd per env as
// prompt_commit_kernel, then (longest next row, any bad, count) as next_rows_stats_kernel
template <bool V8>
__global__ __launch_bounds__(kRedBlock) void prompt_commit_stats_kernel(
    const uint8_t* __restrict__ bpe_err, const uint8_t* __restrict__ text_err, const uint8_t* __restrict__ active,
    const int32_t* __restrict__ mark_tok, int32_t* __restrict__ len_upd, int64_t B, uint8_t* __restrict__ bad,
    const int32_t* __restrict__ len, const uint8_t* __restrict__ has, const uint8_t* __restrict__ flags,
    int32_t* __restrict__ stats) {
  __shared__ int red[kRedBlock / 64];
  int m = 0, any = 0, cnt = 0;
  if (V8) {  // eight envs per thread, 8- and 16-B accesses (B % 8 == 0, aligned arrays)
    for (int64_t g = threadIdx.x; g < (B >> 3); g += kRedBlock) {
      const int64_t e = g << 3;
      const uint64_t be = ld_u8x8(bpe_err + e), te = ld_u8x8(text_err + e), f = ld_u8x8(flags + e);
      const uint64_t ac = active ? ld_u8x8(active + e) : ~0ull, h = has ? ld_u8x8(has + e) : ~0ull;
      const int4 l0 = ld_i4(len + e), l1 = ld_i4(len + e + 4);
      int4 k0 = make_int4(0, 0, 0, 0), k1 = k0, u0 = k0, u1 = k0;
      if (mark_tok) {
        k0 = ld_i4(mark_tok + e);
        k1 = ld_i4(mark_tok + e + 4);
        u0 = ld_i4(len_upd + e);
        u1 = ld_i4(len_upd + e + 4);
      }
      const int lv[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
      const int kv[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
      int uv[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
      uint64_t bw = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int sh = 8 * j;
        const bool on = ((ac >> sh) & 0xFFu) != 0;
        const bool b = on && (((be >> sh) & 0xFFu) != 0 || ((te >> sh) & 0xFFu) != 0);
        bw |= (uint64_t)(b ? 1 : 0) << sh;
        any |= b;
        if (on) uv[j] = kv[j];
        if (((h >> sh) & 0xFFu) != 0 && !((f >> sh) & RMI_FLAG_DONE)) {
          m = max(m, lv[j]);
          ++cnt;
        }
      }
      *reinterpret_cast<uint64_t*>(bad + e) = bw;
      if (mark_tok) {
        *reinterpret_cast<int4*>(len_upd + e) = make_int4(uv[0], uv[1], uv[2], uv[3]);
        *reinterpret_cast<int4*>(len_upd + e + 4) = make_int4(uv[4], uv[5], uv[6], uv[7]);
      }
    }
  } else
  for (int64_t e = threadIdx.x; e < B; e += kRedBlock) {
    const bool on = active ? active[e] != 0 : true;
    const bool b = on && (bpe_err[e] != 0 || text_err[e] != 0);
    bad[e] = b ? 1 : 0;
    if (mark_tok && on) len_upd[e] = mark_tok[e];
    any |= b;
    if ((has ? has[e] != 0 : true) && !(flags[e] & RMI_FLAG_DONE)) {
      m = max(m, len[e]);
      ++cnt;
    }
  }
  m = block_max(m, red);
  any = block_max(any, red);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int c = 0;
#pragma unroll
    for (int w = 0; w < kRedBlock / 64; ++w) c += red[w];
    stats[0] = m;
    stats[1] = any;
    stats[2] = c;
  }
}

// exclusive prefix sum of one int per thread over the kRedBlock-thread workgroup (thread order);
// *total = the sum.  red: kRedBlock / 64 ints of LDS.
__device__ __forceinline__ int block_exclusive_scan(int v, int* red, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) red[w] = x;
  __syncthreads();
  int before = 0, all = 0;
#pragma unroll
  for (int i = 0; i < kRedBlock / 64; ++i) {
    const int t = red[i];
    before += i < w ? t : 0;
    all += t;
  }
  __syncthreads();
  *total = all;
  return before + x - v;
}

// The next generation batch's rows on the device: rows[k] = the k-th env (ascending) with has[e]
// (NULL: every env) and no RMI_FLAG_DONE -- the envs es_manager.step hands back (es_manager.py:
// 168-169) when the turn's envs came in ascending order -- and src[e] = its k, or -1.  (The turn
// chain writes them after the commit; the next turn's gen_rows and pad_rows read them instead of
// an upload of the ids the host derived.)  Eight envs per thread, one block-wide scan per 8192.
__global__ __launch_bounds__(kRedBlock) void next_rows_list_kernel(const uint8_t* __restrict__ has,
                                                                   const uint8_t* __restrict__ flags, int64_t B,
                                                                   int64_t* __restrict__ rows,
                                                                   int64_t* __restrict__ src) {
  __shared__ int red[kRedBlock / 64];
  int64_t base = 0;
  for (int64_t e0 = 0; e0 < B; e0 += 8 * kRedBlock) {
    const int64_t e = e0 + 8 * (int64_t)threadIdx.x;
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (e + j < B && (has ? has[e + j] != 0 : true) && !(flags[e + j] & RMI_FLAG_DONE)) bits |= 1u << j;
    int total;
    int64_t k = base + block_exclusive_scan(__builtin_popcount(bits), red, &total);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (e + j >= B) break;
      if ((bits >> j) & 1u) {
        rows[k] = e + j;
        src[e + j] = k++;
      } else {
        src[e + j] = -1;
      }
    }
    base += total;
  }
}

// formulate_rollouts' first pass (ctx_manager.py:52-62, :278-306 on the device record): the
// update rows' longest, whether a row waits for the host, the most turns (zip_longest's length)
// -> stats i32[3], and the per-env turn counts widened for the assembly -> n_sc i32[B]
__global__ __launch_bounds__(kRedBlock) void formulate_stats_kernel(const int32_t* __restrict__ len,
                                                                    const uint8_t* __restrict__ bad,
                                                                    const uint8_t* __restrict__ n_turns, int64_t B,
                                                                    int32_t* __restrict__ n_sc,
                                                                    int32_t* __restrict__ stats) {
  __shared__ int red[kRedBlock / 64];
  int m = 0, any = 0, mt = 0;
  for (int64_t e = threadIdx.x; e < B; e += kRedBlock) {
    m = max(m, len[e]);
    if (bad) any |= bad[e];
    const int nt = n_turns[e];
    n_sc[e] = nt;
    mt = max(mt, nt);
  }
  m = block_max(m, red);
  any = block_max(any != 0 ? 1 : 0, red);
  mt = block_max(mt, red);
  if (threadIdx.x == 0) {
    stats[0] = m;
    stats[1] = any;
    stats[2] = mt;
  }
}

// formulate_rollouts' reductions after the assembly: the response tokens of every row summed
// (response_length's numerator, ctx_manager.py:305: exact in 64 bits), and the assembly's error
// bytes OR-ed -> out i64[2]
__global__ __launch_bounds__(kRedBlock) void formulate_tail_kernel(const int32_t* __restrict__ resp_count,
                                                                   const uint8_t* __restrict__ err, int64_t B,
                                                                   int64_t* __restrict__ out) {
  __shared__ long long lred[kRedBlock / 64];
  __shared__ int red[kRedBlock / 64];
  long long tot = 0;
  int bits = 0;
  for (int64_t e = threadIdx.x; e < B; e += kRedBlock) {
    tot += resp_count[e];
    bits |= err[e];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    tot += __shfl_xor(tot, o);
    bits |= __shfl_xor(bits, o);
  }
  if ((threadIdx.x & 63) == 0) {
    lred[threadIdx.x >> 6] = tot;
    red[threadIdx.x >> 6] = bits;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0;
    int b = 0;
#pragma unroll
    for (int w = 0; w < kRedBlock / 64; ++w) {
      t += lred[w];
      b |= red[w];
    }
    out[0] = t;
    out[1] = b;
  }
}

__global__ __launch_bounds__(kRedBlock) void rows_stats_kernel(const int32_t* __restrict__ len,
                                                               const int64_t* __restrict__ rows, int64_t n_rows,
                                                               const uint8_t* __restrict__ bad, int64_t B,
                                                               int32_t* __restrict__ stats) {
  __shared__ int red[kRedBlock / 64];
  int m = 0, any = 0;
  for (int64_t i = threadIdx.x; i < n_rows; i += kRedBlock) {
    const int64_t r = rows ? rows[i] : i;
    if (r >= 0 && r < B) m = max(m, len[r]);  // (the host validated the rows: a guard, not a rule)
  }
  if (bad)
    for (int64_t e = threadIdx.x; e < B; e += kRedBlock) any |= bad[e];
  m = block_max(m, red);
  any = block_max(any != 0 ? 1 : 0, red);
  if (threadIdx.x == 0) {
    stats[0] = m;
    stats[1] = any;
  }
}

template <bool V8>
__global__ __launch_bounds__(kRedBlock) void next_rows_stats_kernel(const int32_t* __restrict__ len,
                                                                    const uint8_t* __restrict__ has,
                                                                    const uint8_t* __restrict__ flags,
                                                                    const uint8_t* __restrict__ bad, int64_t B,
                                                                    int32_t* __restrict__ stats) {
  __shared__ int red[kRedBlock / 64];
  int m = 0, any = 0, cnt = 0;
  if (V8) {
    for (int64_t g = threadIdx.x; g < (B >> 3); g += kRedBlock) {
      const int64_t e = g << 3;
      const uint64_t f = ld_u8x8(flags + e), h = has ? ld_u8x8(has + e) : ~0ull;
      const int4 l0 = ld_i4(len + e), l1 = ld_i4(len + e + 4);
      if (bad) any |= ld_u8x8(bad + e) != 0;
      const int lv[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool next = ((h >> (8 * j)) & 0xFFu) != 0 && !((f >> (8 * j)) & RMI_FLAG_DONE);
        if (next) {
          m = max(m, lv[j]);
          ++cnt;
        }
      }
    }
  } else {
    for (int64_t e = threadIdx.x; e < B; e += kRedBlock) {
      const bool next = (has ? has[e] != 0 : true) && !(flags[e] & RMI_FLAG_DONE);
      if (next) {
        m = max(m, len[e]);
        ++cnt;
      }
      if (bad) any |= bad[e];
    }
  }
  m = block_max(m, red);
  any = block_max(any != 0 ? 1 : 0, red);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int c = 0;
#pragma unroll
    for (int w = 0; w < kRedBlock / 64; ++w) c += red[w];
    stats[0] = m;
    stats[1] = any;
    stats[2] = c;
  }
}

inline unsigned glue_grid(int64_t B) {
  const int64_t g = (B + kGlueBlock - 1) / kGlueBlock;
  return (unsigned)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

}  // namespace
}  // namespace rmi

RMI_API int rmi_turn_inputs(const uint8_t* has_t, const uint8_t* dec_err, int64_t B, uint8_t* has, uint8_t* err,
                            rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0) return RMI_EINVAL;
  if (B == 0) return RMI_OK;
  if (!dec_err || !has || !err) return RMI_EINVAL;
  hipLaunchKernelGGL(turn_inputs_kernel, dim3(glue_grid(B)), dim3(kGlueBlock), 0, as_stream(stream), has_t, dec_err,
                     B, has, err);
  return launch_status();
}

RMI_API int rmi_turn_readback(const uint8_t* flags, const uint8_t* err, const uint8_t* dec_err,
                              const uint8_t* num_actions, const int32_t* max_actions, const int32_t* text_len,
                              const int32_t* obs_len, int64_t B, uint8_t* flags_copy, int32_t* left, uint8_t* pack,
                              rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0) return RMI_EINVAL;
  if (!pack || (B > 0 && (!flags || !err || !dec_err || !num_actions || !max_actions || !flags_copy || !left)))
    return RMI_EINVAL;
  if (reinterpret_cast<uintptr_t>(pack) & 3u) return RMI_EINVAL;
  const bool v8 = B % 8 == 0 && aligned(flags, 8) && aligned(err, 8) && aligned(dec_err, 8) &&
                  aligned(num_actions, 8) && aligned(flags_copy, 8) && aligned(pack, 8) && aligned(max_actions, 16) &&
                  aligned(left, 16) && aligned(text_len, 16) && aligned(obs_len, 16);
  if (v8)
    hipLaunchKernelGGL(turn_readback_kernel<true>, dim3(1), dim3(kRedBlock), 0, as_stream(stream), flags, err, dec_err,
                       num_actions, max_actions, text_len, obs_len, B, flags_copy, left, pack);
  else
    hipLaunchKernelGGL(turn_readback_kernel<false>, dim3(1), dim3(kRedBlock), 0, as_stream(stream), flags, err,
                       dec_err, num_actions, max_actions, text_len, obs_len, B, flags_copy, left, pack);
  return launch_status();
}

RMI_API int rmi_turn_readback_pad(const uint8_t* flags, const uint8_t* err, const uint8_t* dec_err,
                                  const uint8_t* num_actions, const int32_t* max_actions, const int32_t* text_len,
                                  const int32_t* obs_len, int64_t B, uint8_t* flags_copy, int32_t* left, uint8_t* pack,
                                  const uint8_t* pad_err, int64_t n_pad, rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || n_pad < 0 || (n_pad > 0 && !pad_err)) return RMI_EINVAL;
  if (!pad_err) n_pad = 0;
  if (!pack || (B > 0 && (!flags || !err || !dec_err || !num_actions || !max_actions || !flags_copy || !left)))
    return RMI_EINVAL;
  if (reinterpret_cast<uintptr_t>(pack) & 3u) return RMI_EINVAL;
  const bool v8 = B % 8 == 0 && aligned(flags, 8) && aligned(err, 8) && aligned(dec_err, 8) &&
                  aligned(num_actions, 8) && aligned(flags_copy, 8) && aligned(pack, 8) && aligned(max_actions, 16) &&
                  aligned(left, 16) && aligned(text_len, 16) && aligned(obs_len, 16);
  if (v8)
    hipLaunchKernelGGL(turn_readback_kernel<true>, dim3(1), dim3(kRedBlock), 0, as_stream(stream), flags, err, dec_err,
                       num_actions, max_actions, text_len, obs_len, B, flags_copy, left, pack, pad_err, n_pad, true);
  else
    hipLaunchKernelGGL(turn_readback_kernel<false>, dim3(1), dim3(kRedBlock), 0, as_stream(stream), flags, err,
                       dec_err, num_actions, max_actions, text_len, obs_len, B, flags_copy, left, pack, pad_err, n_pad, true);
  return launch_status();
}

RMI_API int rmi_prompt_commit(const uint8_t* bpe_err, const uint8_t* text_err, const uint8_t* active,
                              const int32_t* mark_tok, int32_t* len_upd, int64_t B, uint8_t* bad, rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || (mark_tok && !len_upd)) return RMI_EINVAL;
  if (B == 0) return RMI_OK;
  if (!bpe_err || !text_err || !bad) return RMI_EINVAL;
  hipLaunchKernelGGL(prompt_commit_kernel, dim3(glue_grid(B)), dim3(kGlueBlock), 0, as_stream(stream), bpe_err,
                     text_err, active, mark_tok, len_upd, B, bad);
  return launch_status();
}

RMI_API int rmi_prompt_commit_stats(const uint8_t* bpe_err, const uint8_t* text_err, const uint8_t* active,
                                    const int32_t* mark_tok, int32_t* len_upd, int64_t B, uint8_t* bad,
                                    const int32_t* len, const uint8_t* has, const uint8_t* flags, int32_t* stats,
                                    rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || (mark_tok && !len_upd) || !stats) return RMI_EINVAL;
  if (B > 0 && (!bpe_err || !text_err || !bad || !len || !flags)) return RMI_EINVAL;
  if (reinterpret_cast<uintptr_t>(stats) & 3u) return RMI_EINVAL;
  const bool v8 = B % 8 == 0 && aligned(bpe_err, 8) && aligned(text_err, 8) && aligned(active, 8) &&
                  aligned(mark_tok, 16) && aligned(len_upd, 16) && aligned(bad, 8) && aligned(len, 16) &&
                  aligned(has, 8) && aligned(flags, 8);
  if (v8)
    hipLaunchKernelGGL(prompt_commit_stats_kernel<true>, dim3(1), dim3(kRedBlock), 0, as_stream(stream), bpe_err,
                       text_err, active, mark_tok, len_upd, B, bad, len, has, flags, stats);
  else
    hipLaunchKernelGGL(prompt_commit_stats_kernel<false>, dim3(1), dim3(kRedBlock), 0, as_stream(stream), bpe_err,
                       text_err, active, mark_tok, len_upd, B, bad, len, has, flags, stats);
  return launch_status();
}

RMI_API int rmi_next_rows_list(const uint8_t* has, const uint8_t* flags, int64_t B, int64_t* rows, int64_t* src,
                               rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || (B > 0 && (!flags || !rows || !src))) return RMI_EINVAL;
  if (B == 0) return RMI_OK;
  hipLaunchKernelGGL(next_rows_list_kernel, dim3(1), dim3(kRedBlock), 0, as_stream(stream), has, flags, B, rows, src);
  return launch_status();
}

RMI_API int rmi_rows_stats(const int32_t* len, const int64_t* rows, int64_t n_rows, const uint8_t* bad, int64_t B,
                           int32_t* stats, rmi_stream_t stream) {
  using namespace rmi;
  if (n_rows < 0 || B < 0 || !stats || (n_rows > 0 && !len)) return RMI_EINVAL;
  if (reinterpret_cast<uintptr_t>(stats) & 3u) return RMI_EINVAL;
  hipLaunchKernelGGL(rows_stats_kernel, dim3(1), dim3(kRedBlock), 0, as_stream(stream), len, rows, n_rows, bad, B,
                     stats);
  return launch_status();
}

RMI_API int rmi_next_rows_stats(const int32_t* len, const uint8_t* has, const uint8_t* flags, const uint8_t* bad,
                                int64_t B, int32_t* stats, rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || !stats || (B > 0 && (!len || !flags))) return RMI_EINVAL;
  if (reinterpret_cast<uintptr_t>(stats) & 3u) return RMI_EINVAL;
  const bool v8 = B % 8 == 0 && aligned(len, 16) && aligned(has, 8) && aligned(flags, 8) && aligned(bad, 8);
  if (v8)
    hipLaunchKernelGGL(next_rows_stats_kernel<true>, dim3(1), dim3(kRedBlock), 0, as_stream(stream), len, has, flags,
                       bad, B, stats);
  else
    hipLaunchKernelGGL(next_rows_stats_kernel<false>, dim3(1), dim3(kRedBlock), 0, as_stream(stream), len, has, flags,
                       bad, B, stats);
  return launch_status();
}

RMI_API int rmi_formulate_stats(const int32_t* len, const uint8_t* bad, const uint8_t* n_turns, int64_t B,
                                int32_t* n_sc, int32_t* stats, rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || !stats || (B > 0 && (!len || !n_turns || !n_sc))) return RMI_EINVAL;
  hipLaunchKernelGGL(formulate_stats_kernel, dim3(1), dim3(kRedBlock), 0, as_stream(stream), len, bad, n_turns, B,
                     n_sc, stats);
  return launch_status();
}

RMI_API int rmi_formulate_tail(const int32_t* resp_count, const uint8_t* err, int64_t B, int64_t* out,
                               rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || !out || (B > 0 && (!resp_count || !err))) return RMI_EINVAL;
  hipLaunchKernelGGL(formulate_tail_kernel, dim3(1), dim3(kRedBlock), 0, as_stream(stream), resp_count, err, B, out);
  return launch_status();
}
