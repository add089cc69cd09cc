// render.hip — text observations on the device (gfx950), SURVEY §8(f) rank 2.
//
//  rmi_sokoban_render     SokobanEnv.render text mode (sokoban/env.py:53-61)
//  rmi_frozenlake_render  FrozenLakeEnv.render text mode (frozen_lake/env.py:47-61)
//
// One env per 16-lane DPP row (4 envs per 64-thread workgroup): the observation's tokens (H*W
// cells and the H-1 newlines, in order) are split into contiguous runs of ceil(T/16) per lane;
// each lane sums its tokens' UTF-8 lengths, a DPP row scan gives every lane its byte offset, the
// lanes write their bytes into the row's LDS buffer, and the row is copied out as dwords (the
// bytes past the end of the last dword are zero).  Every cell maps to a glyph of the env
// config's grid_lookup (up to 4 UTF-8 bytes; codes outside the table render as '?', like the
// reference's dict.get(c, "?") in this build's host path).  No loop depends on a glyph's length
// except the byte writes (≤ 4), so the row costs a few dozen instructions per lane.  The host
// decodes each row with one bytes(...).decode() — no per-cell Python.
#include "common.hpp"

namespace rmi {
namespace {

constexpr int kGlyphs = 16;

struct GlyphTable {
  uint32_t bytes[kGlyphs];  // UTF-8 bytes, little-endian packed
  uint8_t len[kGlyphs];     // 0 => '?'
};

constexpr int kRenderBlock = 64;
constexpr int kRRow = 16;                                     // lanes per env
constexpr int kMaxCellsR = 64;
constexpr int kTokLane = 8;                                   // tokens per lane at most: T <= 128
constexpr int kRBufWords = (4 * kMaxCellsR + kMaxCellsR + 3) / 4;  // glyph bytes + newlines, in dwords

// the glyph table in LDS (a dynamic index into the kernel-argument struct would be a memory load
// per cell)
__device__ __forceinline__ void stage_glyphs(const GlyphTable& g, uint32_t* gb, uint8_t* gl) {
  if (threadIdx.x < kGlyphs) {
    gb[threadIdx.x] = g.bytes[threadIdx.x];
    gl[threadIdx.x] = g.len[threadIdx.x];
  }
  __syncthreads();
}

// exclusive prefix sum over the 16 lanes of a DPP row
__device__ __forceinline__ int row_excl_scan(int x) {
  int v = x;
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);  // row_shr:8
  return v - x;
}

// One env's observation: lane j of its row, `code(cell)` the glyph code of a cell.  Tokens:
// t = r * (W + 1) + c is cell (r, c); t = r * (W + 1) + W (r < H - 1) is a newline.
template <class CodeOf>
__device__ __forceinline__ void render_row(int j, int H, int W, const uint32_t* gb, const uint8_t* gl, uint8_t* buf,
                                           uint32_t* out, int32_t* len_out, CodeOf code_of) {
  const int T = H * (W + 1) - 1;
  const int per = (T + kRRow - 1) / kRRow;
  const int t0 = j * per;
  uint32_t gbytes[kTokLane];
  int glen[kTokLane], n = 0;
#pragma unroll
  for (int i = 0; i < kTokLane; ++i) {  // per <= kTokLane (the launcher checks T <= 16 * kTokLane)
    const int t = t0 + i;
    const bool tok = i < per && t < T;
    const int r = t / (W + 1), c = t - r * (W + 1);
    const bool nl = c == W;
    const int code = (tok && !nl) ? code_of(r * W + c) : 0;
    const int gl_c = (code >= 0 && code < kGlyphs) ? gl[code] : 0;
    const uint32_t gb_c = (code >= 0 && code < kGlyphs) ? gb[code] : 0u;
    glen[i] = !tok ? 0 : nl ? 1 : (gl_c ? gl_c : 1);
    gbytes[i] = nl ? (uint32_t)'\n' : (gl_c ? gb_c : (uint32_t)'?');
    n += glen[i];
  }
  const int off = row_excl_scan(n);
  const int total = __shfl(off + n, (threadIdx.x & 63 & ~(kRRow - 1)) + kRRow - 1);
  uint32_t* b4 = reinterpret_cast<uint32_t*>(buf);
  for (int w = j; w < (total + 3) / 4; w += kRRow) b4[w] = 0u;  // the last dword's unused bytes stay 0
  wave_sync();
  int o = off;
#pragma unroll
  for (int i = 0; i < kTokLane; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < glen[i]) buf[o + k] = (uint8_t)(gbytes[i] >> (8 * k));
    o += glen[i];
  }
  wave_sync();
  for (int w = j; w < (total + 3) / 4; w += kRRow) out[w] = b4[w];
  if (j == 0) *len_out = total;
}

__global__ __launch_bounds__(kRenderBlock) void sokoban_render_kernel(rmi_sokoban_t env, int B, GlyphTable g,
                                                                      uint8_t* __restrict__ out, int stride,
                                                                      int32_t* __restrict__ len) {
  __shared__ uint32_t gb[kGlyphs];
  __shared__ uint8_t gl[kGlyphs];
  __shared__ uint32_t bufs[kRenderBlock / kRRow][kRBufWords];
  stage_glyphs(g, gb, gl);
  const int j = threadIdx.x & (kRRow - 1);
  const int64_t b = ((int64_t)blockIdx.x * kRenderBlock + threadIdx.x) / kRRow;
  if (b >= B) return;
  const int H = env.H, W = env.W, n = H * W;
  const uint8_t* st = env.room_state + b * n;
  const uint8_t* fx = env.room_fixed + b * n;
  render_row(j, H, W, gb, gl, reinterpret_cast<uint8_t*>(bufs[threadIdx.x / kRRow]),
             reinterpret_cast<uint32_t*>(out + b * stride), len + b, [&](int i) {
               const int v = st[i];
               return (v == 5 && fx[i] == 2) ? 6 : v;  // player on target -> 6 (sokoban/env.py:55)
             });
}

__global__ __launch_bounds__(kRenderBlock) void frozenlake_render_kernel(rmi_frozenlake_t env, int B, GlyphTable g,
                                                                         uint8_t* __restrict__ out, int stride,
                                                                         int32_t* __restrict__ len) {
  __shared__ uint32_t gb[kGlyphs];
  __shared__ uint8_t gl[kGlyphs];
  __shared__ uint32_t bufs[kRenderBlock / kRRow][kRBufWords];
  stage_glyphs(g, gb, gl);
  const int j = threadIdx.x & (kRRow - 1);
  const int64_t b = ((int64_t)blockIdx.x * kRenderBlock + threadIdx.x) / kRRow;
  if (b >= B) return;
  const int nr = env.nrow, nc = env.ncol;
  const int s = env.s[b];
  const uint8_t* d = env.desc + b * nr * nc;
  render_row(j, nr, nc, gb, gl, reinterpret_cast<uint8_t*>(bufs[threadIdx.x / kRRow]),
             reinterpret_cast<uint32_t*>(out + b * stride), len + b, [&](int i) {
               const uint8_t l = d[i];
               if (i == s) return l == 'H' ? 4 : (l == 'G' ? 5 : 0);  // player / in a hole / on the goal
               return l == 'H' ? 2 : (l == 'G' ? 3 : 1);             // S and F render as floor
             });
}

inline int make_table(const uint32_t* glyph_bytes, const uint8_t* glyph_len, GlyphTable& g) {
  if (!glyph_bytes || !glyph_len) return RMI_EINVAL;
  for (int i = 0; i < kGlyphs; ++i) {
    if (glyph_len[i] > 4) return RMI_EINVAL;
    g.bytes[i] = glyph_bytes[i];
    g.len[i] = glyph_len[i];
  }
  return RMI_OK;
}

}  // namespace
}  // namespace rmi

RMI_API int rmi_sokoban_render(const rmi_sokoban_t* env, int32_t B, const uint32_t* glyph_bytes,
                               const uint8_t* glyph_len, uint8_t* out, int32_t stride, int32_t* len,
                               rmi_stream_t stream) {
  using namespace rmi;
  if (!env || B < 0 || env->H <= 0 || env->W <= 0) return RMI_EINVAL;
  GlyphTable g;
  if (make_table(glyph_bytes, glyph_len, g) != RMI_OK) return RMI_EINVAL;
  if (stride < env->H * env->W * 4 + env->H - 1 || stride % 4) return RMI_EINVAL;
  if (B == 0) return RMI_OK;
  if (!env->room_state || !env->room_fixed || !out || !len || (reinterpret_cast<uintptr_t>(out) & 3u))
    return RMI_EINVAL;
  if (env->H * env->W > kMaxCellsR || env->H * (env->W + 1) - 1 > kTokLane * kRRow) return RMI_EUNSUP;
  hipLaunchKernelGGL(sokoban_render_kernel, dim3((unsigned)(((int64_t)B * kRRow + kRenderBlock - 1) / kRenderBlock)),
                     dim3(kRenderBlock), 0,
                     as_stream(stream), *env, B, g, out, stride, len);
  return launch_status();
}

RMI_API int rmi_frozenlake_render(const rmi_frozenlake_t* env, int32_t B, const uint32_t* glyph_bytes,
                                  const uint8_t* glyph_len, uint8_t* out, int32_t stride, int32_t* len,
                                  rmi_stream_t stream) {
  using namespace rmi;
  if (!env || B < 0 || env->nrow <= 0 || env->ncol <= 0) return RMI_EINVAL;
  GlyphTable g;
  if (make_table(glyph_bytes, glyph_len, g) != RMI_OK) return RMI_EINVAL;
  if (stride < env->nrow * env->ncol * 4 + env->nrow - 1 || stride % 4) return RMI_EINVAL;
  if (B == 0) return RMI_OK;
  if (!env->desc || !env->s || !out || !len || (reinterpret_cast<uintptr_t>(out) & 3u)) return RMI_EINVAL;
  if (env->nrow * env->ncol > kMaxCellsR || env->nrow * (env->ncol + 1) - 1 > kTokLane * kRRow) return RMI_EUNSUP;
  hipLaunchKernelGGL(frozenlake_render_kernel, dim3((unsigned)(((int64_t)B * kRRow + kRenderBlock - 1) / kRenderBlock)),
                     dim3(kRenderBlock), 0,
                     as_stream(stream), *env, B, g, out, stride, len);
  return launch_status();
}
