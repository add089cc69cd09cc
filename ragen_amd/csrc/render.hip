// render.hip — text observations on the device (gfx950), SURVEY §8(f) rank 2.
//
//  rmi_sokoban_render     SokobanEnv.render text mode (sokoban/env.py:53-61)
//  rmi_frozenlake_render  FrozenLakeEnv.render text mode (frozen_lake/env.py:47-61)
//
// One thread per env writes its observation as UTF-8 bytes into a fixed-stride row: every cell
// maps to a glyph of the env config's grid_lookup (up to 4 UTF-8 bytes; codes outside the
// table render as '?', like the reference's dict.get(c, "?") in this build's host path), rows
// joined by '\n'.  Bytes are packed into dwords in registers and stored as dwords, so a 6x6
// room costs ~30 stores per env instead of ~113 byte stores.  The host decodes each row with
// one bytes(...).decode() — no per-cell Python.
#include "common.hpp"

namespace rmi {
namespace {

constexpr int kGlyphs = 16;

struct GlyphTable {
  uint32_t bytes[kGlyphs];  // UTF-8 bytes, little-endian packed
  uint8_t len[kGlyphs];     // 0 => '?'
};

// One wave per workgroup (8192 envs = 128 workgroups, not 32), the glyph table in LDS (a
// dynamic index into the kernel-argument struct would be a memory load per cell), and each
// env's grid rows staged into LDS with dword loads when the row is dword-aligned.
constexpr int kRenderBlock = 64;
constexpr int kMaxCellsR = 64;
__device__ __forceinline__ void stage_glyphs(const GlyphTable& g, uint32_t* gb, uint8_t* gl) {
  if (threadIdx.x < kGlyphs) {
    gb[threadIdx.x] = g.bytes[threadIdx.x];
    gl[threadIdx.x] = g.len[threadIdx.x];
  }
  __syncthreads();
}
// this env's n-byte row -> LDS (dwords when aligned)
__device__ __forceinline__ const uint8_t* stage_row(const uint8_t* src, int n, uint8_t* dst) {
  if ((n & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 3u) == 0) {
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d4 = reinterpret_cast<uint32_t*>(dst);
    for (int i = 0; i < (n >> 2); ++i) d4[i] = s4[i];
  } else {
    for (int i = 0; i < n; ++i) dst[i] = src[i];
  }
  return dst;
}

struct ByteWriter {
  uint32_t* out;  // this env's row (4-B aligned)
  uint32_t word;
  int fill, pos;  // bytes in `word`, bytes written in total
  __device__ __forceinline__ void put(uint32_t b) {
    word |= (b & 0xFFu) << (8 * fill);
    if (++fill == 4) {
      out[pos >> 2] = word;
      word = 0;
      fill = 0;
    }
    ++pos;
  }
  __device__ __forceinline__ void glyph(const uint32_t* gb, const uint8_t* gl, int code) {
    const int n = (code < 0 || code >= kGlyphs) ? 0 : gl[code];
    if (n == 0) {
      put('?');
      return;
    }
    const uint32_t v = gb[code];
    for (int i = 0; i < n; ++i) put(v >> (8 * i));
  }
  __device__ __forceinline__ void flush() {
    if (fill) out[pos >> 2] = word;
  }
};

__global__ __launch_bounds__(kRenderBlock) void sokoban_render_kernel(rmi_sokoban_t env, int B, GlyphTable g,
                                                                      uint8_t* __restrict__ out, int stride,
                                                                      int32_t* __restrict__ len) {
  __shared__ uint32_t gb[kGlyphs];
  __shared__ uint8_t gl[kGlyphs];
  __shared__ __attribute__((aligned(4))) uint8_t rows[kRenderBlock][2][kMaxCellsR];
  stage_glyphs(g, gb, gl);
  const int64_t b = (int64_t)blockIdx.x * kRenderBlock + threadIdx.x;
  if (b >= B) return;
  const int H = env.H, W = env.W, n = H * W;
  const uint8_t* st = stage_row(env.room_state + b * n, n, rows[threadIdx.x][0]);
  const uint8_t* fx = stage_row(env.room_fixed + b * n, n, rows[threadIdx.x][1]);
  ByteWriter w{reinterpret_cast<uint32_t*>(out + b * stride), 0u, 0, 0};
  for (int r = 0; r < H; ++r) {
    if (r) w.put('\n');
    for (int c = 0; c < W; ++c) {
      const int v = st[r * W + c];
      w.glyph(gb, gl, (v == 5 && fx[r * W + c] == 2) ? 6 : v);  // player on target -> 6 (sokoban/env.py:55)
    }
  }
  w.flush();
  len[b] = w.pos;
}

__global__ __launch_bounds__(kRenderBlock) void frozenlake_render_kernel(rmi_frozenlake_t env, int B, GlyphTable g,
                                                                         uint8_t* __restrict__ out, int stride,
                                                                         int32_t* __restrict__ len) {
  __shared__ uint32_t gb[kGlyphs];
  __shared__ uint8_t gl[kGlyphs];
  __shared__ __attribute__((aligned(4))) uint8_t rows[kRenderBlock][kMaxCellsR];
  stage_glyphs(g, gb, gl);
  const int64_t b = (int64_t)blockIdx.x * kRenderBlock + threadIdx.x;
  if (b >= B) return;
  const int nr = env.nrow, nc = env.ncol;
  const int s = env.s[b];
  const uint8_t* d = stage_row(env.desc + b * nr * nc, nr * nc, rows[threadIdx.x]);
  ByteWriter w{reinterpret_cast<uint32_t*>(out + b * stride), 0u, 0, 0};
  for (int r = 0; r < nr; ++r) {
    if (r) w.put('\n');
    for (int c = 0; c < nc; ++c) {
      const int i = r * nc + c;
      const uint8_t l = d[i];
      int code;
      if (i == s) code = l == 'H' ? 4 : (l == 'G' ? 5 : 0);  // player / in a hole / on the goal
      else code = l == 'H' ? 2 : (l == 'G' ? 3 : 1);         // S and F render as floor
      w.glyph(gb, gl, code);
    }
  }
  w.flush();
  len[b] = w.pos;
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
  if (env->H * env->W > kMaxCellsR) return RMI_EUNSUP;
  hipLaunchKernelGGL(sokoban_render_kernel, dim3((B + kRenderBlock - 1) / kRenderBlock), dim3(kRenderBlock), 0,
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
  if (env->nrow * env->ncol > kMaxCellsR) return RMI_EUNSUP;
  hipLaunchKernelGGL(frozenlake_render_kernel, dim3((B + kRenderBlock - 1) / kRenderBlock), dim3(kRenderBlock), 0,
                     as_stream(stream), *env, B, g, out, stride, len);
  return launch_status();
}
