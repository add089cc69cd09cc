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
  __device__ __forceinline__ void glyph(const GlyphTable& g, int code) {
    if (code < 0 || code >= kGlyphs || g.len[code] == 0) {
      put('?');
      return;
    }
    const uint32_t v = g.bytes[code];
    for (int i = 0; i < g.len[code]; ++i) put(v >> (8 * i));
  }
  __device__ __forceinline__ void flush() {
    if (fill) out[pos >> 2] = word;
  }
};

__global__ __launch_bounds__(kBlock) void sokoban_render_kernel(rmi_sokoban_t env, int B, GlyphTable g,
                                                                uint8_t* __restrict__ out, int stride,
                                                                int32_t* __restrict__ len) {
  const int64_t b = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (b >= B) return;
  const int H = env.H, W = env.W;
  const uint8_t* st = env.room_state + b * H * W;
  const uint8_t* fx = env.room_fixed + b * H * W;
  ByteWriter w{reinterpret_cast<uint32_t*>(out + b * stride), 0u, 0, 0};
  for (int r = 0; r < H; ++r) {
    if (r) w.put('\n');
    for (int c = 0; c < W; ++c) {
      const int v = st[r * W + c];
      w.glyph(g, (v == 5 && fx[r * W + c] == 2) ? 6 : v);  // player on target -> 6 (sokoban/env.py:55)
    }
  }
  w.flush();
  len[b] = w.pos;
}

__global__ __launch_bounds__(kBlock) void frozenlake_render_kernel(rmi_frozenlake_t env, int B, GlyphTable g,
                                                                   uint8_t* __restrict__ out, int stride,
                                                                   int32_t* __restrict__ len) {
  const int64_t b = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (b >= B) return;
  const int nr = env.nrow, nc = env.ncol;
  const uint8_t* d = env.desc + b * nr * nc;
  const int s = env.s[b];
  ByteWriter w{reinterpret_cast<uint32_t*>(out + b * stride), 0u, 0, 0};
  for (int r = 0; r < nr; ++r) {
    if (r) w.put('\n');
    for (int c = 0; c < nc; ++c) {
      const int i = r * nc + c;
      const uint8_t l = d[i];
      int code;
      if (i == s) code = l == 'H' ? 4 : (l == 'G' ? 5 : 0);  // player / in a hole / on the goal
      else code = l == 'H' ? 2 : (l == 'G' ? 3 : 1);         // S and F render as floor
      w.glyph(g, code);
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
  hipLaunchKernelGGL(sokoban_render_kernel, dim3((B + kBlock - 1) / kBlock), dim3(kBlock), 0, as_stream(stream),
                     *env, B, g, out, stride, len);
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
  hipLaunchKernelGGL(frozenlake_render_kernel, dim3((B + kBlock - 1) / kBlock), dim3(kBlock), 0, as_stream(stream),
                     *env, B, g, out, stride, len);
  return launch_status();
}
