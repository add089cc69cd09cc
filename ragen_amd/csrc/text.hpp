// text.hpp — Python str whitespace on UTF-8 bytes (device helpers shared by the parse and the
// prompt-text kernels).
#pragma once
#include "common.hpp"

namespace rmi {

// Length of the Unicode whitespace character (str.isspace / re \s) whose bytes are c, c1, c2.
__device__ __forceinline__ int ws_len3(uint32_t c, uint32_t c1, uint32_t c2) {
  if (c < 0x80) return ((c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x20)) ? 1 : 0;
  if (c == 0xC2) return (c1 == 0x85 || c1 == 0xA0) ? 2 : 0;
  if (c == 0xE1) return (c1 == 0x9A && c2 == 0x80) ? 3 : 0;
  if (c == 0xE2) {
    if (c1 == 0x80) return ((c2 >= 0x80 && c2 <= 0x8A) || c2 == 0xA8 || c2 == 0xA9 || c2 == 0xAF) ? 3 : 0;
    return (c1 == 0x81 && c2 == 0x9F) ? 3 : 0;
  }
  if (c == 0xE3) return (c1 == 0x80 && c2 == 0x80) ? 3 : 0;
  return 0;
}
// str.isspace of an ASCII byte (ws_len3's first line)
__device__ __forceinline__ bool ascii_space(uint32_t c) { return (c >= 9u && c <= 13u) || (c >= 0x1Cu && c <= 0x20u); }
// ... starting at p inside [.., lim), or 0
__device__ __forceinline__ int ws_fwd(const uint8_t* V, int p, int lim) {
  if (p >= lim) return 0;
  const uint32_t c = V[p];
  if (c < 0x80) return ws_len3(c, 0, 0);
  const uint32_t c1 = p + 1 < lim ? V[p + 1] : 0u, c2 = p + 2 < lim ? V[p + 2] : 0u;
  return ws_len3(c, c1, c2);
}
// ... ending at e (within [s, e)), or 0
__device__ __forceinline__ int ws_back(const uint8_t* V, int s, int e) {
  if (e <= s) return 0;
  const uint32_t c = V[e - 1];
  if (c < 0x80) return ws_len3(c, 0, 0);
  if (e - 2 >= s && V[e - 2] == 0xC2 && (c == 0x85 || c == 0xA0)) return 2;
  if (e - 3 < s) return 0;
  return ws_len3(V[e - 3], V[e - 2], c) == 3 ? 3 : 0;
}
__device__ __forceinline__ void strip(const uint8_t* V, int& a, int& z) {
  for (int l; (l = ws_fwd(V, a, z)) != 0;) a += l;
  for (int l; (l = ws_back(V, a, z)) != 0;) z -= l;
}

}  // namespace rmi
