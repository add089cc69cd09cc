// seed.hip — numpy Generator(PCG64(SeedSequence(seed))) seeding on the device (gfx950).
//
// Replaces the per-env host seeding of BanditEnv.reset (bandit/env.py:25-39, via
// gymnasium.utils.seeding.np_random) and FrozenLakeEnv.reset's env RNG (frozen_lake/env.py:28-37):
// each reset builds a fresh numpy Generator from an int seed and draws from it.  One thread per
// seed computes, with numpy's published algorithms:
//   SeedSequence(seed): the seed's little-endian 32-bit words hashed into a 4-word pool
//     (mix_entropy: hashmix with the running INIT_A / MULT_A constant, then every pool word
//     mixed into every other), generate_state(4, uint64): the pool cycled through the
//     INIT_B / MULT_B hash into 8 words, read as 4 little-endian uint64 v0..v3;
//   PCG64 seeding (pcg64_set_seed -> pcg_setseq_128_srandom_r): inc = (v2:v3 << 1) | 1,
//     state = 0, step, state += v0:v1, step;
// then `draws` Generator.random() calls (the last one returned), leaving the stream where the
// reference's Generator is after them.  Bit-exact against numpy (tests/test_gpu_parity.py).
#include "common.hpp"

namespace rmi {
namespace {

constexpr uint32_t kInitA = 0x43b0d7e5u, kMultA = 0x931e8875u, kInitB = 0x8b51f9ddu, kMultB = 0x58f38dedu;
constexpr uint32_t kMixL = 0xca01f9ddu, kMixR = 0x4973f715u;

__device__ __forceinline__ uint32_t hashmix(uint32_t v, uint32_t& h) {
  v ^= h;
  h *= kMultA;
  v *= h;
  return v ^ (v >> 16);
}
__device__ __forceinline__ uint32_t mix(uint32_t x, uint32_t y) {
  const uint32_t r = kMixL * x - kMixR * y;
  return r ^ (r >> 16);
}

__device__ __forceinline__ Pcg64 seed_pcg64(uint64_t seed) {
  // SeedSequence entropy: the int's 32-bit words, least significant first ([0] for 0)
  const uint32_t e0 = (uint32_t)seed, e1 = (uint32_t)(seed >> 32);
  const int ne = e1 ? 2 : 1;
  uint32_t pool[4];
  uint32_t h = kInitA;
#pragma unroll
  for (int i = 0; i < 4; ++i) pool[i] = hashmix(i == 0 ? e0 : (i < ne ? e1 : 0u), h);
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int d = 0; d < 4; ++d)
      if (s != d) pool[d] = mix(pool[d], hashmix(pool[s], h));
  // generate_state(4, uint64)
  uint32_t w[8];
  uint32_t hb = kInitB;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t v = pool[i & 3] ^ hb;
    hb *= kMultB;
    v *= hb;
    w[i] = v ^ (v >> 16);
  }
  const uint64_t v0 = w[0] | (uint64_t)w[1] << 32, v1 = w[2] | (uint64_t)w[3] << 32;
  const uint64_t v2 = w[4] | (uint64_t)w[5] << 32, v3 = w[6] | (uint64_t)w[7] << 32;
  Pcg64 p;
  p.i_hi = (v2 << 1) | (v3 >> 63);
  p.i_lo = (v3 << 1) | 1ull;
  p.s_hi = 0;
  p.s_lo = 0;
  (void)p.next64();
  const uint64_t lo = p.s_lo + v1;
  p.s_hi += v0 + (lo < p.s_lo ? 1ull : 0ull);
  p.s_lo = lo;
  (void)p.next64();
  return p;
}

__global__ __launch_bounds__(256) void pcg64_seed_kernel(const int64_t* __restrict__ seeds, int64_t n, int draws,
                                                         uint64_t* __restrict__ rng, int64_t ld,
                                                         double* __restrict__ last, uint8_t* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t sd = seeds[i];
  Pcg64 p = seed_pcg64((uint64_t)(sd < 0 ? 0 : sd));
  double u = 0.0;
  for (int k = 0; k < draws; ++k) u = p.next_double();
  rng[i] = p.s_hi;
  rng[ld + i] = p.s_lo;
  rng[2 * ld + i] = p.i_hi;
  rng[3 * ld + i] = p.i_lo;
  if (last) last[i] = u;
  if (err) err[i] = sd < 0 ? RMI_ERR_STATE : 0;  // SeedSequence raises ValueError on a negative seed
}

}  // namespace
}  // namespace rmi

RMI_API int rmi_pcg64_seed(const int64_t* seeds, int64_t n, int32_t draws, uint64_t* rng, int64_t ld,
                           double* last_draw, uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (n < 0 || draws < 0 || ld < n) return RMI_EINVAL;
  if (n == 0) return RMI_OK;
  if (!seeds || !rng) return RMI_EINVAL;
  hipLaunchKernelGGL(pcg64_seed_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), seeds, n,
                     (int)draws, rng, ld, last_draw, err);
  return launch_status();
}
