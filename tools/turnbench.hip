// turnbench.hip — cycles of one board turn (K=5 steps on u32 window bitboards) for a lone wave,
// in isolation: the turn is chained N times (each turn's box / player feed the next) and timed
// with s_memtime.  Diagnostic only; compares formulations of board_turn_k.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Iinclude -Iragen_amd/csrc tools/turnbench.hip -o tools/turnbench
#include "../ragen_amd/csrc/sokoban.hip"

#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void turn_loop(const uint32_t* in, int n, unsigned long long* cyc, uint32_t* out, int W, int n_act,
                          int left, int num_boxes, int max_steps) {
  const int i = threadIdx.x;
  const uint32_t wall = in[i], target = in[64 + i];
  uint32_t box = in[128 + i];
  int jp = (int)in[192 + i];
  uint64_t acts = ((uint64_t)in[256 + i] << 32) | in[320 + i];
  int nes = 0, bot = 0;
  double acc = 0.0;
  uint32_t sink = 0;
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < n; ++it) {
    rmi::BoardTurn t =
        rmi::board_turn_k<uint32_t, 5>(wall, target, box, jp, W, acts, n_act, left, nes & 63, bot, num_boxes, max_steps);
    acc += t.acc;
    sink += t.info + t.taken + t.stop + t.succ + t.moved;
    nes = t.nes;
    bot = t.bot;
    acts = (acts >> 8) | (acts << 32);  // rotate the action bytes (stays 1..4)
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (i == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * 64 + i] = sink ^ box ^ (uint32_t)jp ^ (uint32_t)nes ^ (uint32_t)(acc * 10.0);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 2000, blocks = argc > 2 ? atoi(argv[2]) : 1;
  // 6x6 room, interior 4x4 open, box at (2,3), target at (3,1), player at (1,2); window = cells 6..
  std::vector<uint32_t> h(384);
  uint64_t wall64 = 0, target64 = 1ull << (3 * 6 + 1), box64 = 1ull << (2 * 6 + 3);
  for (int r = 0; r < 6; ++r)
    for (int c = 0; c < 6; ++c)
      if (r == 0 || c == 0 || r == 5 || c == 5) wall64 |= 1ull << (r * 6 + c);
  for (int i = 0; i < 64; ++i) {
    h[i] = (uint32_t)(wall64 >> 6) | ~((1u << 30) - 1);
    h[64 + i] = (uint32_t)(target64 >> 6);
    h[128 + i] = (uint32_t)(box64 >> 6);
    h[192 + i] = (1 * 6 + 2) - 6;
    uint64_t a = 0;
    for (int k = 0; k < 8; ++k) a |= (uint64_t)(1 + (i + k) % 4) << (8 * k);
    h[256 + i] = (uint32_t)(a >> 32);
    h[320 + i] = (uint32_t)a;
  }
  uint32_t *din, *dout;
  unsigned long long* dcyc;
  CK(hipMalloc(&din, h.size() * 4));
  CK(hipMalloc(&dout, blocks * 64 * 4));
  CK(hipMalloc(&dcyc, blocks * 8));
  CK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(turn_loop, dim3(blocks), dim3(64), 0, 0, din, n, dcyc, dout, 6, 5, 1000, 1, 1 << 30);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> c(blocks);
    CK(hipMemcpy(c.data(), dcyc, blocks * 8, hipMemcpyDeviceToHost));
    double s = 0;
    for (auto x : c) s += (double)x;
    printf("n=%d blocks=%d: %.1f shader cycles per 5-step turn (s_memtime units)\n", n, blocks, s / blocks / n);
  }
  return 0;
}
