// microbench.hip — latency anatomy of one Sokoban turn launch (diagnostic, not product).
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench.hip -Iinclude -Lragen_amd/_build -lragen_amd -o mb
// Prints average GPU time per launch (hipEvents over N back-to-back launches) for:
//   empty kernel (same grid) | loads+stores only | full turn | full turn with 0 actions.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../include/ragen_amd.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void empty_kernel(int* p) { if (p && threadIdx.x == 1000) p[0] = 1; }

__global__ __launch_bounds__(64) void touch_kernel(uint8_t* state, const uint8_t* fixed, int8_t* player, int32_t* a,
                                                   int32_t* b, uint8_t* flags, int B) {
  __shared__ uint32_t ls[64 * 9], lf[64 * 9];
  const int lane = threadIdx.x;
  const long b0 = (long)blockIdx.x * 64, i = b0 + lane;
  uint8_t f = flags[i];
  int32_t x = a[i], y = b[i];
  int8_t p = player[2 * i];
  for (int k = lane; k < 64 * 9; k += 64) {
    ls[k] = reinterpret_cast<const uint32_t*>(state + b0 * 36)[k];
    lf[k] = reinterpret_cast<const uint32_t*>(fixed + b0 * 36)[k];
  }
  __syncthreads();
  uint32_t v = ls[lane * 9] ^ lf[lane * 9 + 1];
  flags[i] = f + 1;
  a[i] = x + (int)v;
  b[i] = y + 1;
  player[2 * i] = p;
  __syncthreads();
  for (int k = lane; k < 64 * 9; k += 64) reinterpret_cast<uint32_t*>(state + b0 * 36)[k] = ls[k];
}

template <class F>
float time_it(F f, int n, hipStream_t s) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 10; ++i) f();
  CK(hipEventRecord(a, s));
  for (int i = 0; i < n; ++i) f();
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / n;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 8192, T = 5, K = 5, HW = 36;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  uint8_t *fixed, *state, *flags, *info, *exec, *n_act, *init_state;
  int8_t *player, *acts, *init_player;
  int32_t *nes, *bot, *num_actions, *n_turns;
  double *pen, *rw;
  CK(hipMalloc(&fixed, B * HW));
  CK(hipMalloc(&state, B * HW));
  CK(hipMalloc(&init_state, B * HW));
  CK(hipMalloc(&player, B * 2));
  CK(hipMalloc(&init_player, B * 2));
  CK(hipMalloc(&nes, B * 4));
  CK(hipMalloc(&bot, B * 4));
  CK(hipMalloc(&num_actions, B * 4));
  CK(hipMalloc(&n_turns, B * 4));
  CK(hipMalloc(&flags, B));
  CK(hipMalloc(&pen, B * 8));
  CK(hipMalloc(&rw, T * B * 8));
  CK(hipMalloc(&info, T * B));
  CK(hipMalloc(&exec, T * B));
  CK(hipMalloc(&acts, B * K));
  CK(hipMalloc(&n_act, B));
  // a fixed room: walls around a 4x4 floor, target at (3,1), box at (2,3), player at (1,2)
  std::vector<uint8_t> fx(B * HW), st(B * HW);
  std::vector<int8_t> pl(B * 2), ac(B * K);
  std::vector<uint8_t> na(B);
  for (int e = 0; e < B; ++e) {
    for (int r = 0; r < 6; ++r)
      for (int c = 0; c < 6; ++c) {
        const int v = (r == 0 || c == 0 || r == 5 || c == 5) ? 0 : 1;
        fx[e * HW + r * 6 + c] = v;
        st[e * HW + r * 6 + c] = v;
      }
    fx[e * HW + 3 * 6 + 1] = 2;
    st[e * HW + 3 * 6 + 1] = 2;
    st[e * HW + 2 * 6 + 3] = 4;
    st[e * HW + 1 * 6 + 2] = 5;
    pl[2 * e] = 1;
    pl[2 * e + 1] = 2;
    na[e] = 5;
    for (int k = 0; k < K; ++k) ac[e * K + k] = (int8_t)(1 + (e + k) % 4);
  }
  CK(hipMemcpy(fixed, fx.data(), B * HW, hipMemcpyHostToDevice));
  CK(hipMemcpy(init_state, st.data(), B * HW, hipMemcpyHostToDevice));
  CK(hipMemcpy(init_player, pl.data(), B * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(acts, ac.data(), B * K, hipMemcpyHostToDevice));
  CK(hipMemcpy(n_act, na.data(), B, hipMemcpyHostToDevice));
  rmi_sokoban_t env = {6, 6, 1, 100, fixed, state, player, nes, bot};
  rmi_episode_t ep = {B, T, num_actions, flags, n_turns, pen, rw, info, exec};
  rmi_turn_t in = {0, K, acts, n_act, nullptr, 1000000, -0.1};
  const int n = 200;
  const unsigned grid = (B + 63) / 64;
  float t_empty = time_it([&] { hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(64), 0, s, nullptr); }, n, s);
  float t_touch = time_it([&] {
    hipLaunchKernelGGL(touch_kernel, dim3(grid), dim3(64), 0, s, state, fixed, player, nes, bot, flags, B);
  }, n, s);
  // full turn: reset then turn 0 each iteration (reset timed separately)
  float t_reset = time_it([&] { rmi_sokoban_reset(&env, &ep, init_state, init_player, s); }, n, s);
  float t_pair = time_it([&] {
    rmi_sokoban_reset(&env, &ep, init_state, init_player, s);
    rmi_sokoban_step_turn(&env, &ep, &in, nullptr, s);
  }, n, s);
  rmi_turn_t in0 = in;
  std::vector<uint8_t> zero(B, 0);
  uint8_t* n0;
  CK(hipMalloc(&n0, B));
  CK(hipMemcpy(n0, zero.data(), B, hipMemcpyHostToDevice));
  in0.n_actions = n0;
  float t_pair0 = time_it([&] {
    rmi_sokoban_reset(&env, &ep, init_state, init_player, s);
    rmi_sokoban_step_turn(&env, &ep, &in0, nullptr, s);
  }, n, s);
  printf("B=%d  empty %.2f us | touch(loads+stores) %.2f us | reset %.2f us | turn(5 actions) %.2f us | "
         "turn(0 actions) %.2f us\n",
         B, t_empty, t_touch, t_reset, t_pair - t_reset, t_pair0 - t_reset);
  return 0;
}
