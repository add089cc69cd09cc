// stampbench.hip — where the time of one Sokoban turn launch goes (diagnostic, not product).
// Compiles the kernel source itself with RMI_STAMPS so every wave records s_memtime (shader
// clock) and s_memrealtime (100 MHz) at its phase boundaries:
// (kept in SGPRs, written at the end: no memory traffic inside the phases)
//   0 kernel entry | 1 loads landed | 2 exec list + board decode done | 3 turn done | 4 outputs issued
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Iinclude -Iragen_amd/csrc tools/stampbench.hip -o tools/stampbench
#define RMI_STAMPS 1
#include "../ragen_amd/csrc/sokoban.hip"

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 8192, T = 5, K = 5, HW = 36;
  const int per = 64 / RMI_SPREAD_LPE;
  const int grid = B <= RMI_SPREAD_MAX_ENVS ? (B + per - 1) / per : (B + 63) / 64;  // the launcher's lanes-per-env choice
  uint8_t *fixed, *state, *flags, *info, *exec, *n_act, *init_state;
  int8_t *player, *acts, *init_player;
  int32_t *nes, *bot, *num_actions, *n_turns;
  double *pen, *rw;
  unsigned long long* stamps;
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
  CK(hipMalloc(&stamps, (size_t)grid * 16 * 8));
  CK(hipMemset(stamps, 0, (size_t)grid * 16 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(rmi::g_stamps), &stamps, sizeof(stamps)));
  std::vector<uint8_t> fx(B * HW), st(B * HW), na(B, 5);
  std::vector<int8_t> pl(B * 2), ac(B * K);
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
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 20;
  std::vector<double> phase(5, 0.0);
  double span_rt = 0.0, ev_us = 0.0, clk = 0.0;
  std::vector<unsigned long long> h((size_t)grid * 16);
  for (int it = 0; it < reps + 3; ++it) {
    CK(rmi_sokoban_reset(&env, &ep, init_state, init_player, nullptr) == RMI_OK ? hipSuccess : hipErrorUnknown);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, nullptr));
    CK(rmi_sokoban_step_turn(&env, &ep, &in, nullptr, nullptr) == RMI_OK ? hipSuccess : hipErrorUnknown);
    CK(hipEventRecord(b, nullptr));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
    if (it < 3) continue;
    ev_us += ms * 1000.0;
    unsigned long long rt_min = ~0ull, rt_max = 0;
    double cyc = 0, rts = 0;
    for (int g = 0; g < grid; ++g) {
      const unsigned long long* s = &h[(size_t)g * 16];
      for (int p = 1; p < 5; ++p) {
        phase[p] += (double)(s[2 * p] - s[2 * (p - 1)]) / grid;
      }
      rt_min = std::min(rt_min, s[1]);
      rt_max = std::max(rt_max, s[9]);
      cyc += (double)(s[8] - s[0]);
      rts += (double)(s[9] - s[1]);
    }
    span_rt += (double)(rt_max - rt_min);
    clk += cyc / rts * 100.0;  // MHz
  }
  printf("B=%d grid=%d  event %.2f us/launch | first-entry..last-store span %.2f us | shader clock %.0f MHz\n", B, grid,
         ev_us / reps, span_rt / reps / 100.0, clk / reps);
  // back-to-back: (reset + turn) pairs minus resets alone
  auto run_pairs = [&](bool turn) {
    for (int i = 0; i < 210; ++i) {
      if (i == 10) CK(hipEventRecord(a, nullptr));
      rmi_sokoban_reset(&env, &ep, init_state, init_player, nullptr);
      if (turn) rmi_sokoban_step_turn(&env, &ep, &in, nullptr, nullptr);
    }
    CK(hipEventRecord(b, nullptr));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.0 / 200;
  };
  const double t_reset = run_pairs(false), t_pair = run_pairs(true);
  printf("  back-to-back: reset %.2f us, turn %.2f us (spread<=%d)\n", t_reset, t_pair - t_reset, RMI_SPREAD_MAX_ENVS);
  const char* names[5] = {"", "loads", "decode", "turn", "outputs"};
  for (int p = 1; p < 5; ++p)
    printf("  %-12s %8.0f cycles  %6.2f us\n", names[p], phase[p] / reps, phase[p] / reps / (clk / reps));
  return 0;
}
