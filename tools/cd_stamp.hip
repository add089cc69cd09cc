// cd_stamp.hip — cycle cost of one Countdown answer evaluation (diagnostic, not product).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Iragen_amd/csrc
//        tools/cd_stamp.hip -o tools/cd_stamp
// One wave; lane 0 (or every lane) evaluates the same answer R times from LDS, stamping the
// shader clock around each repetition: the first repetition pays the cold instruction cache,
// the later ones the evaluation itself.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../ragen_amd/csrc/countdown.hip"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int kR = 6;

__global__ __launch_bounds__(64) void stamp_kernel(const uint8_t* ans, int n, const int32_t* nums_in, int n_nums,
                                                   int all_lanes, long long* cyc, int* res) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[64 * (128 + rmi::kMachineBytes)];
  const int lane = threadIdx.x;
  if (!all_lanes && lane) return;
  uint8_t* row = lds + lane * (128 + rmi::kMachineBytes);
  for (int i = 0; i < n; ++i) row[i] = ans[i];
  int32_t nums[rmi::kMaxNums];
  for (int k = 0; k < rmi::kMaxNums; ++k) nums[k] = k < n_nums ? nums_in[k] : -1;
  int acc = 0;
  for (int r = 0; r < kR; ++r) {
    const long long t0 = __builtin_amdgcn_s_memtime();
    bool fmt = false;
    int st = 0;
    rmi::Val v;
    const bool fast = rmi::fast_reward(row, n, nums, n_nums, fmt, st, v, row + 128);
    acc += (int)fast + 2 * (int)fmt + 4 * st + (int)v.i;
    __builtin_amdgcn_s_waitcnt(0);
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[r] = t1 - t0;
  }
  if (lane == 0) res[0] = acc;
}

int main(int argc, char** argv) {
  const char* a = argc > 1 ? argv[1] : "(44 - 19) * (3 + 7)";
  const int all = argc > 2 ? atoi(argv[2]) : 0;
  const int n = (int)strlen(a);
  int32_t nums_h[4] = {44, 19, 3, 7};
  uint8_t* ans;
  int32_t *nums, *res;
  long long* cyc;
  CK(hipMalloc(&ans, 128));
  CK(hipMalloc(&nums, 16));
  CK(hipMalloc(&res, 4));
  CK(hipMalloc(&cyc, kR * 8));
  CK(hipMemcpy(ans, a, n, hipMemcpyHostToDevice));
  CK(hipMemcpy(nums, nums_h, 16, hipMemcpyHostToDevice));
  for (int launch = 0; launch < 3; ++launch) {
    hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, 0, ans, n, nums, 4, all, cyc, res);
    CK(hipDeviceSynchronize());
    long long c[kR];
    int r;
    CK(hipMemcpy(c, cyc, sizeof c, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&r, res, 4, hipMemcpyDeviceToHost));
    printf("'%s' all_lanes=%d launch %d: cycles per repetition (s_memtime, core clock):", a, all, launch);
    for (int i = 0; i < kR; ++i) printf(" %lld", c[i]);
    printf("  (res %d)\n", r);
  }
  return 0;
}
