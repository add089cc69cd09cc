// kernarg_probe.hip — does kernel-argument preloading shorten a latency-bound launch? (diagnostic)
// Three kernels with the same work (8192 lanes each load one value from 12 arrays, sum, store):
//   A: the 12 pointers in a by-value struct (read with s_load from the kernarg segment)
//   B: one base pointer + B as the first two scalar arguments (preloaded into SGPRs with
//      -mllvm -amdgpu-kernarg-preload-count=16); the 12 arrays are fixed offsets of the base
//   C: like B but without preloading (build without the flag) — compile twice.
// Timed as 200 back-to-back launches captured in a hipGraph (µs per launch).
// Build: hipcc --offload-arch=gfx950 -O3 [-mllvm -amdgpu-kernarg-preload-count=16] tools/kernarg_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct Ptrs { const int* p[12]; int* out; int B; };

__global__ __launch_bounds__(64) void kA(Ptrs a) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= a.B) return;
  int s = 0;
#pragma unroll
  for (int k = 0; k < 12; ++k) s += a.p[k][i];
  a.out[i] = s;
}

__global__ __launch_bounds__(64) void kB(const int* __restrict__ base, int B, int* __restrict__ out) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= B) return;
  int s = 0;
#pragma unroll
  for (int k = 0; k < 12; ++k) s += base[(long)k * B + i];
  out[i] = s;
}

template <class F>
float graph_us(F launch, hipStream_t st, int n) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int r = 0; r < n; ++r) launch();
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, st));
  for (int w = 0; w < 5; ++w) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / (5 * n);
}

int main() {
  const int B = 8192;
  int *base, *out;
  CK(hipMalloc(&base, 12L * B * 4));
  CK(hipMalloc(&out, B * 4));
  CK(hipMemset(base, 1, 12L * B * 4));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  Ptrs p;
  for (int k = 0; k < 12; ++k) p.p[k] = base + (long)k * B;
  p.out = out;
  p.B = B;
  const int grid = B / 64;
  for (int rep = 0; rep < 3; ++rep) {
    float ua = graph_us([&] { hipLaunchKernelGGL(kA, dim3(grid), dim3(64), 0, st, p); }, st, 200);
    float ub = graph_us([&] { hipLaunchKernelGGL(kB, dim3(grid), dim3(64), 0, st, base, B, out); }, st, 200);
    printf("struct args %.3f us/launch | base pointer args %.3f us/launch\n", ua, ub);
  }
  return 0;
}
