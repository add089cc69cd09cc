// pmc_calib.hip — calibration kernels for rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950
// (MI355X_MICROARCH.md §HBM: "other access widths are uncalibrated: calibrate on a known byte
// count in your own access pattern").  Each kernel moves a known number of bytes in one of the
// access patterns the Sokoban turn kernel uses; tools/pmc_calib.py runs them past the 256 MiB
// Infinity Cache and divides the counters by the known bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>

struct Dw4 { uint32_t x, y, z, w; };

// one lane per 36-byte row: two 16-B loads + one dword (the turn kernel's row load, LPE = 1)
__global__ __launch_bounds__(64) void rows36_read(const uint8_t* __restrict__ rows, int64_t B, uint32_t* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  const Dw4* r4 = reinterpret_cast<const Dw4*>(rows + b * 36);
  const Dw4 a = r4[0], c = r4[1];
  const uint32_t d = reinterpret_cast<const uint32_t*>(rows + b * 36)[8];
  out[b] = a.x ^ a.y ^ a.z ^ a.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d;
}

// one lane per 36-byte row, dword stores of `n` of its 9 dwords (the changed-cell stores)
__global__ __launch_bounds__(64) void rows36_write(uint8_t* __restrict__ rows, int64_t B, int n) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  uint32_t* r1 = reinterpret_cast<uint32_t*>(rows + b * 36);
  for (int i = 0; i < n; ++i) r1[2 * i + 1] = (uint32_t)b + i;
}

// one byte per lane, coalesced (the u8 SoA fields: flags, counters, actions)
__global__ __launch_bounds__(256) void bytes_read(const uint8_t* __restrict__ x, int64_t n, uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = x[i] + 1;
}

// one f64 per lane, coalesced (penalty, turn_reward)
__global__ __launch_bounds__(256) void f64_rw(double* __restrict__ x, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) x[i] += 1.0;
}

extern "C" {
int calib_rows36_read(const void* rows, int64_t B, void* out, void* s) {
  hipLaunchKernelGGL(rows36_read, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, (hipStream_t)s, (const uint8_t*)rows, B,
                     (uint32_t*)out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
int calib_rows36_write(void* rows, int64_t B, int n, void* s) {
  hipLaunchKernelGGL(rows36_write, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, (hipStream_t)s, (uint8_t*)rows, B, n);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
int calib_bytes_read(const void* x, int64_t n, void* out, void* s) {
  hipLaunchKernelGGL(bytes_read, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)s, (const uint8_t*)x, n,
                     (uint8_t*)out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
int calib_f64_rw(void* x, int64_t n, void* s) {
  hipLaunchKernelGGL(f64_rw, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)s, (double*)x, n);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
}
