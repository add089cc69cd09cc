// copy_probe.hip — achievable HBM bandwidth on this box: variants of a 16-B-per-lane streaming
// copy of 1 GiB (read + write, far past the 256 MiB Infinity Cache), timed with HIP events over
// 20 launches each.  Variants: loads in flight per lane (U), nontemporal vs plain loads/stores,
// grid-stride vs one contiguous chunk per block, and the grid size (blocks per CU).
//   hipcc --offload-arch=gfx950 -O3 -o tools/_build/copy_probe tools/copy_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void grid_stride(v4u* __restrict__ dst, const v4u* __restrict__ src, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    v4u r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(r[u], dst + i + u * stride); else dst[i + u * stride] = r[u];
    }
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

// block b copies the contiguous chunk [b*chunk, (b+1)*chunk) in steps of 256*U vectors
template <int U, bool NT>
__global__ __launch_bounds__(256) void chunked(v4u* __restrict__ dst, const v4u* __restrict__ src, int64_t n16,
                                               int64_t chunk) {
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = lo + chunk < n16 ? lo + chunk : n16;
  int64_t i = lo + threadIdx.x;
  for (; i + (U - 1) * 256 < hi; i += U * 256) {
    v4u r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = NT ? __builtin_nontemporal_load(src + i + u * 256) : src[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(r[u], dst + i + u * 256); else dst[i + u * 256] = r[u];
    }
  }
  for (; i < hi; i += 256) dst[i] = src[i];
}

template <int U, bool NT>
static double run(bool grid, int blocks, v4u* d, const v4u* s, int64_t n16, int reps, hipEvent_t a, hipEvent_t b) {
  const int64_t chunk = (n16 + blocks - 1) / blocks;
  auto launch = [&]() {
    if (grid) hipLaunchKernelGGL((grid_stride<U, NT>), dim3(blocks), dim3(256), 0, 0, d, s, n16);
    else hipLaunchKernelGGL((chunked<U, NT>), dim3(blocks), dim3(256), 0, 0, d, s, n16, chunk);
  };
  launch();
  hipDeviceSynchronize();
  hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return 2.0 * n16 * 16 * reps / (ms * 1e-3) / 1e12;
}

int main() {
  const int64_t bytes = 1ll << 30, n16 = bytes / 16;
  v4u *s, *d;
  CHECK(hipMalloc(&s, bytes));
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMemset(s, 1, bytes));
  CHECK(hipMemset(d, 0, bytes));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("{\"cus\": %d, \"bytes\": %lld, \"rows\": [\n", cus, (long long)bytes);
  const int per_cu[] = {2, 4, 8, 16};
  bool first = true;
  for (int g = 0; g < 2; ++g) {
    for (int nt = 0; nt < 2; ++nt) {
      for (int pc : per_cu) {
        const int blocks = pc * cus;
        double r[4];
        if (nt) {
          r[0] = run<1, true>(g == 0, blocks, d, s, n16, 20, a, b);
          r[1] = run<2, true>(g == 0, blocks, d, s, n16, 20, a, b);
          r[2] = run<4, true>(g == 0, blocks, d, s, n16, 20, a, b);
          r[3] = run<8, true>(g == 0, blocks, d, s, n16, 20, a, b);
        } else {
          r[0] = run<1, false>(g == 0, blocks, d, s, n16, 20, a, b);
          r[1] = run<2, false>(g == 0, blocks, d, s, n16, 20, a, b);
          r[2] = run<4, false>(g == 0, blocks, d, s, n16, 20, a, b);
          r[3] = run<8, false>(g == 0, blocks, d, s, n16, 20, a, b);
        }
        const int us[4] = {1, 2, 4, 8};
        for (int k = 0; k < 4; ++k) {
          printf("%s{\"grid_stride\": %d, \"nontemporal\": %d, \"blocks_per_cu\": %d, \"loads_per_lane\": %d, "
                 "\"TBs\": %.3f}", first ? "" : ",\n", g == 0 ? 1 : 0, nt, pc, us[k], r[k]);
          first = false;
        }
      }
    }
  }
  printf("\n]}\n");
  // verify the last copy
  std::vector<unsigned char> h(4096);
  hipMemcpy(h.data(), d, 4096, hipMemcpyDeviceToHost);
  for (int i = 0; i < 4096; ++i)
    if (h[i] != 1) { printf("copy mismatch at %d\n", i); return 2; }
  return 0;
}
