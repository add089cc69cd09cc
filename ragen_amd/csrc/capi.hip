// capi.hip — library-level helpers of the C ABI.
#include "common.hpp"

namespace rmi {
namespace {

// 16 B per lane, grid-stride, nontemporal (MI355X_MICROARCH.md: the float4 copy that measures
// the achievable HBM bandwidth).  The grid is what sets the rate: tools/copy_probe.hip swept
// loads in flight per lane (1, 2, 4, 8), nontemporal vs plain, grid-stride vs one chunk per
// block and 2 / 4 / 8 / 16 blocks per CU over a 1 GiB copy (profiles/r04_copy_probe.json):
// 4 blocks per CU with one 16-B load per lane per step reads + writes 6.00 TB/s, 2 per CU with
// two loads 5.98, while the 8-per-CU grid this used before (2048 blocks) reached 4.86.
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kBlock) void stream_copy_kernel(v4u* __restrict__ dst, const v4u* __restrict__ src,
                                                             int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n16; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__global__ void tail_copy_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

}  // namespace
}  // namespace rmi

RMI_API const char* rmi_version(void) { return "ragen_amd 0.2.0 (gfx950)"; }

RMI_API int rmi_stream_synchronize(rmi_stream_t stream) {
  return hipStreamSynchronize(rmi::as_stream(stream)) == hipSuccess ? RMI_OK : RMI_EDEVICE;
}

RMI_API int rmi_upload(void* dst, const void* src, size_t bytes, rmi_stream_t stream) {
  if (!bytes) return RMI_OK;
  if (!dst || !src) return RMI_EINVAL;
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, rmi::as_stream(stream)) == hipSuccess ? RMI_OK
                                                                                                   : RMI_EDEVICE;
}

namespace rmi {
namespace {
constexpr int kCopyBlock = 256;
// 16-B stores (fewer PCIe writes) while both ends are 16-B aligned, then the dword tail
__global__ __launch_bounds__(kCopyBlock) void readback_kernel(const uint32_t* __restrict__ src, uint32_t* dst,
                                                              int64_t n32) {
  const bool v4 = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) == 0;
  const int64_t n4 = v4 ? n32 / 4 : 0;
  const int64_t t = (int64_t)blockIdx.x * kCopyBlock + threadIdx.x, step = (int64_t)gridDim.x * kCopyBlock;
  for (int64_t i = t; i < n4; i += step)
    reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
  for (int64_t i = 4 * n4 + t; i < n32; i += step) dst[i] = src[i];
}

// the device address of a pinned host buffer, or nullptr (pageable memory).  Looked up on every
// call, never cached: a pinned buffer may be released (hipHostFree, hipHostUnregister, torch's
// host-cache flush) and its address reused by pageable memory or another registration, and a
// remembered mapping would then send the readback kernel's stores to a stale device address.
// The lookup is a runtime map search (well under a microsecond against a launch).
void* host_mapping(void* host) {
  hipPointerAttribute_t attr;
  // (only where the runtime's host address is the one asked about: its device address is then
  // that byte's, whether or not the runtime offsets interior pointers)
  if (hipPointerGetAttributes(&attr, host) == hipSuccess && attr.type == hipMemoryTypeHost && attr.devicePointer &&
      attr.hostPointer == host)
    return attr.devicePointer;
  (void)hipGetLastError();  // (clear the lookup's error: pageable memory)
  return nullptr;
}
}  // namespace

int readback_async(void* host, const void* dev, size_t bytes, hipStream_t s) {
  const bool a4 = bytes % 4 == 0 && ((reinterpret_cast<uintptr_t>(host) | reinterpret_cast<uintptr_t>(dev)) & 3u) == 0;
  void* hdev = a4 ? host_mapping(host) : nullptr;
  if (!hdev)
    return hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, s) == hipSuccess ? RMI_OK : RMI_EDEVICE;
  const int64_t n32 = (int64_t)(bytes / 4);
  int64_t grid = (n32 / 4 + kCopyBlock - 1) / kCopyBlock;  // (one 16-B store a thread)
  grid = grid < 1 ? 1 : (grid > 1024 ? 1024 : grid);
  hipLaunchKernelGGL(readback_kernel, dim3((unsigned)grid), dim3(kCopyBlock), 0, s, static_cast<const uint32_t*>(dev),
                     static_cast<uint32_t*>(hdev), n32);
  return hipGetLastError() == hipSuccess ? RMI_OK : RMI_EDEVICE;
}
}  // namespace rmi

RMI_API int64_t rmi_host_live_ids(const uint8_t* flags, int64_t n, uint32_t done_bits, int64_t lo, int64_t* out,
                                  int64_t cap) {
  if (!flags || n < 0 || (!out && cap > 0)) return -1;
  // branch-free in the flags (their pattern is random: a branch per env mispredicted often)
  int64_t k = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (k < cap) out[k] = lo + i;
    k += (flags[i] & done_bits) == 0;
  }
  return k <= cap ? k : -1;
}

RMI_API int rmi_readback(void* dst, const void* src, size_t bytes, rmi_stream_t stream) {
  if (!bytes) return RMI_OK;
  if (!dst || !src) return RMI_EINVAL;
  hipStream_t s = rmi::as_stream(stream);
  const int rc = rmi::readback_async(dst, src, bytes, s);
  if (rc) return rc;
  return hipStreamSynchronize(s) == hipSuccess ? RMI_OK : RMI_EDEVICE;
}

RMI_API int rmi_device_copy(void* dst, const void* src, size_t bytes, rmi_stream_t stream) {
  using namespace rmi;
  if ((!dst || !src) && bytes) return RMI_EINVAL;
  if (!bytes) return RMI_OK;
  hipStream_t s = as_stream(stream);
  const bool aligned = ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15u) == 0;
  const int64_t n16 = aligned ? (int64_t)(bytes / 16) : 0;
  if (n16) {
    static int cus = 0;  // the device's CU count, queried once
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
    }
    int64_t blocks = (n16 + kBlock - 1) / kBlock;
    if (blocks > 4 * (int64_t)cus) blocks = 4 * (int64_t)cus;
    hipLaunchKernelGGL(stream_copy_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, static_cast<v4u*>(dst),
                       static_cast<const v4u*>(src), n16);
  }
  const int64_t done = n16 * 16, rest = (int64_t)bytes - done;
  if (rest > 0)
    hipLaunchKernelGGL(tail_copy_kernel, dim3((unsigned)((rest + 255) / 256)), dim3(256), 0, s,
                       static_cast<uint8_t*>(dst) + done, static_cast<const uint8_t*>(src) + done, rest);
  return launch_status();
}

// Host-side: the packed vocabulary of rmi_detokenize from the plain byte table (run once per
// tokenizer; CPU memory in and out).
RMI_API int rmi_vocab_pack(const int64_t* vocab_off, const uint8_t* vocab_bytes, int64_t n_bytes, int64_t V,
                           const uint8_t* skip, uint32_t* packed) {
  if (V < 1 || n_bytes < 0 || !vocab_off || !packed || (n_bytes > 0 && !vocab_bytes)) return RMI_EINVAL;
  for (int64_t t = 0; t < V; ++t) {
    const int64_t o = vocab_off[t], len = vocab_off[t + 1] - o;
    if (o < 0 || len < 0 || o + len > n_bytes) return RMI_EINVAL;
    if (len > 0xFFFFFF || o > 0xFFFFFFFFll) return RMI_EUNSUP;
    uint32_t w[3] = {0u, 0u, 0u};
    if (len <= 12) {
      for (int64_t k = 0; k < len; ++k) w[k >> 2] |= (uint32_t)vocab_bytes[o + k] << (8 * (k & 3));
    } else {
      w[0] = (uint32_t)o;
    }
    uint32_t* e = packed + 4 * t;
    e[0] = w[0];
    e[1] = w[1];
    e[2] = w[2];
    e[3] = (uint32_t)len | ((skip && skip[t]) ? 0x80000000u : 0u);
  }
  return RMI_OK;
}
