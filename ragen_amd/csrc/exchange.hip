// exchange.hip — the one-shot all-gather of the per-rank episode arena (include/ragen_amd.h,
// "the one-shot arena exchange").
//
// Why not RCCL's all-gather: a ring all-gather of W ranks moves every rank's bytes over W-1
// serial hops, one xGMI link per hop, plus a per-step handshake; at W = 8 that is 7 hops of the
// 0.5-MB arena after every rollout (~23 us on the link alone, about the rollout's
// own time).  The MI355X node is a full xGMI mesh (7 links per GPU), so the direct form is one
// hop: each rank stores its arena into every peer's receive region, all 7 links at once, and
// the gather is complete when all W senders' arrival counts reached the epoch's.
//
// Memory model (MI355X_MICROARCH.md / cdna_hip_programming.md §6 G16, in its no-release form,
// carried to system scope because the readers are other devices): every store of the handed-off
// bytes is a system-scope (sc0 sc1) store, written through to the receiving memory, and drained
// (vmcnt 0) before the block barrier; then ONE lane adds the block's arrival.  No release fence:
// a system-scope release writes back the whole L2 of the XCD (buffer_wbl2), which the rollout
// just filled with dirty lines — measured +4 us per exchange at W = 1.  The waiting lanes poll
// relaxed at system scope (these loads bypass the caches) and fence once with a system-scope
// acquire.  The receive regions are fine-grained device memory, whose L2
// lines (MTYPE NC) are invalidated by that acquire and at every kernel boundary, so no L2 on the
// receiving GPU serves a stale copy of a slot a peer rewrote.
// Every wait is bounded by the constant 100-MHz clock: a missing peer sets an error bit and the
// grid drains.
#include <string.h>

#include "common.hpp"

namespace rmi {
namespace {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

constexpr int kXgBlock = 256;
constexpr int64_t kXgHdr = 4096;   // header bytes: consumed at 0, arrivals[q] at 64 + 8q
constexpr int64_t kXgAlign = 4096;  // row alignment inside a slot
constexpr int kArrivals = 8;        // u64 index of arrivals[0]
constexpr int kSysStore = 1 | 16;   // buffer cache policy: sc0 | sc1 = system scope (write-through)
constexpr int kRsrcWord3 = 0x00020000;  // gfx9 raw buffer descriptor word 3 (32-bit data format)

struct XgArgs {
  const v4u* src;
  uint8_t* region[RMI_XG_MAX_RANKS];
  u64* state;
  uint32_t* err;
  int64_t n16, nbp, slot_bytes;
  u64 ticks;
  int32_t W, rank, nb, flags;
};

__device__ __forceinline__ u64 clock100() { return __builtin_amdgcn_s_memrealtime(); }

// poll *p (relaxed, system scope) until >= target or the deadline; one acquire on success
__device__ bool wait_ge(const u64* p, u64 target, u64 deadline) {
  while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
    if (clock100() > deadline) return false;
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return true;
}

__global__ __launch_bounds__(kXgBlock) void xgather_kernel(XgArgs a) {
  __shared__ int s_ok;
  const int tid = threadIdx.x;
  // the epoch this launch moves: every block reads it before the waiting half can advance it
  // (the waiter advances only after all this rank's storing blocks counted themselves done)
  const u64 e = __hip_atomic_load(a.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  const u64 deadline = clock100() + a.ticks;
  const int n_pub = (a.flags & RMI_XG_PUBLISH) ? a.W * a.nb : 0;
  const int b = blockIdx.x;
  if (b < n_pub) {
    const int p = b / a.nb, c = b - p * a.nb;
    u64* hdr = reinterpret_cast<u64*>(a.region[p]);
    // everything enqueued before this launch has finished reading slot (e - 1) & 1 of our region
    // (a kernel boundary: reads need no release)
    if (b == 0 && tid == 0)
      __hip_atomic_store(reinterpret_cast<u64*>(a.region[a.rank]), e - 1, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    if (tid == 0) {
      // slot e & 1 of peer p last held epoch e - 2: p must be done with it
      const bool ok = e < 3 || wait_ge(hdr, e - 2, deadline);
      if (!ok) atomicOr(a.err, (uint32_t)RMI_XG_ERR_PEER_BUSY);
      s_ok = ok;
    }
    __syncthreads();
    if (!s_ok) return;
    const int64_t per = (a.n16 + a.nb - 1) / a.nb;
    const int64_t lo = (int64_t)c * per, hi = lo + per < a.n16 ? lo + per : a.n16;
    // this block's chunk of the row, as system-scope (sc0 sc1: write-through) 16-B buffer stores
    uint8_t* dst = a.region[p] + kXgHdr + (int64_t)(e & 1) * a.slot_bytes + (int64_t)a.rank * a.nbp + lo * 16;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7FFFFFF0, kRsrcWord3);
    // two 16-B pieces per lane per step, both loads issued before either store (a block holds
    // ~8 KB: one step for most lanes)
    for (int64_t i0 = lo + tid; i0 < hi; i0 += 2 * kXgBlock) {
      const int64_t i1 = i0 + kXgBlock;
      const v4u v0 = __builtin_nontemporal_load(a.src + i0);
      const v4u v1 = __builtin_nontemporal_load(a.src + (i1 < hi ? i1 : i0));
      __builtin_amdgcn_raw_buffer_store_b128(v0, rs, (int)((i0 - lo) * 16), 0, kSysStore);
      if (i1 < hi) __builtin_amdgcn_raw_buffer_store_b128(v1, rs, (int)((i1 - lo) * 16), 0, kSysStore);
    }
    __builtin_amdgcn_s_waitcnt(0);  // every store acknowledged by the memory it was written to
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(hdr + kArrivals + a.rank, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_fetch_add(a.state + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  // the waiting block: every sender's arrivals in our region, and our own storing blocks done
  const u64* own = reinterpret_cast<const u64*>(a.region[a.rank]);
  bool ok = true;
  if (tid < a.W)
    ok = wait_ge(own + kArrivals + tid, e * (u64)a.nb, deadline);
  else if (tid == 64)  // (another wave: it polls beside the first)
    ok = wait_ge(a.state + 1, e * (u64)a.W * (u64)a.nb, deadline);
  if (!ok) atomicOr(a.err, (uint32_t)RMI_XG_ERR_ARRIVALS);
  __syncthreads();
  if (tid == 0) __hip_atomic_store(a.state, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // read after the kernel boundary
}

int64_t row_bytes(int64_t nbytes) { return (nbytes + kXgAlign - 1) / kXgAlign * kXgAlign; }

}  // namespace
}  // namespace rmi

RMI_API int64_t rmi_xgather_region_bytes(int32_t world, int64_t nbytes) {
  if (world < 1 || world > RMI_XG_MAX_RANKS || nbytes < 1) return -1;
  return rmi::kXgHdr + 2 * (int64_t)world * rmi::row_bytes(nbytes);
}

RMI_API int64_t rmi_xgather_slot_offset(int32_t world, int64_t nbytes, int64_t epoch) {
  if (world < 1 || world > RMI_XG_MAX_RANKS || nbytes < 1 || epoch < 1) return -1;
  return rmi::kXgHdr + (epoch & 1) * (int64_t)world * rmi::row_bytes(nbytes);
}

RMI_API int32_t rmi_xgather_blocks_per_peer(int64_t nbytes) {
  // ~8 KB per storing block: two 16-B pieces per lane, one step, so a block's latency is one
  // load and one write-through store; 61 blocks per peer for the 0.5-MB SK arena (the first
  // form, 32 KB per block in 8 dependent steps, measured 6.3 us per exchange at W = 1)
  int64_t nb = (nbytes + 8191) / 8192;
  return (int32_t)(nb < 1 ? 1 : (nb > 256 ? 256 : nb));
}

RMI_API int rmi_xgather_alloc(int64_t bytes, int32_t mode, void** region, uint8_t* handle) {
  if (bytes < 1 || !region || !handle) return RMI_EINVAL;
  unsigned flags = mode == RMI_XG_MEM_UNCACHED ? hipDeviceMallocUncached
                   : mode == RMI_XG_MEM_FINEGRAINED ? hipDeviceMallocFinegrained
                                                    : 0u;
  if (!flags) return RMI_EINVAL;
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, (size_t)bytes, flags) != hipSuccess || !p) {
    (void)hipGetLastError();
    return RMI_EDEVICE;
  }
  hipIpcMemHandle_t h;
  static_assert(sizeof(h) == 64, "HIP IPC handle is 64 bytes");
  if (hipMemset(p, 0, (size_t)bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
      hipIpcGetMemHandle(&h, p) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFree(p);
    return RMI_EDEVICE;
  }
  memcpy(handle, &h, sizeof(h));
  *region = p;
  return RMI_OK;
}

RMI_API int rmi_xgather_open(const uint8_t* handle, void** region) {
  if (!handle || !region) return RMI_EINVAL;
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess || !p) {
    (void)hipGetLastError();
    return RMI_EDEVICE;
  }
  *region = p;
  return RMI_OK;
}

RMI_API int rmi_xgather_close(void* region) {
  if (!region) return RMI_EINVAL;
  return hipIpcCloseMemHandle(region) == hipSuccess ? RMI_OK : RMI_EDEVICE;
}

RMI_API int rmi_xgather_free(void* region) {
  if (!region) return RMI_EINVAL;
  return hipFree(region) == hipSuccess ? RMI_OK : RMI_EDEVICE;
}

RMI_API int rmi_xgather(const rmi_xgather_t* x, const void* src, int32_t flags, rmi_stream_t stream) {
  using namespace rmi;
  if (!x || flags < 1 || flags > (RMI_XG_PUBLISH | RMI_XG_WAIT)) return RMI_EINVAL;
  const int W = x->world;
  if (W < 1 || W > RMI_XG_MAX_RANKS || x->rank < 0 || x->rank >= W || x->nbytes < 16 || x->nbytes % 16 ||
      !x->state || !x->err || x->blocks_per_peer < 0)
    return RMI_EINVAL;
  if ((flags & RMI_XG_PUBLISH) && (!src || (reinterpret_cast<uintptr_t>(src) & 15u))) return RMI_EINVAL;
  XgArgs a;
  for (int q = 0; q < RMI_XG_MAX_RANKS; ++q) {
    a.region[q] = static_cast<uint8_t*>(q < W ? x->region[q] : nullptr);
    if (q < W && !a.region[q]) return RMI_EINVAL;
  }
  a.src = static_cast<const v4u*>(src);
  a.state = reinterpret_cast<u64*>(x->state);
  a.err = x->err;
  a.n16 = x->nbytes / 16;
  a.nbp = row_bytes(x->nbytes);
  a.slot_bytes = (int64_t)W * a.nbp;
  a.ticks = (x->timeout_us ? x->timeout_us : 2000000ull) * 100ull;
  a.W = W;
  a.rank = x->rank;
  a.nb = x->blocks_per_peer ? x->blocks_per_peer : rmi_xgather_blocks_per_peer(x->nbytes);
  a.flags = flags;
  const int grid = ((flags & RMI_XG_PUBLISH) ? W * a.nb : 0) + ((flags & RMI_XG_WAIT) ? 1 : 0);
  hipLaunchKernelGGL(xgather_kernel, dim3(grid), dim3(kXgBlock), 0, as_stream(stream), a);
  return launch_status();
}
