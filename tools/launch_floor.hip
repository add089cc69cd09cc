// launch_floor.hip — the floor under a short chain of small launches (diagnostic).
//
// A rollout is T dependent launches over B envs.  This probe replays, in one HIP graph, T
// launches of the same grid doing (a) nothing, (b) only a turn's memory traffic: each env
// loads L u64 words and stores S u64 words (SoA planes, coalesced), with no arithmetic between
// beyond a dependence on every load.  Their per-rollout times bound what any rewrite of a
// turn's arithmetic can reach at that shape.
//   hipcc --offload-arch=gfx950 -O3 tools/launch_floor.hip -o /tmp/launch_floor
//   /tmp/launch_floor B T L S WAVES_PER_BLOCK ROLLOUTS_PER_GRAPH   (defaults: FrozenLake 4096 8 9 4 1 1;
//   bench.py replays 8 rollouts per graph, which spreads the replay's own overhead)
//   e.g. Sokoban 6x6 bench: 8192 5 12 6 2 (141 B per env-turn ~ 12 loads + 6 stores of 8 B)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int kMaxWords = 32;

__global__ void empty_kernel(uint64_t* in, uint64_t* out, int B, int L, int S) {}

__global__ void touch_kernel(uint64_t* in, uint64_t* out, int B, int L, int S) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  uint64_t v[kMaxWords];
#pragma unroll
  for (int k = 0; k < kMaxWords; ++k) v[k] = k < L ? in[(int64_t)k * B + b] : 0ull;
  uint64_t mix = 0;
#pragma unroll
  for (int k = 0; k < kMaxWords; ++k) mix ^= v[k];
#pragma unroll
  for (int k = 0; k < kMaxWords; ++k)
    if (k < S) out[(int64_t)k * B + b] = v[k] ^ (mix & 1);
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 4096, T = argc > 2 ? atoi(argv[2]) : 8;
  const int L = argc > 3 ? atoi(argv[3]) : 9, S = argc > 4 ? atoi(argv[4]) : 4;
  const int wpb = argc > 5 ? atoi(argv[5]) : 1, R = argc > 6 ? atoi(argv[6]) : 1;
  const int REPS = 2000;
  if (L > kMaxWords || S > kMaxWords || S > L) {
    fprintf(stderr, "L, S <= %d and S <= L\n", kMaxWords);
    return 1;
  }
  uint64_t *in, *out;
  CK(hipMalloc(&in, 8ull * L * B));
  CK(hipMalloc(&out, 8ull * S * B));
  CK(hipMemset(in, 0, 8ull * L * B));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int threads = 64 * wpb, grid = (B + threads - 1) / threads;
  const char* names[2] = {"empty", "touch"};
  for (int which = 0; which < 2; ++which) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int t = 0; t < T * R; ++t) {
      if (which == 0) empty_kernel<<<grid, threads, 0, st>>>(in, out, B, L, S);
      else touch_kernel<<<grid, threads, 0, st>>>(in, out, B, L, S);
    }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 200; ++i) CK(hipGraphLaunch(ge, st));
    hipEvent_t a, z;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&z));
    CK(hipEventRecord(a, st));
    for (int i = 0; i < REPS; ++i) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(z, st));
    CK(hipEventSynchronize(z));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, z));
    printf("{\"probe\": \"%s\", \"envs\": %d, \"launches_per_rollout\": %d, \"bytes_per_env\": %d, "
           "\"waves_per_block\": %d, \"rollouts_per_graph\": %d, \"us_per_rollout\": %.3f, \"us_per_launch\": %.3f}\n",
           names[which], B, T, 8 * (L + S), wpb, R, 1e3 * ms / REPS / R, 1e3 * ms / REPS / R / T);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipStreamSynchronize(st));
  return 0;
}
