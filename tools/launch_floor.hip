// launch_floor.hip — the floor under a short chain of small launches (diagnostic).
//
// A FrozenLake rollout is 8 dependent launches of 64 one-wave workgroups (4096 envs).  This
// probe replays, in one HIP graph, 8 launches of the same grid doing (a) nothing, (b) the turn's
// memory traffic only: each lane loads the bytes a FrozenLake env-turn reads (desc 16 B, s,
// PCG64 state 32 B, flags / counters / penalty, has_input, n_actions, 8 action bytes) and
// stores what it writes back, with no arithmetic between.  Their per-rollout times bound what
// any rewrite of the turn's arithmetic can reach.
//   hipcc --offload-arch=gfx950 -O3 tools/launch_floor.hip -o /tmp/launch_floor && /tmp/launch_floor
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

struct Env {
  const uint4* desc;
  int32_t* s;
  uint64_t* rng;  // [4, B]
  uint8_t* flags;
  int32_t* num_actions;
  int32_t* n_turns;
  double* penalty;
  const uint8_t* has_input;
  const int32_t* n_act;
  const uint64_t* acts;
  double* turn_reward;  // [T, B]
  uint8_t* turn_info;
  uint8_t* turn_exec;
  int B;
};

__global__ __launch_bounds__(64) void empty_kernel(Env e, int t) {}

__global__ __launch_bounds__(64) void touch_kernel(Env e, int t) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= e.B) return;
  const uint4 d = e.desc[b];
  int32_t s = e.s[b];
  uint64_t r0 = e.rng[b], r1 = e.rng[e.B + b], r2 = e.rng[2 * e.B + b], r3 = e.rng[3 * e.B + b];
  uint8_t f = e.flags[b];
  int32_t na = e.num_actions[b], nt = e.n_turns[b];
  double p = e.penalty[b];
  const uint8_t h = e.has_input[b];
  const int32_t n = e.n_act[b];
  const uint64_t a = e.acts[b];
  // a dependence on every load (so none is dead), then the turn's stores
  const uint64_t mix = d.x ^ d.y ^ d.z ^ d.w ^ (uint64_t)s ^ r0 ^ r1 ^ r2 ^ r3 ^ f ^ (uint64_t)na ^ (uint64_t)nt ^ h ^
                       (uint64_t)n ^ a ^ (uint64_t)p;
  const int64_t tb = (int64_t)t * e.B + b;
  e.s[b] = s ^ (int32_t)(mix & 1);
  e.rng[b] = r0;
  e.rng[e.B + b] = r1 ^ (mix & 2);
  e.flags[b] = f;
  e.num_actions[b] = na + 1;
  e.n_turns[b] = nt + 1;
  e.penalty[b] = p;
  e.turn_reward[tb] = (double)(mix & 3);
  e.turn_info[tb] = (uint8_t)mix;
  e.turn_exec[tb] = (uint8_t)(mix >> 8);
}

int main() {
  const int B = 4096, T = 8, REPS = 2000;
  Env e;
  e.B = B;
  void* p;
  CK(hipMalloc(&p, 16 * B)); CK(hipMemset(p, 0, 16 * B)); e.desc = (const uint4*)p;
  CK(hipMalloc(&p, 4 * B)); CK(hipMemset(p, 0, 4 * B)); e.s = (int32_t*)p;
  CK(hipMalloc(&p, 32 * B)); CK(hipMemset(p, 0, 32 * B)); e.rng = (uint64_t*)p;
  CK(hipMalloc(&p, B)); CK(hipMemset(p, 0, B)); e.flags = (uint8_t*)p;
  CK(hipMalloc(&p, 4 * B)); CK(hipMemset(p, 0, 4 * B)); e.num_actions = (int32_t*)p;
  CK(hipMalloc(&p, 4 * B)); CK(hipMemset(p, 0, 4 * B)); e.n_turns = (int32_t*)p;
  CK(hipMalloc(&p, 8 * B)); CK(hipMemset(p, 0, 8 * B)); e.penalty = (double*)p;
  CK(hipMalloc(&p, B)); CK(hipMemset(p, 1, B)); e.has_input = (const uint8_t*)p;
  CK(hipMalloc(&p, 4 * B)); CK(hipMemset(p, 0, 4 * B)); e.n_act = (const int32_t*)p;
  CK(hipMalloc(&p, 8 * B)); CK(hipMemset(p, 0, 8 * B)); e.acts = (const uint64_t*)p;
  CK(hipMalloc(&p, 8 * B * T)); e.turn_reward = (double*)p;
  CK(hipMalloc(&p, B * T)); e.turn_info = (uint8_t*)p;
  CK(hipMalloc(&p, B * T)); e.turn_exec = (uint8_t*)p;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const char* names[2] = {"empty", "touch"};
  for (int which = 0; which < 2; ++which) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int t = 0; t < T; ++t) {
      if (which == 0) empty_kernel<<<B / 64, 64, 0, st>>>(e, t);
      else touch_kernel<<<B / 64, 64, 0, st>>>(e, t);
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
    printf("{\"probe\": \"%s\", \"envs\": %d, \"launches_per_rollout\": %d, \"us_per_rollout\": %.3f, "
           "\"us_per_launch\": %.3f}\n",
           names[which], B, T, 1e3 * ms / REPS, 1e3 * ms / REPS / T);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipStreamSynchronize(st));
  return 0;
}
