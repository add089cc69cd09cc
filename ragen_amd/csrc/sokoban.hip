// sokoban.hip — one whole EnvStateManager turn for a batch of Sokoban envs (gfx950).
//
// Replaces es_manager.py:105-171 driving sokoban/env.py:44-51 -> gym_sokoban step
// (SURVEY.md App. A.1).  One lane owns one env; a 256-thread workgroup owns 256 envs.
//
// HBM layout (caller-owned SoA, include/ragen_amd.h): room grids are [B, H*W] u8 rows.
// The workgroup stages its 256 rows of room_state and room_fixed through LDS with fully
// coalesced dword loads (row stride H*W/4 dwords = 9 for 6x6 — coprime with the 32 LDS
// banks, so each lane's row read is conflict-free).  Each lane turns its row into 64-bit
// bit-planes with SWAR multiplies (3 planes for room_state values 0..7, 2 for room_fixed),
// runs up to K pushes/moves with shift/mask arithmetic — cell writes are byte-exact with
// the numpy writes upstream makes, including the untouched cells — and keeps the number
// of open targets incrementally (no per-step grid scan).  Rows go back the same way.
// The kernel is latency-bound (8192 envs = 128 waves): the work per lane is kept short.
#include "common.hpp"

namespace rmi {
namespace {

// 4 bytes -> 4 bits: bit p of byte j of x lands at bit j   (no carries: distinct products)
__device__ __forceinline__ uint32_t gather_bit(uint32_t x, int p) {
  return (((x >> p) & 0x01010101u) * 0x01020408u) >> 24 & 0xFu;
}
// 4 bits -> 4 bytes (bit j of n -> bit 0 of byte j)
__device__ __forceinline__ uint32_t spread_bits(uint32_t n) { return (n * 0x00204081u) & 0x01010101u; }

struct SokobanEnvDev {
  uint64_t s0, s1, s2, f0, f1, tgt;  // state planes, fixed planes, fixed == 2
  int H, W, r, c;
  int num_env_steps, boxes_on_target, num_boxes, max_steps, n_open;
  uint8_t err;

  __device__ __forceinline__ int sval(int i) const {
    return (int)((s0 >> i) & 1ull) | ((int)((s1 >> i) & 1ull) << 1) | ((int)((s2 >> i) & 1ull) << 2);
  }
  __device__ __forceinline__ int fval(int i) const {
    return (int)((f0 >> i) & 1ull) | ((int)((f1 >> i) & 1ull) << 1);
  }
  // contribution of a cell to the open-target count of _calc_reward:
  // (room_state == 2) | ((room_fixed == 2) & (room_state == 5))
  __device__ __forceinline__ int open_of(int i, int v) const {
    return (v == 2) | ((v == 5) & (int)((tgt >> i) & 1ull));
  }
  __device__ __forceinline__ void sset(int i, int v) {
    n_open += open_of(i, v) - open_of(i, sval(i));
    const uint64_t m = 1ull << i;
    s0 = (s0 & ~m) | ((v & 1) ? m : 0ull);
    s1 = (s1 & ~m) | ((v & 2) ? m : 0ull);
    s2 = (s2 & ~m) | ((v & 4) ? m : 0ull);
  }
  // numpy indexing of room_state[row, col]: negative indices wrap once, else IndexError
  __device__ __forceinline__ bool cell(int row, int col, int& idx) const {
    if (row < -H || row >= H || col < -W || col >= W) return false;
    idx = (row < 0 ? row + H : row) * W + (col < 0 ? col + W : col);
    return true;
  }
  // action 1..4 push (falls back to move), 5..8 move  (gym_sokoban ACTION_LOOKUP)
  __device__ __forceinline__ bool step(int a, double& reward, bool& done, bool& eff, bool& success) {
    if (a < 1 || a > 8) return false;
    const int d = (a - 1) & 3;  // CHANGE_COORDINATES[(a-1) % 4]
    const int dr = d == 0 ? -1 : (d == 1 ? 1 : 0);
    const int dc = d == 2 ? -1 : (d == 3 ? 1 : 0);
    const int pr = r, pc = c;
    num_env_steps += 1;
    const int nr = r + dr, nc = c + dc;
    bool try_move = a > 4;
    if (a <= 4) {  // _push
      const int br = nr + dr, bc = nc + dc;
      if (!(br >= H || bc >= W)) {  // upstream only bounds-checks the high side: else no push, no move
        int ni, bi;
        if (!cell(nr, nc, ni) || !cell(br, bc, bi)) {
          err |= RMI_ERR_INDEX;
          return false;
        }
        const int vn = sval(ni), vb = sval(bi);
        if ((vn == 3 || vn == 4) && (vb == 1 || vb == 2)) {
          int oi;
          cell(r, c, oi);
          sset(ni, 5);
          sset(oi, fval(oi));
          sset(bi, ((tgt >> bi) & 1ull) ? 3 : 4);
          r = nr;
          c = nc;
        } else {
          try_move = true;  // _push falls back to _move
        }
      }
    }
    if (try_move) {  // _move
      int ni;
      if (!cell(nr, nc, ni)) {
        err |= RMI_ERR_INDEX;
        return false;
      }
      const int vn = sval(ni);
      if (vn == 1 || vn == 2) {
        int oi;
        cell(r, c, oi);
        sset(ni, 5);
        sset(oi, fval(oi));
        r = nr;
        c = nc;
      }
    }
    // _calc_reward + _check_if_done
    const int cur = num_boxes - n_open;
    double rw = -0.1;                              // penalty_for_step
    if (cur > boxes_on_target) rw += 1.0;          // reward_box_on_target
    else if (cur < boxes_on_target) rw += -1.0;    // penalty_box_off_target
    const bool all_on = n_open == 0;
    if (all_on) rw += 10.0;                        // reward_finished
    boxes_on_target = cur;
    reward = rw;
    done = all_on || (max_steps == num_env_steps);
    success = boxes_on_target == num_boxes;        // sokoban/env.py:49
    eff = !(pr == r && pc == c);                   // sokoban/env.py:48
    return true;
  }
};

constexpr int kRowWordsMax = 16;  // 64 cells

template <int HW>  // HW = H*W (compile-time for the common sizes, 0 = runtime)
__device__ __forceinline__ void to_planes(const uint32_t* ms, const uint32_t* mf, int hw, SokobanEnvDev& e) {
  const int row_words = (hw + 3) >> 2;
  e.s0 = e.s1 = e.s2 = e.f0 = e.f1 = 0;
#pragma unroll
  for (int w = 0; w < kRowWordsMax; ++w) {
    if (w < row_words) {
      uint32_t xs = ms[w], xf = mf[w];
      const int valid = hw - 4 * w;  // cells of this word inside the row
      if (valid < 4) {
        const uint32_t keep = (1u << (8 * valid)) - 1u;
        xs &= keep;
        xf &= keep;
      }
      if ((xs | xf) & 0xF8F8F8F8u) e.err |= RMI_ERR_STATE;  // byte > 7
      if (xf & 0x04040404u) e.err |= RMI_ERR_STATE;         // fixed > 3
      e.s0 |= (uint64_t)gather_bit(xs, 0) << (4 * w);
      e.s1 |= (uint64_t)gather_bit(xs, 1) << (4 * w);
      e.s2 |= (uint64_t)gather_bit(xs, 2) << (4 * w);
      e.f0 |= (uint64_t)gather_bit(xf, 0) << (4 * w);
      e.f1 |= (uint64_t)gather_bit(xf, 1) << (4 * w);
    }
  }
  e.tgt = e.f1 & ~e.f0;  // fixed == 2
  // initial open-target count
  const uint64_t eq2 = ~e.s0 & e.s1 & ~e.s2, eq5 = e.s0 & ~e.s1 & e.s2;
  e.n_open = __popcll(eq2 | (e.tgt & eq5));
}

template <int HW>
__global__ __launch_bounds__(kBlock) void sokoban_step_turn_kernel(
    rmi_sokoban_t env, rmi_episode_t ep, rmi_turn_t in, int hw_rt, int word_path, uint8_t* __restrict__ err_out) {
  __shared__ uint32_t lds_state[kBlock * kRowWordsMax];
  __shared__ uint32_t lds_fixed[kBlock * kRowWordsMax];
  const int hw = HW ? HW : hw_rt;
  const int row_words = (hw + 3) >> 2;
  const int B = ep.B;
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * kBlock;
  const int64_t b = b0 + tid;
  const int nb = (int)min<int64_t>(kBlock, B - b0);

  bool act = false;
  uint8_t flags = 0;
  if (b < B) {
    flags = ep.flags[b];
    act = in.has_input ? (in.has_input[b] != 0) : !(flags & RMI_FLAG_DONE);
  }
  if (!__syncthreads_or(act)) return;  // nothing to step in this workgroup

  // ---- stage the workgroup's rows through LDS (coalesced)
  if (word_path) {
    const uint32_t* gs = reinterpret_cast<const uint32_t*>(env.room_state + b0 * hw);
    const uint32_t* gf = reinterpret_cast<const uint32_t*>(env.room_fixed + b0 * hw);
    const int nwords = nb * row_words;
    for (int i = tid; i < nwords; i += kBlock) {
      lds_state[i] = gs[i];
      lds_fixed[i] = gf[i];
    }
  } else {
    uint8_t* ls = reinterpret_cast<uint8_t*>(lds_state);
    uint8_t* lf = reinterpret_cast<uint8_t*>(lds_fixed);
    const int nbytes = nb * hw;
    for (int i = tid; i < nbytes; i += kBlock) {
      const int row = i / hw, col = i - row * hw;
      ls[row * row_words * 4 + col] = env.room_state[b0 * hw + i];
      lf[row * row_words * 4 + col] = env.room_fixed[b0 * hw + i];
    }
  }
  __syncthreads();

  bool changed = false;
  if (act) {
    // per-env scalars: issue every load before the dependent work
    const int8_t pr = env.player[2 * b], pc = env.player[2 * b + 1];
    const int32_t nes = env.num_env_steps[b], bot = env.boxes_on_target[b];
    int32_t num_actions = ep.num_actions[b];
    int32_t n_turns = ep.n_turns[b];
    double penalty = ep.penalty[b];
    const int n_act = in.n_actions[b];
    const uint64_t acts = load_actions(in.actions + b * (int64_t)in.K, in.K);

    SokobanEnvDev e;
    e.H = env.H;
    e.W = env.W;
    e.err = 0;
    uint32_t* ms = lds_state + tid * row_words;
    to_planes<HW>(ms, lds_fixed + tid * row_words, hw, e);
    e.r = pr;
    e.c = pc;
    e.num_env_steps = nes;
    e.boxes_on_target = bot;
    e.num_boxes = env.num_boxes;
    e.max_steps = env.max_steps;

    uint8_t err = 0;
    TurnOut o = run_turn(e, acts, n_act, in.K, num_actions, flags, n_turns, penalty, in.max_actions_per_traj,
                         in.format_penalty, err);
    err |= e.err;
    changed = o.stepped_any_state;

    ep.num_actions[b] = num_actions;
    ep.flags[b] = flags;
    ep.n_turns[b] = n_turns;
    ep.penalty[b] = penalty;
    const int64_t tb = (int64_t)in.turn * B + b;
    ep.turn_reward[tb] = o.acc;
    ep.turn_info[tb] = o.info;
    ep.turn_exec[tb] = o.exec;
    if (changed) {
      env.player[2 * b] = (int8_t)e.r;
      env.player[2 * b + 1] = (int8_t)e.c;
      env.num_env_steps[b] = e.num_env_steps;
      env.boxes_on_target[b] = e.boxes_on_target;
#pragma unroll
      for (int w = 0; w < kRowWordsMax; ++w) {
        if (w < row_words) {
          const int sh = 4 * w;
          uint32_t x = spread_bits((uint32_t)(e.s0 >> sh) & 0xFu) | (spread_bits((uint32_t)(e.s1 >> sh) & 0xFu) << 1) |
                       (spread_bits((uint32_t)(e.s2 >> sh) & 0xFu) << 2);
          const int valid = hw - 4 * w;
          if (valid < 4) {  // keep the padding bytes of a partial last word
            const uint32_t keep = (1u << (8 * valid)) - 1u;
            x = (x & keep) | (ms[w] & ~keep);
          }
          ms[w] = x;
        }
      }
    }
    if (err_out && err) err_out[b] |= err;
  }
  if (!__syncthreads_or(changed)) return;
  if (word_path) {
    uint32_t* gs = reinterpret_cast<uint32_t*>(env.room_state + b0 * hw);
    const int nwords = nb * row_words;
    for (int i = tid; i < nwords; i += kBlock) gs[i] = lds_state[i];
  } else {
    const uint8_t* ls = reinterpret_cast<const uint8_t*>(lds_state);
    const int nbytes = nb * hw;
    for (int i = tid; i < nbytes; i += kBlock) {
      const int row = i / hw, col = i - row * hw;
      env.room_state[b0 * hw + i] = ls[row * row_words * 4 + col];
    }
  }
}

// Fused reset: room_state/player from the post-generation snapshot, counters and the whole
// episode record zeroed, in one launch (SokobanEnv.reset sokoban/env.py:37 + EnvStatus()).
__global__ __launch_bounds__(kBlock) void sokoban_reset_kernel(rmi_sokoban_t env, rmi_episode_t ep, int hw,
                                                               const uint8_t* __restrict__ init_state,
                                                               const int8_t* __restrict__ init_player) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t B = ep.B;
  const int64_t nwords = (B * hw) >> 2;
  if (i < nwords) reinterpret_cast<uint32_t*>(env.room_state)[i] = reinterpret_cast<const uint32_t*>(init_state)[i];
  if (i < B) {
    env.player[2 * i] = init_player[2 * i];
    env.player[2 * i + 1] = init_player[2 * i + 1];
    env.num_env_steps[i] = 0;
    env.boxes_on_target[i] = 0;
    ep.num_actions[i] = 0;
    ep.flags[i] = 0;
    ep.n_turns[i] = 0;
    ep.penalty[i] = 0.0;
    for (int t = 0; t < ep.T; ++t) {
      ep.turn_reward[t * B + i] = 0.0;
      ep.turn_info[t * B + i] = 0;
      ep.turn_exec[t * B + i] = 0;
    }
  }
}

}  // namespace
}  // namespace rmi

RMI_API int rmi_sokoban_step_turn(const rmi_sokoban_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                  uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (!env) return RMI_EINVAL;
  const int hw = env->H * env->W;
  if (env->H <= 0 || env->W <= 0 || hw > 64) return RMI_EUNSUP;
  const int rc = check_turn_args(ep, in);
  if (rc != RMI_OK) return rc > 0 ? RMI_OK : rc;
  if (!env->room_fixed || !env->room_state || !env->player || !env->num_env_steps || !env->boxes_on_target)
    return RMI_EINVAL;
  const bool aligned = ((reinterpret_cast<uintptr_t>(env->room_state) | reinterpret_cast<uintptr_t>(env->room_fixed)) &
                        3u) == 0;
  const int word_path = (hw % 4 == 0) && aligned;
  const unsigned grid = (unsigned)((ep->B + kBlock - 1) / kBlock);
  hipStream_t s = as_stream(stream);
  if (hw == 36 && word_path)
    hipLaunchKernelGGL(sokoban_step_turn_kernel<36>, dim3(grid), dim3(kBlock), 0, s, *env, *ep, *in, hw, 1, err);
  else if (hw == 64 && word_path)
    hipLaunchKernelGGL(sokoban_step_turn_kernel<64>, dim3(grid), dim3(kBlock), 0, s, *env, *ep, *in, hw, 1, err);
  else
    hipLaunchKernelGGL(sokoban_step_turn_kernel<0>, dim3(grid), dim3(kBlock), 0, s, *env, *ep, *in, hw, word_path,
                       err);
  return launch_status();
}

RMI_API int rmi_sokoban_reset(const rmi_sokoban_t* env, const rmi_episode_t* ep, const uint8_t* init_state,
                              const int8_t* init_player, rmi_stream_t stream) {
  using namespace rmi;
  if (!env || !ep || ep->B < 0 || ep->T <= 0) return RMI_EINVAL;
  const int hw = env->H * env->W;
  if (hw <= 0 || hw > 64) return RMI_EUNSUP;
  if (ep->B == 0) return RMI_OK;
  if (!init_state || !init_player || !env->room_state || !env->player || !env->num_env_steps ||
      !env->boxes_on_target || !ep->num_actions || !ep->flags || !ep->n_turns || !ep->penalty || !ep->turn_reward ||
      !ep->turn_info || !ep->turn_exec)
    return RMI_EINVAL;
  if (((int64_t)ep->B * hw) % 4 != 0 ||
      ((reinterpret_cast<uintptr_t>(env->room_state) | reinterpret_cast<uintptr_t>(init_state)) & 3u))
    return RMI_EUNSUP;
  const int64_t n = ((int64_t)ep->B * hw / 4) > ep->B ? ((int64_t)ep->B * hw / 4) : ep->B;
  hipLaunchKernelGGL(sokoban_reset_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     as_stream(stream), *env, *ep, hw, init_state, init_player);
  return launch_status();
}
