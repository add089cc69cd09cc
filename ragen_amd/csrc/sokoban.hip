// sokoban.hip — one whole EnvStateManager turn for a batch of Sokoban envs (gfx950).
//
// Replaces es_manager.py:105-171 driving sokoban/env.py:44-51 -> gym_sokoban step
// (SURVEY.md App. A.1).  One thread owns one env; a 256-thread workgroup owns 256 envs.
//
// HBM layout (caller-owned SoA, see include/ragen_amd.h): room grids are [B, H*W] u8
// rows.  The workgroup stages its 256 rows of room_state and room_fixed through LDS with
// fully coalesced dword loads (row stride H*W/4 dwords = 9 for 6x6, coprime with the 32
// LDS banks, so the per-lane row reads are conflict-free), converts each row to 3 (state)
// + 2 (fixed) 64-bit bit-planes in registers, runs up to K pushes/moves on the planes with
// shift/mask arithmetic (byte-exact with numpy cell writes), and writes the rows back the
// same way.  Per-turn outputs go to turn-major [T,B] rows (coalesced).
#include "common.hpp"

namespace rmi {
namespace {

struct SokobanEnvDev {
  // bit-planes of room_state (values 0..7) and room_fixed (0..3); bit c = cell c
  uint64_t s0, s1, s2, f0, f1, cells;
  int H, W, r, c;
  int num_env_steps, boxes_on_target, num_boxes, max_steps;
  uint8_t err;

  __device__ __forceinline__ int sval(int i) const {
    return (int)((s0 >> i) & 1ull) | ((int)((s1 >> i) & 1ull) << 1) | ((int)((s2 >> i) & 1ull) << 2);
  }
  __device__ __forceinline__ int fval(int i) const {
    return (int)((f0 >> i) & 1ull) | ((int)((f1 >> i) & 1ull) << 1);
  }
  __device__ __forceinline__ void sset(int i, int v) {
    const uint64_t m = 1ull << i;
    s0 = (s0 & ~m) | ((v & 1) ? m : 0ull);
    s1 = (s1 & ~m) | ((v & 2) ? m : 0ull);
    s2 = (s2 & ~m) | ((v & 4) ? m : 0ull);
  }
  __device__ __forceinline__ uint64_t s_eq(int v) const {
    return ((v & 1) ? s0 : ~s0) & ((v & 2) ? s1 : ~s1) & ((v & 4) ? s2 : ~s2) & cells;
  }
  // numpy indexing of room_state[row, col]: negative indices wrap once, else IndexError
  __device__ __forceinline__ bool cell(int row, int col, int& idx) const {
    if (row < -H || row >= H || col < -W || col >= W) return false;
    idx = (row < 0 ? row + H : row) * W + (col < 0 ? col + W : col);
    return true;
  }
  // gym_sokoban _calc_reward + _check_if_done (App. A.1)
  __device__ __forceinline__ void finish_step(double& reward, bool& done, bool& success) {
    const uint64_t open_targets = s_eq(2) | ((f1 & ~f0 & cells) & s_eq(5));  // fixed==2 & state==5
    const int n_open = __popcll(open_targets);
    const int cur = num_boxes - n_open;
    double rw = -0.1;  // penalty_for_step
    if (cur > boxes_on_target) rw += 1.0;       // reward_box_on_target
    else if (cur < boxes_on_target) rw += -1.0;  // penalty_box_off_target
    const bool all_on = (n_open == 0);
    if (all_on) rw += 10.0;  // reward_finished
    boxes_on_target = cur;
    reward = rw;
    done = all_on || (max_steps == num_env_steps);
    success = (boxes_on_target == num_boxes);  // sokoban/env.py:49
  }
  __device__ __forceinline__ bool move_player(int dr, int dc, bool& moved) {  // _move
    moved = false;
    int ni, oi;
    if (!cell(r + dr, c + dc, ni) || !cell(r, c, oi)) { err |= RMI_ERR_INDEX; return false; }
    const int v = sval(ni);
    if (v == 1 || v == 2) {
      r += dr;
      c += dc;
      sset(ni, 5);
      sset(oi, fval(oi));
      moved = true;
    }
    return true;
  }
  // action 1..4 push (falls back to move), 5..8 move; (gym_sokoban ACTION_LOOKUP)
  __device__ __forceinline__ bool step(int a, double& reward, bool& done, bool& eff, bool& success) {
    if (a < 1 || a > 8) return false;
    const int d = (a - 1) & 3;
    const int dr = d == 0 ? -1 : (d == 1 ? 1 : 0);
    const int dc = d == 2 ? -1 : (d == 3 ? 1 : 0);
    const int pr = r, pc = c;
    num_env_steps += 1;
    bool moved = false;
    if (a <= 4) {
      const int nr = r + dr, nc = c + dc, br = nr + dr, bc = nc + dc;
      if (!(br >= H || bc >= W)) {  // upstream only bounds-checks the high side
        int ni, bi, oi;
        if (!cell(nr, nc, ni) || !cell(br, bc, bi) || !cell(r, c, oi)) {
          err |= RMI_ERR_INDEX;
          return false;
        }
        const int vn = sval(ni), vb = sval(bi);
        if ((vn == 3 || vn == 4) && (vb == 1 || vb == 2)) {
          r = nr;
          c = nc;
          sset(ni, 5);
          sset(oi, fval(oi));
          sset(bi, fval(bi) == 2 ? 3 : 4);
          moved = true;
        } else if (!move_player(dr, dc, moved)) {
          return false;
        }
      }
    } else if (!move_player(dr, dc, moved)) {
      return false;
    }
    finish_step(reward, done, success);
    eff = !(pr == r && pc == c);  // sokoban/env.py:48
    return true;
  }
};

template <int HW>  // HW = H*W (compile-time for the common sizes, 0 = runtime)
__global__ __launch_bounds__(kBlock) void sokoban_step_turn_kernel(
    rmi_sokoban_t env, rmi_episode_t ep, rmi_turn_t in, int hw_rt, uint8_t* __restrict__ err_out) {
  constexpr int kRowWordsMax = 16;  // 64 cells
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
  if ((hw & 3) == 0) {
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
    SokobanEnvDev e;
    e.H = env.H;
    e.W = env.W;
    e.err = 0;
    e.cells = hw == 64 ? ~0ull : ((1ull << hw) - 1ull);
    e.s0 = e.s1 = e.s2 = e.f0 = e.f1 = 0;
    const uint32_t* ms = lds_state + tid * row_words;
    const uint32_t* mf = lds_fixed + tid * row_words;
#pragma unroll
    for (int w = 0; w < kRowWordsMax; ++w) {
      if (w < row_words) {
        const uint32_t xs = ms[w], xf = mf[w];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int cidx = 4 * w + j;
          if (cidx < hw) {
            const uint32_t vs = (xs >> (8 * j)) & 0xffu, vf = (xf >> (8 * j)) & 0xffu;
            if (vs > 7u || vf > 3u) e.err |= RMI_ERR_STATE;
            e.s0 |= (uint64_t)(vs & 1u) << cidx;
            e.s1 |= (uint64_t)((vs >> 1) & 1u) << cidx;
            e.s2 |= (uint64_t)((vs >> 2) & 1u) << cidx;
            e.f0 |= (uint64_t)(vf & 1u) << cidx;
            e.f1 |= (uint64_t)((vf >> 1) & 1u) << cidx;
          }
        }
      }
    }
    e.r = env.player[2 * b];
    e.c = env.player[2 * b + 1];
    e.num_env_steps = env.num_env_steps[b];
    e.boxes_on_target = env.boxes_on_target[b];
    e.num_boxes = env.num_boxes;
    e.max_steps = env.max_steps;

    int32_t num_actions = ep.num_actions[b];
    int32_t n_turns = ep.n_turns[b];
    double penalty = ep.penalty[b];
    const int8_t* acts = in.actions + b * (int64_t)in.K;
    const int n_act = in.n_actions[b];
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
      uint32_t* wsd = lds_state + tid * row_words;
#pragma unroll
      for (int w = 0; w < kRowWordsMax; ++w) {
        if (w < row_words) {
          uint32_t x = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int cidx = 4 * w + j;
            if (cidx < hw) x |= (uint32_t)e.sval(cidx) << (8 * j);
            else x |= ms[w] & (0xffu << (8 * j));
          }
          wsd[w] = x;
        }
      }
    }
    if (err_out) err_out[b] |= err;
  }
  if (!__syncthreads_or(changed)) return;
  if ((hw & 3) == 0) {
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

}  // namespace
}  // namespace rmi

RMI_API int rmi_sokoban_step_turn(const rmi_sokoban_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                  uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (!env || !ep || !in) return RMI_EINVAL;
  const int hw = env->H * env->W;
  if (env->H <= 0 || env->W <= 0 || hw > 64) return RMI_EUNSUP;
  if (in->K < 0 || in->K > kMaxK || in->turn < 0 || in->turn >= ep->T) return RMI_EINVAL;
  if (ep->B < 0) return RMI_EINVAL;
  if (ep->B == 0) return RMI_OK;
  if (!env->room_fixed || !env->room_state || !env->player || !env->num_env_steps || !env->boxes_on_target ||
      !ep->num_actions || !ep->flags || !ep->n_turns || !ep->penalty || !ep->turn_reward || !ep->turn_info ||
      !ep->turn_exec || (in->K > 0 && !in->actions) || !in->n_actions)
    return RMI_EINVAL;
  const unsigned grid = (unsigned)((ep->B + kBlock - 1) / kBlock);
  hipStream_t s = as_stream(stream);
  if (hw == 36)
    hipLaunchKernelGGL(sokoban_step_turn_kernel<36>, dim3(grid), dim3(kBlock), 0, s, *env, *ep, *in, hw, err);
  else if (hw == 64)
    hipLaunchKernelGGL(sokoban_step_turn_kernel<64>, dim3(grid), dim3(kBlock), 0, s, *env, *ep, *in, hw, err);
  else
    hipLaunchKernelGGL(sokoban_step_turn_kernel<0>, dim3(grid), dim3(kBlock), 0, s, *env, *ep, *in, hw, err);
  return launch_status();
}
