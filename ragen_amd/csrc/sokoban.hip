// sokoban.hip — one whole EnvStateManager turn for a batch of Sokoban envs (gfx950).
//
// Replaces es_manager.py:105-171 driving sokoban/env.py:44-51 -> gym_sokoban step
// (SURVEY.md App. A.1).  One lane owns one env; a 64-lane workgroup (one wave) owns 64 envs.
//
// HBM layout (caller-owned SoA, include/ragen_amd.h): room grids are [B, H*W] u8 rows.
// The kernel is latency-bound (8192 envs = 128 waves < 256 CUs), so it is organised to
// minimise the length of each lane's serial chain:
//   1. every global load of the turn is issued up front: the wave's 64 rows of room_state
//      and room_fixed as coalesced dwords (16 B / lane where aligned) staged through LDS,
//      and the per-env scalars / actions (one round trip);
//   2. each lane turns its row into 64-bit bit-planes with SWAR multiplies (3 planes for
//      room_state values 0..7, 2 for room_fixed) — read back from LDS with a row stride of
//      H*W/4 dwords (9 for 6x6: coprime with the 32 banks, conflict-free);
//   3. each action is a branch-free predicated update of at most three cells (player,
//      previous player cell, box), byte-exact with upstream's numpy writes, with the
//      open-target count of _calc_reward maintained incrementally (no grid scan);
//   4. rows go back through LDS with coalesced stores, only if some env of the wave moved.
#include "common.hpp"

namespace rmi {
namespace {

constexpr int kWave = 64;
constexpr int kRowWordsMax = 16;  // 64 cells

// 4 bytes -> 4 bits: bit p of byte j lands at bit j (the 4 partial products never overlap)
__device__ __forceinline__ uint32_t gather_bit(uint32_t x, int p) {
  return ((((x >> p) & 0x01010101u) * 0x01020408u) >> 24) & 0xFu;
}
// 4 bits -> 4 bytes: bit j of n -> bit 0 of byte j
__device__ __forceinline__ uint32_t spread_bits(uint32_t n) { return (n * 0x00204081u) & 0x01010101u; }

__device__ __forceinline__ uint32_t bit_at(uint64_t x, int i) { return (uint32_t)(x >> i) & 1u; }

struct SokobanEnvDev {
  uint64_t s0, s1, s2, f0, f1, tgt;  // state planes, fixed planes, fixed == 2
  int H, W, r, c;
  int num_env_steps, boxes_on_target, num_boxes, max_steps, n_open;
  uint8_t err;

  __device__ __forceinline__ int sval(int i) const {
    return (int)(bit_at(s0, i) | (bit_at(s1, i) << 1) | (bit_at(s2, i) << 2));
  }
  __device__ __forceinline__ int fval(int i) const { return (int)(bit_at(f0, i) | (bit_at(f1, i) << 1)); }
  // contribution of a cell to _calc_reward's open-target count:
  // (room_state == 2) | ((room_fixed == 2) & (room_state == 5))
  __device__ __forceinline__ int open_of(int i, int v) const { return (v == 2) | ((v == 5) & (int)bit_at(tgt, i)); }
  // numpy indexing room_state[row, col]: a negative index wraps once; otherwise IndexError
  __device__ __forceinline__ int wrap(int row, int col, bool& ok) const {
    ok = row >= -H && row < H && col >= -W && col < W;
    const int rr = row < 0 ? row + H : row, cc = col < 0 ? col + W : col;
    return ok ? rr * W + cc : 0;
  }

  // One env.step(a): a = 1..4 push (falls back to move), 5..8 move (gym_sokoban ACTION_LOOKUP).
  __device__ __forceinline__ bool step(int a, double& reward, bool& done, bool& eff, bool& success) {
    if (a < 1 || a > 8) return false;
    const int d = (a - 1) & 3;  // CHANGE_COORDINATES[(a-1) % 4]
    const int dr = d == 0 ? -1 : (d == 1 ? 1 : 0);
    const int dc = d == 2 ? -1 : (d == 3 ? 1 : 0);
    const int nr = r + dr, nc = c + dc, br = nr + dr, bc = nc + dc;
    bool ok_n, ok_b, ok_o;
    const int ni = wrap(nr, nc, ok_n), bi = wrap(br, bc, ok_b), oi = wrap(r, c, ok_o);
    const bool push_act = a <= 4;
    const bool high = br >= H || bc >= W;  // _push only bounds-checks the high side
    const int vn = sval(ni), vb = sval(bi), vo = sval(oi), fo = fval(oi);
    const bool is_push = push_act && !high && (vn == 3 || vn == 4) && (vb == 1 || vb == 2);
    const bool try_move = !push_act || (!high && !is_push);  // _push falls back to _move
    const bool moved_only = try_move && (vn == 1 || vn == 2);
    const bool bad = (push_act && !high && (!ok_n || !ok_b)) || (try_move && !ok_n) || !ok_o;
    if (bad) {  // the reference raises IndexError; flag it and leave the env untouched
      err |= RMI_ERR_INDEX;
      return false;
    }
    num_env_steps += 1;
    const bool moved = is_push || moved_only;
    const int vbn = bit_at(tgt, bi) ? 3 : 4;  // box_type
    // incremental open-target count over the (at most three) written cells
    n_open += moved ? (open_of(ni, 5) - open_of(ni, vn) + open_of(oi, fo) - open_of(oi, vo)) : 0;
    n_open += is_push ? (open_of(bi, vbn) - open_of(bi, vb)) : 0;
    const uint64_t mn = moved ? (1ull << ni) : 0ull, mo = moved ? (1ull << oi) : 0ull,
                   mb = is_push ? (1ull << bi) : 0ull;
    const uint64_t clr = ~(mn | mo | mb);
    // new values: player cell 5 (0b101), old player cell fixed (fo), box cell 3 / 4
    s0 = (s0 & clr) | mn | ((fo & 1) ? mo : 0ull) | ((vbn & 1) ? mb : 0ull);
    s1 = (s1 & clr) | ((fo & 2) ? mo : 0ull) | ((vbn & 2) ? mb : 0ull);
    s2 = (s2 & clr) | mn | ((vbn & 4) ? mb : 0ull);
    r = moved ? nr : r;
    c = moved ? nc : c;
    // _calc_reward + _check_if_done
    const int cur = num_boxes - n_open;
    double rw = -0.1;                                                  // penalty_for_step
    rw += cur > boxes_on_target ? 1.0 : (cur < boxes_on_target ? -1.0 : 0.0);  // on / off target
    const bool all_on = n_open == 0;
    rw += all_on ? 10.0 : 0.0;                                         // reward_finished
    boxes_on_target = cur;
    reward = rw;
    done = all_on || (max_steps == num_env_steps);
    success = boxes_on_target == num_boxes;  // sokoban/env.py:49
    eff = moved;                             // position changed (sokoban/env.py:48)
    return true;
  }
};

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
      if (((xs | xf) & 0xF8F8F8F8u) | (xf & 0x04040404u)) e.err |= RMI_ERR_STATE;  // state > 7, fixed > 3
      e.s0 |= (uint64_t)gather_bit(xs, 0) << (4 * w);
      e.s1 |= (uint64_t)gather_bit(xs, 1) << (4 * w);
      e.s2 |= (uint64_t)gather_bit(xs, 2) << (4 * w);
      e.f0 |= (uint64_t)gather_bit(xf, 0) << (4 * w);
      e.f1 |= (uint64_t)gather_bit(xf, 1) << (4 * w);
    }
  }
  e.tgt = e.f1 & ~e.f0;  // fixed == 2
  const uint64_t eq2 = ~e.s0 & e.s1 & ~e.s2, eq5 = e.s0 & ~e.s1 & e.s2;
  e.n_open = __popcll(eq2 | (e.tgt & eq5));
}

// Stage `nwords` dwords of a wave's rows global -> LDS (16 B per lane when aligned).
__device__ __forceinline__ void stage_in(uint32_t* lds, const uint8_t* g, int nwords, int lane, bool vec) {
  if (vec) {
    const uint4* g4 = reinterpret_cast<const uint4*>(g);
    uint4* l4 = reinterpret_cast<uint4*>(lds);
    const int n4 = nwords >> 2;
    for (int i = lane; i < n4; i += kWave) l4[i] = g4[i];
    for (int i = (n4 << 2) + lane; i < nwords; i += kWave) lds[i] = reinterpret_cast<const uint32_t*>(g)[i];
  } else {
    const uint32_t* g1 = reinterpret_cast<const uint32_t*>(g);
    for (int i = lane; i < nwords; i += kWave) lds[i] = g1[i];
  }
}

template <int HW>  // HW = H*W for the common sizes (0 = runtime); word path only (hw % 4 == 0)
__global__ __launch_bounds__(kWave) void sokoban_step_turn_kernel(rmi_sokoban_t env, rmi_episode_t ep, rmi_turn_t in,
                                                                  int hw_rt, uint8_t* __restrict__ err_out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_state[kWave * kRowWordsMax];
  __shared__ __attribute__((aligned(16))) uint32_t lds_fixed[kWave * kRowWordsMax];
  const int hw = HW ? HW : hw_rt;
  const int row_words = hw >> 2;
  const int B = ep.B;
  const int lane = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * kWave;
  const int64_t b = b0 + lane;
  const int nb = (int)min<int64_t>(kWave, B - b0);
  const bool live = b < B;

  // ---- 1. every load of the turn, issued together
  const uint8_t flags0 = live ? ep.flags[b] : (uint8_t)RMI_FLAG_DONE;
  const bool act = live && (in.has_input ? (in.has_input[b] != 0) : !(flags0 & RMI_FLAG_DONE));
  int8_t pr = 0, pc = 0;
  int32_t nes = 0, bot = 0, num_actions = 0, n_turns = 0, n_act = 0;
  double penalty = 0.0;
  uint64_t acts = 0;
  if (live) {
    pr = env.player[2 * b];
    pc = env.player[2 * b + 1];
    nes = env.num_env_steps[b];
    bot = env.boxes_on_target[b];
    num_actions = ep.num_actions[b];
    n_turns = ep.n_turns[b];
    penalty = ep.penalty[b];
    n_act = in.n_actions[b];
    acts = load_actions(in.actions + b * (int64_t)in.K, in.K);
  }
  const int nwords = nb * row_words;
  const bool vec = ((reinterpret_cast<uintptr_t>(env.room_state + b0 * hw) |
                     reinterpret_cast<uintptr_t>(env.room_fixed + b0 * hw)) & 15u) == 0;
  stage_in(lds_state, env.room_state + b0 * hw, nwords, lane, vec);
  stage_in(lds_fixed, env.room_fixed + b0 * hw, nwords, lane, vec);
  __syncthreads();

  // ---- 2-3. the turn
  bool changed = false;
  uint32_t* ms = lds_state + lane * row_words;
  SokobanEnvDev e;
  if (act) {
    e.H = env.H;
    e.W = env.W;
    e.err = 0;
    to_planes(ms, lds_fixed + lane * row_words, hw, e);
    e.r = pr;
    e.c = pc;
    e.num_env_steps = nes;
    e.boxes_on_target = bot;
    e.num_boxes = env.num_boxes;
    e.max_steps = env.max_steps;

    uint8_t err = 0, flags = flags0;
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
          ms[w] = spread_bits((uint32_t)(e.s0 >> sh) & 0xFu) | (spread_bits((uint32_t)(e.s1 >> sh) & 0xFu) << 1) |
                  (spread_bits((uint32_t)(e.s2 >> sh) & 0xFu) << 2);
        }
      }
    }
    if (err_out && err) err_out[b] |= err;
  }
  // ---- 4. rows back (only if some env of the wave changed)
  if (!__syncthreads_or(changed)) return;
  if (vec) {
    uint4* g4 = reinterpret_cast<uint4*>(env.room_state + b0 * hw);
    const uint4* l4 = reinterpret_cast<const uint4*>(lds_state);
    const int n4 = nwords >> 2;
    for (int i = lane; i < n4; i += kWave) g4[i] = l4[i];
    for (int i = (n4 << 2) + lane; i < nwords; i += kWave)
      reinterpret_cast<uint32_t*>(env.room_state + b0 * hw)[i] = lds_state[i];
  } else {
    uint32_t* g1 = reinterpret_cast<uint32_t*>(env.room_state + b0 * hw);
    for (int i = lane; i < nwords; i += kWave) g1[i] = lds_state[i];
  }
}

// Fused reset: room_state/player from the generated rooms, counters and the whole episode
// record zeroed, in one launch (SokobanEnv.reset sokoban/env.py:37-38 + EnvStatus()).
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
  // rows are staged as dwords: H*W must be a multiple of 4 and the grids 4-byte aligned
  if (hw % 4 != 0 ||
      ((reinterpret_cast<uintptr_t>(env->room_state) | reinterpret_cast<uintptr_t>(env->room_fixed)) & 3u))
    return RMI_EUNSUP;
  const unsigned grid = (unsigned)((ep->B + kWave - 1) / kWave);
  hipStream_t s = as_stream(stream);
  if (hw == 36)
    hipLaunchKernelGGL(sokoban_step_turn_kernel<36>, dim3(grid), dim3(kWave), 0, s, *env, *ep, *in, hw, err);
  else if (hw == 64)
    hipLaunchKernelGGL(sokoban_step_turn_kernel<64>, dim3(grid), dim3(kWave), 0, s, *env, *ep, *in, hw, err);
  else
    hipLaunchKernelGGL(sokoban_step_turn_kernel<0>, dim3(grid), dim3(kWave), 0, s, *env, *ep, *in, hw, err);
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
  if (hw % 4 != 0 || ((reinterpret_cast<uintptr_t>(env->room_state) | reinterpret_cast<uintptr_t>(init_state)) & 3u))
    return RMI_EUNSUP;
  const int64_t nw = (int64_t)ep->B * hw / 4;
  const int64_t n = nw > ep->B ? nw : ep->B;
  hipLaunchKernelGGL(sokoban_reset_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     as_stream(stream), *env, *ep, hw, init_state, init_player);
  return launch_status();
}
