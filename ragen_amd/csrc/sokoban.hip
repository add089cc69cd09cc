// sokoban.hip — one whole EnvStateManager turn for a batch of Sokoban envs (gfx950).
//
// Replaces es_manager.py:105-171 driving sokoban/env.py:44-51 -> gym_sokoban step
// (SURVEY.md App. A.1).  One lane owns one env; a 64-lane workgroup (one wave) owns 64 envs.
//
// HBM layout (caller-owned SoA, include/ragen_amd.h): room grids are [B, H*W] u8 rows.
// The kernel is latency-bound (8192 envs = 128 waves < 256 CUs), so it minimises each
// lane's serial chain:
//   1. every global load of the turn is issued up front: the wave's 64 rows of room_state
//      and room_fixed as coalesced 16-B loads staged into LDS, and the per-env scalars and
//      actions — one memory round trip;
//   2. the grids stay in LDS; a lane's row starts at lane*H*W bytes (stride 9 dwords for
//      6x6: coprime with the 32 banks).  An action reads its <= 6 cells as independent
//      ds_read_u8 (one LDS round trip), decides push / move / blocked branch-free and
//      writes <= 3 cells — byte-exact with upstream's numpy writes;
//   3. _calc_reward's open-target count is computed once per turn with SWAR byte compares
//      on the row's dwords and then maintained incrementally from the written cells;
//   4. updated rows go back with coalesced 16-B stores, only if some env of the wave moved.
#include "common.hpp"

namespace rmi {
namespace {

constexpr int kWave = 64;
constexpr int kMaxCells = 64;

// exact per-byte "== 0" test: high bit of each byte set iff the byte is zero
__device__ __forceinline__ uint32_t zero_bytes(uint32_t y) {
  return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
}
__device__ __forceinline__ uint32_t eq_bytes(uint32_t x, uint32_t v) { return zero_bytes(x ^ (v * 0x01010101u)); }

struct SokobanLdsEnv {
  uint8_t* st;        // this env's room_state row (LDS)
  const uint8_t* fx;  // this env's room_fixed row (LDS)
  int H, W, r, c;
  int num_env_steps, boxes_on_target, num_boxes, max_steps, n_open;
  uint8_t err;

  // numpy indexing room_state[row, col]: a negative index wraps once; otherwise IndexError
  __device__ __forceinline__ int wrap(int row, int col, bool& ok) const {
    ok = row >= -H && row < H && col >= -W && col < W;
    const int rr = row < 0 ? row + H : row, cc = col < 0 ? col + W : col;
    return ok ? rr * W + cc : 0;
  }
  // contribution of a cell to the open-target count: (state == 2) | ((fixed == 2) & (state == 5))
  __device__ __forceinline__ static int open_of(int v, int f) { return (v == 2) | ((v == 5) & (f == 2)); }

  // One env.step(a): a = 1..4 push (falls back to move), 5..8 move (gym_sokoban ACTION_LOOKUP).
  __device__ __forceinline__ bool step(int a, double& reward, bool& done, bool& eff, bool& success) {
    if (a < 1 || a > 8) return false;
    const int d = (a - 1) & 3;  // CHANGE_COORDINATES[(a-1) % 4]
    const int dr = d == 0 ? -1 : (d == 1 ? 1 : 0);
    const int dc = d == 2 ? -1 : (d == 3 ? 1 : 0);
    const int nr = r + dr, nc = c + dc, br = nr + dr, bc = nc + dc;
    bool ok_n, ok_b, ok_o;
    const int ni = wrap(nr, nc, ok_n), bi = wrap(br, bc, ok_b), oi = wrap(r, c, ok_o);
    // independent LDS reads, one round trip
    const int vn = st[ni], vb = st[bi], vo = st[oi];
    const int fn = fx[ni], fb = fx[bi], fo = fx[oi];
    const bool push_act = a <= 4;
    const bool high = br >= H || bc >= W;  // _push only bounds-checks the high side
    const bool is_push = push_act && !high && (vn == 3 || vn == 4) && (vb == 1 || vb == 2);
    const bool try_move = !push_act || (!high && !is_push);  // _push falls back to _move
    const bool moved = is_push || (try_move && (vn == 1 || vn == 2));
    if ((push_act && !high && (!ok_n || !ok_b)) || (try_move && !ok_n) || !ok_o) {
      err |= RMI_ERR_INDEX;  // the reference raises IndexError; flag it, leave the env untouched
      return false;
    }
    num_env_steps += 1;
    const int vbn = fb == 2 ? 3 : 4;  // box_type
    if (moved) {
      n_open += open_of(5, fn) - open_of(vn, fn) + open_of(fo, fo) - open_of(vo, fo);
      st[ni] = 5;
      st[oi] = (uint8_t)fo;
      r = nr;
      c = nc;
    }
    if (is_push) {
      n_open += open_of(vbn, fb) - open_of(vb, fb);
      st[bi] = (uint8_t)vbn;
    }
    // _calc_reward + _check_if_done
    const int cur = num_boxes - n_open;
    double rw = -0.1;                                                           // penalty_for_step
    rw += cur > boxes_on_target ? 1.0 : (cur < boxes_on_target ? -1.0 : 0.0);  // box on / off target
    const bool all_on = n_open == 0;
    rw += all_on ? 10.0 : 0.0;  // reward_finished
    boxes_on_target = cur;
    reward = rw;
    done = all_on || (max_steps == num_env_steps);
    success = boxes_on_target == num_boxes;  // sokoban/env.py:49
    eff = moved;                             // player position changed (sokoban/env.py:48)
    return true;
  }
};

// One EnvStateManager turn for one Sokoban env (es_manager.py:149-169), specialised for the
// latency of a lone wave: the executed-action list valid[:left] is built up front with
// predicated byte ops, then each step is straight-line code — the index arithmetic of an
// interior player (every generated room: the border is wall) and six independent LDS reads;
// the rare player that can reach the border (hand-made rooms) takes the exact numpy-wrap path
// of SokobanLdsEnv::step.  Same results as run_turn + step, bit for bit.
__device__ __forceinline__ TurnOut sokoban_turn(SokobanLdsEnv& e, uint64_t acts, int n_act, int K, int32_t& num_actions,
                                                uint8_t& flags, int32_t& n_turns, double& penalty, int max_actions,
                                                double format_penalty, uint8_t& err) {
  TurnOut o;
  o.acc = 0.0;
  o.info = 0;
  o.exec = 0;
  o.stepped_any_state = false;
  flags &= (uint8_t)~RMI_FLAG_DONE;
  if (n_act > K) n_act = K;
  const int left = max_actions - num_actions;
  // valid = [ids of known names]; exec list = valid[:left]  (es_manager.py:156-157)
  uint64_t run = 0;
  int nv = 0, cnt = 0;
#pragma unroll
  for (int k = 0; k < kMaxK; ++k) {
    const uint32_t a = (uint32_t)(acts >> (8 * k)) & 0xFFu;
    const bool valid = k < n_act && a != 0;
    const bool take = valid && cnt < left;
    run |= take ? ((uint64_t)a << (8 * cnt)) : 0ull;
    cnt += take;
    nv += valid;
  }
  if (nv != n_act || nv == 0) penalty += format_penalty;  // :158-159
  const int W = e.W, H = e.H;
  int p = e.r * W + e.c;  // player cell (fast path: interior player)
  bool stop = false, turn_done = false, succ_last = false;
  for (int i = 0; i < kMaxK; ++i) {
    const bool go = i < cnt && !stop;
    if (!__any(go)) break;  // wave-uniform trip count
    if (!go) continue;
    const int a = (int)(int8_t)(uint8_t)(run >> (8 * i));
    const int d = (a - 1) & 3;
    const int dr = (d == 1) - (d == 0), dc = (d == 3) - (d == 2);
    const int nr = e.r + dr, nc = e.c + dc, br = nr + dr, bc = nc + dc;
    const bool in_n = (unsigned)nr < (unsigned)H && (unsigned)nc < (unsigned)W;
    const bool in_b = (unsigned)br < (unsigned)H && (unsigned)bc < (unsigned)W;
    const bool high = br >= H || bc >= W;
    const bool fast = a >= 1 && a <= 8 && in_n && (in_b || high) && (unsigned)e.r < (unsigned)H &&
                      (unsigned)e.c < (unsigned)W;
    double r;
    bool done, eff, succ;
    if (fast) {
      const int delta = dr * W + dc;
      const int ni = p + delta, bi = in_b ? ni + delta : p;
      const int vn = e.st[ni], vb = e.st[bi], vo = e.st[p];
      const int fn = e.fx[ni], fb = e.fx[bi], fo = e.fx[p];
      const bool push_act = a <= 4;
      const bool is_push = push_act && !high && (vn == 3 || vn == 4) && (vb == 1 || vb == 2);
      const bool try_move = !push_act || (!high && !is_push);  // _push falls back to _move
      const bool moved = is_push || (try_move && (vn == 1 || vn == 2));
      const int vbn = fb == 2 ? 3 : 4;  // box_type
      e.num_env_steps += 1;
      if (moved) {
        e.n_open += SokobanLdsEnv::open_of(5, fn) - SokobanLdsEnv::open_of(vn, fn) + (fo == 2) -
                    SokobanLdsEnv::open_of(vo, fo);
        e.st[ni] = 5;
        e.st[p] = (uint8_t)fo;
        e.r = nr;
        e.c = nc;
        p = ni;
      }
      if (is_push) {
        e.n_open += SokobanLdsEnv::open_of(vbn, fb) - SokobanLdsEnv::open_of(vb, fb);
        e.st[bi] = (uint8_t)vbn;
      }
      const int cur = e.num_boxes - e.n_open;
      double rw = -0.1;
      rw += cur > e.boxes_on_target ? 1.0 : (cur < e.boxes_on_target ? -1.0 : 0.0);
      const bool all_on = e.n_open == 0;
      rw += all_on ? 10.0 : 0.0;
      e.boxes_on_target = cur;
      r = rw;
      done = all_on || (e.max_steps == e.num_env_steps);
      succ = cur == e.num_boxes;
      eff = moved;
    } else if (!e.step(a, r, done, eff, succ)) {  // exact numpy-wrap / error path
      err |= (a < 1 || a > 8) ? RMI_ERR_ACTION : 0;
      stop = true;
      continue;
    } else {
      p = e.r * W + e.c;
    }
    o.acc += r;
    o.exec++;
    o.stepped_any_state = true;
    o.info = (uint8_t)(RMI_INFO_PRESENT | (eff ? RMI_INFO_EFFECTIVE : 0) | RMI_INFO_VALID | (succ ? RMI_INFO_SUCCESS : 0));
    succ_last = succ;
    if (done) {
      stop = true;
      turn_done = true;
    }
  }
  num_actions += o.exec;
  n_turns += 1;
  if (turn_done) {
    flags |= RMI_FLAG_TERMINATED | RMI_FLAG_DONE;
    flags = succ_last ? (uint8_t)(flags & ~RMI_FLAG_TRUNCATED) : (uint8_t)(flags | RMI_FLAG_TRUNCATED);
  } else if (num_actions >= max_actions) {
    flags |= RMI_FLAG_TERMINATED | RMI_FLAG_TRUNCATED | RMI_FLAG_DONE;
  }
  return o;
}

// Stage `nwords` dwords global -> LDS (16 B per lane when both are 16-B aligned).
__device__ __forceinline__ void stage_in(uint32_t* lds, const uint8_t* g, int nwords, int lane, bool vec) {
  const uint32_t* g1 = reinterpret_cast<const uint32_t*>(g);
  int done = 0;
  if (vec) {
    const uint4* g4 = reinterpret_cast<const uint4*>(g);
    uint4* l4 = reinterpret_cast<uint4*>(lds);
    const int n4 = nwords >> 2;
#pragma unroll 4
    for (int i = lane; i < n4; i += kWave) l4[i] = g4[i];
    done = n4 << 2;
  }
  for (int i = done + lane; i < nwords; i += kWave) lds[i] = g1[i];
}

__device__ __forceinline__ void stage_out(uint8_t* g, const uint32_t* lds, int nwords, int lane, bool vec) {
  uint32_t* g1 = reinterpret_cast<uint32_t*>(g);
  int done = 0;
  if (vec) {
    uint4* g4 = reinterpret_cast<uint4*>(g);
    const uint4* l4 = reinterpret_cast<const uint4*>(lds);
    const int n4 = nwords >> 2;
#pragma unroll 4
    for (int i = lane; i < n4; i += kWave) g4[i] = l4[i];
    done = n4 << 2;
  }
  for (int i = done + lane; i < nwords; i += kWave) g1[i] = lds[i];
}

template <int HW>  // H*W for the common sizes (0 = runtime); H*W % 4 == 0
__global__ __launch_bounds__(kWave) void sokoban_step_turn_kernel(rmi_sokoban_t env, rmi_episode_t ep, rmi_turn_t in,
                                                                  int hw_rt, uint8_t* __restrict__ err_out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_state[kWave * kMaxCells / 4];
  __shared__ __attribute__((aligned(16))) uint32_t lds_fixed[kWave * kMaxCells / 4];
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
  uint8_t* gstate = env.room_state + b0 * hw;
  const uint8_t* gfixed = env.room_fixed + b0 * hw;
  const bool vec = ((reinterpret_cast<uintptr_t>(gstate) | reinterpret_cast<uintptr_t>(gfixed)) & 15u) == 0;
  stage_in(lds_state, gstate, nwords, lane, vec);
  stage_in(lds_fixed, gfixed, nwords, lane, vec);
  __syncthreads();

  // ---- 2-3. the turn
  bool changed = false;
  if (act) {
    SokobanLdsEnv e;
    e.st = reinterpret_cast<uint8_t*>(lds_state) + lane * hw;
    e.fx = reinterpret_cast<const uint8_t*>(lds_fixed) + lane * hw;
    e.H = env.H;
    e.W = env.W;
    e.err = 0;
    // open targets of _calc_reward, SWAR over the row's dwords
    const uint32_t* ws = lds_state + lane * row_words;
    const uint32_t* wf = lds_fixed + lane * row_words;
    int n_open = 0;
#pragma unroll
    for (int w = 0; w < kMaxCells / 4; ++w) {
      if (w < row_words) {
        const uint32_t xs = ws[w], xf = wf[w];
        n_open += __popc(eq_bytes(xs, 2u) | (eq_bytes(xs, 5u) & eq_bytes(xf, 2u)));
      }
    }
    e.n_open = n_open;
    e.r = pr;
    e.c = pc;
    e.num_env_steps = nes;
    e.boxes_on_target = bot;
    e.num_boxes = env.num_boxes;
    e.max_steps = env.max_steps;

    uint8_t err = 0, flags = flags0;
    TurnOut o = sokoban_turn(e, acts, n_act, in.K, num_actions, flags, n_turns, penalty, in.max_actions_per_traj,
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
    }
    if (err_out && err) err_out[b] |= err;
  }
  // ---- 4. rows back (only if some env of the wave changed)
  if (!__syncthreads_or(changed)) return;
  stage_out(gstate, lds_state, nwords, lane, vec);
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
  if (env->H <= 0 || env->W <= 0 || hw > kMaxCells) return RMI_EUNSUP;
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
  if (hw <= 0 || hw > kMaxCells) return RMI_EUNSUP;
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
