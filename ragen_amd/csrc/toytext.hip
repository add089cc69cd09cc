// toytext.hip — FrozenLake and Bandit turns (gfx950), one thread per env.
//
// FrozenLake: replaces es_manager.py:105-171 driving frozen_lake/env.py:39-45 ->
//   gymnasium FrozenLakeEnv.step + categorical_sample (App. A.2) with numpy PCG64
//   draws (App. A.5).  Every step consumes exactly one Generator.random() draw, also on
//   non-slippery maps and from terminal cells, as upstream does.
// Bandit: replaces bandit/env.py:62-76 (one draw only when the hi arm is pulled).
//
// Per-env state is tiny (FrozenLake: desc row <= 64 B + s + 32 B of PCG64 state), so
// the kernels are plain coalesced SoA loads: rng is [4,B] u64 planes, desc is [B,n] u8.
#include "common.hpp"

namespace rmi {
namespace {

// One wave per workgroup for the turn kernels: a turn is a latency-bound chain per env, and
// 4096 envs in 256-thread blocks would occupy only 16 CUs (64 one-wave blocks spread over 64).
constexpr int kToyBlock = 64;
#ifndef RMI_FL_BLOCK
#define RMI_FL_BLOCK 64
#endif
constexpr int kFlBlock = RMI_FL_BLOCK;  // FrozenLake turn: threads per workgroup (envs, one per lane)

struct FrozenLakeDev {
  const uint8_t* desc;  // this env's row
  uint64_t d_lo, d_hi;  // the row itself when it has <= 16 cells (loaded once; no per-step load)
  bool in_regs;
  int nrow, ncol, s;
  bool slippery;
  double cs0, cs1, cs2;
  Pcg64 rng;

  __device__ __forceinline__ int inc(int s0, int a) const {
    int row = s0 / ncol, col = s0 - (s0 / ncol) * ncol;
    if (a == 0) col = col - 1 < 0 ? 0 : col - 1;                       // LEFT
    else if (a == 1) row = row + 1 > nrow - 1 ? nrow - 1 : row + 1;    // DOWN
    else if (a == 2) col = col + 1 > ncol - 1 ? ncol - 1 : col + 1;    // RIGHT
    else row = row - 1 < 0 ? 0 : row - 1;                              // UP
    return row * ncol + col;
  }
  __device__ __forceinline__ uint8_t cell(int i) const {
    if (in_regs) return (uint8_t)((i < 8 ? d_lo >> (8 * i) : d_hi >> (8 * (i - 8))) & 0xFF);
    return desc[i];
  }
  // action ids 1..4 -> gym 0..3 via FrozenLakeEnvConfig.action_map (frozen_lake/config.py:15)
  __device__ __forceinline__ bool step(int a, double& reward, bool& done, bool& eff, bool& success) {
    if (a < 1 || a > 4) return false;
    const int ga = a - 1;
    const int prev = s;
    const double u = rng.next_double();  // categorical_sample draw
    const uint8_t letter = cell(s);
    if (letter == 'G' || letter == 'H') {  // P[s][a] = [(1.0, s, 0, True)]
      reward = 0.0;
      done = true;
    } else {
      int b = ga;
      if (slippery) {  // argmax(cumsum(p) > u) over [(a-1)%4, a, (a+1)%4]
        const int i = (cs0 > u) ? 0 : (cs1 > u) ? 1 : (cs2 > u) ? 2 : 0;
        b = (ga + 3 + i) & 3;
      }
      s = inc(s, b);
      const uint8_t nl = cell(s);
      reward = (nl == 'G') ? 1.0 : 0.0;
      done = (nl == 'G' || nl == 'H');
    }
    eff = prev != s;                   // frozen_lake/env.py:43
    success = cell(s) == 'G';
    return true;
  }
};

// ---- the 4x4 turn, straight-line (the bench's and RAGEN's FrozenLake: size 4)
// The generic turn (run_turn over FrozenLakeDev::step) is a data-dependent loop: a wave pays
// every branch side of every lane, ~300 instructions per step.  For 4x4 maps the whole turn is
// written as K predicated steps on bitboards (hole / goal bits of the 16 cells, s in 0..15):
//  * the exec list (known-name actions in order, es_manager.py:156) is compacted first, so
//    step k always consumes draw k of the turn;
//  * the turn's <= K PCG64 draws are the LCG chain's next K outputs, computed up front in one
//    block (their only dependence is the chain itself, not the steps) — the state after the
//    turn is chain state number `exec`;
//  * categorical_sample's argmax(cumsum(p) > u) with u = (x >> 11) * 2^-53 compares the 53-bit
//    integer against ceil(cs_i * 2^53) (exact: cs_i * 2^53 is an exact double);
//  * each step is a 16-cell transition table (4 bits per cell) built from its draw and action
//    alone, so the turn's dependent chain is one table lookup per step (see fl4_turn).
// Same results bit for bit as the generic turn (FrozenLakeDev::step); taken when every lane
// of the wave has a 4x4 map, a state in range and action ids in 0..4.
struct Fl4Out {
  TurnOut o;
  bool turn_done, succ_last;
  int s;
  int nv;  // known-name actions among the first n_act slots
  Pcg64 rng;
#ifdef RMI_STAMPS
  unsigned long long t_draws;  // diagnostic: s_memtime once the turn's draws are computed
#endif
};

__device__ __forceinline__ uint64_t pcg_out(uint64_t hi, uint64_t lo) {
  const uint64_t x = hi ^ lo;
  const unsigned rot = (unsigned)(hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

template <int K>
__device__ __forceinline__ Fl4Out fl4_turn(uint32_t hole, uint32_t goal, int s, Pcg64 rng, uint64_t acts, int n_act,
                                           int left, bool slippery, uint64_t t0, uint64_t t1, uint64_t t2) {
  Fl4Out r;
  r.o.acc = 0.0;
  r.o.info = 0;
  r.o.exec = 0;
  r.o.stepped_any_state = false;
  r.turn_done = false;
  r.succ_last = false;
  // exec list: the first min(nv, left) known-name ids, in order
  uint64_t cl = 0;
  int nv = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint64_t a = (acts >> (8 * k)) & 0xFF;
    const bool use = k < n_act && a != 0;
    cl |= use ? a << (8 * nv) : 0ull;
    nv += use ? 1 : 0;
  }
  r.nv = nv;
  const int n_try = nv < left ? nv : (left > 0 ? left : 0);
  // the chain's next K states and outputs (draw k of the turn = output of state k + 1)
  uint64_t shi[K + 1], slo[K + 1], draw[K];
  shi[0] = rng.s_hi;
  slo[0] = rng.s_lo;
  {
    Pcg64 c = rng;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      c.next64();
      shi[k + 1] = c.s_hi;
      slo[k + 1] = c.s_lo;
      draw[k] = pcg_out(c.s_hi, c.s_lo) >> 11;
    }
  }
#ifdef RMI_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  r.t_draws = __builtin_amdgcn_s_memtime();
#endif
  // Step k's transition is a map of the 16 cells, fixed once the draw and the action are known:
  // a terminal cell stays, any other moves by direction b_k (a wall keeps it).  Its table
  // (4 bits per cell) is built for every k at once — b_k depends on the draw and the action
  // only, not on the cell — so the dependent chain of the turn is one shift and mask per step:
  // s_{k+1} = table_k[s_k].  The steps' outputs are then read off the chain (the steps run
  // while k < n_try and until the first done, exactly the loop's `go`).
  const uint64_t kMove[4] = {0xedcca98865442100ull, 0xfedcfedcba987654ull,  // LEFT, DOWN
                             0xffedbba977653321ull, 0xba98765432103210ull}; // RIGHT, UP
  const uint32_t term16 = hole | goal;
  uint64_t tm = term16;  // bit j -> nibble j all ones
  tm = (tm | (tm << 24)) & 0x000000FF000000FFull;
  tm = (tm | (tm << 12)) & 0x000F000F000F000Full;
  tm = (tm | (tm << 6)) & 0x0303030303030303ull;
  tm = (tm | (tm << 3)) & 0x1111111111111111ull;
  tm *= 0xFull;
  const uint64_t stay = 0xfedcba9876543210ull & tm;
  uint64_t chain = (uint64_t)s;  // nibble k = the cell before step k
  uint32_t done_m = 0, rw_m = 0, eff_m = 0, g_m = 0;
  int cur = s;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int ga = (int)((cl >> (8 * k)) & 0xFF) - 1;  // gym action 0..3 (a step past the list is never used)
    const uint64_t u = draw[k];
    const int i = (u < t0) ? 0 : (u < t1) ? 1 : (u < t2) ? 2 : 0;
    const int b = (slippery ? ga + 3 + i : ga) & 3;
    const uint64_t table = (kMove[b] & ~tm) | stay;
    const int ns = (int)((table >> (4 * cur)) & 0xFull);
    const uint32_t term = (term16 >> cur) & 1u, g = (goal >> ns) & 1u, h = (hole >> ns) & 1u;
    done_m |= (term | g | h) << k;
    rw_m |= ((term ^ 1u) & g) << k;
    eff_m |= (uint32_t)(ns != cur) << k;
    g_m |= g << k;
    cur = ns;
    chain |= (uint64_t)ns << (4 * (k + 1));
  }
  // executed steps: the first n_try, cut after the first done
  const int first_done = __builtin_ctz(done_m | (1u << K));
  const int ex = n_try < first_done + 1 ? n_try : first_done + 1;
  const uint32_t ran = (1u << ex) - 1u;
  const int last = ex - 1;
  // the reward sum: 0.0 / 1.0 terms added in order from +0.0 are exact, so it is their count
  r.o.acc = (double)__builtin_popcount(rw_m & ran);
  const uint32_t eff = last >= 0 ? (eff_m >> last) & 1u : 0u, gl = last >= 0 ? (g_m >> last) & 1u : 0u;
  r.o.info = ex ? (uint8_t)(RMI_INFO_PRESENT | RMI_INFO_VALID | (eff << 1) | (gl << 3)) : (uint8_t)0;
  r.succ_last = ex && gl;
  r.turn_done = ex && ((done_m >> last) & 1u);
  r.o.exec = (uint8_t)ex;
  r.o.stepped_any_state = ex > 0;
  r.s = (int)((chain >> (4 * ex)) & 0xFull);
  r.rng = rng;
#pragma unroll
  for (int k = 1; k <= K; ++k)
    if (k == ex) {
      r.rng.s_hi = shi[k];
      r.rng.s_lo = slo[k];
    }
  return r;
}

// bit i = (cell i == letter) for a 16-cell map held as two u64 (cell i in byte i): SWAR byte
// compare, then each dword's 4 byte flags gathered by one multiply (bit 8j -> bit 24 + j).
__device__ __forceinline__ uint32_t cell_bits(uint64_t lo, uint64_t hi, uint32_t letter) {
  const uint32_t pat = letter * 0x01010101u;
  const uint32_t w[4] = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
  uint32_t bits = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t x = w[j] ^ pat;                                              // zero byte = match
    const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;  // high bit of a zero byte
    bits |= (((z >> 7) * 0x01020408u) >> 24) << (4 * j);
  }
  return bits;
}

// ceil(cs * 2^53): u = (x >> 11) * 2^-53 satisfies cs > u  <=>  (x >> 11) < ceil(cs * 2^53)
__device__ __forceinline__ uint64_t draw_threshold(double cs) {
  return (uint64_t)ceil(cs * 9007199254740992.0);
}

__device__ __forceinline__ Fl4Out fl4_dispatch(int K, uint32_t hole, uint32_t goal, int s, const Pcg64& rng,
                                              uint64_t acts, int n_act, int left, bool slip, uint64_t t0,
                                              uint64_t t1, uint64_t t2) {
  switch (K) {  // wave-uniform
    case 1: return fl4_turn<1>(hole, goal, s, rng, acts, n_act, left, slip, t0, t1, t2);
    case 2: return fl4_turn<2>(hole, goal, s, rng, acts, n_act, left, slip, t0, t1, t2);
    case 3: return fl4_turn<3>(hole, goal, s, rng, acts, n_act, left, slip, t0, t1, t2);
    case 4: return fl4_turn<4>(hole, goal, s, rng, acts, n_act, left, slip, t0, t1, t2);
    case 5: return fl4_turn<5>(hole, goal, s, rng, acts, n_act, left, slip, t0, t1, t2);
    case 6: return fl4_turn<6>(hole, goal, s, rng, acts, n_act, left, slip, t0, t1, t2);
    case 7: return fl4_turn<7>(hole, goal, s, rng, acts, n_act, left, slip, t0, t1, t2);
    default: return fl4_turn<8>(hole, goal, s, rng, acts, n_act, left, slip, t0, t1, t2);
  }
}

// kFirst: a fresh episode's first turn fused with its reset (rmi_frozenlake_reset): desc, s and
// the PCG64 state come from the init arrays, the counters and the record start at zero without
// being read, and the env's reset state and whole record are written before the turn runs.
// kFin: the launch is the rollout's last turn and also runs rmi_rollout_finalize for uniform
// contiguous groups of fin.group_size envs (each group inside the launch's one wave): every
// lane, live or not, reaches the group shuffles of finalize_envs.
template <bool kFirst, bool kFin>
__global__ __launch_bounds__(kFlBlock) void frozenlake_step_turn_kernel(rmi_frozenlake_t env, rmi_episode_t ep,
                                                                         rmi_turn_t in, uint8_t* __restrict__ err_out,
                                                                         const uint8_t* __restrict__ init_desc,
                                                                         const int32_t* __restrict__ init_s,
                                                                         const uint64_t* __restrict__ init_rng,
                                                                         rmi_finalize_t fin) {
  const int64_t b = (int64_t)blockIdx.x * kFlBlock + threadIdx.x;
  const int B = ep.B;
  if (!kFin && b >= B) return;
  const bool live = b < B;
  const int64_t bc = live ? b : (int64_t)B - 1;  // clamped: every load below is valid
  RMI_STAMP_DECL;
  RMI_STAMP(0);
  // every load of the turn is issued before the first use (one memory round trip); the env
  // state first (its pointers and the record's come from different kernel-argument fetches)
  const int n = env.nrow * env.ncol;
  FrozenLakeDev e;
  e.desc = (kFirst ? init_desc : env.desc) + bc * n;
  e.in_regs = n <= 16;
  e.d_lo = e.d_hi = 0;
  e.s = kFirst ? init_s[bc] : env.s[bc];
  e.rng = load_pcg(kFirst ? init_rng : env.rng, B, bc);
  if (n == 16 && (reinterpret_cast<uintptr_t>(kFirst ? init_desc : env.desc) & 15u) == 0) {  // 4x4: one 16-B load
    const uint4 q = *reinterpret_cast<const uint4*>(e.desc);
    e.d_lo = ((uint64_t)q.y << 32) | q.x;
    e.d_hi = ((uint64_t)q.w << 32) | q.z;
  }
  uint8_t flags = 0;
  int32_t num_actions = 0, n_turns = 0;
  double penalty = 0.0;
  if (!kFirst) {  // a fresh episode's record is all zero (EnvStatus(), es_manager.py:95)
    flags = ep.flags[bc];
    num_actions = ep.num_actions[bc];
    n_turns = ep.n_turns[bc];
    penalty = ep.penalty[bc];
  }
  // branch-free: a conditional load would make the compiler wait for the earlier loads
  const uint8_t has_in = *(in.has_input ? in.has_input + bc : ep.flags + bc);
  const int n_act = in.n_actions[bc];
  const uint64_t acts = load_actions(in.actions + bc * (int64_t)in.K, in.K, ep.flags + bc);
  if (!(n == 16 && (reinterpret_cast<uintptr_t>(kFirst ? init_desc : env.desc) & 15u) == 0) && e.in_regs) {
    for (int i = 0; i < n; ++i) {  // small maps other than an aligned 4x4: byte by byte
      const uint64_t c = e.desc[i];
      if (i < 8) e.d_lo |= c << (8 * i);
      else e.d_hi |= c << (8 * (i - 8));
    }
  }
  e.nrow = env.nrow;
  e.ncol = env.ncol;
  e.slippery = env.is_slippery != 0;
  e.cs0 = env.cs0;
  e.cs1 = env.cs1;
  e.cs2 = env.cs2;
  FinRecord rec;
  if (kFin) rec.load(ep, bc);
  if (kFirst && live) {  // the reset, then the turn (same thread, later stores win)
    uint8_t* desc = const_cast<uint8_t*>(env.desc) + b * n;
    if (n == 16 && ((reinterpret_cast<uintptr_t>(env.desc) & 15u) == 0)) {
      *reinterpret_cast<uint4*>(desc) = make_uint4((uint32_t)e.d_lo, (uint32_t)(e.d_lo >> 32), (uint32_t)e.d_hi,
                                                   (uint32_t)(e.d_hi >> 32));
    } else {
      for (int i = 0; i < n; ++i) desc[i] = e.desc[i];
    }
    env.s[b] = e.s;
#pragma unroll
    for (int k = 0; k < 4; ++k) env.rng[k * (int64_t)B + b] = init_rng[k * (int64_t)B + b];
    ep.num_actions[b] = 0;
    ep.flags[b] = 0;
    ep.n_turns[b] = 0;
    ep.penalty[b] = 0.0;
    for (int t = 0; t < ep.T; ++t) {
      ep.turn_reward[(int64_t)t * B + b] = 0.0;
      ep.turn_info[(int64_t)t * B + b] = 0;
      ep.turn_exec[(int64_t)t * B + b] = 0;
    }
  }
  RMI_STAMP_WAIT(1);
  const bool act = live && (in.has_input ? has_in != 0 : !(flags & RMI_FLAG_DONE));
  TurnOut o;
  o.acc = 0.0;
  o.info = 0;
  o.exec = 0;
  o.stepped_any_state = false;
  bool stepped = false;
  // the 4x4 straight-line turn when every lane of the wave can take it (see fl4_turn)
  const bool ids_ok = ((((acts & 0x7F7F7F7F7F7F7F7Full) + 0x7B7B7B7B7B7B7B7Bull) | acts) &  // every id byte <= 4
                       0x8080808080808080ull) == 0;
  const bool fast = n == 16 && env.ncol == 4 && e.in_regs && in.K >= 1 && ids_ok && e.s >= 0 && e.s < 16;
  if (__all(fast || !act)) {
    if (act) {
      const uint32_t hole = cell_bits(e.d_lo, e.d_hi, 'H'), goal = cell_bits(e.d_lo, e.d_hi, 'G');
      int n_a = n_act > in.K ? in.K : n_act;
      flags &= (uint8_t)~RMI_FLAG_DONE;  // done-ness is decided per stepped turn (es_manager.py:168)
      RMI_STAMP(2);
      const Fl4Out f = fl4_dispatch(in.K, hole, goal, e.s, e.rng, acts, n_a, in.max_actions_per_traj - num_actions,
                                    e.slippery, draw_threshold(e.cs0), draw_threshold(e.cs1), draw_threshold(e.cs2));
      RMI_STAMP(3);
#ifdef RMI_STAMPS
      if ((threadIdx.x & 63) == 0) g_stamps[(blockIdx.x * blockDim.x + threadIdx.x) / 64 * 16 + 11] = f.t_draws;
#endif
      // the format penalty (es_manager.py:158-159): not every parsed name known, or none
      // (fl4_turn counted the known names; selects, no branches, down to the stores)
      penalty = ((f.nv != n_a) | (f.nv == 0)) ? penalty + in.format_penalty : penalty;
      o = f.o;
      num_actions += o.exec;
      n_turns += 1;
      const uint8_t fd = (uint8_t)(RMI_FLAG_TERMINATED | RMI_FLAG_DONE);
      const uint8_t f_done = f.succ_last ? (uint8_t)((flags | fd) & ~RMI_FLAG_TRUNCATED)
                                         : (uint8_t)(flags | fd | RMI_FLAG_TRUNCATED);
      const uint8_t f_cap = (uint8_t)(flags | fd | RMI_FLAG_TRUNCATED);
      flags = f.turn_done ? f_done : (num_actions >= in.max_actions_per_traj ? f_cap : flags);
      stepped = true;
      ep.num_actions[b] = num_actions;
      ep.flags[b] = flags;
      ep.n_turns[b] = n_turns;
      ep.penalty[b] = penalty;
      const int64_t tb = (int64_t)in.turn * B + b;
      ep.turn_reward[tb] = o.acc;
      ep.turn_info[tb] = o.info;
      ep.turn_exec[tb] = o.exec;
      // s and the PCG64 state: written back whether or not a step ran (unchanged then)
      e.s = f.s;
      e.rng = f.rng;
      env.s[b] = e.s;
      store_pcg(env.rng, B, b, e.rng);
    }
  } else if (act) {
    if (e.s < 0 || e.s >= n) {
      if (err_out) err_out[b] |= RMI_ERR_STATE;
    } else {
      uint8_t err = 0;
      o = run_turn(e, acts, n_act, in.K, num_actions, flags, n_turns, penalty, in.max_actions_per_traj,
                   in.format_penalty, err);
      stepped = true;
      ep.num_actions[b] = num_actions;
      ep.flags[b] = flags;
      ep.n_turns[b] = n_turns;
      ep.penalty[b] = penalty;
      const int64_t tb = (int64_t)in.turn * B + b;
      ep.turn_reward[tb] = o.acc;
      ep.turn_info[tb] = o.info;
      ep.turn_exec[tb] = o.exec;
      if (o.stepped_any_state) {
        env.s[b] = e.s;
        store_pcg(env.rng, B, b, e.rng);
      }
      if (err_out && err) err_out[b] |= err;
    }
  }
  if (kFin) {
    if (stepped) rec.set(in.turn, o.acc, o.info);  // this turn's record is still in registers
    finalize_envs<1>(ep, fin, rec, b, live, flags, n_turns, num_actions, penalty, stepped ? in.turn : -1, o.acc,
                     o.info);
  }
  RMI_STAMP(4);
}

struct BanditDev {
  int start;
  bool hi_first;
  double lo_score, hi_lo, hi_hi, hi_prob;
  Pcg64 rng;
  __device__ __forceinline__ bool step(int a, double& reward, bool& done, bool& eff, bool& success) {
    if (a != start && a != start + 1) return false;  // assert action in ACTION_LOOKUP
    const bool is_hi = (a == start) == hi_first;
    if (is_hi) reward = rng.next_double() < hi_prob ? hi_hi : hi_lo;  // _hi_arm_reward
    else reward = lo_score;                                            // _lo_arm_reward
    done = true;
    eff = true;
    success = is_hi;
    return true;
  }
};

__global__ __launch_bounds__(kToyBlock) void bandit_step_turn_kernel(rmi_bandit_t env, rmi_episode_t ep, rmi_turn_t in,
                                                                  uint8_t* __restrict__ err_out) {
  const int64_t b = (int64_t)blockIdx.x * kToyBlock + threadIdx.x;
  const int B = ep.B;
  if (b >= B) return;
  uint8_t flags = ep.flags[b];
  const bool act = in.has_input ? (in.has_input[b] != 0) : !(flags & RMI_FLAG_DONE);
  if (!act) return;
  BanditDev e;
  e.start = env.action_space_start;
  e.hi_first = env.hi_is_first[b] != 0;
  e.lo_score = env.lo_arm_score;
  e.hi_lo = env.hi_arm_loscore;
  e.hi_hi = env.hi_arm_hiscore;
  e.hi_prob = env.hi_arm_hiscore_prob;
  e.rng = load_pcg(env.rng, B, b);
  uint8_t err = 0;
  int32_t num_actions = ep.num_actions[b], n_turns = ep.n_turns[b];
  double penalty = ep.penalty[b];
  TurnOut o = run_turn(e, load_actions(in.actions + b * (int64_t)in.K, in.K, ep.flags + b), in.n_actions[b], in.K, num_actions, flags, n_turns,
                       penalty, in.max_actions_per_traj, in.format_penalty, err);
  ep.num_actions[b] = num_actions;
  ep.flags[b] = flags;
  ep.n_turns[b] = n_turns;
  ep.penalty[b] = penalty;
  const int64_t tb = (int64_t)in.turn * B + b;
  ep.turn_reward[tb] = o.acc;
  ep.turn_info[tb] = o.info;
  ep.turn_exec[tb] = o.exec;
  if (o.stepped_any_state) store_pcg(env.rng, B, b, e.rng);
  if (err_out && err) err_out[b] |= err;
}

// Device part of FrozenLakeEnv.reset (frozen_lake/env.py:28-37) + EnvStatus(): desc / s / PCG64
// state := the generated map, start state and seeded generator, and the episode record zeroed,
// in one launch (thread i: env i's scalars and record, plus desc word i of the flat [B, n] map).
__global__ __launch_bounds__(kBlock) void frozenlake_reset_kernel(rmi_frozenlake_t env, rmi_episode_t ep,
                                                                  const uint8_t* __restrict__ init_desc,
                                                                  const int32_t* __restrict__ init_s,
                                                                  const uint64_t* __restrict__ init_rng) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t B = ep.B, n = (int64_t)env.nrow * env.ncol;
  const int64_t nbytes = B * n;
  uint8_t* desc = const_cast<uint8_t*>(env.desc);
  if (i < (nbytes >> 2)) reinterpret_cast<uint32_t*>(desc)[i] = reinterpret_cast<const uint32_t*>(init_desc)[i];
  if (i < (nbytes & 3)) desc[(nbytes & ~3ll) + i] = init_desc[(nbytes & ~3ll) + i];
  if (i < B) {
    env.s[i] = init_s[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) env.rng[k * B + i] = init_rng[k * B + i];
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

#ifdef RMI_STAMPS
RMI_API int rmi_toytext_set_stamps(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(rmi::g_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -2;
}
#endif

RMI_API int rmi_frozenlake_reset(const rmi_frozenlake_t* env, const rmi_episode_t* ep, const uint8_t* init_desc,
                                 const int32_t* init_s, const uint64_t* init_rng, rmi_stream_t stream) {
  using namespace rmi;
  if (!env || !ep || ep->B < 0 || ep->T <= 0) return RMI_EINVAL;
  if (env->nrow <= 0 || env->ncol <= 0 || env->nrow * env->ncol > 64) return RMI_EUNSUP;
  if (ep->B == 0) return RMI_OK;
  if (!env->desc || !env->s || !env->rng || !init_desc || !init_s || !init_rng || !ep->num_actions || !ep->flags ||
      !ep->n_turns || !ep->penalty || !ep->turn_reward || !ep->turn_info || !ep->turn_exec)
    return RMI_EINVAL;
  if ((reinterpret_cast<uintptr_t>(env->desc) | reinterpret_cast<uintptr_t>(init_desc)) & 3u) return RMI_EUNSUP;
  const int64_t nw = (int64_t)ep->B * env->nrow * env->ncol / 4;
  const int64_t n = nw > ep->B ? nw : ep->B;
  hipLaunchKernelGGL(frozenlake_reset_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     as_stream(stream), *env, *ep, init_desc, init_s, init_rng);
  return launch_status();
}

RMI_API int rmi_frozenlake_step_turn(const rmi_frozenlake_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                     uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (!env) return RMI_EINVAL;
  if (env->nrow <= 0 || env->ncol <= 0 || env->nrow * env->ncol > 64) return RMI_EUNSUP;
  const int rc = check_turn_args(ep, in);
  if (rc != RMI_OK) return rc > 0 ? RMI_OK : rc;
  if (!env->desc || !env->s || !env->rng) return RMI_EINVAL;
  const unsigned grid = (unsigned)((ep->B + kFlBlock - 1) / kFlBlock);
  hipLaunchKernelGGL((frozenlake_step_turn_kernel<false, false>), dim3(grid), dim3(kFlBlock), 0, as_stream(stream),
                     *env, *ep, *in, err, nullptr, nullptr, nullptr, rmi_finalize_t{});
  return launch_status();
}

RMI_API int rmi_frozenlake_step_turn_first(const rmi_frozenlake_t* env, const rmi_episode_t* ep,
                                           const rmi_turn_t* in, const uint8_t* init_desc, const int32_t* init_s,
                                           const uint64_t* init_rng, uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (!env) return RMI_EINVAL;
  if (env->nrow <= 0 || env->ncol <= 0 || env->nrow * env->ncol > 64) return RMI_EUNSUP;
  const int rc = check_turn_args(ep, in);
  if (rc != RMI_OK) return rc > 0 ? RMI_OK : rc;
  if (!env->desc || !env->s || !env->rng || !init_desc || !init_s || !init_rng) return RMI_EINVAL;
  const unsigned grid = (unsigned)((ep->B + kFlBlock - 1) / kFlBlock);
  hipLaunchKernelGGL((frozenlake_step_turn_kernel<true, false>), dim3(grid), dim3(kFlBlock), 0, as_stream(stream),
                     *env, *ep, *in, err, init_desc, init_s, init_rng, rmi_finalize_t{});
  return launch_status();
}

RMI_API int rmi_frozenlake_step_turn_finalize(const rmi_frozenlake_t* env, const rmi_episode_t* ep,
                                              const rmi_turn_t* in, uint8_t* err, const rmi_finalize_t* fin,
                                              rmi_stream_t stream) {
  using namespace rmi;
  if (!env || !fin) return RMI_EINVAL;
  if (env->nrow <= 0 || env->ncol <= 0 || env->nrow * env->ncol > 64) return RMI_EUNSUP;
  const int rc = check_turn_args(ep, in);
  if (rc < 0) return rc;
  if (ep->B == 0) return RMI_OK;
  if (!env->desc || !env->s || !env->rng) return RMI_EINVAL;
  if (fin->method < 0 || fin->method > 3 || fin->group_size < 1) return RMI_EINVAL;
  // every group inside the one-wave workgroup, and no partial group
  if (64 % fin->group_size != 0 || ep->B % fin->group_size != 0) return RMI_EUNSUP;  // groups inside one wave
  rmi_finalize_t f = *fin;
  if (f.group_size == 1) f.method = RMI_NORM_IDENTITY;  // ctx_manager.py:220: no group with > 1 member
  const unsigned grid = (unsigned)((ep->B + kFlBlock - 1) / kFlBlock);
  hipLaunchKernelGGL((frozenlake_step_turn_kernel<false, true>), dim3(grid), dim3(kFlBlock), 0, as_stream(stream),
                     *env, *ep, *in, err, nullptr, nullptr, nullptr, f);
  return launch_status();
}

RMI_API int rmi_bandit_step_turn(const rmi_bandit_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                 uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (!env) return RMI_EINVAL;
  const int rc = check_turn_args(ep, in);
  if (rc != RMI_OK) return rc > 0 ? RMI_OK : rc;
  if (!env->hi_is_first || !env->rng) return RMI_EINVAL;
  const unsigned grid = (unsigned)((ep->B + kToyBlock - 1) / kToyBlock);
  hipLaunchKernelGGL(bandit_step_turn_kernel, dim3(grid), dim3(kToyBlock), 0, as_stream(stream), *env, *ep, *in, err);
  return launch_status();
}
