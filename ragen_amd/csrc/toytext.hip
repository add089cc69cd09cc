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
constexpr int kFlBlock = RMI_FL_BLOCK;  // FrozenLake turn: threads per workgroup
// FrozenLake turn: lanes per env (see fl4_turn).  8 lanes (one jump per lane) measured 30.7 us
// per rollout against 29.7 for 4: the wave span shrinks, the dispatch of twice the waves costs
// more.  The fused finalize needs its group of 16 envs inside one wave (4 lanes at most).
constexpr int kFlLpe = 4, kFlLpeFin = 4;

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
  Pcg64 rng;       // the state after the turn: valid on the owner lane only
  bool rng_owner;  // this lane ran the turn's last executed step (stores the PCG64 state)
#ifdef RMI_STAMPS
  unsigned long long t_draws;  // diagnostic: s_memtime once the turn's draws are computed
#endif
};

__device__ __forceinline__ uint64_t pcg_out(uint64_t hi, uint64_t lo) {
  const uint64_t x = hi ^ lo;
  const unsigned rot = (unsigned)(hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

// Jump-ahead constants of the PCG64 LCG: the state k steps on is A_k * state + S_k * inc
// (mod 2^128) with A_k = M^k and S_k = 1 + M + ... + M^(k-1); row k-1 = {A_k hi, lo, S_k hi, lo}.
typedef unsigned __int128 u128;
constexpr u128 kPcgMult = ((u128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
constexpr u128 jump_a(int k) {
  u128 a = 1;
  for (int i = 0; i < k; ++i) a *= kPcgMult;
  return a;
}
constexpr u128 jump_s(int k) {
  u128 s = 0, p = 1;
  for (int i = 0; i < k; ++i) {
    s += p;
    p *= kPcgMult;
  }
  return s;
}
#define RMI_JROW(k) \
  {(uint64_t)(jump_a(k) >> 64), (uint64_t)jump_a(k), (uint64_t)(jump_s(k) >> 64), (uint64_t)jump_s(k)}
__constant__ uint64_t kPcgJump[kMaxK][4] = {RMI_JROW(1), RMI_JROW(2), RMI_JROW(3), RMI_JROW(4),
                                            RMI_JROW(5), RMI_JROW(6), RMI_JROW(7), RMI_JROW(8)};
#undef RMI_JROW

// low 128 bits of (a_hi:a_lo) * (b_hi:b_lo)
__device__ __forceinline__ void mul128lo(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl, uint64_t& h,
                                         uint64_t& l) {
  l = al * bl;
  h = __umul64hi(al, bl) + al * bh + ah * bl;
}

// The PCG64 state j steps after (s, inc), from row j-1 of kPcgJump (already loaded).
__device__ __forceinline__ void pcg_jump(const Pcg64& r, const uint64_t* J, uint64_t& h, uint64_t& l) {
  uint64_t ph, pl, qh, ql;
  mul128lo(J[0], J[1], r.s_hi, r.s_lo, ph, pl);
  mul128lo(J[2], J[3], r.i_hi, r.i_lo, qh, ql);
  l = pl + ql;
  h = ph + qh + (l < pl ? 1ull : 0ull);
}

// The cell after step k to the lane of step k + 1: L = 4, lane q of a quad <- lane (q + 3) & 3
// (DPP quad_perm [3, 0, 1, 2]); L = 8, lane i <- lane i - 1 (row_shr:1; K <= 8 never wraps).
template <int L>
__device__ __forceinline__ int chain_pass(int x) {
  if (L == 4) return __builtin_amdgcn_mov_dpp(x, 0x93, 0xF, 0xF, false);
  return __builtin_amdgcn_update_dpp(x, x, 0x111, 0xF, 0xF, false);
}

// The turn of one env on L lanes (lane q = its index in the env's group of L): lane q owns
// steps q and q + L.  It computes their PCG64 states by jump-ahead from the turn's start state
// (the K draws no longer form a chain of K 128-bit multiply-adds) and their transition
// tables; the steps' dependent chain then walks the lanes, one table lookup per step and one
// DPP move between (chain_pass).  Every lane of the group ends with the same outputs; the
// PCG64 state after the turn stays on the lane of the last executed step (Fl4Out.rng_owner),
// which stores it.
template <int K, int L>
__device__ __forceinline__ Fl4Out fl4_turn(int q, int grp, uint32_t hole, uint32_t goal, int s, const Pcg64& rng,
                                           uint64_t acts, int n_act, int left, bool slippery, uint64_t t0,
                                           uint64_t t1, uint64_t t2, const uint64_t* J0, const uint64_t* J1) {
  constexpr int P = (K + L - 1) / L;  // steps per lane
  constexpr uint64_t kGrpMask = (1ull << L) - 1;
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
  // this lane's steps q + L p: the PCG64 state after them (draw k = output of state k + 1)
  uint64_t sh[P], sl[P], table[P];
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
#pragma unroll
  for (int p = 0; p < P; ++p) {
    pcg_jump(rng, p ? J1 : J0, sh[p], sl[p]);
    const uint64_t u = pcg_out(sh[p], sl[p]) >> 11;
    // Step k's transition is a map of the 16 cells fixed by its draw and action alone: a
    // terminal cell stays, any other moves by direction b (a wall keeps it); 4 bits per cell.
    const int k = q + L * p;
    const int ga = (int)((cl >> (8 * k)) & 0xFF) - 1;  // gym action 0..3 (a step past the list is never used)
    const int i = (u < t0) ? 0 : (u < t1) ? 1 : (u < t2) ? 2 : 0;
    const int b = (slippery ? ga + 3 + i : ga) & 3;
    table[p] = (kMove[b] & ~tm) | stay;
  }
#ifdef RMI_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  r.t_draws = __builtin_amdgcn_s_memtime();
#endif
  // the chain: step k runs on lane k % L from the cell the previous step's lane passed to it
  int c = s, pre[P], post[P];
#pragma unroll
  for (int p = 0; p < P; ++p) pre[p] = post[p] = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int p = k / L;
    const int ns = (int)((table[p] >> (4 * c)) & 0xFull);
    const bool mine = q == k % L;
    pre[p] = mine ? c : pre[p];
    post[p] = mine ? ns : post[p];
    if (k + 1 < K) c = chain_pass<L>(ns);
  }
  // per-step outcomes of this lane's steps, gathered over the group by ballots (bit k = step k)
  uint32_t done_m = 0, rw_m = 0, eff_m = 0, g_m = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const uint32_t term = (term16 >> pre[p]) & 1u, g = (goal >> post[p]) & 1u, h = (hole >> post[p]) & 1u;
    done_m |= (uint32_t)((__ballot((term | g | h) != 0) >> grp) & kGrpMask) << (L * p);
    rw_m |= (uint32_t)((__ballot(((term ^ 1u) & g) != 0) >> grp) & kGrpMask) << (L * p);
    eff_m |= (uint32_t)((__ballot(post[p] != pre[p]) >> grp) & kGrpMask) << (L * p);
    g_m |= (uint32_t)((__ballot(g != 0) >> grp) & kGrpMask) << (L * p);
  }
  done_m &= (1u << K) - 1u;  // lanes of steps >= K computed throw-away steps
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
  // the cell after the last executed step, from the lane that ran it (same group: all active)
  const int lp = last >= L ? 1 : 0;
  const int post_last = P > 1 && lp ? post[P - 1] : post[0];
  const int from = __shfl(post_last, grp + (last & (L - 1)), 64);
  r.s = ex ? from : s;
  r.rng = rng;
  r.rng_owner = ex > 0 && q == (last & (L - 1));
  r.rng.s_hi = P > 1 && lp ? sh[P - 1] : sh[0];
  r.rng.s_lo = P > 1 && lp ? sl[P - 1] : sl[0];
  return r;
}

// The hole / goal bits of a 4x4 map (bit i = cell i is 'H' / 'G') on the lanes of an env's quad:
// lane q compares dword q of the row (cells 4q..4q+3; SWAR: a zero byte of row ^ letter, then
// the dword's 4 byte flags gathered by one multiply), two DPP quad swaps OR the parts together.
__device__ __forceinline__ uint32_t quad_cell_bits(uint64_t lo, uint64_t hi, int q) {
  const uint64_t w64 = (q & 2) ? hi : lo;
  const uint32_t w = (uint32_t)(w64 >> (32 * (q & 1)));
  uint32_t bits = 0;
#pragma unroll
  for (int j = 0; j < 2; ++j) {  // 'H' -> bits 0..15, 'G' -> bits 16..31
    const uint32_t x = w ^ ((j ? 'G' : 'H') * 0x01010101u);                      // zero byte = match
    const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;  // high bit of a zero byte
    bits |= (((z >> 7) * 0x01020408u) >> 24) << (4 * (q & 3) + 16 * j);
  }
  bits |= (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0xB1, 0xF, 0xF, false);  // quad_perm [1, 0, 3, 2]
  bits |= (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0x4E, 0xF, 0xF, false);  // quad_perm [2, 3, 0, 1]
  return bits;
}

// ceil(cs * 2^53): u = (x >> 11) * 2^-53 satisfies cs > u  <=>  (x >> 11) < ceil(cs * 2^53)
__device__ __forceinline__ uint64_t draw_threshold(double cs) {
  return (uint64_t)ceil(cs * 9007199254740992.0);
}

template <int L>
__device__ __forceinline__ Fl4Out fl4_dispatch(int K, int q, int grp, uint32_t hole, uint32_t goal, int s,
                                              const Pcg64& rng, uint64_t acts, int n_act, int left, bool slip,
                                              uint64_t t0, uint64_t t1, uint64_t t2, const uint64_t* J0,
                                              const uint64_t* J1) {
#define RMI_FL4(k) fl4_turn<k, L>(q, grp, hole, goal, s, rng, acts, n_act, left, slip, t0, t1, t2, J0, J1)
  switch (K) {  // wave-uniform
    case 1: return RMI_FL4(1);
    case 2: return RMI_FL4(2);
    case 3: return RMI_FL4(3);
    case 4: return RMI_FL4(4);
    case 5: return RMI_FL4(5);
    case 6: return RMI_FL4(6);
    case 7: return RMI_FL4(7);
    default: return RMI_FL4(8);
  }
#undef RMI_FL4
}

// kFirst: a fresh episode's first turn fused with its reset (rmi_frozenlake_reset): desc, s and
// the PCG64 state come from the init arrays, the counters and the record start at zero without
// being read, and the env's reset state and whole record are written before the turn runs.
// kFin: the launch is the rollout's last turn and also runs rmi_rollout_finalize for uniform
// contiguous groups of fin.group_size envs (each group inside the launch's one wave): every
// lane, live or not, reaches the group shuffles of finalize_envs.
template <bool kFirst, bool kFin, int L>
__global__ __launch_bounds__(kFlBlock) void frozenlake_step_turn_kernel(rmi_frozenlake_t env, rmi_episode_t ep,
                                                                         rmi_turn_t in, uint8_t* __restrict__ err_out,
                                                                         const uint8_t* __restrict__ init_desc,
                                                                         const int32_t* __restrict__ init_s,
                                                                         const uint64_t* __restrict__ init_rng,
                                                                         rmi_finalize_t fin) {
  const int64_t gt = (int64_t)blockIdx.x * kFlBlock + threadIdx.x;
  const int64_t b = gt / L;  // the env of this lane's group of L
  const int q = (int)(gt & (L - 1)), grp = (int)(threadIdx.x & 63) & ~(L - 1);
  const int B = ep.B;
  if (!kFin && b >= B) return;  // whole groups (B * L lanes)
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
  // jump-ahead rows of this lane's steps q and q + L (loaded with the rest)
  const uint64_t* J0 = kPcgJump[q];
  const uint64_t* J1 = kPcgJump[L < kMaxK ? q + L : q];
  uint64_t j0[4], j1[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    j0[i] = J0[i];
    j1[i] = J1[i];
  }
  FinRecord rec;
  if (kFin) rec.load(ep, bc);
  if (kFirst && live) {  // the reset, spread over the env's lanes, then the turn (later stores win)
    uint8_t* desc = const_cast<uint8_t*>(env.desc) + b * n;
    if (n == 16 && ((reinterpret_cast<uintptr_t>(env.desc) & 15u) == 0)) {
      const uint64_t w = q < 2 ? e.d_lo : e.d_hi;
      if (q < 4) reinterpret_cast<uint32_t*>(desc)[q] = (uint32_t)(w >> (32 * (q & 1)));
    } else if (q == 0) {
      for (int i = 0; i < n; ++i) desc[i] = e.desc[i];
    }
    if (q < 4) env.rng[q * (int64_t)B + b] = init_rng[q * (int64_t)B + bc];  // lane q: plane q
    if (q == 0) {
      env.s[b] = e.s;
      ep.num_actions[b] = 0;
      ep.flags[b] = 0;
      ep.n_turns[b] = 0;
      ep.penalty[b] = 0.0;
    }
    for (int t = q; t < ep.T; t += L) {
      ep.turn_reward[(int64_t)t * B + b] = 0.0;
      ep.turn_info[(int64_t)t * B + b] = 0;
      ep.turn_exec[(int64_t)t * B + b] = 0;
    }
  }
  // the jump rows are used deep inside the turn: tie them to this point so that their loads go
  // out with the others (sunk next to their use they cost a second memory round trip)
  asm volatile("" ::"v"(j0[0]), "v"(j0[1]), "v"(j0[2]), "v"(j0[3]), "v"(j1[0]), "v"(j1[1]), "v"(j1[2]), "v"(j1[3]));
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
  const bool wave_fast = __all(fast || !act);
  if (wave_fast) {
    if (act) {
      const uint32_t hg = quad_cell_bits(e.d_lo, e.d_hi, q);  // every lane of the quad is active here
      const uint32_t hole = hg & 0xFFFFu, goal = hg >> 16;
      int n_a = n_act > in.K ? in.K : n_act;
      flags &= (uint8_t)~RMI_FLAG_DONE;  // done-ness is decided per stepped turn (es_manager.py:168)
      RMI_STAMP(2);
      const Fl4Out f = fl4_dispatch<L>(in.K, q, grp, hole, goal, e.s, e.rng, acts, n_a,
                                    in.max_actions_per_traj - num_actions, e.slippery, draw_threshold(e.cs0),
                                    draw_threshold(e.cs1), draw_threshold(e.cs2), j0, j1);
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
      if (q == 0) {
        ep.num_actions[b] = num_actions;
        ep.flags[b] = flags;
        ep.n_turns[b] = n_turns;
        ep.penalty[b] = penalty;
        const int64_t tb = (int64_t)in.turn * B + b;
        ep.turn_reward[tb] = o.acc;
        ep.turn_info[tb] = o.info;
        ep.turn_exec[tb] = o.exec;
        env.s[b] = f.s;  // unchanged when no step ran
      }
      if (f.rng_owner) store_pcg(env.rng, B, b, f.rng);  // the lane of the last executed step
    }
  } else if (act && q == 0) {  // the generic turn: one lane of the quad
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
    // every lane of a group holds its env's values after the fast turn; after the generic one
    // (lane 0 only) the group's other lanes take them from it
    if (!wave_fast) {
      const int l0 = grp;
      flags = (uint8_t)__shfl((int)flags, l0, 64);
      n_turns = __shfl(n_turns, l0, 64);
      num_actions = __shfl(num_actions, l0, 64);
      penalty = __shfl(penalty, l0, 64);
      o.acc = __shfl(o.acc, l0, 64);
      o.info = (uint8_t)__shfl((int)o.info, l0, 64);
      stepped = __shfl((int)stepped, l0, 64) != 0;
    }
    if (stepped) rec.set(in.turn, o.acc, o.info);  // this turn's record is still in registers
    finalize_envs<L>(ep, fin, rec, b, live && q == 0, flags, n_turns, num_actions, penalty,
                          stepped ? in.turn : -1, o.acc, o.info);
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
  const unsigned grid = (unsigned)(((int64_t)ep->B * kFlLpe + kFlBlock - 1) / kFlBlock);
  hipLaunchKernelGGL((frozenlake_step_turn_kernel<false, false, kFlLpe>), dim3(grid), dim3(kFlBlock), 0, as_stream(stream),
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
  const unsigned grid = (unsigned)(((int64_t)ep->B * kFlLpe + kFlBlock - 1) / kFlBlock);
  hipLaunchKernelGGL((frozenlake_step_turn_kernel<true, false, kFlLpe>), dim3(grid), dim3(kFlBlock), 0, as_stream(stream),
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
  if (64 % (fin->group_size * kFlLpeFin) != 0 || ep->B % fin->group_size != 0) return RMI_EUNSUP;  // groups in one wave
  rmi_finalize_t f = *fin;
  if (f.group_size == 1) f.method = RMI_NORM_IDENTITY;  // ctx_manager.py:220: no group with > 1 member
  const unsigned grid = (unsigned)(((int64_t)ep->B * kFlLpeFin + kFlBlock - 1) / kFlBlock);
  hipLaunchKernelGGL((frozenlake_step_turn_kernel<false, true, kFlLpeFin>), dim3(grid), dim3(kFlBlock), 0, as_stream(stream),
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
