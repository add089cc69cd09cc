// board_step.hpp — the K action slots of one EnvStateManager turn of a regular Sokoban room,
// on window bitboards (es_manager.py:149-169 driving gym_sokoban's step through
// sokoban/env.py:44-51).
//
// The turn kernel runs 64 envs per wave and, at the bench's 8192 envs, one wave per SIMD: a
// lone wave issues about one instruction per 4 cycles, so this block's cost is its instruction
// count.  Everything that does not depend on the walk is therefore computed once per turn, four
// slots at a time, on the action dwords (byte k = slot k):
//   V  slot k runs if the turn is still going: a known name (id != 0), k < n_act, and one of the
//      first `left` such slots (valid[:left], es_manager.py:156-157);
//   P  V and a push action (id <= 4: _push, else _move);
//   D  V and the slot whose step brings num_env_steps to max_steps (_check_if_done);
//   S  the slot's window offset (-W, +W, -1, +1), one v_perm from a 4-byte table.
// The walk itself keeps 0/1 values and takes single bits with v_bfe (`alive` = the turn has not
// hit done is the extract width, so a stopped env's slot extracts 0).  What a slot leaves behind
// that only the turn's end needs (info, success, num_env_steps) is rebuilt once at the end.
//
// This file also builds for the host (tests/board_step_check.cpp checks it against the
// straight restatement of the same turn over random rooms), so the three bit primitives are
// given both as gfx950 instructions and in portable C++.
#pragma once
#include <stdint.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#endif

#include "ragen_amd.h"

#if defined(__HIP_DEVICE_COMPILE__)
#define RMI_BS_FN __device__ __forceinline__
#elif defined(__HIPCC__)
#define RMI_BS_FN __host__ __device__ __forceinline__
#else
#define RMI_BS_FN inline
#endif

namespace rmi {
namespace bs {

// (x >> off) & ((1 << w) - 1), offset and width taken mod 32 (v_bfe_u32)
RMI_BS_FN uint32_t ubfe(uint32_t x, uint32_t off, uint32_t w) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_ubfe(x, off, w);
#else
  off &= 31u;
  w &= 31u;
  return w ? (x >> off) & ((1u << w) - 1u) : 0u;
#endif
}
// bits [off, off + w) sign-extended, offset and width mod 32 (v_bfe_i32): with w = 1 a bit
// becomes a 0 / all-ones mask, with w = 0 the result is 0
RMI_BS_FN uint32_t smask(uint32_t x, uint32_t off, uint32_t w) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_sbfe((int32_t)x, off, w);
#else
  off &= 31u;
  w &= 31u;
  return w ? (uint32_t)((int32_t)(x << (32u - off - w)) >> (32u - w)) : 0u;
#endif
}
// hides a value's range from the compiler, which would otherwise turn the int -> f64
// conversions of small ranges below into chains of compare + select (each pair also costs a
// hazard wait on gfx950): no instruction
template <class T>
RMI_BS_FN void opaque(T& x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(x));
#else
  (void)x;
#endif
}
// the signed byte at bit `off` (v_bfe_i32, off <= 24)
RMI_BS_FN int32_t sbyte(uint32_t x, uint32_t off) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_sbfe((int32_t)x, off, 8u);
#else
  return (int32_t)(int8_t)(uint8_t)(x >> off);
#endif
}
// byte i of the result = byte sel_i of `table` (selectors 0..3; v_perm_b32)
RMI_BS_FN uint32_t pick_bytes(uint32_t table, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(0u, table, sel);
#else
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) r |= ((table >> (8 * ((sel >> (8 * i)) & 3u))) & 0xFFu) << (8 * i);
  return r;
#endif
}
RMI_BS_FN int popc32(uint32_t x) { return __builtin_popcount(x); }
RMI_BS_FN int popc64(uint64_t x) { return __builtin_popcountll(x); }

template <class M>
struct Word;
template <>
struct Word<uint32_t> {
  static RMI_BS_FN uint32_t mask(uint32_t x, int j) { return smask(x, (uint32_t)j, 1u); }  // bit j mod 32
  static RMI_BS_FN uint32_t at(int j) { return 1u << (j & 31); }
  static RMI_BS_FN uint32_t widen(uint32_t m) { return m; }  // a 0 / all-ones mask as a word
  static RMI_BS_FN int popc(uint32_t x) { return popc32(x); }
};
template <>
struct Word<uint64_t> {
  static RMI_BS_FN uint32_t mask(uint64_t x, int j) { return 0u - ((uint32_t)(x >> (j & 63)) & 1u); }
  static RMI_BS_FN uint64_t at(int j) { return 1ull << (j & 63); }
  static RMI_BS_FN uint64_t widen(uint32_t m) { return (uint64_t)(int64_t)(int32_t)m; }
  static RMI_BS_FN int popc(uint64_t x) { return popc64(x); }
};

// high bit of each byte: a known name (id != 0) in a slot < n_act (`in_range`)
RMI_BS_FN uint32_t valid_bytes(uint32_t x, uint32_t in_range) {
  return ((((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u) & in_range;
}

// The per-slot byte vectors of four slots (one action dword x, its valid bytes, `below` = the
// valid slots before it, broadcast).  pc = the inclusive count of valid slots up to each byte
// (at most 8, so no byte ever carries or borrows into the next).
struct Slots4 {
  uint32_t V, P, D, S;
};
RMI_BS_FN Slots4 slots4(uint32_t x, uint32_t valid, uint32_t below, uint32_t left_b, uint32_t m_b, uint32_t dir_table) {
  Slots4 s;
  const uint32_t pc = (valid >> 7) * 0x01010101u + below;
  s.V = ((left_b | 0x80808080u) - pc) & valid;      // pc <= left
  s.P = s.V & ~((x & 0x7F7F7F7Fu) + 0x7B7B7B7Bu);  // id <= 4 (valid ids are 1..8)
  s.D = s.V & ~((pc ^ m_b) + 0x7F7F7F7Fu);          // pc == max_steps - num_env_steps
  s.S = pick_bytes(dir_table, x & 0x03030303u);      // id & 3: 1 up, 2 down, 3 left, 0 right
  return s;
}

struct BoardTurn {
  double acc;
  uint32_t info, taken, stop, succ, moved;
  int nes, bot;
};

// One turn: K action slots (K <= 8) of the regular room (wall, target, box; player at window
// bit jp).  acts = the slots' action ids (byte k = slot k, each 1..8 where it is valid: the
// caller checks), n_act <= K.  Bit-identical to exact gym_sokoban steps (the LDS path and
// oracle/sokoban.c's sokoban_turn); box and jp are left at the turn's end.
template <class M, int K>
RMI_BS_FN BoardTurn board_turn_k(M wall, M target, M& box, int& jp, int W, uint64_t acts, int n_act, int left,
                                 int nes, int bot, int num_boxes, int max_steps) {
  const M box0 = box;
  const int jp0 = jp;
  // wave-uniform: the direction table (byte (id & 3) -> signed window offset)
  const uint32_t dir_table = 0x01u | ((uint32_t)(-W) & 0xFFu) << 8 | ((uint32_t)W & 0xFFu) << 16 | 0xFF000000u;
  // per lane: the slot range, the left budget and the max_steps slot, broadcast to bytes
  const uint64_t range = n_act >= 8 ? ~0ull : (1ull << (8 * n_act)) - 1;
  const uint32_t l8 = left <= 0 ? 0u : (left >= 8 ? 8u : (uint32_t)left);
  const int m = max_steps - nes;  // the 1-based count of steps that ends the episode
  const uint32_t m8 = (m >= 1 && m <= 8) ? (uint32_t)m : 0x7Fu;
  const uint32_t left_b = l8 * 0x01010101u, m_b = m8 * 0x01010101u;
  const uint32_t xl = (uint32_t)acts, xh = (uint32_t)(acts >> 32);
  const uint32_t vl = valid_bytes(xl, (uint32_t)range);
  Slots4 q[2];
  q[0] = slots4(xl, vl, 0u, left_b, m_b, dir_table);
  if (K > 4) q[1] = slots4(xh, valid_bytes(xh, (uint32_t)(range >> 32)), (uint32_t)popc32(vl) * 0x01010101u, left_b, m_b, dir_table);
  // the walk: booleans are 0 / all-ones masks (selects become v_bfi), except `alive` (0 / 1:
  // the width of the slot extracts)
  uint32_t alive = 1u, taken = 0u, last_moved = 0u, z = 1u;
  int open_bot = num_boxes - bot;  // the open-target count the env's boxes_on_target implies
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const Slots4& v = q[k >> 2];
    const uint32_t hb = 8u * (uint32_t)(k & 3) + 7u;  // the slot's byte's high bit
    const int s = sbyte(v.S, 8u * (uint32_t)(k & 3));
    const uint32_t go = smask(v.V, hb, alive), go_push = smask(v.P, hb, alive), go_done = smask(v.D, hb, alive);
    const int jn = jp + s, jb = jn + s;
    const M occ = wall | box;
    const uint32_t n_box = Word<M>::mask(box, jn), n_occ = Word<M>::mask(occ, jn), b_occ = Word<M>::mask(occ, jb);
    const uint32_t is_push = go_push & n_box & ~b_occ;  // _push: a box ahead, floor behind it
    const uint32_t moved = go & (is_push | ~n_occ);     // else _move: floor ahead
    box ^= (Word<M>::at(jn) | Word<M>::at(jb)) & Word<M>::widen(is_push);
    jp = (int)((moved & (uint32_t)jn) | (~moved & (uint32_t)jp));
    // _calc_reward: open targets = targets without a box; the box-count term is the sign of the
    // change against boxes_on_target (num_boxes - open_bot)
    const int n_open = Word<M>::popc(target & ~box);
    int sg = n_open - open_bot;
    sg = sg > 1 ? 1 : (sg < -1 ? -1 : sg);  // -(box on / off target)
    z = n_open < 1 ? (uint32_t)n_open : 1u;  // 0: every target covered (reward_finished, done)
    uint32_t fin = 1u - z;
    opaque(sg);
    opaque(fin);
    double rw = -0.1 - (double)sg;                // == penalty_for_step + (+1 / -1 / 0)
    rw = __builtin_fma(10.0, (double)fin, rw);    // + 10 (exact: one rounding, as the add)
    acc = __builtin_fma(-(double)(int32_t)go, rw, acc);  // acc += go ? rw : 0 (acc is never -0.0)
    open_bot = (int)((go & (uint32_t)n_open) | (~go & (uint32_t)open_bot));
    taken -= go;
    last_moved = (go & moved) | (~go & last_moved);
    alive &= ~(go_done | (go & fin));  // done: all targets covered or max_steps reached
  }
  BoardTurn t;
  t.acc = acc;
  t.taken = taken;
  t.stop = alive ^ 1u;
  // the last slot that ran decides info / success; box does not change after it
  t.succ = taken ? (z ^ 1u) : 0u;
  t.info = taken ? (RMI_INFO_PRESENT | RMI_INFO_VALID | (last_moved & 2u) | (t.succ << 3)) : 0u;
  t.moved = (box != box0) | (jp != jp0);  // the room changed (a walk back to the start stores nothing)
  t.nes = nes + (int)taken;
  t.bot = num_boxes - open_bot;
  return t;
}

}  // namespace bs
}  // namespace rmi
