// sokoban.hip — one whole EnvStateManager turn for a batch of Sokoban envs (gfx950).
//
// Replaces es_manager.py:105-171 driving sokoban/env.py:44-51 -> gym_sokoban step
// (SURVEY.md App. A.1).  One lane owns one env; a 64-lane workgroup (one wave) owns 64 envs.
//
// HBM layout (caller-owned SoA, include/ragen_amd.h): room grids are [B, H*W] u8 rows.
// The kernel is latency-bound (8192 envs = 128 waves < 256 CUs), so it minimises each
// lane's serial chain (DESIGN.md §3.1 has the measurements behind each point):
//   1. every global load of the turn is issued up front, branch-free from clamped addresses:
//      the lane's own rows of room_state and room_fixed (16-B pieces), the per-env scalars and
//      the actions — one memory round trip;
//   2. the rows stay in VGPRs.  A regular room (every generated one) becomes wall / target /
//      box bitboards; the K steps are one unrolled, predicated block of shifts and masks, and
//      _calc_reward's open-target count is popc(target & ~box);
//   3. only the changed cells (old / new player, moved boxes) are stored back;
//   4. any irregular room sends its whole wave to the exact path (env-private LDS rows,
//      numpy's negative-index wrap, gym_sokoban's IndexError points).
#include "common.hpp"
#include "board_step.hpp"
#include "parse_core.hpp"

#include <type_traits>

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
    // _push indexes new and new_box whenever the box side is not high; the player's own cell
    // is indexed only when the player actually moves (gym_sokoban _push / _move)
    if ((push_act && !high && (!ok_n || !ok_b)) || (try_move && !ok_n) || (moved && !ok_o)) {
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

// valid = [ids of known names], exec list = valid[:left] (es_manager.py:156-157), packed one
// byte per action (exact LDS path).
struct ExecList {
  uint64_t run;
  int cnt;
};
__device__ __forceinline__ ExecList exec_list(uint64_t acts, int n_act, int left) {  // n_act <= K
  ExecList x;
  x.run = 0;
  x.cnt = 0;
#pragma unroll
  for (int k = 0; k < kMaxK; ++k) {
    const uint32_t a = (uint32_t)(acts >> (8 * k)) & 0xFFu;
    const bool take = k < n_act && a != 0 && x.cnt < left;
    x.run |= take ? ((uint64_t)a << (8 * x.cnt)) : 0ull;
    x.cnt += take;
  }
  return x;
}

// End of the turn: counters and done / truncated flags (es_manager.py:160-169).
__device__ __forceinline__ void finish_turn(const TurnOut& o, bool turn_done, bool succ_last, int32_t& num_actions,
                                            uint8_t& flags, int32_t& n_turns, int max_actions) {
  num_actions += o.exec;
  n_turns += 1;
  if (turn_done) {
    flags |= RMI_FLAG_TERMINATED | RMI_FLAG_DONE;
    flags = succ_last ? (uint8_t)(flags & ~RMI_FLAG_TRUNCATED) : (uint8_t)(flags | RMI_FLAG_TRUNCATED);
  } else if (num_actions >= max_actions) {
    flags |= RMI_FLAG_TERMINATED | RMI_FLAG_TRUNCATED | RMI_FLAG_DONE;
  }
}

// _calc_reward + _check_if_done after one executed step (gym_sokoban sokoban_env.py).
__device__ __forceinline__ double step_reward(int n_open, int num_boxes, int& boxes_on_target, bool& all_on) {
  const int cur = num_boxes - n_open;
  double rw = -0.1;                                                           // penalty_for_step
  rw += cur > boxes_on_target ? 1.0 : (cur < boxes_on_target ? -1.0 : 0.0);  // box on / off target
  all_on = n_open == 0;
  rw += all_on ? 10.0 : 0.0;  // reward_finished
  boxes_on_target = cur;
  return rw;
}

// ------------------------------------------------------------------ bitboard fast path
// A room is "regular" when room_state is exactly what room_fixed + box set + player imply
// (every state byte equals the fixed byte, except boxes = 3 on a target / 4 on floor and the
// player's 5 on a non-wall cell), room_fixed holds only {0,1,2}, its whole border is wall and
// the player is interior.  Every generated room is regular and gym_sokoban's writes keep it
// so.  A regular room steps on bitboards held in registers — a handful of bit operations
// per action, no memory access — and numpy's negative-index wrap can never trigger (the
// player never reaches the border).  Anything else takes the exact LDS path.
//
// Board window: bit j = cell W + j (row 0, all wall, is left out), so a 6x6 room's rows
// 1..5 fit a u32 (an 8x8 one a u64).  The only cells a step can address outside the window
// are row-0 cells (j in [1-W, -1]); shift amounts are taken mod the word size, which aliases
// them onto the top bits — the bottom border row and the padding above it, all wall.  So the
// hot loop needs no range test at all.  Requires (H-1)*W <= bits of the word type.

__device__ __forceinline__ uint32_t nonzero_bytes(uint32_t y) {  // high bit of each byte != 0
  return (((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
}
__device__ __forceinline__ uint32_t gt8_bytes(uint32_t y) {  // high bit of each byte > 8
  return (y | ((y & 0x7F7F7F7Fu) + 0x77777777u)) & 0x80808080u;
}
// bit 0 of each byte of a dword -> 4-bit nibble (byte j -> bit j); exact, no carries.
// (One multiply beats the 5-instruction shift/or gather on a latency-bound lone wave.)
__device__ __forceinline__ uint32_t nib(uint32_t x) { return (x * 0x01020408u) >> 24; }
// Two such dwords at once: y = x0 | x1 << 4 (bits 8j and 8j+4) -> byte nib(x0) | nib(x1) << 4.
// The multiplier's shifts {21, 14, 7, 0} send bit 8j and bit 8j+4 to 21+j and 25+j; every
// other partial product lands on a distinct bit outside 21..28, so nothing carries.  One
// quarter-rate v_mul_lo_u32 per two dwords instead of two (host-checked exhaustively).
__device__ __forceinline__ uint32_t nib2(uint32_t x0, uint32_t x1) {
  return ((x0 | (x1 << 4)) * 0x00204081u) >> 21 & 0xFFu;
}
// 0/1 per byte -> 0x00/0xFF per byte.  Written as a subtract/xor on purpose: (x << 8) - x is
// folded by the compiler into x * 255, a quarter-rate v_mul_lo_u32.  0x80 - {0,1} never borrows.
__device__ __forceinline__ uint32_t byte_mask(uint32_t x) { return (0x80808080u - x) ^ 0x80808080u; }

// OR across the LPE lanes that share an env (consecutive lanes; DPP inside a row of 16).
template <int LPE>
__device__ __forceinline__ uint32_t env_or(uint32_t x) {
  if (LPE >= 2) x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  if (LPE >= 4) x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  if (LPE >= 8) x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
  if (LPE >= 16) x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false);  // row_mirror
  static_assert(LPE <= 16, "an env's lanes lie in one DPP row");
  return x;
}
template <int LPE>
__device__ __forceinline__ uint64_t env_or64(uint64_t x) {
  return ((uint64_t)env_or<LPE>((uint32_t)(x >> 32)) << 32) | env_or<LPE>((uint32_t)x);
}

// Bitboards (cell i = bit i, row-major) of one room, and whether it is consistent: fixed
// bytes in {0,1,2}, and the state row equals its rebuild from (fixed, boxes, player p).
// Lane `sub` of the env's LPE lanes holds row dwords w = sub + LPE * i; the partial boards
// are OR-combined across those lanes, so every lane ends with the whole room.
template <int NWL, int LPE>
__device__ __forceinline__ bool decode_rows(const uint32_t (&xs)[NWL], const uint32_t (&xf)[NWL], int sub,
                                            int row_words, int p, uint64_t& wall, uint64_t& target, uint64_t& box) {
  constexpr uint32_t L = 0x01010101u;
  const int pw = p >> 2;
  const uint32_t pmask = 0xFFu << (8 * (p & 3)), p5 = 5u << (8 * (p & 3));
  uint32_t bad = 0;
  uint64_t wl = 0, tl = 0, bl = 0;
  uint32_t fw[NWL], ft[NWL], bx[NWL];
#pragma unroll
  for (int i = 0; i < NWL; ++i) {
    const int w = sub + LPE * i;
    fw[i] = ft[i] = bx[i] = 0;
    if (w < row_words) {
      const uint32_t f = xf[i], s = xs[i];
      const uint32_t f1 = f >> 1, s1 = s >> 1, s2 = s >> 2;
      bad |= (f & 0xFCFCFCFCu) | (f & f1 & L);                   // fixed byte in {0, 1, 2}
      fw[i] = ~(f | f1) & L;                                       // fixed == 0 (wall)
      ft[i] = f1 & L;                                              // fixed == 2 (target)
      bx[i] = ((s & s1 & ~s2) | (s2 & ~s1 & ~s)) & L;            // low bits 011 / 100: 3 or 4
      const uint32_t bm = byte_mask(bx[i]);
      uint32_t reb = (f & ~bm) | ((0x05050505u - f) & bm);  // boxes: 5 - fixed = 3 on target, 4 on floor
      reb = w == pw ? ((reb & ~pmask) | p5) : reb;           // the player's 5
      bad |= reb ^ s;
    }
  }
  // gather bit 0 of every byte into the boards, two dwords per multiply (dwords w, w + LPE);
  // dwords past the row are all-zero, so they add nothing
#pragma unroll
  for (int i = 0; i < NWL; i += 2) {
    const int w = sub + LPE * i;
    if (i + 1 < NWL) {
      const uint64_t n_w = nib2(fw[i], fw[i + 1]), n_t = nib2(ft[i], ft[i + 1]), n_b = nib2(bx[i], bx[i + 1]);
      if (LPE == 1) {  // adjacent nibbles: one byte at 4w
        wl |= n_w << (4 * w);
        tl |= n_t << (4 * w);
        bl |= n_b << (4 * w);
      } else {
        const int w1 = w + LPE;
        wl |= ((n_w & 0xF) << (4 * w)) | ((n_w >> 4) << (4 * w1));
        tl |= ((n_t & 0xF) << (4 * w)) | ((n_t >> 4) << (4 * w1));
        bl |= ((n_b & 0xF) << (4 * w)) | ((n_b >> 4) << (4 * w1));
      }
    } else {
      wl |= (uint64_t)nib(fw[i]) << (4 * w);
      tl |= (uint64_t)nib(ft[i]) << (4 * w);
      bl |= (uint64_t)nib(bx[i]) << (4 * w);
    }
  }
  wall = env_or64<LPE>(wl);
  target = env_or64<LPE>(tl);
  box = env_or64<LPE>(bl);
  return env_or<LPE>(bad) == 0;
}

template <class M>
struct WordBits;
template <>
struct WordBits<uint32_t> {
  static constexpr int kBits = 32;
  __device__ __forceinline__ static int popc(uint32_t x) { return __popc(x); }
  __device__ __forceinline__ static int ctz(uint32_t x) { return __builtin_ctz(x); }
};
template <>
struct WordBits<uint64_t> {
  static constexpr int kBits = 64;
  __device__ __forceinline__ static int popc(uint64_t x) { return __popcll(x); }
  __device__ __forceinline__ static int ctz(uint64_t x) { return __builtin_ctzll(x); }
};

// One EnvStateManager turn (es_manager.py:149-169) of one regular room on window bitboards:
// board_step.hpp (the K slots as one unrolled, branch-free block; K is a template parameter).
using bs::board_turn_k;
using bs::BoardTurn;

template <class M>
__device__ __forceinline__ TurnOut board_turn(M wall, M target, M& box, int& jp, int W, uint64_t acts, int K, int n_act,
                                              int left, int& num_env_steps, int& boxes_on_target, int num_boxes,
                                              int max_steps, bool& turn_done, bool& succ_last, bool& moved_any) {
  BoardTurn t;
#define RMI_BOARD_K(k_)                                                                                           \
  case k_:                                                                                                      \
    t = board_turn_k<M, k_>(wall, target, box, jp, W, acts, n_act, left, num_env_steps, boxes_on_target, num_boxes, \
                            max_steps);                                                                         \
    break;
  switch (K) {  // wave-uniform
    RMI_BOARD_K(1)
    RMI_BOARD_K(2)
    RMI_BOARD_K(3)
    RMI_BOARD_K(4)
    RMI_BOARD_K(5)
    RMI_BOARD_K(6)
    RMI_BOARD_K(7)
    RMI_BOARD_K(8)
    default:  // K == 0: no action slots
      t = board_turn_k<M, 0>(wall, target, box, jp, W, acts, n_act, left, num_env_steps, boxes_on_target, num_boxes,
                             max_steps);
  }
#undef RMI_BOARD_K
  TurnOut o;
  o.acc = t.acc;
  o.info = (uint8_t)t.info;
  o.exec = (uint8_t)t.taken;
  o.stepped_any_state = t.taken > 0;
  num_env_steps = t.nes;
  boxes_on_target = t.bot;
  turn_done = t.stop != 0;
  succ_last = t.succ != 0;
  moved_any = t.moved != 0;
  return o;
}

// --------------------------------------------------------------------- exact LDS path
// One EnvStateManager turn for one Sokoban env on its LDS row: interior players take
// straight-line index arithmetic, the rest SokobanLdsEnv::step's exact numpy-wrap code.
__device__ __forceinline__ TurnOut lds_turn(SokobanLdsEnv& e, const ExecList& x, uint8_t& err, bool& turn_done,
                                            bool& succ_last) {
  TurnOut o;
  o.acc = 0.0;
  o.info = 0;
  o.exec = 0;
  o.stepped_any_state = false;
  const int W = e.W, H = e.H;
  int p = e.r * W + e.c;
  bool stop = false;
  for (int i = 0; i < kMaxK; ++i) {
    const bool go = i < x.cnt && !stop;
    if (!__any(go)) break;
    if (!go) continue;
    const int a = (int)(int8_t)(uint8_t)(x.run >> (8 * i));
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
      bool all_on;
      r = step_reward(e.n_open, e.num_boxes, e.boxes_on_target, all_on);
      done = all_on || (e.max_steps == e.num_env_steps);
      succ = e.boxes_on_target == e.num_boxes;
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
  return o;
}

// A lane's row dwords w = sub + LPE*i.  With one lane per env and a compile-time row size the
// row is moved as 16-B pieces (global_load/store_dwordx4 need only dword alignment): 3
// instructions per 36-B row instead of 9, i.e. fewer address passes through the TA.
struct __attribute__((packed, aligned(4))) Dw4 {
  uint32_t x, y, z, w;
};
template <int NWL, int LPE, bool kWide>
__device__ __forceinline__ void load_row(const uint8_t* row, uint32_t (&x)[NWL], int sub, int row_words) {
  const uint32_t* r1 = reinterpret_cast<const uint32_t*>(row);
  if (kWide && LPE == 1) {
    const Dw4* r4 = reinterpret_cast<const Dw4*>(row);
#pragma unroll
    for (int i = 0; i < NWL / 4; ++i) {
      const Dw4 v = r4[i];
      x[4 * i] = v.x;
      x[4 * i + 1] = v.y;
      x[4 * i + 2] = v.z;
      x[4 * i + 3] = v.w;
    }
#pragma unroll
    for (int i = NWL / 4 * 4; i < NWL; ++i) x[i] = r1[i];
  } else {
#pragma unroll
    for (int i = 0; i < NWL; ++i) {
      const int w = sub + LPE * i;
      if (w < row_words) x[i] = r1[w];
    }
  }
}
template <int NWL, int LPE, bool kWide>
__device__ __forceinline__ void store_row(uint8_t* row, const uint32_t (&x)[NWL], int sub, int row_words) {
  uint32_t* r1 = reinterpret_cast<uint32_t*>(row);
  if (kWide && LPE == 1) {
    Dw4* r4 = reinterpret_cast<Dw4*>(row);
#pragma unroll
    for (int i = 0; i < NWL / 4; ++i) r4[i] = Dw4{x[4 * i], x[4 * i + 1], x[4 * i + 2], x[4 * i + 3]};
#pragma unroll
    for (int i = NWL / 4 * 4; i < NWL; ++i) r1[i] = x[i];
  } else {
#pragma unroll
    for (int i = 0; i < NWL; ++i) {
      const int w = sub + LPE * i;
      if (w < row_words) r1[w] = x[i];
    }
  }
}

constexpr int kMaxWords = kMaxCells / 4;
#ifndef RMI_SPREAD_MAX_ENVS  // (tools/stampbench.hip overrides it to compare the layouts)
#define RMI_SPREAD_MAX_ENVS 4096
#endif
#ifndef RMI_SPREAD_LPE
#define RMI_SPREAD_LPE 4
#endif
constexpr int64_t kSpreadMaxEnvs = RMI_SPREAD_MAX_ENVS;  // RMI_SPREAD_LPE lanes per env up to this batch
constexpr int kSpreadLpe = RMI_SPREAD_LPE;
#ifndef RMI_SOK_WPB  // waves per workgroup of the turn kernel (every wave owns its own envs)
#define RMI_SOK_WPB 2
#endif
constexpr int kSokWpb = RMI_SOK_WPB;
__host__ __device__ inline bool spread_lanes(int64_t B) { return B <= kSpreadMaxEnvs; }

// ---- the observation a turn launch renders itself (rmi_sokoban_step_turn_render, kObs): the
// text of SokobanEnv.render (sokoban/env.py:53-61) of every env's state after the turn, byte for
// byte rmi_sokoban_render's rows (render.hip), with no launch and no reload of the rows of its
// own.  A turn lane leaves its env's final state in LDS (the row dwords, or for a stepped
// regular room the bitboards, which hold it); the workgroup then renders its envs with
// kObsLpe lanes each — the turn's waves plus kObsFan - 1 helper waves per turn wave, which skip
// the turn (one lane per env would make the render a ~40-step serial chain per lane: measured
// 11.4 us per launch against 4.5 for the turn alone) — into an LDS block laid out like the
// output rows, and copies the block out with coalesced 16-B stores.
struct ObsOut {
  uint32_t gb[16];  // glyph bytes of each code (absent codes: '?'), little-endian
  uint64_t glen;    // glyph byte count of each code, 4 bits per code (1..4)
  uint8_t* out;     // [B, stride]
  int32_t* len;     // [B]
  int stride;
};
constexpr int kObsFan = 4;  // waves per turn wave in a kObs workgroup (the render's lanes)
constexpr int kObsLpe = 4;  // render lanes per env
constexpr int obs_pitch_max(int HW) { return HW * 5; }  // >= H*W*4 + H - 1 for any H <= H*W (bytes)

template <int HW, class M>
struct ObsLds {  // the workgroup's envs after the turn, and its output block
  static constexpr int kEnvs = kWave * kSokWpb;
  uint32_t xs[kEnvs][HW / 4], xf[kEnvs][HW / 4];
  M wall[kEnvs], target[kEnvs], box[kEnvs];
  int jp[kEnvs];  // the player's window bit for a stepped regular room, else INT32_MIN (use the rows)
  uint32_t gb[18];  // the glyph bytes of codes 0..15, then '?' and '\n'
  uint32_t blk[kEnvs * (obs_pitch_max(HW) / 4)];
};

// The workgroup's render (every thread): env e = threadIdx.x / kObsLpe of the group, its tokens
// (H*W cells and H - 1 newlines, in order) split into kObsLpe contiguous runs; each lane sizes
// its run's glyphs, a 4-lane scan places them, the bytes go into the block, the block goes out.
template <int HW, class M>
__device__ __forceinline__ void render_group(const ObsOut& o, ObsLds<HW, M>& L, int64_t B, int H, int W) {
  constexpr int kTokMax = (2 * HW + kObsLpe - 1) / kObsLpe;  // T = H*(W+1) - 1 < 2*H*W
  const int e = threadIdx.x / kObsLpe, j = threadIdx.x % kObsLpe;
  const int64_t g0 = (int64_t)blockIdx.x * ObsLds<HW, M>::kEnvs;
  const int T = H * (W + 1) - 1;
  const int per = (T + kObsLpe - 1) / kObsLpe;
  const int t0 = j * per;
  const int r0 = t0 / (W + 1), c0 = t0 - r0 * (W + 1);
  // the env's record (its row bytes are read per cell below: LDS byte reads, issued together)
  const int jp = L.jp[e];
  const M wall = L.wall[e], target = L.target[e], box = L.box[e];
  const uint8_t* rs = reinterpret_cast<const uint8_t*>(L.xs[e]);
  const uint8_t* rf = reinterpret_cast<const uint8_t*>(L.xf[e]);
  const bool bits = jp != INT32_MIN;
  uint32_t code[kTokMax];
  int r = r0, c = c0;
#pragma unroll
  for (int k = 0; k < kTokMax; ++k) {
    const bool tok = k < per && t0 + k < T;
    const bool newline = c == W;
    const int i = r * W + c;
    int cd = 0xFF;  // 0xFF: newline / no token
    if (tok && !newline) {
      const int ic = i < HW ? i : HW - 1;
      const uint32_t s = rs[ic], f = rf[ic];
      cd = (s == 5u && f == 2u) ? 6 : (int)s;  // the player on a target shown as 6 (sokoban/env.py:55)
      // a stepped regular room: from the bitboards (window bit q = cell W + q; row 0 all wall)
      const int qb = i - W;
      const int qq = qb >= 0 ? qb : 0;
      const uint32_t wl = qb >= 0 ? (uint32_t)(wall >> qq) & 1u : 1u;
      const int tg = (int)((target >> qq) & 1u), bx = (int)((box >> qq) & 1u);
      const int bc = wl ? 0 : (qb == jp ? 5 + tg : (bx ? 4 - tg : 1 + tg));
      cd = bits ? bc : cd;
      cd = cd > 0xFE ? 0xFE : cd;
    }
    code[k] = tok ? (uint32_t)cd : 0x100u;  // 0x100: no token
    if (++c > W) {
      c = 0;
      ++r;
    }
  }
  // the glyphs: LDS table reads ([16] = '?', [17] = '\n'), all issued before any is used
  uint32_t gl[kTokMax];
  int n = 0;
#pragma unroll
  for (int k = 0; k < kTokMax; ++k) {
    const uint32_t cd = code[k];
    gl[k] = L.gb[cd < 16 ? cd : (cd == 0xFF ? 17 : 16)];
  }
  int nl[kTokMax];
#pragma unroll
  for (int k = 0; k < kTokMax; ++k) {
    const uint32_t cd = code[k];
    nl[k] = cd == 0x100u ? 0 : cd == 0xFF ? 1 : (cd < 16 ? (int)((o.glen >> (4 * (cd & 15))) & 15u) : 1);
    n += nl[k];
  }
  // exclusive scan of the byte counts over the env's kObsLpe lanes
  int incl = n;
#pragma unroll
  for (int d = 1; d < kObsLpe; d <<= 1) {
    const int v = __shfl_up(incl, d, kObsLpe);
    if (j >= d) incl += v;
  }
  const int off = incl - n;
  const int total = __shfl(incl, kObsLpe - 1, kObsLpe);
  uint8_t* row = reinterpret_cast<uint8_t*>(L.blk) + e * o.stride;
  int p = off;
#pragma unroll
  for (int k = 0; k < kTokMax; ++k) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q < nl[k]) row[p + q] = (uint8_t)(gl[k] >> (8 * q));
    p += nl[k];
  }
  if (j == kObsLpe - 1)
    for (int q = total; q < ((total + 3) & ~3); ++q) row[q] = 0;  // the last dword's unused bytes
  if (j == 0 && g0 + e < B) o.len[g0 + e] = total;
  __syncthreads();
  // the block out: the group's rows are one contiguous run of n_live * stride bytes
  const int64_t left = B - g0;
  const int n_live = left < ObsLds<HW, M>::kEnvs ? (int)left : ObsLds<HW, M>::kEnvs;
  const int nb = n_live * o.stride;
  uint8_t* dst = o.out + g0 * (int64_t)o.stride;
  const int nt = blockDim.x;
  if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
    const int n16 = nb >> 4;
    for (int k = threadIdx.x; k < n16; k += nt) reinterpret_cast<uint4*>(dst)[k] = reinterpret_cast<const uint4*>(L.blk)[k];
    for (int k = (n16 << 2) + threadIdx.x; k < (nb >> 2); k += nt) reinterpret_cast<uint32_t*>(dst)[k] = L.blk[k];
  } else {
    for (int k = threadIdx.x; k < (nb >> 2); k += nt) reinterpret_cast<uint32_t*>(dst)[k] = L.blk[k];
  }
}

// One launch = one turn of every env.  LPE consecutive lanes own one env (LPE = 1 for big
// batches; 4 when the batch is too small to fill the chip, so the per-wave instruction
// chain — decode, row rebuild, loads, stores — is split LPE ways; the steps themselves run
// redundantly on the env's lanes).  Each lane loads and stores only its own row dwords
// w = sub + LPE*i (no barriers); every load of the turn is issued up front (one memory
// round trip), rows live in VGPRs, and a wave of regular rooms steps on bitboards of word
// type M.  `border` = bitmask of the border cells (row-major), precomputed by the launcher.
// kFin: the launch is the rollout's last turn and also runs rmi_rollout_finalize for uniform
// contiguous groups of fin.group_size envs (each group inside one wave): see finalize_envs.
// kFirst: the launch is a fresh episode's first turn fused with the reset (rmi_sokoban_reset):
// the rows and players come from init_state / init_player, the counters and the episode record
// start at zero without being read, and every env's state and whole record are written.
// kLate (large batches, plain and last turns): the rows are loaded after the activity test and only by
// the lanes whose env acts this turn, a second memory round trip that a batch this size hides,
// so the rows of done envs are not fetched (HBM-bound there: done envs were ≈18 % of the bench
// rollout's env-turns, their rows ≈9 % of its traffic).
// kObs (HW == 36, LPE == 1): the launch also renders every env's observation after the turn
// (render_group; kObsFan times the waves per workgroup, the extra ones only render).
// The turn of env b (this lane is its sub-th of LPE): the body of sokoban_step_turn_kernel and of the
// token turn (sokoban_token_turn_kernel).  ls / lf: the env's exact-path LDS rows (row_words dwords
// each).  at_end(xs, xf, wall, target, box, jp): the env's state after the turn, for a fused render
// (jp = the player's window bit of a stepped regular room — read the bitboards — else INT32_MIN:
// read the rows); called by every lane after the turn's stores, before the fused finalize.
// kBoards (HW == 36, M = u32, one lane per env, not kLate): env.boards / boards_mode are honoured
// (include/ragen_amd.h: the board cache).  BUILD decodes every live env's rows (acting or not)
// and stores its entry; USE loads the 16-B entry instead of the two rows and skips the decode,
// unless some acting env of the wave has an untagged entry or actions off the regular path:
// that wave then loads its rows (a second round trip) and decodes them as without a cache.
template <int HW, class M, int LPE, bool kFin, bool kFirst, bool kLate, bool kBoards, class Ix, class AtEnd>
__device__ __forceinline__ void turn_env(const rmi_sokoban_t& env, const rmi_episode_t& ep, const rmi_turn_t& in,
                                         int hw_rt, uint64_t border, uint8_t* __restrict__ err_out,
                                         const rmi_finalize_t& fin, const uint8_t* __restrict__ init_state,
                                         const int8_t* __restrict__ init_player, int64_t b, int sub, uint32_t* ls,
                                         uint32_t* lf, AtEnd&& at_end) {
  constexpr int NW = HW ? HW / 4 : kMaxWords;
  constexpr int NWL = (NW + LPE - 1) / LPE;      // row dwords per lane
  const int hw = HW ? HW : hw_rt;
  const int row_words = hw >> 2;
  const int B = ep.B;
  const bool live = b < B;
  const int H = env.H, W = env.W;
  const uint32_t w_magic = (65536u + (uint32_t)W - 1u) / (uint32_t)W;  // off the critical path
  static_assert(!kBoards || (HW == 36 && LPE == 1 && !kLate && sizeof(M) == 4), "the board cache: 6x6, u32 window");
  // the cache mode of this launch (wave-uniform).  A fresh episode's first turn (kFirst) reads
  // the RESET state: under USE from env.init_boards (the reset rows' entries, written by a
  // first turn under BUILD), its rows still loaded -- they are the reset's store
  const int bmode = kBoards && env.boards ? (kFirst && !env.init_boards ? RMI_BOARDS_BUILD : env.boards_mode)
                                          : RMI_BOARDS_NONE;
  const bool use = bmode == RMI_BOARDS_USE;
  RMI_STAMP_DECL;
  RMI_STAMP(0);

  // ---- 1. every load of the turn, issued together: branch-free from clamped (always valid)
  //         addresses, rows first, nothing consumed before the last load is issued — so the
  //         compiler's vmcnt waits all fall after one memory round trip
  const int64_t bc = live ? b : (int64_t)B - 1;
  uint32_t xs[NWL], xf[NWL];
#pragma unroll
  for (int i = 0; i < NWL; ++i) xs[i] = xf[i] = 0;
  Dw4 ent = {0u, 0u, 0u, 0u};  // the env's board-cache entry (USE)
  if (use) ent = *elem<Ix>(reinterpret_cast<const Dw4*>(kFirst ? env.init_boards : env.boards), bc);
  if ((!use || kFirst) && !kLate) {
    load_row<NWL, LPE, HW != 0>(elem<Ix>(kFirst ? init_state : env.room_state, bc * hw), xs, sub, row_words);
    load_row<NWL, LPE, HW != 0>(elem<Ix>(env.room_fixed, bc * hw), xf, sub, row_words);
  }
  const int8_t* pl = kFirst ? init_player : env.player;
  int r = 0, c = 0;
  if (!use || kFirst) {  // (plain USE turns: the entry holds the player cell and the two counters)
    const uint16_t rc = *elem<Ix>(reinterpret_cast<const uint16_t*>(pl), bc);  // (row, col): one load
    r = (int)(int8_t)(rc & 0xFFu);
    c = (int)(int8_t)(rc >> 8);
  }
  // branch-free: a conditional load here would make the compiler wait for the rows first
  const uint8_t has_in = *elem<Ix>(in.has_input ? in.has_input : ep.flags, bc);
  uint8_t flags = 0;
  int nes = 0, bot = 0;
  int32_t num_actions = 0, n_turns = 0;
  double penalty = 0.0;
  if (!kFirst) {  // a fresh episode's record is all zero (EnvStatus(), es_manager.py:95)
    flags = *elem<Ix>(ep.flags, bc);
    if (!use) {
      nes = *elem<Ix>(env.num_env_steps, bc);
      bot = *elem<Ix>(env.boxes_on_target, bc);
    }
    num_actions = *elem<Ix>(ep.num_actions, bc);
    n_turns = *elem<Ix>(ep.n_turns, bc);
    penalty = *elem<Ix>(ep.penalty, bc);
  }
  int n_act = *elem<Ix>(in.n_actions, bc);
  const uint64_t acts = load_actions_at<Ix>(in.actions, bc, in.K, ep.flags);
  FinRecord rec;
  if (kFin) rec.load<Ix>(ep, bc);
  if (!live) flags = RMI_FLAG_DONE;
  const bool act = live && (in.has_input ? has_in != 0 : !(flags & RMI_FLAG_DONE));
  if (kLate && act) {
    load_row<NWL, LPE, HW != 0>(elem<Ix>(env.room_state, bc * hw), xs, sub, row_words);
    load_row<NWL, LPE, HW != 0>(elem<Ix>(env.room_fixed, bc * hw), xf, sub, row_words);
  }
  RMI_STAMP_WAIT(1);
  if (kFirst && live) store_row<NWL, LPE, HW != 0>(elem<Ix>(env.room_state, b * hw), xs, sub, row_words);  // the reset

  // ---- 2. format penalty and the regular-room test
  if (n_act > in.K) n_act = in.K;
  const int left = in.max_actions_per_traj - num_actions;
  // valid = action slots < n_act holding a known name (id != 0)  (es_manager.py:156, :239)
  const uint64_t slots = n_act >= 8 ? ~0ull : (1ull << (8 * n_act)) - 1;
  const uint32_t sl = (uint32_t)slots, sh = (uint32_t)(slots >> 32);
  const uint32_t al = (uint32_t)acts, ah = (uint32_t)(acts >> 32);
  const uint32_t vl = nonzero_bytes(al) & sl, vh = nonzero_bytes(ah) & sh;
  const bool acts_ok = ((gt8_bytes(al) & vl) | (gt8_bytes(ah) & vh)) == 0;
  // USE: the entry stands in for the rows while it is tagged and the actions stay on the
  // regular path; else this wave loads its rows now and decodes them
  // (an env that does not act needs no actions check: a first turn writes its reset entry)
  bool from_cache = use && (ent.w >> 8 & 0xFFu) == 1u && (acts_ok || !act);
  if (use) {
    // the tagged entry's player cell and counters (entry word 3: cell | tag << 8 | nes << 16 |
    // bot << 24); an untagged entry's are reloaded below with the rows
    const int p = (int)(ent.w & 0xFFu);
    r = (int)(((uint32_t)p * w_magic) >> 16);
    c = p - r * W;
    nes = (int)(ent.w >> 16 & 0xFFu);
    bot = (int)(int8_t)(ent.w >> 24);
  }
  if (use && !__all(from_cache || !live || (!act && !kFirst))) {
    from_cache = false;
    if (kFirst) {  // the reset rows and player are loaded already; the counters start at 0
      r = elem<Ix>(pl, 2 * bc)[0];
      c = elem<Ix>(pl, 2 * bc)[1];
      nes = bot = 0;
    } else {
      load_row<NWL, LPE, HW != 0>(elem<Ix>(env.room_state, bc * hw), xs, sub, row_words);
      load_row<NWL, LPE, HW != 0>(elem<Ix>(env.room_fixed, bc * hw), xf, sub, row_words);
      r = elem<Ix>(env.player, 2 * bc)[0];
      c = elem<Ix>(env.player, 2 * bc)[1];
      nes = *elem<Ix>(env.num_env_steps, bc);
      bot = *elem<Ix>(env.boxes_on_target, bc);
    }
  }
  bool regular = true, room_ok = false;
  M wall = 0, target = 0, box = 0;
  int jp = 0;
  if (act) {
    flags &= (uint8_t)~RMI_FLAG_DONE;  // done-ness is decided per stepped turn (:168)
    const int nv = __popc(vl) + __popc(vh);
    if (nv != n_act || nv == 0) penalty += in.format_penalty;  // :158-159
  }
  if (from_cache && (act || kFirst)) {  // the tagged entry: a regular room's window boards and player cell
    wall = (M)ent.x;
    target = (M)ent.y;
    box = (M)ent.z;
    jp = (int)(ent.w & 0xFFu) - W;
  } else if (act || ((bmode == RMI_BOARDS_BUILD || kFirst) && bmode != RMI_BOARDS_NONE && live)) {
    // (BUILD, and a first turn that fell back: every live env's entry)
    const bool interior = r >= 1 && r <= H - 2 && c >= 1 && c <= W - 2;
    const int p = interior ? r * W + c : 0;
    uint64_t wall64, target64, box64;
    const bool consistent = decode_rows<NWL, LPE>(xs, xf, sub, row_words, p, wall64, target64, box64);
    room_ok = consistent && interior && (border & ~wall64) == 0 && ((wall64 >> p) & 1) == 0;
    regular = !act || (room_ok && acts_ok);
    // window: bit j = cell W + j; the cells past row H-1 are padding walls
    const int used = (H - 1) * W;
    const M pad = used >= WordBits<M>::kBits ? (M)0 : ~(((M)1 << used) - 1);
    wall = (M)(wall64 >> W) | pad;
    target = (M)(target64 >> W);
    box = (M)(box64 >> W);
    jp = p - W;
    // a first turn under BUILD also keeps the reset state's entry for the next rollouts' first
    // turns (USE reads it instead of decoding the reset rows again)
    if (kFirst && bmode == RMI_BOARDS_BUILD && env.init_boards && live)
      *elem<Ix>(reinterpret_cast<Dw4*>(env.init_boards), b) =
          Dw4{(uint32_t)wall, (uint32_t)target, (uint32_t)box, ((uint32_t)p & 0xFFu) | (room_ok ? 1u : 0u) << 8};
  }
  RMI_STAMP(2);

  // ---- 3. the turn
  TurnOut o;
  o.acc = 0.0;
  o.info = 0;
  o.exec = 0;
  o.stepped_any_state = false;
  bool turn_done = false, succ_last = false, row_changed = false;
  uint8_t err = 0;
  // kFirst: the reset row's store (above) has completed before any lane of the env writes
  // cells of it (with several lanes per env they are other lanes' dwords)
  if (kFirst) __builtin_amdgcn_s_waitcnt(0);
  const bool fast = __all(regular);
  if (fast) {
    if (act) {
      const M box0 = box;
      const int jp0 = jp;
      o = board_turn<M>(wall, target, box, jp, W, acts, in.K, n_act, left, nes, bot, env.num_boxes, env.max_steps,
                        turn_done, succ_last, row_changed);
      if (row_changed) {
        const int p = jp + W;
        r = (int)(((uint32_t)p * w_magic) >> 16);  // p / W (exact for p < 2^10, W < 2^10)
        c = p - r * W;
        // The room was regular before the turn (state == rebuild(fixed, box0, player p0)) and
        // is after it, so the new row differs from the old one only at the old and new player
        // cells and at the cells whose box bit flipped.  Those bytes are stored directly
        // (rebuild values: player 5, box 3 on a target / 4, else the fixed byte 2 / 1) instead
        // of rebuilding and storing the whole row.
        M m = (box0 ^ box) | ((M)1 << jp0) | ((M)1 << jp);
#ifdef RMI_SOKOBAN_DWORD_STORES
        if (LPE == 1) {
          // measured variant (tools/prof_sokoban_scale.py), not built by default:
          // every dword holding a changed cell is rebuilt from the bitboards (a regular room's
          // state byte is wall 0 / player 5 / box 4 or 3 on a target / floor 1 or target 2) and
          // stored whole.  +1.1 us per launch at 8192 envs against the byte stores below.
          uint32_t dirty = 0;
          while (m) {
            const int j = WordBits<M>::ctz(m);
            m &= m - 1;
            dirty |= 1u << ((j + W) >> 2);
          }
          uint32_t* r1 = reinterpret_cast<uint32_t*>(elem<Ix>(env.room_state, b * hw));
          while (dirty) {
            const int dw = __builtin_ctz(dirty);
            dirty &= dirty - 1;
            uint32_t word = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const int j = 4 * dw + k - W;  // window bit of the cell (row 0 is all wall)
              uint32_t v = 0;
              if (j >= 0) {
                const uint32_t wl = (uint32_t)(wall >> j) & 1u, tg = (uint32_t)(target >> j) & 1u;
                const uint32_t bx = (uint32_t)(box >> j) & 1u;
                v = wl ? 0u : (j == jp ? 5u : (bx ? 4u - tg : 1u + tg));
              }
              word |= v << (8 * k);
            }
            r1[dw] = word;
          }
        } else
#endif
        if (sub == 0) {
          // the changed cells: the old and new player cells and the cells whose box bit
          // flipped — 2 to 4 for one box pushed any number of times.  The first 4 are stored
          // straight-line (a missing one repeats the first: the same byte, the same value); only
          // a turn that moved several boxes loops over the rest.
          const int64_t win = b * hw + W;  // window bit j = cell W + j
          int jj[4];
          jj[0] = WordBits<M>::ctz(m);
          m &= m - 1;
#pragma unroll
          for (int k = 1; k < 4; ++k) {
            jj[k] = m ? WordBits<M>::ctz(m) : jj[0];
            m &= m - 1;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int j = jj[k];
            const uint32_t t = (uint32_t)(target >> j) & 1u, bx = (uint32_t)(box >> j) & 1u;
            *elem<Ix>(env.room_state, win + j) = (uint8_t)(j == jp ? 5u : (bx ? 4u - t : 1u + t));
          }
          while (m) {
            const int j = WordBits<M>::ctz(m);
            m &= m - 1;
            const uint32_t t = (uint32_t)(target >> j) & 1u, bx = (uint32_t)(box >> j) & 1u;
            *elem<Ix>(env.room_state, win + j) = (uint8_t)(j == jp ? 5u : (bx ? 4u - t : 1u + t));
          }
        }
        row_changed = false;  // stored
      }
    }
  } else {
    // rare: some room of the wave is irregular -> the exact path on an env-private LDS row,
    // assembled from the env's lanes and stepped by its first lane
    if (act) {
#pragma unroll
      for (int i = 0; i < NWL; ++i) {
        const int w = sub + LPE * i;
        if (w < row_words) {
          ls[w] = xs[i];
          lf[w] = xf[i];
        }
      }
    }
    wave_sync();  // the rows are wave-private; the workgroup's other waves may be on the fast path
    if (act && sub == 0) {
      int n_open = 0;
      for (int w = 0; w < row_words; ++w)
        n_open += __popc(eq_bytes(ls[w], 2u) | (eq_bytes(ls[w], 5u) & eq_bytes(lf[w], 2u)));
      SokobanLdsEnv e;
      e.st = reinterpret_cast<uint8_t*>(ls);
      e.fx = reinterpret_cast<const uint8_t*>(lf);
      e.H = H;
      e.W = W;
      e.r = r;
      e.c = c;
      e.num_env_steps = nes;
      e.boxes_on_target = bot;
      e.num_boxes = env.num_boxes;
      e.max_steps = env.max_steps;
      e.n_open = n_open;
      e.err = 0;
      const ExecList x = exec_list(acts, n_act, left);
      o = lds_turn(e, x, err, turn_done, succ_last);
      err |= e.err;
      r = e.r;
      c = e.c;
      nes = e.num_env_steps;
      bot = e.boxes_on_target;
      row_changed = o.stepped_any_state;
    }
    wave_sync();  // the rows are wave-private; the workgroup's other waves may be on the fast path
    row_changed = env_or<LPE>(row_changed) != 0;  // the env's other lanes store their dwords too
    if (act && row_changed) {
#pragma unroll
      for (int i = 0; i < NWL; ++i) {
        const int w = sub + LPE * i;
        if (w < row_words) xs[i] = ls[w];
      }
    }
  }
  RMI_STAMP(3);

  // ---- 4. outputs: scalars from the env's first lane, row dwords from every lane
  if (kFirst && live && !act && sub == 0) {  // no input this turn: the env keeps its reset state
    elem<Ix>(env.player, 2 * b)[0] = (int8_t)r;
    elem<Ix>(env.player, 2 * b)[1] = (int8_t)c;
    *elem<Ix>(env.num_env_steps, b) = 0;
    *elem<Ix>(env.boxes_on_target, b) = 0;
    *elem<Ix>(ep.num_actions, b) = 0;
    *elem<Ix>(ep.flags, b) = 0;
    *elem<Ix>(ep.n_turns, b) = 0;
    *elem<Ix>(ep.penalty, b) = 0.0;
  }
  if (kFirst && live && sub == 0)
    for (int t = 0; t < ep.T; ++t)
      if (t != in.turn || !act) {
        *elem<Ix>(ep.turn_reward + (int64_t)t * B, b) = 0.0;
        *elem<Ix>(ep.turn_info + (int64_t)t * B, b) = 0;
        *elem<Ix>(ep.turn_exec + (int64_t)t * B, b) = 0;
      }
  if (act) {
    if (sub == 0) {
      finish_turn(o, turn_done, succ_last, num_actions, flags, n_turns, in.max_actions_per_traj);
      *elem<Ix>(ep.num_actions, b) = num_actions;
      *elem<Ix>(ep.flags, b) = flags;
      *elem<Ix>(ep.n_turns, b) = n_turns;
      *elem<Ix>(ep.penalty, b) = penalty;
      const int64_t tb = (int64_t)in.turn * B;  // this turn's row of the record
      *elem<Ix>(ep.turn_reward + tb, b) = o.acc;
      *elem<Ix>(ep.turn_info + tb, b) = o.info;
      *elem<Ix>(ep.turn_exec + tb, b) = o.exec;
      if (kFirst || o.stepped_any_state) {
        elem<Ix>(env.player, 2 * b)[0] = (int8_t)r;
        elem<Ix>(env.player, 2 * b)[1] = (int8_t)c;
        *elem<Ix>(env.num_env_steps, b) = nes;
        *elem<Ix>(env.boxes_on_target, b) = bot;
      }
      if (err_out && err) *elem<Ix>(err_out, b) |= err;
    }
    if (row_changed) store_row<NWL, LPE, HW != 0>(elem<Ix>(env.room_state, b * hw), xs, sub, row_words);
  }
  if (bmode != RMI_BOARDS_NONE && live) {
    // the entry after the turn: an acting env of a fast wave (its boards were stepped), every
    // decoded env under BUILD; an env of the exact path is untagged (its room may not be
    // regular any more); a USE env that did not act keeps its entry
    const bool stepped_fast = fast && act;
    const bool write = bmode == RMI_BOARDS_BUILD || act || kFirst;
    const uint32_t tag = (stepped_fast || !act) ? (from_cache || room_ok ? 1u : 0u) : 0u;
    if (write) {
      const uint32_t cell = (uint32_t)(jp + W) & 0xFFu;
      *elem<Ix>(reinterpret_cast<Dw4*>(env.boards), b) = Dw4{(uint32_t)wall, (uint32_t)target, (uint32_t)box,
                                                   cell | (tag << 8) | ((uint32_t)nes & 0xFFu) << 16 |
                                                       ((uint32_t)bot & 0xFFu) << 24};
    }
  }
  RMI_STAMP(4);
  at_end(xs, xf, wall, target, box, (fast && act) ? jp : INT32_MIN);
  if (kFin) {
    if (act) rec.set(in.turn, o.acc, o.info);  // this turn's record is still in registers
    finalize_envs<LPE, Ix>(ep, fin, rec, b, live && sub == 0, flags, n_turns, num_actions, penalty, act ? in.turn : -1,
                       o.acc, o.info);
  }
}

template <int HW, class M, int LPE, bool kFin, bool kFirst = false, bool kLate = false, bool kObs = false,
          class Ix = int64_t>  // HW = H*W (0 = runtime); H*W % 4 == 0
__global__ __launch_bounds__(kWave * kSokWpb * (kObs ? kObsFan : 1)) void sokoban_step_turn_kernel(rmi_sokoban_t env, rmi_episode_t ep, rmi_turn_t in,
                                                                  int hw_rt, uint64_t border,
                                                                  uint8_t* __restrict__ err_out, rmi_finalize_t fin,
                                                                  const uint8_t* __restrict__ init_state = nullptr,
                                                                  const int8_t* __restrict__ init_player = nullptr,
                                                                  ObsOut obs = ObsOut{}) {
  static_assert(!kObs || (HW == 36 && LPE == 1 && !kLate), "the fused render: 36-cell rooms, one lane per env");
  constexpr int NW = HW ? HW / 4 : kMaxWords;
  constexpr int kEnvs = kWave / LPE;             // envs per wave
  __shared__ uint32_t lds_state[kSokWpb * kEnvs * NW];  // exact path only: env-private rows
  __shared__ uint32_t lds_fixed[kSokWpb * kEnvs * NW];
  using ObsL = ObsLds<kObs ? HW : 36, M>;
  __shared__ typename std::conditional<kObs, ObsL, char>::type lds_obs;  // kObs: the group's envs and rows
  const int B = ep.B;
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int sub = lane % LPE, slot = lane / LPE;
  const bool turn_wave = !kObs || wave < kSokWpb;  // kObs helper waves only render
  const int64_t b = turn_wave ? ((int64_t)blockIdx.x * kSokWpb + wave) * kEnvs + slot : (int64_t)B;
  const int row_words = (HW ? HW : hw_rt) >> 2;
  auto at_end = [&](const auto& xs, const auto& xf, M wall, M target, M box, int jp) {
        if constexpr (kObs) {
          const int H = env.H, W = env.W;
          if (turn_wave) {  // this env's state after the turn, for the group's render
            const int e = wave * kWave + lane;
#pragma unroll
            for (int i = 0; i < NW; ++i) {
              lds_obs.xs[e][i] = xs[i];
              lds_obs.xf[e][i] = xf[i];
            }
            lds_obs.wall[e] = wall;
            lds_obs.target[e] = target;
            lds_obs.box[e] = box;
            lds_obs.jp[e] = jp;
          }
          if (threadIdx.x < 18) lds_obs.gb[threadIdx.x] = threadIdx.x < 16 ? obs.gb[threadIdx.x] : (threadIdx.x == 16 ? '?' : '\n');
          __syncthreads();
#ifndef RMI_OBS_SKIP_RENDER  // (diagnostic variant: the record and the barrier only)
          render_group<HW, M>(obs, lds_obs, B, H, W);
#endif
        }
      };
  constexpr bool kBoards = HW == 36 && LPE == 1 && !kLate && !kObs && sizeof(M) == 4;
  static_assert(sizeof(Ix) == 8 || kBoards, "32-bit env offsets: the SK layout only (launched below kOff32MaxB envs)");
  turn_env<HW, M, LPE, kFin, kFirst, kLate, kBoards, Ix>(env, ep, in, hw_rt, border, err_out, fin, init_state,
                                                         init_player, b, sub, lds_state + (wave * kEnvs + slot) * row_words,
                                                         lds_fixed + (wave * kEnvs + slot) * row_words, at_end);
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

// Reset from the distinct generated rooms (rmi_sokoban_load_rooms): env i takes row room_of[i]
// of rooms [n_rooms, 2HW+2] (fixed | state | player bytes) into room_fixed / init_state /
// init_player, then the reset above (room_state, player, counters, record).  A thread per
// (env, cell) for the rooms, a thread per env for the rest.
__global__ __launch_bounds__(kBlock) void sokoban_load_rooms_kernel(rmi_sokoban_t env, rmi_episode_t ep, int hw,
                                                                    const uint8_t* __restrict__ rooms, int n_rooms,
                                                                    const int32_t* __restrict__ room_of,
                                                                    uint8_t* __restrict__ init_state,
                                                                    int8_t* __restrict__ init_player,
                                                                    uint8_t* __restrict__ err) {
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t B = ep.B;
  const int64_t pitch = 2 * hw + 2;
  if (t < B * hw) {  // cell k of env i
    const int64_t i = t / hw;
    const int k = (int)(t - i * hw);
    const int r = room_of ? room_of[i] : (int)i;
    const bool bad = r < 0 || r >= n_rooms;
    const uint8_t f = bad ? 0 : rooms[(int64_t)r * pitch + k], v = bad ? 0 : rooms[(int64_t)r * pitch + hw + k];
    const_cast<uint8_t*>(env.room_fixed)[t] = f;  // (read-only to the turn; the reset writes it)
    env.room_state[t] = v;
    init_state[t] = v;
  }
  if (t < B) {
    const int64_t i = t;
    const int r = room_of ? room_of[i] : (int)i;
    const bool bad = r < 0 || r >= n_rooms;
    if (err) err[i] = bad ? RMI_ERR_INDEX : 0;
    const uint8_t* src = rooms + (int64_t)(bad ? 0 : r) * pitch + 2 * hw;
    const int8_t p0 = bad ? 0 : (int8_t)src[0], p1 = bad ? 0 : (int8_t)src[1];
    init_player[2 * i] = p0;
    init_player[2 * i + 1] = p1;
    env.player[2 * i] = p0;
    env.player[2 * i + 1] = p1;
    env.num_env_steps[i] = 0;
    env.boxes_on_target[i] = 0;
    ep.num_actions[i] = 0;
    ep.flags[i] = 0;
    ep.n_turns[i] = 0;
    ep.penalty[i] = 0.0;
    for (int u = 0; u < ep.T; ++u) {
      ep.turn_reward[u * B + i] = 0.0;
      ep.turn_info[u * B + i] = 0;
      ep.turn_exec[u * B + i] = 0;
    }
  }
}


// ---- the token turn (rmi_sokoban_token_turn): the decode + parse, the turn and the render of a
// Sokoban turn in one launch.  A workgroup holds kTokEnvs envs = kTokEnvs waves: wave w decodes and
// parses env b0 + w's generation (detok_parse_kernel's body, its rows in the wave's LDS); after
// the barrier wave 0 steps the group's envs, one lane each (turn_env: the turn kernel's code, and
// its fused finalize for groups inside the 16 envs), leaving each env's state after the turn in
// LDS; after the second barrier wave w renders env b0 + w, one lane per token (cell or newline),
// into an LDS row copied out as dwords — the bytes rmi_sokoban_render writes.  The per-turn launch
// count of the token path drops from three (decode + parse, turn, render) to one, and the turn's
// and the render's launches (their ramps and tails) go with it.
constexpr int kTokEnvs = 16;
// Diagnostic build only (tools/prof_token_turn.py compiles this file with RMI_TOK_STAMPS): per wave
// s_memtime at the phase boundaries and s_memrealtime at entry / exit, written once at the end.
#ifdef RMI_TOK_STAMPS
__device__ unsigned long long* g_tok_stamps;
#define TST_DECL unsigned long long tst_[8] = {0}; tst_[0] = __builtin_amdgcn_s_memrealtime(); tst_[1] = __builtin_amdgcn_s_memtime()
#define TST(i) (tst_[i] = __builtin_amdgcn_s_memtime())
#define TST_FLUSH(w)                                                                              \
  do {                                                                                            \
    tst_[7] = __builtin_amdgcn_s_memrealtime();                                                   \
    if ((threadIdx.x & 63) == 0 && g_tok_stamps)                                                  \
      for (int s_ = 0; s_ < 8; ++s_) g_tok_stamps[((int64_t)blockIdx.x * kTokEnvs + (w)) * 8 + s_] = tst_[s_]; \
  } while (0)
#else
#define TST_DECL do {} while (0)
#define TST(i) do {} while (0)
#define TST_FLUSH(w) do {} while (0)
#endif
constexpr int kTokRowWords = 48;  // >= (36 * 4 + 35 + 3) / 4: the longest 36-cell observation, in dwords
struct TokRec {                  // an env's state after the turn (36-cell room, u32 board window)
  uint32_t xs[9], xf[9];
  uint32_t wall, target, box;
  int jp;                        // a stepped regular room's player bit (the bitboards hold it), else INT32_MIN
};
__host__ __device__ constexpr size_t tok_static_lds() {
  return 2 * kTokEnvs * 9 * 4 + kTokEnvs * sizeof(TokRec) + kTokEnvs * kTokRowWords * 4 + 18 * 4;
}

template <bool kFin, bool kFirst>
__global__ __launch_bounds__(kWave* kTokEnvs) __attribute__((amdgpu_waves_per_eu(8))) void sokoban_token_turn_kernel(
    DetokArgs d, ParseArgs a, rmi_sokoban_t env, rmi_episode_t ep, rmi_turn_t in, uint64_t border,
    uint8_t* __restrict__ err_out, rmi_finalize_t fin, const uint8_t* __restrict__ init_state,
    const int8_t* __restrict__ init_player, ObsOut obs, const uint8_t* __restrict__ has_t, uint8_t* __restrict__ has) {
  extern __shared__ uint64_t lds_q[];  // kTokEnvs parse regions (parse_lds(stride) each)
  __shared__ uint32_t lds_state[kTokEnvs * 9], lds_fixed[kTokEnvs * 9];
  __shared__ TokRec rec[kTokEnvs];
  __shared__ uint32_t blk[kTokEnvs][kTokRowWords];
  __shared__ uint32_t gb[18];  // glyph bytes of codes 0..15, then '?' and '\n'
  // the render's scalars, staged here so that none of them stays live in registers across the
  // decode, the parse and the turn (the kernel runs at the parse's 64-VGPR budget)
  __shared__ struct {
    uint8_t* out;
    int32_t* len;
    uint64_t glen;
    int stride, H, W, B;
  } rp;
  // wave-uniform in SGPRs (a VGPR copy of the wave index was spilled and reloaded from scratch)
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t b0 = (int64_t)blockIdx.x * kTokEnvs, b = b0 + wv;
  TST_DECL;
  if (threadIdx.x < 18) gb[threadIdx.x] = threadIdx.x < 16 ? obs.gb[threadIdx.x] : (threadIdx.x == 16 ? '?' : '\n');
  if (threadIdx.x == 64) {
    rp.out = obs.out;
    rp.len = obs.len;
    rp.glen = obs.glen;
    rp.stride = obs.stride;
    rp.H = env.H;
    rp.W = env.W;
    rp.B = ep.B;
  }

  // ---- 1. env b's generation: decoded into the parse's LDS row (and written out), parsed in place
  if (b < a.B) {
    uint8_t* lds = reinterpret_cast<uint8_t*>(lds_q) + wv * parse_lds(a.stride);
    const int cap = list_cap(a.stride);
    uint8_t* T = lds + 4;
    uint8_t* Wb = lds + row_bytes(a.stride) + 4;
    uint16_t* EL = reinterpret_cast<uint16_t*>(lds + 2 * row_bytes(a.stride));
    uint16_t* ES = EL + cap;
    uint8_t* EI = reinterpret_cast<uint8_t*>(ES + cap);
    const Names nm = load_names(a.cfg, (a.sel && a.sel[b]) ? 1 : 0);
#ifdef RMI_PARSE_STAMPS
    unsigned long long pst_[10], dst_[6];
#endif
    uint8_t derr;
    const int n = detok_row(d, T + kPre, Wb + kPre, b, lane DSTAMP_ARG, &derr);
    if (has && lane == 0) {  // rmi_turn_inputs: the env steps when it has a generation decoded without error
      has[b] = ((!has_t || has_t[b]) && derr == 0) ? 1 : 0;
      err_out[b] = 0;
    }
    parse_row(a, T, Wb, EL, ES, EI, b, n, 0, nm, lane PSTAMP_ARG);
  }
  TST(2);
  __syncthreads();  // the group's actions (global stores of its parse waves) visible to wave 0
  TST(3);

  // ---- 2. the turn of the group's envs: kLpeT = 16 lanes per env on the first 4 waves (env
  //         b0 + t / 16 for thread t): one row dword per lane keeps the turn inside the parse's
  //         64-VGPR budget.  The last turn's finalize runs after it (section 3)
  constexpr int kLpeT = 16;
  constexpr int kTurnWaves = kTokEnvs * kLpeT / kWave;
#ifndef RMI_TOK_NO_TURN  // (diagnostic variants: tools/bench_token_turn.py)
  if (wv < kTurnWaves) {
    const int t = wv * kWave + lane, e = t / kLpeT, sub = t % kLpeT;
    const int64_t be = b0 + e;
    turn_env<36, uint32_t, kLpeT, false, kFirst, false, false, int64_t>(
        env, ep, in, 36, border, err_out, fin, init_state, init_player, be, sub, lds_state + e * 9, lds_fixed + e * 9,
        [&](const auto& xs, const auto& xf, uint32_t wall, uint32_t target, uint32_t box, int jp) {
#pragma unroll
          for (int i = 0; i < (9 + kLpeT - 1) / kLpeT; ++i) {
            const int w = sub + kLpeT * i;
            if (w < 9) {
              rec[e].xs[w] = xs[i];
              rec[e].xf[w] = xf[i];
            }
          }
          if (sub == 0) {
            rec[e].wall = wall;
            rec[e].target = target;
            rec[e].box = box;
            rec[e].jp = jp;
          }
        });
  }
#endif
  TST(4);
  __syncthreads();
  TST(5);
  // ---- 3. the last turn: rmi_rollout_finalize's work for the group's envs on wave 0, one lane per
  //         env (finalize_envs, as the fused turn form runs it), from the record the turn just wrote
  if constexpr (kFin) {
    if (wv == 0) {
      const int64_t be = b0 + (lane & (kTokEnvs - 1)), bc = be < ep.B ? be : (int64_t)ep.B - 1;
      FinRecord fr;
      fr.load(ep, bc);
      finalize_envs<1>(ep, fin, fr, be, lane < kTokEnvs && be < ep.B, ep.flags[bc], ep.n_turns[bc],
                       ep.num_actions[bc], ep.penalty[bc], -1, 0.0, 0);
    }
  }
#ifdef RMI_TOK_NO_RENDER
  return;
#endif

  // ---- 4. env b's observation (rmi_sokoban_render's row): token t = lane, t = r * (W + 1) + c is
  //         cell (r, c) for c < W, a newline for c == W
  if (b >= rp.B) {
    TST_FLUSH(wv);
    return;
  }
  const int H = rp.H, W = rp.W, T = H * (W + 1) - 1;
  const TokRec& R = rec[wv];
  const int r = lane / (W + 1), c = lane - r * (W + 1);
  uint32_t cd = 0x100u;  // no token
  if (lane < T) {
    if (c == W) {
      cd = 0xFFu;  // newline
    } else {
      const int i = r * W + c;
      const uint32_t s_ = (R.xs[i >> 2] >> (8 * (i & 3))) & 0xFFu, f_ = (R.xf[i >> 2] >> (8 * (i & 3))) & 0xFFu;
      int v = (s_ == 5u && f_ == 2u) ? 6 : (int)s_;  // the player on a target shown as 6 (sokoban/env.py:55)
      if (R.jp != INT32_MIN) {  // a stepped regular room: from the bitboards (window bit q = cell W + q)
        const int qb = i - W, qq = qb >= 0 ? qb : 0;
        const uint32_t wl = qb >= 0 ? (R.wall >> qq) & 1u : 1u;
        const int tg = (int)((R.target >> qq) & 1u), bx = (int)((R.box >> qq) & 1u);
        v = wl ? 0 : (qb == R.jp ? 5 + tg : (bx ? 4 - tg : 1 + tg));
      }
      cd = (uint32_t)(v > 0xFE ? 0xFE : v);
    }
  }
  const uint32_t g = gb[cd < 16u ? cd : (cd == 0xFFu ? 17u : 16u)];
  const int len = cd == 0x100u ? 0 : (cd < 16u ? (int)((rp.glen >> (4 * cd)) & 15u) : 1);
  const int incl = wave_inclusive_scan(len);
  const int off = incl - len, total = __builtin_amdgcn_readlane(incl, 63), nw = (total + 3) >> 2;
  uint32_t* row = blk[wv];
  if (lane < nw) row[lane] = 0u;  // the last dword's unused bytes stay 0
  wave_sync();
  uint8_t* rb = reinterpret_cast<uint8_t*>(row);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < len) rb[off + q] = (uint8_t)(g >> (8 * q));
  wave_sync();
  if (lane < nw) reinterpret_cast<uint32_t*>(rp.out + b * (int64_t)rp.stride)[lane] = row[lane];
  if (lane == 0) rp.len[b] = total;
  TST(6);
  TST_FLUSH(wv);
}

}  // namespace
}  // namespace rmi

#ifndef RMI_SOK_LATE_MIN
#define RMI_SOK_LATE_MIN (1 << 17)  // envs from which plain and last turns take the late row loads (kLate)
#endif
namespace rmi {
namespace {
template <bool kFin, bool kFirst = false>
int sokoban_step_turn_launch(const rmi_sokoban_t* env, const rmi_episode_t* ep, const rmi_turn_t* in, uint8_t* err,
                             const rmi_finalize_t& fin, hipStream_t s, const uint8_t* init_state = nullptr,
                             const int8_t* init_player = nullptr) {
  const int hw = env->H * env->W;
  const unsigned grid = (unsigned)((ep->B + kWave * kSokWpb - 1) / (kWave * kSokWpb));
  const int H = env->H, W = env->W;
  uint64_t border = 0;  // border cells, row-major
  for (int r = 0; r < H; ++r)
    for (int c = 0; c < W; ++c)
      if (r == 0 || c == 0 || r == H - 1 || c == W - 1) border |= 1ull << (r * W + c);
  const bool w32 = (H - 1) * W <= 32;  // the board window fits a u32
  // lanes per env: spread a batch too small to fill the chip over 4 lanes per env
  const bool spread = spread_lanes(ep->B);
  const bool late = !kFirst && !spread && ep->B >= RMI_SOK_LATE_MIN;
  // the board cache is kept only by the 6x6 one-lane-per-env launch (include/ragen_amd.h)
  if (env->boards && (hw != 36 || !w32 || spread || ep->B >= RMI_SOK_LATE_MIN ||
                      (env->boards_mode != RMI_BOARDS_BUILD && env->boards_mode != RMI_BOARDS_USE) ||
                      ((reinterpret_cast<uintptr_t>(env->boards) | reinterpret_cast<uintptr_t>(env->init_boards)) & 15u)))
    return RMI_EUNSUP;
#define RMI_LAUNCH(HW_, M_)                                                                                   \
  do {                                                                                                        \
    if (spread)                                                                                               \
      hipLaunchKernelGGL((sokoban_step_turn_kernel<HW_, M_, kSpreadLpe, kFin, kFirst>),                       \
                         dim3((unsigned)((ep->B + kWave * kSokWpb / kSpreadLpe - 1) /                          \
                                         (kWave * kSokWpb / kSpreadLpe))),                                   \
                         dim3(kWave * kSokWpb), 0, s, *env, *ep, *in, hw, border, err, fin, init_state,      \
                         init_player);                                                                        \
    else if (late) {                                                                                          \
      if constexpr (!kFirst)                                                                                  \
        hipLaunchKernelGGL((sokoban_step_turn_kernel<HW_, M_, 1, kFin, false, true>), dim3(grid),            \
                           dim3(kWave * kSokWpb), 0, s, *env, *ep, *in, hw, border, err, fin, init_state,    \
                           init_player);                                                                      \
    } else {                                                                                                  \
      if constexpr (HW_ == 36 && sizeof(M_) == 4) {                                                           \
        if (ep->B < kOff32MaxB) {                                                                             \
          hipLaunchKernelGGL((sokoban_step_turn_kernel<HW_, M_, 1, kFin, kFirst, false, false, uint32_t>),    \
                             dim3(grid), dim3(kWave * kSokWpb), 0, s, *env, *ep, *in, hw, border, err, fin,   \
                             init_state, init_player);                                                        \
          break;                                                                                              \
        }                                                                                                     \
      }                                                                                                       \
      hipLaunchKernelGGL((sokoban_step_turn_kernel<HW_, M_, 1, kFin, kFirst>), dim3(grid), dim3(kWave * kSokWpb), \
                         0, s, *env, *ep, *in, hw, border, err, fin, init_state, init_player);                \
    }                                                                                                         \
  } while (0)
  // (the SK layout -- 6x6 u32 window, one lane per env, early row loads -- addresses the env
  // arrays with 32-bit offsets below kOff32MaxB envs, elem<uint32_t>; every other form with
  // 64-bit ones)
  if (hw == 36 && w32)
    RMI_LAUNCH(36, uint32_t);
  else if (hw == 36)
    RMI_LAUNCH(36, uint64_t);
  else if (hw == 64)
    RMI_LAUNCH(64, uint64_t);
  else if (w32)
    RMI_LAUNCH(0, uint32_t);
  else
    RMI_LAUNCH(0, uint64_t);
#undef RMI_LAUNCH
  return launch_status();
}

// The turn with the render fused (kObs): 36-cell rooms, one lane per env.
// -> RMI_EUNSUP for any other layout (the caller launches the turn and the render separately).
template <bool kFin, bool kFirst>
int sokoban_step_turn_obs_launch(const rmi_sokoban_t* env, const rmi_episode_t* ep, const rmi_turn_t* in, uint8_t* err,
                                 const rmi_finalize_t& fin, hipStream_t s, const uint8_t* init_state,
                                 const int8_t* init_player, const ObsOut& obs) {
  const int hw = env->H * env->W;
  const int H = env->H, W = env->W;
  if (spread_lanes(ep->B) || hw != 36 || obs.stride > obs_pitch_max(hw)) return RMI_EUNSUP;
  uint64_t border = 0;
  for (int r = 0; r < H; ++r)
    for (int c = 0; c < W; ++c)
      if (r == 0 || c == 0 || r == H - 1 || c == W - 1) border |= 1ull << (r * W + c);
  const bool w32 = (H - 1) * W <= 32;
  const dim3 grid((unsigned)((ep->B + kWave * kSokWpb - 1) / (kWave * kSokWpb))), block(kWave * kSokWpb * kObsFan);
  if (w32)
    hipLaunchKernelGGL((sokoban_step_turn_kernel<36, uint32_t, 1, kFin, kFirst, false, true>), grid, block, 0, s, *env,
                       *ep, *in, hw, border, err, fin, init_state, init_player, obs);
  else
    hipLaunchKernelGGL((sokoban_step_turn_kernel<36, uint64_t, 1, kFin, kFirst, false, true>), grid, block, 0, s, *env,
                       *ep, *in, hw, border, err, fin, init_state, init_player, obs);
  return launch_status();
}

int sokoban_check(const rmi_sokoban_t* env) {
  if (!env) return RMI_EINVAL;
  const int hw = env->H * env->W;
  if (env->H <= 0 || env->W <= 0 || hw > kMaxCells) return RMI_EUNSUP;
  if (!env->room_fixed || !env->room_state || !env->player || !env->num_env_steps || !env->boxes_on_target)
    return RMI_EINVAL;
  // rows are staged as dwords: H*W must be a multiple of 4 and the grids 4-byte aligned
  if (hw % 4 != 0 ||
      ((reinterpret_cast<uintptr_t>(env->room_state) | reinterpret_cast<uintptr_t>(env->room_fixed)) & 3u))
    return RMI_EUNSUP;
  return RMI_OK;
}
}  // namespace
}  // namespace rmi

#ifdef RMI_TOK_STAMPS
RMI_API int rmi_tok_set_stamps(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(rmi::g_tok_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -2;
}
#endif
#ifdef RMI_STAMPS
RMI_API int rmi_sokoban_set_stamps(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(rmi::g_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -2;
}
#endif

namespace rmi {
namespace {
constexpr int kSkip = 1;  // (validate_turn: an empty batch, nothing to launch)
// The argument checks of the three turn forms (plain; fin: the last turn fused with the
// finalize; init_state: the first turn fused with the reset).  -> RMI_OK (f = the finalize
// arguments to launch with), kSkip, or the error.
int validate_turn(const rmi_sokoban_t* env, const rmi_episode_t* ep, const rmi_turn_t* in, const rmi_finalize_t* fin,
                  const uint8_t* init_state, const int8_t* init_player, rmi_finalize_t& f, bool boards_ok = false) {
  if (!env || (init_state && !ep)) return RMI_EINVAL;
  if (env->boards && !boards_ok) return RMI_EUNSUP;  // only the plain turn forms keep the board cache
  if (env->H <= 0 || env->W <= 0 || env->H * env->W > kMaxCells) return RMI_EUNSUP;
  const int rc = check_turn_args(ep, in);
  if (rc != RMI_OK) return rc > 0 ? kSkip : rc;
  const int ec = sokoban_check(env);
  if (ec != RMI_OK) return ec;
  f = rmi_finalize_t{};
  if (fin) {
    if (fin->method < 0 || fin->method > 3 || fin->group_size < 1) return RMI_EINVAL;
    // every group inside one wave (64 envs, or 16 when 4 lanes share an env), and no partial group
    const int per_wave = spread_lanes(ep->B) ? kWave / kSpreadLpe : kWave;
    if (per_wave % fin->group_size != 0 || ep->B % fin->group_size != 0) return RMI_EUNSUP;
    f = *fin;
    if (f.group_size == 1) f.method = RMI_NORM_IDENTITY;  // ctx_manager.py:220: no group with > 1 member
  }
  if (init_state) {
    if (!init_player) return RMI_EINVAL;
    if (reinterpret_cast<uintptr_t>(init_state) & 3u) return RMI_EUNSUP;
  }
  return RMI_OK;
}
}  // namespace
}  // namespace rmi

RMI_API int rmi_sokoban_step_turn(const rmi_sokoban_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                  uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  rmi_finalize_t f;
  const int rc = validate_turn(env, ep, in, nullptr, nullptr, nullptr, f, true);
  if (rc != RMI_OK) return rc == kSkip ? RMI_OK : rc;
  return sokoban_step_turn_launch<false>(env, ep, in, err, f, as_stream(stream));
}

RMI_API int rmi_sokoban_step_turn_finalize(const rmi_sokoban_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                           uint8_t* err, const rmi_finalize_t* fin, rmi_stream_t stream) {
  using namespace rmi;
  if (!fin) return RMI_EINVAL;
  rmi_finalize_t f;
  const int rc = validate_turn(env, ep, in, fin, nullptr, nullptr, f, true);
  if (rc != RMI_OK) return rc == kSkip ? RMI_OK : rc;
  return sokoban_step_turn_launch<true>(env, ep, in, err, f, as_stream(stream));
}

RMI_API int rmi_sokoban_step_turn_first(const rmi_sokoban_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                        const uint8_t* init_state, const int8_t* init_player, uint8_t* err,
                                        rmi_stream_t stream) {
  using namespace rmi;
  if (!init_state || !init_player) return RMI_EINVAL;
  rmi_finalize_t f;
  const int rc = validate_turn(env, ep, in, nullptr, init_state, init_player, f, true);
  if (rc != RMI_OK) return rc == kSkip ? RMI_OK : rc;
  return sokoban_step_turn_launch<false, true>(env, ep, in, err, f, as_stream(stream), init_state, init_player);
}

namespace rmi {
namespace {
// rmi_sokoban_step_turn_render's glyph table and output checks -> the kernel's ObsOut.
int obs_out(const rmi_sokoban_t* env, const rmi_render_t* obs, ObsOut& o) {
  if (!obs || !env || env->H <= 0 || env->W <= 0) return RMI_EINVAL;
  for (int k = 0; k < 16; ++k)
    if (obs->glyph_len[k] > 4) return RMI_EINVAL;
  if (obs->stride < env->H * env->W * 4 + env->H - 1 || obs->stride % 4) return RMI_EINVAL;
  o.glen = 0;
  for (int k = 0; k < 16; ++k) {  // absent glyphs render '?' (as rmi_sokoban_render)
    o.gb[k] = obs->glyph_len[k] ? obs->glyph_bytes[k] : (uint32_t)'?';
    o.glen |= (uint64_t)(obs->glyph_len[k] ? obs->glyph_len[k] : 1) << (4 * k);
  }
  o.out = obs->out;
  o.len = obs->len;
  o.stride = obs->stride;
  return RMI_OK;
}
}  // namespace
}  // namespace rmi

RMI_API int rmi_sokoban_step_turn_render(const rmi_sokoban_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                         uint8_t* err, const rmi_finalize_t* fin, const uint8_t* init_state,
                                         const int8_t* init_player, const rmi_render_t* obs, rmi_stream_t stream) {
  using namespace rmi;
  if (!obs || (fin && init_state) || (!init_state) != (!init_player)) return RMI_EINVAL;
  ObsOut o;
  const int oc = obs_out(env, obs, o);
  if (oc != RMI_OK) return oc;
  rmi_finalize_t f;
  const int rc = validate_turn(env, ep, in, fin, init_state, init_player, f);
  if (rc != RMI_OK) return rc == kSkip ? RMI_OK : rc;
  if (!obs->out || !obs->len || (reinterpret_cast<uintptr_t>(obs->out) & 3u)) return RMI_EINVAL;
  hipStream_t s = as_stream(stream);
  int lc = fin ? sokoban_step_turn_obs_launch<true, false>(env, ep, in, err, f, s, nullptr, nullptr, o)
           : init_state ? sokoban_step_turn_obs_launch<false, true>(env, ep, in, err, f, s, init_state, init_player, o)
                        : sokoban_step_turn_obs_launch<false, false>(env, ep, in, err, f, s, nullptr, nullptr, o);
  if (lc != RMI_EUNSUP) return lc;
  // another layout: the turn, then the render
  lc = fin ? sokoban_step_turn_launch<true>(env, ep, in, err, f, s)
       : init_state ? sokoban_step_turn_launch<false, true>(env, ep, in, err, f, s, init_state, init_player)
                    : sokoban_step_turn_launch<false>(env, ep, in, err, f, s);
  if (lc != RMI_OK) return lc;
  return rmi_sokoban_render(env, ep->B, obs->glyph_bytes, obs->glyph_len, obs->out, obs->stride, obs->len, stream);
}

RMI_API int rmi_sokoban_load_rooms(const rmi_sokoban_t* env, const rmi_episode_t* ep, const uint8_t* rooms,
                                   int32_t n_rooms, const int32_t* room_of, uint8_t* init_state,
                                   int8_t* init_player, uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (!env || !ep || ep->B < 0 || ep->T <= 0 || n_rooms < 0) return RMI_EINVAL;
  if (env->boards) return RMI_EUNSUP;  // a writer of the state: the caller's cache is invalid after it
  const int hw = env->H * env->W;
  if (hw <= 0 || hw > kMaxCells) return RMI_EUNSUP;
  if (ep->B == 0) return RMI_OK;
  if (!rooms || n_rooms == 0 || (!room_of && n_rooms < ep->B) || !init_state || !init_player || !env->room_fixed ||
      !env->room_state || !env->player || !env->num_env_steps || !env->boxes_on_target || !ep->num_actions ||
      !ep->flags || !ep->n_turns || !ep->penalty || !ep->turn_reward || !ep->turn_info || !ep->turn_exec)
    return RMI_EINVAL;
  const int64_t nt = (int64_t)ep->B * hw;  // >= B (hw >= 1)
  hipLaunchKernelGGL(sokoban_load_rooms_kernel, dim3((unsigned)((nt + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     as_stream(stream), *env, *ep, hw, rooms, (int)n_rooms, room_of, init_state, init_player, err);
  return launch_status();
}

RMI_API int rmi_sokoban_reset(const rmi_sokoban_t* env, const rmi_episode_t* ep, const uint8_t* init_state,
                              const int8_t* init_player, rmi_stream_t stream) {
  using namespace rmi;
  if (!env || !ep || ep->B < 0 || ep->T <= 0) return RMI_EINVAL;
  if (env->boards) return RMI_EUNSUP;  // a writer of the state: the caller's cache is invalid after it
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


RMI_API int rmi_sokoban_token_turn(const rmi_token_rows_t* tok, const rmi_sokoban_t* env, const rmi_episode_t* ep,
                                   const rmi_turn_t* in, uint8_t* err, const rmi_finalize_t* fin,
                                   const uint8_t* init_state, const int8_t* init_player, const rmi_render_t* obs,
                                   rmi_stream_t stream) {
  using namespace rmi;
  if (!tok || !ep || !in || !obs || !tok->cfg || (fin && init_state) || (!init_state) != (!init_player))
    return RMI_EINVAL;
  if (tok->cfg->K != in->K) return RMI_EINVAL;
  if (tok->has && (in->has_input != tok->has || !tok->decode_err || !err)) return RMI_EINVAL;
  const int64_t B = ep->B;
  DetokArgs d;
  ParseArgs a;
  int rc = detok_parse_args(tok->ids, B, tok->R, tok->n_ids, tok->vocab_packed, tok->vocab_bytes, tok->n_bytes, tok->V,
                            tok->text, tok->stride, tok->text_len, tok->decode_err, tok->cfg, tok->sel, const_cast<int8_t*>(in->actions),
                            const_cast<uint8_t*>(in->n_actions), tok->spans, nullptr, nullptr, 0, tok->parse_err, d, a);
  if (rc < 0) return rc;
  ObsOut o;
  rc = obs_out(env, obs, o);
  if (rc != RMI_OK) return rc;
  rmi_finalize_t f;
  rc = validate_turn(env, ep, in, fin, init_state, init_player, f);
  if (rc != RMI_OK) return rc == kSkip ? RMI_OK : rc;
  if (!obs->out || !obs->len || (reinterpret_cast<uintptr_t>(obs->out) & 3u)) return RMI_EINVAL;
  const int H = env->H, W = env->W;
  const size_t shm = (size_t)kTokEnvs * parse_lds(tok->stride);
  const bool fused = H * W == 36 && (H - 1) * W <= 32 && H * (W + 1) - 1 <= kWave && (!fin || kTokEnvs % fin->group_size == 0) &&
                     shm + tok_static_lds() <= 64 * 1024 && o.stride <= obs_pitch_max(36);
  if (!fused) {  // the two calls
    rc = rmi_detok_parse(tok->ids, B, tok->R, tok->n_ids, tok->vocab_packed, tok->vocab_bytes, tok->n_bytes, tok->V,
                         tok->text, tok->stride, tok->text_len, tok->decode_err, tok->cfg, tok->sel, const_cast<int8_t*>(in->actions),
                         const_cast<uint8_t*>(in->n_actions), tok->spans, nullptr, nullptr, 0, tok->parse_err, stream);
    if (rc != RMI_OK) return rc;
    if (tok->has) {
      rc = rmi_turn_inputs(tok->has_t, tok->decode_err, B, tok->has, err, stream);
      if (rc != RMI_OK) return rc;
    }
    return rmi_sokoban_step_turn_render(env, ep, in, err, fin, init_state, init_player, obs, stream);
  }
  uint64_t border = 0;
  for (int r = 0; r < H; ++r)
    for (int c = 0; c < W; ++c)
      if (r == 0 || c == 0 || r == H - 1 || c == W - 1) border |= 1ull << (r * W + c);
  const dim3 grid((unsigned)((B + kTokEnvs - 1) / kTokEnvs)), block(kWave * kTokEnvs);
  hipStream_t s = as_stream(stream);
  if (fin)
    hipLaunchKernelGGL((sokoban_token_turn_kernel<true, false>), grid, block, shm, s, d, a, *env, *ep, *in, border, err, f,
                       nullptr, nullptr, o, tok->has_t, tok->has);
  else if (init_state)
    hipLaunchKernelGGL((sokoban_token_turn_kernel<false, true>), grid, block, shm, s, d, a, *env, *ep, *in, border, err, f,
                       init_state, init_player, o, tok->has_t, tok->has);
  else
    hipLaunchKernelGGL((sokoban_token_turn_kernel<false, false>), grid, block, shm, s, d, a, *env, *ep, *in, border, err,
                       f, nullptr, nullptr, o, tok->has_t, tok->has);
  return launch_status();
}
