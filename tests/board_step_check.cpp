// Host check of ragen_amd/csrc/board_step.hpp: the slot-vector form of a Sokoban turn on window
// bitboards against the straight per-slot restatement (the form the turn kernel used through
// round 6, itself pinned to gym_sokoban by the GPU parity tests and oracle/sokoban.c).  Every
// output is compared bit for bit (the reward sum as f64 bits) over random rooms, action slots,
// budgets and step counts, for K = 0..8 and both window words.
// Build + run: tests/test_board_step.py (g++ -O2).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>

#include "board_step.hpp"

namespace {

using rmi::bs::BoardTurn;

template <class M, int K>
BoardTurn ref_turn(M wall, M target, M& box, int& jp, int W, uint64_t acts, int n_act, int left, int nes, int bot,
                   int num_boxes, int max_steps) {
  constexpr int kMask = sizeof(M) * 8 - 1;
  BoardTurn t;
  t.acc = 0.0;
  t.info = t.taken = t.stop = t.succ = t.moved = 0;
  for (int k = 0; k < K; ++k) {
    const int a = (int)(acts >> (8 * k)) & 0xFF;
    const uint32_t go = (t.stop == 0) & (k < n_act) & ((int)t.taken < left) & (a != 0);
    const int dir = (a - 1) & 3;
    const int mag = (dir & 2) ? 1 : W;
    const int s = (dir & 1) ? mag : -mag;
    const int jn = jp + s, jb = jn + s;
    const M nb = (M)1 << (jn & kMask), bb = (M)1 << (jb & kMask);
    const M occ = wall | box;
    const uint32_t n_box = (box & nb) != 0;
    const uint32_t n_free = (occ & nb) == 0;
    const uint32_t is_push = go & (a <= 4) & n_box & ((occ & bb) == 0);
    const uint32_t moved = go & (is_push | n_free);
    box ^= is_push ? (nb | bb) : (M)0;
    jp = moved ? jn : jp;
    const int n_open = __builtin_popcountll((uint64_t)(target & ~box));
    const int cur = num_boxes - n_open;
    const double d_box = cur > bot ? 1.0 : (cur < bot ? -1.0 : 0.0);
    const uint32_t all_on = n_open == 0;
    const double rw = (-0.1 + d_box) + (all_on ? 10.0 : 0.0);
    const int nes1 = nes + 1;
    const uint32_t done = all_on | (max_steps == nes1);
    const uint32_t succ = cur == num_boxes;
    nes = go ? nes1 : nes;
    bot = go ? cur : bot;
    t.acc += go ? rw : 0.0;
    t.info = go ? (RMI_INFO_PRESENT | RMI_INFO_VALID | (moved << 1) | (succ << 3)) : t.info;
    t.succ = go ? succ : t.succ;
    t.moved |= moved;
    t.taken += go;
    t.stop |= go & done;
  }
  t.nes = nes;
  t.bot = bot;
  return t;
}

struct Case {
  uint64_t wall, target, box;
  int jp, W, n_act, left, nes, bot, num_boxes, max_steps;
  uint64_t acts;
};

template <class M>
Case make_case(std::mt19937_64& g, int K) {
  Case c;
  std::uniform_int_distribution<int> u(0, 1 << 30);
  const int H = 3 + u(g) % (sizeof(M) == 4 ? 4 : 6);  // (H - 1) * W fits the word
  const int W = 3 + u(g) % (sizeof(M) == 4 ? 4 : 6);
  const int bits = sizeof(M) * 8;
  const bool garbage = u(g) % 8 == 0;  // any words at all: both forms are pure bit functions
  if (garbage || (H - 1) * W > bits) {
    c.wall = g();
    c.target = g();
    c.box = g();
    c.jp = (int)(u(g) % 80) - 8;
  } else {
    const int used = (H - 1) * W;
    uint64_t wall = used >= 64 ? 0 : ~((1ull << used) - 1);  // padding above the window: wall
    uint64_t target = 0, box = 0;
    for (int r = 1; r < H; ++r)
      for (int col = 0; col < W; ++col) {
        const int j = (r - 1) * W + col;  // window bit of cell (r, col)
        const bool border = r == H - 1 || col == 0 || col == W - 1;
        if (border || u(g) % 6 == 0) wall |= 1ull << j;
      }
    for (int j = 0; j < used; ++j)
      if (!((wall >> j) & 1)) {
        if (u(g) % 5 == 0) target |= 1ull << j;
        if (u(g) % 4 == 0) box |= 1ull << j;
      }
    int jp = -1;
    for (int tries = 0; tries < 64 && jp < 0; ++tries) {
      const int j = u(g) % used;
      if (!((wall >> j) & 1) && !((box >> j) & 1)) jp = j;
    }
    c.wall = wall;
    c.target = target;
    c.box = box;
    c.jp = jp < 0 ? W + 1 : jp;
  }
  if (sizeof(M) == 4) {
    c.wall &= 0xFFFFFFFFull;
    c.target &= 0xFFFFFFFFull;
    c.box &= 0xFFFFFFFFull;
  }
  c.W = W;
  c.n_act = K ? u(g) % (K + 1) : 0;
  c.acts = 0;
  for (int k = 0; k < 8; ++k) {
    uint64_t a;
    if (k < c.n_act)
      a = u(g) % 5 == 0 ? 0 : 1 + u(g) % 8;  // in range: unknown (0) or a valid id 1..8
    else
      a = u(g) % 256;  // out of range: anything
    c.acts |= a << (8 * k);
  }
  c.left = u(g) % 15 - 3;
  c.nes = u(g) % 3 == 0 ? u(g) % 200 : u(g) % 12;
  c.max_steps = u(g) % 3 == 0 ? c.nes + u(g) % 12 - 2 : (u(g) % 2 ? 100 : u(g) % 14);
  c.bot = u(g) % 7 - 2;
  c.num_boxes = u(g) % 5;
  return c;
}

template <class M, int K>
int check(std::mt19937_64& g, int n) {
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    const Case c = make_case<M>(g, K);
    M box_a = (M)c.box, box_b = (M)c.box;
    int jp_a = c.jp, jp_b = c.jp;
    const BoardTurn a = rmi::bs::board_turn_k<M, K>((M)c.wall, (M)c.target, box_a, jp_a, c.W, c.acts, c.n_act, c.left,
                                                    c.nes, c.bot, c.num_boxes, c.max_steps);
    const BoardTurn b =
        ref_turn<M, K>((M)c.wall, (M)c.target, box_b, jp_b, c.W, c.acts, c.n_act, c.left, c.nes, c.bot, c.num_boxes,
                       c.max_steps);
    uint64_t ab, bb;
    memcpy(&ab, &a.acc, 8);
    memcpy(&bb, &b.acc, 8);
    // `moved`: the new form reports whether the room changed, the old one whether any slot moved
    // the player; they differ only for a walk that returns to its start, which stores nothing
    const bool moved_ok = a.moved == (uint32_t)(box_b != (M)c.box || jp_b != c.jp) && (!a.moved || b.moved);
    if (ab != bb || a.info != b.info || a.taken != b.taken || (a.stop != 0) != (b.stop != 0) ||
        (a.succ != 0) != (b.succ != 0) || a.nes != b.nes || a.bot != b.bot || box_a != box_b || jp_a != jp_b ||
        !moved_ok) {
      if (bad++ < 5)
        fprintf(stderr,
                "mismatch M=%zu K=%d: acc %.17g/%.17g info %u/%u taken %u/%u stop %u/%u succ %u/%u nes %d/%d "
                "bot %d/%d jp %d/%d moved %u/%u (acts %016llx n_act %d left %d nes %d max %d bot %d nb %d)\n",
                sizeof(M), K, a.acc, b.acc, a.info, b.info, a.taken, b.taken, a.stop, b.stop, a.succ, b.succ, a.nes,
                b.nes, a.bot, b.bot, jp_a, jp_b, a.moved, b.moved, (unsigned long long)c.acts, c.n_act, c.left,
                c.nes, c.max_steps, c.bot, c.num_boxes);
    }
  }
  return bad;
}

template <class M>
int check_all(std::mt19937_64& g, int n) {
  return check<M, 0>(g, n) + check<M, 1>(g, n) + check<M, 2>(g, n) + check<M, 3>(g, n) + check<M, 4>(g, n) +
         check<M, 5>(g, n) + check<M, 6>(g, n) + check<M, 7>(g, n) + check<M, 8>(g, n);
}

}  // namespace

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 200000;
  std::mt19937_64 g(12345);
  const int bad = check_all<uint32_t>(g, n) + check_all<uint64_t>(g, n);
  printf("%s %d cases per (word, K), %d mismatches\n", bad ? "FAIL" : "ok", n, bad);
  return bad ? 1 : 0;
}
