// sokoban_gen.cpp — host-side Sokoban level generation with the reference's exact RNG streams.
//
// Replaces SokobanEnv.reset (sokoban/env.py:28-42) -> generate_room (sokoban/utils.py:221-278),
// room_topology_generation (:281-355), place_boxes_and_player (:358-397),
// reverse_playing (:408-437), depth_first_search (:440-498), reverse_move (:501-542),
// box_displacement_score (:545-560), add_random_player_movement (:152-213), all run under
// all_seed(seed) (ragen/utils.py:7-18).
//
// Reset is a recursive search (host work by design: SURVEY.md A5).  The two RNG streams are
// reproduced bit for bit:
//   * CPython `random` (Python 3.10): MT19937, seed(int) = init_by_array over the 32-bit
//     little-endian words of |seed|; random() = (a>>5, b>>6) 53-bit; _randbelow(n) =
//     rejection on getrandbits(n.bit_length()); randint/sample(k=1)/choice use _randbelow.
//   * numpy legacy `np.random` (RandomState): MT19937 init_genrand(seed & 0xffffffff);
//     randint(n) = masked rejection on 32-bit draws (no draw when n == 1).
// The DFS visits states in the reference's order (actions 0..3, first-visit wins, the
// explored set keyed on grid contents) so ties in room score resolve identically.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <thread>
#include <unordered_set>
#include <vector>
#include <string>

#define RMI_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

struct MT19937 {
  uint32_t mt[624];
  int mti = 625;
  void init_genrand(uint32_t s) {
    mt[0] = s;
    for (int i = 1; i < 624; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    mti = 624;
  }
  void init_by_array(const uint32_t* key, int len) {
    init_genrand(19650218u);
    int i = 1, j = 0;
    for (int k = (624 > len ? 624 : len); k; k--) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
      i++;
      j++;
      if (i >= 624) {
        mt[0] = mt[623];
        i = 1;
      }
      if (j >= len) j = 0;
    }
    for (int k = 623; k; k--) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
      i++;
      if (i >= 624) {
        mt[0] = mt[623];
        i = 1;
      }
    }
    mt[0] = 0x80000000u;
  }
  uint32_t next() {
    static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
    uint32_t y;
    if (mti >= 624) {
      int kk;
      for (kk = 0; kk < 624 - 397; kk++) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
      }
      for (; kk < 623; kk++) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
      }
      y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
      mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1u];
      mti = 0;
    }
    y = mt[mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
};

struct PyRandom {  // CPython 3.10 random.Random
  MT19937 g;
  void seed(int64_t s) {
    uint64_t a = s < 0 ? (uint64_t)(-s) : (uint64_t)s;
    uint32_t key[2];
    int n = 0;
    if (a == 0) {
      key[0] = 0;
      n = 1;
    } else {
      while (a) {
        key[n++] = (uint32_t)(a & 0xffffffffu);
        a >>= 32;
      }
    }
    g.init_by_array(key, n);
  }
  double random() {
    uint32_t a = g.next() >> 5, b = g.next() >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
  }
  uint32_t getrandbits(int k) { return k == 0 ? 0u : (g.next() >> (32 - k)); }
  int randbelow(int n) {
    int k = 0;
    for (int x = n; x; x >>= 1) k++;  // n.bit_length()
    uint32_t r = getrandbits(k);
    while ((int64_t)r >= n) r = getrandbits(k);
    return (int)r;
  }
  int randint(int a, int b) { return a + randbelow(b - a + 1); }
};

struct NpLegacy {  // numpy RandomState (legacy MT19937)
  MT19937 g;
  void seed(int64_t s) { g.init_genrand((uint32_t)((uint64_t)s & 0xffffffffu)); }
  int randint(int n) {  // np.random.randint(n): masked rejection, rng = n - 1
    const uint32_t rng = (uint32_t)(n - 1);
    if (rng == 0) return 0;
    uint32_t mask = rng;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t v;
    while ((v = (g.next() & mask)) > rng) {
    }
    return (int)v;
  }
};

const int CH[4][2] = {{-1, 0}, {1, 0}, {0, -1}, {0, 1}};  // CHANGE_COORDINATES

// The reverse-play search for rooms with <= 64 open cells, <= 256 cells and <= 16 boxes (every
// size RAGEN configures): Gen::dfs's visits in Gen::dfs's order with the same scores and the
// same explored-set semantics, without its allocations: the state lives in fixed arrays on the
// stack, the player's cell is carried instead of rescanned, and the explored set is an
// open-addressing table of 128-bit keys packing the grid (2 bits per open cell: its structure
// value, box 3, box 4, player 5 — given the fixed structure, the same information as the grid
// contents the reference keys on).  About 10x the speed of the std::string-keyed search.
struct FastSearch {
  static constexpr int kMaxHW = 256, kMaxOpen = 64, kMaxBoxes = 16;
  static constexpr size_t kCap = 300000;  // depth_first_search's explored-set limit
  int HW = 0, W = 0, nopen = 0, num_boxes = 0;
  int8_t slot[kMaxHW];  // open cell -> its 2-bit field in the key (-1: wall)
  int8_t structure[kMaxHW];
  int tr[kMaxBoxes], tc[kMaxBoxes];  // box_mapping keys (targets, insertion order)
  // explored set: 16-B slots, the all-zero key free (a grid always holds the player: code 3)
  struct Slot {
    uint64_t a, b;
  };
  std::vector<Slot> tab;
  size_t count = 0, mask = 0;
  // best
  long best_score = -1;
  int8_t best_room[kMaxHW];
  int best_r[kMaxBoxes], best_c[kMaxBoxes];
  bool have_best = false;

  static bool usable(const std::vector<int8_t>& state, const std::vector<int8_t>& st_struct, int HW, int nb) {
    if (HW > kMaxHW || nb > kMaxBoxes) return false;
    int open = 0, players = 0;
    for (int i = 0; i < HW; ++i) {
      open += st_struct[i] != 0;
      players += state[i] == 5;
    }
    return open <= kMaxOpen && players == 1;
  }
  static uint64_t mix(uint64_t x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
  }
  void clear_set() {
    if (tab.size() != 4096) tab.assign(4096, Slot{0, 0});
    else std::fill(tab.begin(), tab.end(), Slot{0, 0});
    mask = 4095;
    count = 0;
  }
  // -> true if the key was absent (and is now present)
  bool insert(uint64_t a, uint64_t b) {
    if (2 * (count + 1) > mask + 1) grow();
    size_t h = mix(a ^ mix(b)) & mask;
    for (;; h = (h + 1) & mask) {
      Slot& e = tab[h];
      if ((e.a | e.b) == 0) {
        e.a = a;
        e.b = b;
        ++count;
        return true;
      }
      if (e.a == a && e.b == b) return false;
    }
  }
  void grow() {
    std::vector<Slot> old;
    old.swap(tab);
    tab.assign(old.size() * 2, Slot{0, 0});
    mask = tab.size() - 1;
    count = 0;
    for (const Slot& e : old)
      if (e.a | e.b) insert(e.a, e.b);
  }
  static uint64_t code(int v) { return v == 5 ? 3u : (v == 4 ? 2u : (v == 3 ? 1u : 0u)); }
  // cell i changes from value u to v: the key's field follows
  void rekey(uint64_t& a, uint64_t& b, int i, int u, int v) const {
    const int j = slot[i];
    const uint64_t d = code(u) ^ code(v);
    if (j < 32) a ^= d << (2 * j);
    else b ^= d << (2 * (j - 32));
  }
  long displacement(const int* br, const int* bc) const {
    long s = 0;
    for (int k = 0; k < num_boxes; ++k) s += std::abs(br[k] - tr[k]) + std::abs(bc[k] - tc[k]);
    return s;
  }
  // state's key (a, b) and its count of value-2 cells (n2) are carried, updated per move
  void dfs(const int8_t* state, uint64_t a, uint64_t b, int n2, int pi, const int* br, const int* bc, long box_swaps,
           int last_pull, int ttl) {
    ttl -= 1;
    if (ttl <= 0 || count >= kCap) return;
    if (!insert(a, b)) return;  // explored (nothing reads the set between the test and the insert)
    long score = box_swaps * displacement(br, bc);
    if (n2 != num_boxes) score = 0;
    if (score > best_score) {
      memcpy(best_room, state, HW);
      memcpy(best_r, br, sizeof(int) * num_boxes);
      memcpy(best_c, bc, sizeof(int) * num_boxes);
      best_score = score;
      have_best = true;
    }
    const int prow = pi / W, pcol = pi % W;
    for (int action = 0; action < 4; ++action) {  // reverse_move, then the recursion
      const int nr = prow + CH[action][0], nc = pcol + CH[action][1];
      const int ni = nr * W + nc;
      if (!(state[ni] == 1 || state[ni] == 2)) {  // no move: the same state, explored already
        dfs(state, a, b, n2, pi, br, bc, box_swaps, last_pull, ttl);
        continue;
      }
      int8_t nxt[kMaxHW];
      int nr_[kMaxBoxes], nc_[kMaxBoxes];
      memcpy(nxt, state, HW);
      memcpy(nr_, br, sizeof(int) * num_boxes);
      memcpy(nc_, bc, sizeof(int) * num_boxes);
      uint64_t na = a, nb = b;
      int nn2 = n2, lp = last_pull;
      auto set = [&](int i, int v) {
        rekey(na, nb, i, nxt[i], v);
        nn2 += (v == 2) - (nxt[i] == 2);
        nxt[i] = (int8_t)v;
      };
      set(pi, structure[pi]);
      set(ni, 5);
      const int brow = prow - CH[action][0], bcol = pcol - CH[action][1];
      const int bi = brow * W + bcol;
      if (nxt[bi] == 3 || nxt[bi] == 4) {
        set(pi, 3);
        set(bi, structure[bi]);
        for (int k = 0; k < num_boxes; ++k)
          if (nr_[k] == brow && nc_[k] == bcol) {
            nr_[k] = prow;
            nc_[k] = pcol;
            lp = k;
          }
      }
      dfs(nxt, na, nb, nn2, ni, nr_, nc_, box_swaps + (lp != last_pull ? 1 : 0), lp, ttl);
    }
  }
};

struct Gen {
  int H, W, HW;
  PyRandom pr;
  NpLegacy np;
  // reverse-play search state
  int num_boxes = 0;
  std::unordered_set<std::string> explored;
  long best_score = -1;
  std::vector<int8_t> best_room;
  std::vector<std::pair<int, int>> best_map;  // box_mapping values, keyed by target order
  std::vector<std::pair<int, int>> targets;   // box_mapping keys (insertion order)
  FastSearch fast;                            // the allocation-free search (most rooms)
  bool force_string_search = false;           // RMI_SOKOBAN_GEN_STRING_SEARCH=1 (A/B tests)

  int at(int r, int c) const { return r * W + c; }

  // room_topology_generation(dim, p_change_directions=0.35, num_steps)
  std::vector<int> topology(int num_steps) {
    static const int masks[5][3][3] = {{{0, 0, 0}, {1, 1, 1}, {0, 0, 0}},
                                       {{0, 1, 0}, {0, 1, 0}, {0, 1, 0}},
                                       {{0, 0, 0}, {1, 1, 0}, {0, 1, 0}},
                                       {{0, 0, 0}, {1, 1, 0}, {1, 1, 0}},
                                       {{0, 0, 0}, {0, 1, 1}, {0, 1, 0}}};
    static const int dirs[4][2] = {{1, 0}, {0, 1}, {-1, 0}, {0, -1}};
    int d = pr.randbelow(4);
    int p0 = pr.randint(1, H - 1);
    int p1 = pr.randint(1, W - 1);
    std::vector<int> level(HW, 0);
    for (int s = 0; s < num_steps; ++s) {
      if (pr.random() < 0.35) d = pr.randbelow(4);
      p0 += dirs[d][0];
      p1 += dirs[d][1];
      p0 = std::max(std::min(p0, H - 2), 1);
      p1 = std::max(std::min(p1, W - 2), 1);
      const int m = pr.randbelow(5);
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          const int rr = p0 - 1 + i, cc = p1 - 1 + j;
          if (rr >= 0 && rr < H && cc >= 0 && cc < W) level[at(rr, cc)] += masks[m][i][j];
        }
    }
    for (int i = 0; i < HW; ++i) level[i] = level[i] > 0 ? 1 : 0;
    for (int r = 0; r < H; ++r) level[at(r, 0)] = level[at(r, W - 1)] = 0;
    for (int c = 0; c < W; ++c) level[at(0, c)] = level[at(H - 1, c)] = 0;
    return level;
  }

  // place_boxes_and_player(room, num_boxes, second_player=False); false => RuntimeError
  bool place(std::vector<int>& room, int nboxes) {
    std::vector<int> pos;
    for (int i = 0; i < HW; ++i)
      if (room[i] == 1) pos.push_back(i);
    if ((int)pos.size() <= nboxes + 1) return false;
    room[pos[np.randint((int)pos.size())]] = 5;
    for (int n = 0; n < nboxes; ++n) {
      pos.clear();
      for (int i = 0; i < HW; ++i)
        if (room[i] == 1) pos.push_back(i);
      room[pos[np.randint((int)pos.size())]] = 2;
    }
    return true;
  }

  static long displacement(const std::vector<std::pair<int, int>>& keys,
                           const std::vector<std::pair<int, int>>& vals) {
    long s = 0;
    for (size_t i = 0; i < keys.size(); ++i)
      s += std::abs(vals[i].first - keys[i].first) + std::abs(vals[i].second - keys[i].second);
    return s;
  }

  void dfs(const std::vector<int8_t>& state, const std::vector<int8_t>& structure,
           const std::vector<std::pair<int, int>>& bmap, long box_swaps, int last_pull, int ttl) {
    ttl -= 1;
    if (ttl <= 0 || explored.size() >= 300000) return;
    std::string key(reinterpret_cast<const char*>(state.data()), state.size());
    if (explored.count(key)) return;
    long score = box_swaps * displacement(targets, bmap);
    int n2 = 0;
    for (int i = 0; i < HW; ++i) n2 += state[i] == 2;
    if (n2 != num_boxes) score = 0;
    if (score > best_score) {
      best_room = state;
      best_score = score;
      best_map = bmap;
    }
    explored.insert(std::move(key));
    for (int action = 0; action < 4; ++action) {
      std::vector<int8_t> nxt = state;
      std::vector<std::pair<int, int>> nmap = bmap;
      int lp = last_pull;
      reverse_move(nxt, structure, nmap, lp, action);
      dfs(nxt, structure, nmap, box_swaps + (lp != last_pull ? 1 : 0), lp, ttl);
    }
  }

  // reverse_move; last_pull is the index of the pulled box's target key (-1 = none)
  void reverse_move(std::vector<int8_t>& st, const std::vector<int8_t>& structure,
                    std::vector<std::pair<int, int>>& bmap, int& last_pull, int action) {
    int pi = -1;
    for (int i = 0; i < HW; ++i)
      if (st[i] == 5) {
        pi = i;
        break;
      }
    const int pr_ = pi / W, pc = pi % W;
    const int nr = pr_ + CH[action % 4][0], nc = pc + CH[action % 4][1];
    const int ni = at(nr, nc);
    if (st[ni] == 1 || st[ni] == 2) {
      st[pi] = structure[pi];
      st[ni] = 5;
      if (action < 4) {
        const int br = pr_ - CH[action % 4][0], bc = pc - CH[action % 4][1];
        const int bi = at(br, bc);
        if (st[bi] == 3 || st[bi] == 4) {
          st[pi] = 3;
          st[bi] = structure[bi];
          for (size_t k = 0; k < bmap.size(); ++k)
            if (bmap[k].first == br && bmap[k].second == bc) {
              bmap[k] = {pr_, pc};
              last_pull = (int)k;
            }
        }
      }
    }
  }

  // returns 0 ok, 1 RuntimeError/RuntimeWarning
  int generate(int64_t seed, int num_gen_steps, int nboxes, int search_depth, uint8_t* out_fixed,
               uint8_t* out_state, int8_t* out_player) {
    pr.seed(seed);
    np.seed(seed);
    std::vector<int8_t> room_state, room_structure;
    long score = 0;
    for (int t = 0; t < 4; ++t) {  // tries=4
      std::vector<int> room = topology(num_gen_steps);
      if (!place(room, nboxes)) return 1;
      room_structure.assign(HW, 0);
      room_state.assign(HW, 0);
      for (int i = 0; i < HW; ++i) {
        room_structure[i] = (int8_t)(room[i] == 5 ? 1 : room[i]);
        room_state[i] = (int8_t)(room[i] == 2 ? 4 : room[i]);
      }
      // reverse_playing
      targets.clear();
      for (int i = 0; i < HW; ++i)
        if (room_structure[i] == 2) targets.push_back({i / W, i % W});
      num_boxes = (int)targets.size();
      if (!force_string_search && FastSearch::usable(room_state, room_structure, HW, num_boxes)) {
        FastSearch& f = fast;
        f.HW = HW;
        f.W = W;
        f.num_boxes = num_boxes;
        f.nopen = 0;
        int pi = 0, n2 = 0;
        uint64_t ka = 0, kb = 0;
        for (int i = 0; i < HW; ++i) {
          f.structure[i] = room_structure[i];
          f.slot[i] = (int8_t)(room_structure[i] != 0 ? f.nopen++ : -1);
          if (f.slot[i] >= 0) f.rekey(ka, kb, i, room_structure[i], room_state[i]);
          if (room_state[i] == 5) pi = i;
          n2 += room_state[i] == 2;
        }
        int br[FastSearch::kMaxBoxes], bc[FastSearch::kMaxBoxes];
        for (int k = 0; k < num_boxes; ++k) {
          f.tr[k] = br[k] = targets[k].first;
          f.tc[k] = bc[k] = targets[k].second;
        }
        f.clear_set();
        f.best_score = -1;
        f.have_best = false;
        f.dfs(room_state.data(), ka, kb, n2, pi, br, bc, 0, -1, search_depth);
        if (!f.have_best) return 1;  // search_depth <= 1: reference would fail later
        room_state.assign(f.best_room, f.best_room + HW);
        best_map.clear();
        for (int k = 0; k < num_boxes; ++k) best_map.push_back({f.best_r[k], f.best_c[k]});
      } else {
        explored.clear();
        best_score = -1;
        best_room.clear();
        best_map = targets;
        dfs(room_state, room_structure, targets, 0, -1, search_depth);
        if (best_room.empty()) return 1;  // search_depth <= 1: reference would fail later
        room_state = best_room;
      }
      for (int i = 0; i < HW; ++i)
        if (room_state[i] == 3) room_state[i] = 4;
      score = displacement(targets, best_map);
      if (score > 0) break;
    }
    if (score == 0) return 1;  // RuntimeWarning('Generated Model with score == 0')
    // add_random_player_movement
    const double move_p = score == 1 ? 0.8 : 0.5;
    if (!(pr.random() > move_p)) {
      int pi = -1;
      for (int i = 0; i < HW; ++i)
        if (room_state[i] == 5) {
          pi = i;
          break;
        }
      int p0 = pi / W, p1 = pi % W;
      std::vector<std::pair<int, int>> prev = {{p0, p1}};
      int steps = 0;
      while (steps < 3) {
        int va[4], vr[4], vc[4], nv = 0;
        for (int a = 0; a < 4; ++a) {
          const int r = p0 + CH[a][0], c = p1 + CH[a][1];
          const int v = room_state[at(r, c)];
          if ((v == 1 || v == 2) &&
              std::find(prev.begin(), prev.end(), std::make_pair(r, c)) == prev.end()) {
            va[nv] = a;
            vr[nv] = r;
            vc[nv] = c;
            nv++;
          }
        }
        if (!nv) break;
        const int k = pr.randbelow(nv);  // random.choice(valid_moves)
        (void)va;
        room_state[at(p0, p1)] = room_structure[at(p0, p1)];
        room_state[at(vr[k], vc[k])] = 5;
        p0 = vr[k];
        p1 = vc[k];
        prev.push_back({p0, p1});
        steps++;
        if (steps >= 3 || pr.random() > 0.5) break;
      }
    }
    int pi = -1;
    for (int i = 0; i < HW; ++i) {
      out_fixed[i] = (uint8_t)room_structure[i];
      out_state[i] = (uint8_t)room_state[i];
      if (pi < 0 && room_state[i] == 5) pi = i;
    }
    out_player[0] = (int8_t)(pi / W);
    out_player[1] = (int8_t)(pi % W);
    return 0;
  }
};

}  // namespace

RMI_HOST_API int rmi_sokoban_generate_rooms(const int64_t* seeds, int32_t n, int32_t H, int32_t W, int32_t num_boxes,
                                            int32_t search_depth, uint8_t* room_fixed, uint8_t* room_state,
                                            int8_t* player, uint8_t* status, int32_t n_threads) {
  if (!seeds || !room_fixed || !room_state || !player || !status || n < 0 || H < 3 || W < 3 || H * W > 4096)
    return -1;
  for (int i = 0; i < n; ++i)
    if (seeds[i] < 0 || seeds[i] > 0xffffffffLL) return -1;  // np.random.seed range
  const int num_gen_steps = (int)(1.7 * (H + W));  // gym_sokoban ctor
  const int HW = H * W;
  const char* ss = getenv("RMI_SOKOBAN_GEN_STRING_SEARCH");  // the std::string-keyed search (tests)
  const bool string_search = ss && ss[0] == '1';
  auto work = [&](int lo, int hi) {
    for (int i = lo; i < hi; ++i) {
      Gen g;
      g.force_string_search = string_search;
      g.H = H;
      g.W = W;
      g.HW = HW;
      status[i] = (uint8_t)g.generate(seeds[i], num_gen_steps, num_boxes, search_depth, room_fixed + (int64_t)i * HW,
                                      room_state + (int64_t)i * HW, player + 2 * (int64_t)i);
    }
  };
  int nt = n_threads > 0 ? n_threads : 1;
  if (nt > n) nt = n > 0 ? n : 1;
  if (nt == 1) {
    work(0, n);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(work, (int)((int64_t)n * t / nt), (int)((int64_t)n * (t + 1) / nt));
    for (auto& x : th) x.join();
  }
  return 0;
}

struct rmi_rooms_job {
  std::thread th;
  int rc = 0;
};

RMI_HOST_API rmi_rooms_job* rmi_sokoban_generate_rooms_start(const int64_t* seeds, int32_t n, int32_t H, int32_t W,
                                                             int32_t num_boxes, int32_t search_depth,
                                                             uint8_t* room_fixed, uint8_t* room_state, int8_t* player,
                                                             uint8_t* status, int32_t n_threads) {
  rmi_rooms_job* j = new (std::nothrow) rmi_rooms_job;
  if (!j) return nullptr;
  try {
    j->th = std::thread([=] {
      j->rc = rmi_sokoban_generate_rooms(seeds, n, H, W, num_boxes, search_depth, room_fixed, room_state, player,
                                         status, n_threads);
    });
  } catch (...) {
    delete j;
    return nullptr;
  }
  return j;
}

RMI_HOST_API int rmi_sokoban_generate_rooms_wait(rmi_rooms_job* job) {
  if (!job) return -1;
  job->th.join();
  const int rc = job->rc;
  delete job;
  return rc;
}
