// Sanitizer driver (TEST INFRASTRUCTURE): the host C++ room generator
// (ragen_amd/csrc/sokoban_gen.cpp) and the C oracle (oracle/ragen_oracle.c), built with
// -fsanitize=address,undefined by tests/test_sanitize.py and run over the golden seeds.
//
//   san_driver H num_boxes search_depth n_threads seeds.bin out.bin
//
// Generates the rooms of every seed (int64 LE in seeds.bin) and writes fixed | state | player |
// status to out.bin for the test to compare with the golden rooms; then drives every oracle
// entry point over those rooms and small seeded rows (5 Sokoban turns, FrozenLake, Bandit,
// masks / scores, metrics, normalisation, GAE, bi-level GAE, whitening, GRPO, REINFORCE++,
// REMAX, RLOO, filter), so that any out-of-bounds access or undefined operation aborts.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../oracle/ragen_oracle.h"

extern "C" int rmi_sokoban_generate_rooms(const int64_t* seeds, int32_t n, int32_t H, int32_t W, int32_t num_boxes,
                                          int32_t search_depth, uint8_t* room_fixed, uint8_t* room_state,
                                          int8_t* player, uint8_t* status, int32_t n_threads);

namespace {

uint64_t g_state = 0x9E3779B97F4A7C15ull;
uint32_t rnd() {  // splitmix64, fixed seed: the driver is deterministic
  uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)((z ^ (z >> 31)) >> 32);
}
float frnd() { return (float)((int)(rnd() % 2001) - 1000) / 500.f; }

struct Episode {
  int B, T;
  std::vector<int32_t> num_actions, n_turns;
  std::vector<uint8_t> flags, turn_info, turn_exec;
  std::vector<double> penalty, turn_reward;
  orc_episode_t v;
  Episode(int B_, int T_)
      : B(B_), T(T_), num_actions(B_), n_turns(B_), flags(B_), turn_info((size_t)T_ * B_), turn_exec((size_t)T_ * B_),
        penalty(B_), turn_reward((size_t)T_ * B_) {
    v = orc_episode_t{B, T, num_actions.data(), flags.data(), n_turns.data(), penalty.data(), turn_reward.data(),
                      turn_info.data(), turn_exec.data()};
  }
};

void turn_inputs(int B, int K, int lo, int hi, std::vector<int8_t>& act, std::vector<uint8_t>& n) {
  for (int b = 0; b < B; ++b) {
    n[b] = (uint8_t)(rnd() % (K + 1));
    for (int k = 0; k < K; ++k) act[(size_t)b * K + k] = (int8_t)(rnd() % 10 == 0 ? 0 : lo + (int)(rnd() % (hi - lo + 1)));
  }
}

void advantage_family(double* sink) {
  const int B = 37, L = 91, G = 5;
  std::vector<float> r((size_t)B * L), v((size_t)B * L), adv((size_t)B * L), ret((size_t)B * L), base(B);
  std::vector<uint8_t> m((size_t)B * L), err(B);
  for (int b = 0; b < B; ++b) {
    int start = (int)(rnd() % 40);
    base[b] = frnd();
    for (int l = 0; l < L; ++l) {
      size_t i = (size_t)b * L + l;
      m[i] = l >= start && rnd() % 4 != 0;
      r[i] = rnd() % 7 == 0 ? frnd() : 0.f;
      v[i] = frnd() * m[i];
    }
    r[(size_t)b * L + L - 1] = 1.f;
    m[(size_t)b * L + L - 1] = 1;
  }
  std::vector<int32_t> seg = {0, 3, 10, 11, 30, B};
  for (int variant = 0; variant < 2; ++variant) {
    orc_gae(r.data(), v.data(), m.data(), B, L, 1.0, 0.95, variant, adv.data(), ret.data());
    *sink += adv[5] + ret[7];
  }
  orc_bilevel_gae(r.data(), v.data(), m.data(), B, L, 1.0, 0.95, 0.95, adv.data(), ret.data(), err.data());
  orc_masked_whiten(adv.data(), m.data(), B, L);
  orc_grpo(r.data(), m.data(), B, L, seg.data(), G, 1e-6, 1, adv.data(), ret.data());
  orc_reinforce_pp(r.data(), m.data(), B, L, 0.99, ret.data());
  orc_remax(r.data(), m.data(), base.data(), B, L, adv.data(), ret.data());
  orc_rloo(r.data(), m.data(), B, L, seg.data(), G, adv.data());
  *sink += adv[11] + ret[13];
}

void masks_family(double* sink) {
  const int64_t B = 23, S = 77, SP = 151644, RT = 151645;
  const int T = 4;
  std::vector<int64_t> ids((size_t)(B * S));
  for (auto& x : ids) x = rnd() % 9 == 0 ? SP : (rnd() % 13 == 0 ? RT : 100 + rnd() % 900);
  std::vector<double> sc((size_t)T * B);
  for (auto& x : sc) x = frnd();
  std::vector<int32_t> nsc(B);
  for (auto& x : nsc) x = (int32_t)(rnd() % (T + 1));
  std::vector<float> so((size_t)(B * (S - 1)));
  std::vector<uint8_t> lm(so.size()), rm(so.size()), err(B);
  for (int flags = 0; flags < 8; ++flags) {
    orc_masks_and_scores(ids.data(), B, S, SP, RT, sc.data(), nsc.data(), T, T, flags, so.data(), lm.data(), rm.data(),
                         err.data());
    *sink += so[(size_t)flags * 3] + lm[flags] + rm[flags];
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 7) {
    std::fprintf(stderr, "usage: %s H num_boxes search_depth n_threads seeds.bin out.bin\n", argv[0]);
    return 2;
  }
  const int H = std::atoi(argv[1]), nb = std::atoi(argv[2]), sd = std::atoi(argv[3]), nt = std::atoi(argv[4]);
  std::FILE* f = std::fopen(argv[5], "rb");
  if (!f) return 2;
  std::vector<int64_t> seeds;
  int64_t s;
  while (std::fread(&s, sizeof s, 1, f) == 1) seeds.push_back(s);
  std::fclose(f);
  const int n = (int)seeds.size(), HW = H * H;
  std::vector<uint8_t> fixed((size_t)n * HW), state((size_t)n * HW), status(n);
  std::vector<int8_t> player((size_t)n * 2);
  if (rmi_sokoban_generate_rooms(seeds.data(), n, H, H, nb, sd, fixed.data(), state.data(), player.data(),
                                 status.data(), nt) != 0)
    return 3;
  std::FILE* o = std::fopen(argv[6], "wb");
  if (!o) return 2;
  std::fwrite(fixed.data(), 1, fixed.size(), o);
  std::fwrite(state.data(), 1, state.size(), o);
  std::fwrite(player.data(), 1, player.size(), o);
  std::fwrite(status.data(), 1, status.size(), o);
  std::fclose(o);

  double sink = 0.0;
  // 5 Sokoban turns over the generated rooms (mixed ids incl. 0 = unknown name, cap 10)
  const int T = 5, K = 5;
  Episode ep(n, T);
  std::vector<int32_t> nes(n), bot(n);
  std::vector<int8_t> act((size_t)n * K);
  std::vector<uint8_t> na(n), err(n);
  for (int t = 0; t < T; ++t) {
    turn_inputs(n, K, 1, 4, act, na);
    orc_turn_t in{t, K, act.data(), na.data(), nullptr, 10, -0.1};
    orc_sokoban_turn(H, H, nb, 100, fixed.data(), state.data(), player.data(), nes.data(), bot.data(), &ep.v, &in,
                     err.data());
  }
  std::vector<double> met((size_t)n * 4);
  std::vector<float> score(n), pen(n), normed(n);
  orc_rollout_metrics(&ep.v, met.data());
  orc_trajectory_scores(&ep.v, score.data(), pen.data());
  std::vector<int32_t> seg;
  for (int g = 0; g <= n; g += 16) seg.push_back(g);
  if (seg.back() != n) seg.push_back(n);
  for (int method = 0; method < 4; ++method)
    orc_group_normalize(score.data(), pen.data(), seg.data(), (int)seg.size() - 1, n, method, normed.data());
  const int G = n / 16;
  if (G > 0) {
    std::vector<float> gs(G), gm(G), gmean(G);
    std::vector<uint8_t> keep(G);
    double fm[6];
    for (int type = 0; type < 2; ++type) orc_filter(score.data(), G, 16, 0.25, type, gs.data(), gm.data(), gmean.data(),
                                                    keep.data(), fm);
    sink += fm[0];
  }
  // FrozenLake 4x4 slippery and Bandit turns on seeded maps / PCG64 states
  {
    const int B = 64;
    std::vector<uint8_t> desc((size_t)B * 16);
    std::vector<int32_t> st(B);
    std::vector<uint64_t> rng((size_t)4 * B);
    for (int b = 0; b < B; ++b) {
      for (int c = 0; c < 16; ++c) desc[(size_t)b * 16 + c] = rnd() % 5 == 0 ? 'H' : 'F';
      desc[(size_t)b * 16] = 'S';
      desc[(size_t)b * 16 + 15] = 'G';
      st[b] = 0;
      for (int k = 0; k < 4; ++k) rng[(size_t)k * B + b] = ((uint64_t)rnd() << 32 | rnd()) | (k == 3 ? 1u : 0u);
    }
    Episode fe(B, 8);
    std::vector<int8_t> fa((size_t)B * K);
    std::vector<uint8_t> fn(B), fer(B), hi(B);
    for (int t = 0; t < 8; ++t) {
      turn_inputs(B, K, 1, 4, fa, fn);
      orc_turn_t in{t, K, fa.data(), fn.data(), nullptr, 10, -0.1};
      orc_frozenlake_turn(4, 4, 1, 1.0 / 3, 2.0 / 3, 1.0, desc.data(), st.data(), rng.data(), &fe.v, &in, fer.data());
    }
    Episode be(B, 1);
    for (int b = 0; b < B; ++b) hi[b] = rnd() & 1;
    turn_inputs(B, 1, 1, 2, fa, fn);
    orc_turn_t bin{0, 1, fa.data(), fn.data(), nullptr, 1, -0.1};
    orc_bandit_turn(0, 0.1, 1.0, 0.0, 0.25, hi.data(), rng.data(), &be.v, &bin, fer.data());
    uint64_t p4[4] = {1, 2, 3, 5};
    sink += orc_pcg64_random(p4) + fe.turn_reward[3] + be.turn_reward[1];
  }
  advantage_family(&sink);
  masks_family(&sink);
  std::printf("rooms %d, checksum %.6f\n", n, sink + met[0] + normed[0]);
  return 0;
}
