/*
 * ragen_oracle.h — CPU restatement of RAGEN's rollout/advantage hot path.
 *
 * TEST INFRASTRUCTURE (the parity oracle).  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it, and only as the checker — never as the thing
 * measured or shipped.  Plain C, one env / one row at a time, written from the reference's
 * Python (file:line cited per function) independently of the HIP kernels.
 *
 * Pinned by tests/test_oracle.py against golden vectors recorded by running the reference
 * itself (tests/golden/make_golden.py).  Third-party semantics the reference calls but does
 * not vendor (gym_sokoban step, gymnasium FrozenLake, numpy PCG64, verl GAE/whiten/GRPO)
 * follow SURVEY.md Appendix A and are pinned through the same recorded traces.
 *
 * Layouts are the product's HBM layouts (include/ragen_amd.h) but on host memory.
 */
#ifndef RAGEN_ORACLE_H
#define RAGEN_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* episode status, identical meaning to rmi_episode_t */
typedef struct {
  int32_t B, T;
  int32_t* num_actions;
  uint8_t* flags;
  int32_t* n_turns;
  double* penalty;
  double* turn_reward; /* [T,B] */
  uint8_t* turn_info;  /* [T,B] */
  uint8_t* turn_exec;  /* [T,B] */
} orc_episode_t;

typedef struct {
  int32_t turn, K;
  const int8_t* actions;   /* [B,K] */
  const uint8_t* n_actions;
  const uint8_t* has_input; /* NULL = not-done envs */
  int32_t max_actions_per_traj;
  double format_penalty;
} orc_turn_t;

int orc_sokoban_turn(int32_t H, int32_t W, int32_t num_boxes, int32_t max_steps, const uint8_t* room_fixed,
                     uint8_t* room_state, int8_t* player, int32_t* num_env_steps, int32_t* boxes_on_target,
                     orc_episode_t* ep, const orc_turn_t* in, uint8_t* err);

int orc_frozenlake_turn(int32_t nrow, int32_t ncol, int32_t is_slippery, double cs0, double cs1, double cs2,
                        const uint8_t* desc, int32_t* s, uint64_t* rng /*[4,B]*/, orc_episode_t* ep,
                        const orc_turn_t* in, uint8_t* err);

int orc_bandit_turn(int32_t start, double lo, double hi_lo, double hi_hi, double hi_prob, const uint8_t* hi_is_first,
                    uint64_t* rng, orc_episode_t* ep, const orc_turn_t* in, uint8_t* err);

double orc_pcg64_random(uint64_t st[4]); /* st = {state_hi, state_lo, inc_hi, inc_lo} */

/* get_masks_and_scores (ctx_manager.py:35-70).  flags: 1 turn scores, 2 response mask, 4 roll (Qwen). */
int orc_masks_and_scores(const int64_t* ids, int64_t B, int64_t S, int64_t sp, int64_t rt, const double* scores,
                         const int32_t* n_scores, int32_t T, int32_t n_slots, int32_t flags, float* score_out,
                         uint8_t* loss_mask, uint8_t* response_mask, uint8_t* err);

void orc_rollout_metrics(const orc_episode_t* ep, double* out /*[B,4]*/);
void orc_trajectory_scores(const orc_episode_t* ep, float* score, float* pen);
void orc_group_normalize(const float* score, const float* pen, const int32_t* seg, int32_t G, int32_t B, int32_t method,
                         float* out);

void orc_gae(const float* r, const float* v, const uint8_t* mask, int64_t B, int64_t L, double gamma, double lam,
             int32_t variant, float* adv, float* ret);
int orc_bilevel_gae(const float* r, const float* v, const uint8_t* mask, int64_t B, int64_t L, double gamma,
                    double lam, double hlg, float* adv, float* ret, uint8_t* err);
int orc_masked_whiten(float* x, const uint8_t* mask, int64_t B, int64_t L);
void orc_grpo(const float* r, const uint8_t* mask, int64_t B, int64_t L, const int32_t* seg, int32_t G, double eps,
              int32_t norm_by_std, float* adv, float* ret);
void orc_reinforce_pp(const float* r, const uint8_t* mask, int64_t B, int64_t L, double gamma, float* ret);
void orc_remax(const float* r, const uint8_t* mask, const float* base, int64_t B, int64_t L, float* adv, float* ret);
void orc_rloo(const float* r, const uint8_t* mask, int64_t B, int64_t L, const int32_t* seg, int32_t G, float* adv);
void orc_filter(const float* scores, int32_t G, int32_t gs, double ratio, int32_t type, float* g_std, float* g_max,
                float* g_mean, uint8_t* keep, double* metrics);

#ifdef __cplusplus
}
#endif
#endif
