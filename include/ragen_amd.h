/*
 * ragen_amd.h — C ABI of the MI355X (gfx950) rollout-and-advantage engine.
 *
 * Drop-in boundary for RAGEN's StarPO hot path (quanwei0/RAGEN @ 2025-07-04).
 * The reference is pure Python; every entry point below replaces a Python loop of the
 * reference, cited per function as  <file>:<line>  relative to the reference root.
 *
 * Conventions
 *  - All pointers are DEVICE pointers (hipMalloc / torch CUDA tensors) unless marked
 *    [host].  The caller owns every buffer; no entry point allocates, frees or
 *    synchronises.  Work is enqueued on `stream` (a hipStream_t; NULL = default stream).
 *  - Env state is updated IN PLACE (the reference mutates env objects in place,
 *    es_manager.py:161-167).
 *  - Return value: RMI_OK (0) when the launch was enqueued; a negative code for an
 *    invalid argument or a HIP launch failure.  Data-dependent errors that the reference
 *    raises as Python exceptions (e.g. IndexError in bi-level GAE, core_algos.py:79)
 *    are reported per row through the optional `err` buffer (u8[B], bit set = error),
 *    readable after the stream has been synchronised.
 *  - Per-turn episode outputs are stored turn-major ([T, B]) so each per-turn kernel
 *    writes one contiguous row of B elements (coalesced).
 */
#ifndef RAGEN_AMD_H
#define RAGEN_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* rmi_stream_t; /* hipStream_t */

enum {
  RMI_OK = 0,
  RMI_EINVAL = -1,  /* bad pointer / shape / parameter */
  RMI_EDEVICE = -2, /* HIP runtime reported an error on launch */
  RMI_EUNSUP = -3   /* configuration outside the kernels' supported envelope */
};

/* Episode-status flag bits (A1: EnvStatus, es_manager.py:17-24). */
enum {
  RMI_FLAG_TERMINATED = 1, /* EnvStatus.terminated */
  RMI_FLAG_TRUNCATED = 2,  /* EnvStatus.truncated */
  RMI_FLAG_DONE = 4        /* env no longer returned by step() (es_manager.py:168-169) */
};

/* Per-turn info bits (the turn_info dict of es_manager.py:116-128). */
enum {
  RMI_INFO_PRESENT = 1,   /* >=1 action executed this turn (turn_info non-empty) */
  RMI_INFO_EFFECTIVE = 2, /* info['action_is_effective'] of the last executed action */
  RMI_INFO_VALID = 4,     /* info['action_is_valid'] */
  RMI_INFO_SUCCESS = 8    /* info['success'] */
};

/* Per-row error bits written to an optional err buffer. */
enum {
  RMI_ERR_ACTION = 1,  /* action id outside the env's action space */
  RMI_ERR_INDEX = 2,   /* grid index out of range (numpy would raise IndexError) */
  RMI_ERR_STATE = 4,   /* malformed state (e.g. grid byte > 7) */
  RMI_ERR_UNSUP = 8    /* expression outside the Countdown evaluator's grammar */
};

/* ------------------------------------------------------------------ A1 episode status
 * Replaces: EnvStatus + rollout_cache bookkeeping of EnvStateManager
 *           (es_manager.py:17-24, :85, :130-144, :158-169).                          */
typedef struct {
  int32_t B;             /* number of envs in this batch (one env tag)                  */
  int32_t T;             /* rows of the per-turn outputs (>= max_turn), <= 255          */
  uint8_t* num_actions;  /* [B]  EnvStatus.num_actions (<= max_actions_per_traj <= 255)  */
  uint8_t* flags;        /* [B]  RMI_FLAG_* bits                                        */
  uint8_t* n_turns;      /* [B]  turns stepped = len(history) - 1 (<= T <= 255)         */
  double* penalty;       /* [B]  rollout_cache[env]['penalty'] (format penalty sum)     */
  double* turn_reward;   /* [T,B] acc_reward of each turn (EnvStatus.rewards)           */
  uint8_t* turn_info;    /* [T,B] RMI_INFO_* bits                                       */
  uint8_t* turn_exec;    /* [T,B] number of actions executed in the turn                */
} rmi_episode_t;

/* Common per-turn inputs (what ContextManager.get_env_inputs hands to
 * EnvStateManager.step, ctx_manager.py:332-352, after name->id mapping
 * es_manager.py:230-240).                                                              */
typedef struct {
  int32_t turn;                /* row of the per-turn outputs to write                  */
  int32_t K;                   /* max actions per turn (agent_proxy.max_actions_per_turn) */
  const int8_t* actions;       /* [B,K] mapped action ids; 0 = name not in action_lookup  */
  const uint8_t* n_actions;    /* [B]  number of parsed action strings (len(actions))     */
  const uint8_t* has_input;    /* [B]  1 = env receives an input this turn; NULL = every
                                  env whose RMI_FLAG_DONE bit is clear                     */
  int32_t max_actions_per_traj;/* custom_envs.<tag>.max_actions_per_traj, 1..255 (u8
                                  counters; a larger cap is RMI_EUNSUP)                    */
  double format_penalty;       /* es_manager.format_penalty                               */
} rmi_turn_t;

/* ------------------------------------------------------------------------ Sokoban
 * Replaces: EnvStateManager.step (es_manager.py:105-171) driving SokobanEnv.step
 *           (sokoban/env.py:44-51) -> gym_sokoban SokobanEnv.step/_push/_move/_calc_reward
 *           (third-party, restated in SURVEY.md App. A.1).
 * One launch executes one whole turn (up to K actions) for every env of the batch.    */
typedef struct {
  int32_t H, W;               /* dim_room; H*W <= 64                                      */
  int32_t num_boxes;          /* SokobanEnvConfig.num_boxes                               */
  int32_t max_steps;          /* SokobanEnvConfig.max_steps                               */
  const uint8_t* room_fixed;  /* [B,H*W]  room_fixed (0 wall, 1 floor, 2 target)           */
  uint8_t* room_state;        /* [B,H*W]  room_state (0..5)                                */
  int8_t* player;             /* [B,2]    player_position (row, col)                       */
  uint8_t* num_env_steps;     /* [B]  (<= num_actions <= 255: one env step per action)     */
  int8_t* boxes_on_target;    /* [B]  num_boxes - open targets: -64..64 for H*W <= 64      */
  /* Optional board cache (NULL: none), caller-owned like every other field: 16 B per env
   * holding the room's state after the last turn (window wall | target | box u32, then the
   * player's cell index, a tag byte -- 1 = the room is regular and the entry is its state --,
   * num_env_steps and boxes_on_target; the SoA fields are written as without a cache).  boards_mode RMI_BOARDS_BUILD: the turn decodes every env's rows as without a
   * cache and writes every live env's entry; RMI_BOARDS_USE: the turn trusts the tagged
   * entries of the acting envs (no row loads, no decode) and keeps them current -- valid only
   * while nothing but rmi_sokoban_step_turn{,_first,_finalize} launches with this cache have
   * written room_state / room_fixed / player since a BUILD launch (the caller tracks that).
   * A wave with an acting env whose entry is untagged (or whose actions leave the regular
   * path) loads and decodes its rows as without a cache.  Only 6x6 rooms (the window in a
   * u32) at one lane per env (4097 <= B < 131072) maintain it: any other launch given a
   * non-NULL boards returns RMI_EUNSUP.                                                    */
  uint8_t* boards;            /* [B,16] or NULL                                            */
  int32_t boards_mode;        /* RMI_BOARDS_*                                              */
  /* The reset state's entries (NULL: none), for rmi_sokoban_step_turn_first: under BUILD that
   * launch decodes the reset rows and writes them here as well; under USE it reads them
   * instead of decoding the reset rows again (the rows are still loaded: they are the reset's
   * store).  Valid while init_state / init_player / room_fixed are unchanged since that BUILD
   * launch (a reset or load_rooms changes them; a restore does not).                       */
  uint8_t* init_boards;       /* [B,16] or NULL                                            */
} rmi_sokoban_t;
enum { RMI_BOARDS_NONE = 0, RMI_BOARDS_BUILD = 1, RMI_BOARDS_USE = 2 };

int rmi_sokoban_step_turn(const rmi_sokoban_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                          uint8_t* err, rmi_stream_t stream);

/* The rollout's last turn fused with its end: rmi_sokoban_step_turn, then exactly what
 * rmi_rollout_finalize computes (get_rollout_states es_manager.py:173-207, trajectory scores,
 * _normalize_score_tensor ctx_manager.py:175-226), in one launch.  Groups must be uniform and
 * contiguous: env b is in group b / group_size (the StarPO "state" grouping of es_manager.py:80-82).
 * Outputs as rmi_rollout_finalize (metrics f64[B,4], score / pen / norm f32[B]; any may be NULL).
 * RMI_EUNSUP when a group would straddle a wave (group_size must divide 64, or 16 for
 * B <= 4096) or B % group_size != 0: then launch the two separately.                          */
typedef struct {
  int32_t group_size;
  int32_t method; /* RMI_NORM_* */
  double* metrics;
  float* score;
  float* pen;
  float* norm;
} rmi_finalize_t;
int rmi_sokoban_step_turn_finalize(const rmi_sokoban_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                   uint8_t* err, const rmi_finalize_t* fin, rmi_stream_t stream);

/* A fresh episode's first turn fused with its reset: exactly rmi_sokoban_reset(init_state,
 * init_player) followed by rmi_sokoban_step_turn, in one launch (SokobanEnv.reset
 * sokoban/env.py:37-38 + EnvStatus() es_manager.py:95, then EnvStateManager.step
 * es_manager.py:105-171).  The counters and the episode record are not read (they start at
 * zero); every env's row, player, counters and whole record (all T rows) are written.   */
int rmi_sokoban_step_turn_first(const rmi_sokoban_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                const uint8_t* init_state, const int8_t* init_player, uint8_t* err,
                                rmi_stream_t stream);

/* Device part of SokobanEnv.reset (sokoban/env.py:37-38) + EnvStatus(seed) (es_manager.py:95):
 * room_state/player := init_state/init_player (the generated rooms), num_env_steps =
 * boxes_on_target = 0, and the whole episode record zeroed — one launch.  B*H*W % 4 == 0. */
int rmi_sokoban_reset(const rmi_sokoban_t* env, const rmi_episode_t* ep, const uint8_t* init_state,
                      const int8_t* init_player, rmi_stream_t stream);

/* rmi_sokoban_reset from the distinct generated rooms, in one launch: env i takes row
 * room_of[i] (NULL: row i) of rooms u8[n_rooms, 2*H*W+2] (device; per row room_fixed |
 * room_state | player as int8 bytes) into env->room_fixed, init_state u8[B, H*W] and init_player
 * i8[B, 2] (kept for a later rmi_sokoban_reset), then room_state / player := those, counters and
 * the whole episode record zeroed.  A row index outside [0, n_rooms) loads an empty room and
 * sets RMI_ERR_INDEX in err u8[B] (optional; else 0 per env).                                */
int rmi_sokoban_load_rooms(const rmi_sokoban_t* env, const rmi_episode_t* ep, const uint8_t* rooms,
                           int32_t n_rooms, const int32_t* room_of, uint8_t* init_state, int8_t* init_player,
                           uint8_t* err, rmi_stream_t stream);

/* Replaces: SokobanEnv.reset (sokoban/env.py:28-42) -> generate_room (sokoban/utils.py:221-278)
 * under all_seed (ragen/utils.py:7-18).  [host] CPU function: exact CPython-random /
 * numpy-legacy MT19937 semantics.  Writes one room per seed.  Returns per seed
 * 0 = ok, 1 = the reference would raise RuntimeError/RuntimeWarning (caller reseeds with
 * abs(hash(str(seed))) % 2**32 exactly as sokoban/env.py:41).                           */
int rmi_sokoban_generate_rooms(const int64_t* seeds /*[host][n]*/, int32_t n, int32_t H, int32_t W,
                               int32_t num_boxes, int32_t search_depth,
                               uint8_t* room_fixed /*[host][n,H*W]*/, uint8_t* room_state /*[host][n,H*W]*/,
                               int8_t* player /*[host][n,2]*/, uint8_t* status /*[host][n]*/,
                               int32_t n_threads);

/* rmi_sokoban_generate_rooms on a host thread of its own (the generation of a later reset, behind
 * the current rollout): returns a job handle (NULL: could not start) at once; every buffer must
 * stay valid until rmi_sokoban_generate_rooms_wait(job), which joins it, frees the handle and
 * returns rmi_sokoban_generate_rooms' result.  Every started job is waited on exactly once. */
typedef struct rmi_rooms_job rmi_rooms_job;
rmi_rooms_job* rmi_sokoban_generate_rooms_start(const int64_t* seeds /*[host][n]*/, int32_t n, int32_t H,
                                                int32_t W, int32_t num_boxes, int32_t search_depth,
                                                uint8_t* room_fixed, uint8_t* room_state, int8_t* player,
                                                uint8_t* status, int32_t n_threads);
int rmi_sokoban_generate_rooms_wait(rmi_rooms_job* job);

/* Replaces: SokobanEnv.render text mode (sokoban/env.py:53-61): room_state, the player on a
 * target shown as code 6, each code through the config's grid_lookup, rows joined by '\n'.
 * glyph_bytes[16] / glyph_len[16] (HOST memory): UTF-8 bytes of each code packed little-endian,
 * length 0..4 (0 = absent: rendered '?').  out u8[B, stride] (device, 4-B aligned, stride a
 * multiple of 4 and >= H*W*4 + H - 1), len i32[B] bytes written.                         */
int rmi_sokoban_render(const rmi_sokoban_t* env, int32_t B, const uint32_t* glyph_bytes, const uint8_t* glyph_len,
                       uint8_t* out, int32_t stride, int32_t* len, rmi_stream_t stream);

/* The turn and the next observation in ONE launch: EnvStateManager.step (es_manager.py:105-171,
 * as rmi_sokoban_step_turn) followed by SokobanEnv.render (sokoban/env.py:53-61) of every env's
 * state after it (es_manager.py:170 `next_state`; the rows rmi_sokoban_render writes, byte for
 * byte).  fin != NULL: the rollout's last turn fused with its end (rmi_sokoban_step_turn_finalize);
 * init_state / init_player != NULL: a fresh episode's first turn fused with its reset
 * (rmi_sokoban_step_turn_first); not both.  The render is fused into the turn's launch for
 * 36-cell rooms (6x6 and other 36-cell shapes) with B > 4096 (one lane per env: the turn waves
 * leave their envs' state in LDS and the workgroup's helper waves render it); any other layout
 * (other room sizes, 64-cell rooms included, or B <= 4096) runs the turn launch, then
 * rmi_sokoban_render (same outputs).                                                          */
typedef struct {
  uint32_t glyph_bytes[16]; /* as rmi_sokoban_render's glyph table                          */
  uint8_t glyph_len[16];    /* 0..4 (0: '?')                                                */
  uint8_t* out;             /* [B, stride] device, 4-B aligned; stride % 4 == 0 and
                               >= H*W*4 + H - 1                                              */
  int32_t stride;
  int32_t* len;             /* [B] bytes written                                            */
} rmi_render_t;
int rmi_sokoban_step_turn_render(const rmi_sokoban_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                 uint8_t* err, const rmi_finalize_t* fin, const uint8_t* init_state,
                                 const int8_t* init_player, const rmi_render_t* obs, rmi_stream_t stream);

/* --------------------------------------------------------------------- FrozenLake
 * Replaces: FrozenLakeEnv.step (frozen_lake/env.py:39-45) -> gymnasium FrozenLakeEnv.step
 *           + categorical_sample (third-party, App. A.2), numpy PCG64 draws (App. A.5). */
typedef struct {
  int32_t nrow, ncol;         /* nrow*ncol <= 64                                          */
  int32_t is_slippery;
  double cs0, cs1, cs2;       /* cumsum of the slippery transition probabilities          */
  const uint8_t* desc;        /* [B,nrow*ncol] ASCII 'S' 'F' 'H' 'G'                       */
  int32_t* s;                 /* [B] current state                                        */
  uint64_t* rng;              /* [4,B] PCG64 state_hi, state_lo, inc_hi, inc_lo            */
} rmi_frozenlake_t;

int rmi_frozenlake_step_turn(const rmi_frozenlake_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                             uint8_t* err, rmi_stream_t stream);

/* Device part of FrozenLakeEnv.reset (frozen_lake/env.py:28-37) + EnvStatus(seed)
 * (es_manager.py:95): desc / s / rng := the generated map, its start state and the seeded PCG64
 * (generate_random_map and the seeding stay on the host), episode record zeroed — one launch.  */
/* The rollout's last turn fused with its end: rmi_frozenlake_step_turn, then exactly what
 * rmi_rollout_finalize computes, in one launch (as rmi_sokoban_step_turn_finalize; the turn
 * runs each env on 4 lanes, so fin->group_size must divide 16 and B, else RMI_EUNSUP).      */
int rmi_frozenlake_step_turn_finalize(const rmi_frozenlake_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                      uint8_t* err, const rmi_finalize_t* fin, rmi_stream_t stream);

/* A fresh episode's first turn fused with its reset: exactly rmi_frozenlake_reset(init_desc,
 * init_s, init_rng) followed by rmi_frozenlake_step_turn, in one launch (FrozenLakeEnv.reset
 * frozen_lake/env.py:28-37 + EnvStatus() es_manager.py:95, then EnvStateManager.step).    */
int rmi_frozenlake_step_turn_first(const rmi_frozenlake_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                                   const uint8_t* init_desc, const int32_t* init_s, const uint64_t* init_rng,
                                   uint8_t* err, rmi_stream_t stream);
int rmi_frozenlake_reset(const rmi_frozenlake_t* env, const rmi_episode_t* ep, const uint8_t* init_desc,
                         const int32_t* init_s, const uint64_t* init_rng, rmi_stream_t stream);

/* Replaces: FrozenLakeEnv.render text mode (frozen_lake/env.py:47-61): codes P=0 (player), floor
 * (S, F) 1, hole 2, goal 3, player in a hole 4, player on the goal 5, through grid_lookup;
 * glyph table and output as rmi_sokoban_render (stride >= nrow*ncol*4 + nrow - 1).        */
int rmi_frozenlake_render(const rmi_frozenlake_t* env, int32_t B, const uint32_t* glyph_bytes,
                          const uint8_t* glyph_len, uint8_t* out, int32_t stride, int32_t* len,
                          rmi_stream_t stream);

/* ------------------------------------------------------------------------- Bandit
 * Replaces: BanditEnv.step/compute_reward (bandit/env.py:62-76).                       */
typedef struct {
  int32_t action_space_start;
  double lo_arm_score, hi_arm_loscore, hi_arm_hiscore, hi_arm_hiscore_prob;
  const uint8_t* hi_is_first; /* [B] ACTION_LOOKUP[start] is the hi arm (bandit/env.py:25-39) */
  uint64_t* rng;              /* [4,B] PCG64 state                                         */
} rmi_bandit_t;

int rmi_bandit_step_turn(const rmi_bandit_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                         uint8_t* err, rmi_stream_t stream);

/* ---------------------------------------------------------------------- Countdown
 * Replaces: CountdownEnv.step/compute_reward, check_format, check_correctness
 *           (countdown/env.py:9-21, :58-78).  Actions are answer strings: in->actions is
 * ignored; answer k of env b is answers[(b*K+k)*Lmax .. +answer_len[b*K+k]).             */
typedef struct {
  int32_t max_nums;           /* row stride of nums                                       */
  double score, format_score; /* CountdownEnvConfig.score / .format_score                  */
  const int32_t* nums;        /* [B,max_nums]                                              */
  const int32_t* n_nums;      /* [B]                                                       */
  const int32_t* target;      /* [B]                                                       */
} rmi_countdown_t;

int rmi_countdown_step_turn(const rmi_countdown_t* env, const rmi_episode_t* ep, const rmi_turn_t* in,
                            const uint8_t* answers, const int32_t* answer_len, int32_t Lmax,
                            uint8_t* err, rmi_stream_t stream);

/* Single reward evaluation (no episode bookkeeping), for parity tests and the reward
 * path of a batch of answers: reward[i] of answer i against nums/target row i.          */
int rmi_countdown_reward(const rmi_countdown_t* env, const uint8_t* answers, const int32_t* answer_len,
                         int32_t Lmax, int32_t n, double* reward, uint8_t* flags /*bit0 format bit1 correct*/,
                         uint8_t* err, rmi_stream_t stream);

/* --------------------------------------------------------- A16 rollout-state metrics
 * Replaces: EnvStateManager.get_rollout_states (es_manager.py:173-207).
 * out[B,4] f64: success, num_actions, action_is_effective, action_is_valid
 * (the last two NaN when no turn carried info, i.e. the key is absent).                 */
int rmi_rollout_metrics(const rmi_episode_t* ep, double* out, rmi_stream_t stream);

/* Trajectory scores (ctx_manager.py:282 + get_masks_and_scores:64-65 + :217):
 * score[b] = f32(sum over turns of turn_reward), pen[b] = f32(penalty[b]).              */
int rmi_trajectory_scores(const rmi_episode_t* ep, float* score, float* pen, rmi_stream_t stream);

/* Fused end of rollout: rmi_rollout_metrics + rmi_trajectory_scores + rmi_group_normalize in
 * one launch (any output pointer may be NULL except norm when G > 0).                    */
int rmi_rollout_finalize(const rmi_episode_t* ep, const int32_t* seg, int32_t G, int32_t method, double* metrics,
                         float* score, float* pen, float* norm, rmi_stream_t stream);

/* ------------------------------------------------------- A10 reward normalisation
 * Replaces: ContextManager._normalize_score_tensor (ctx_manager.py:175-226).
 * Groups are contiguous segments [seg[g], seg[g+1]) (state: group_size runs, inductive:
 * tag runs, batch: one segment).  out[b] = norm(score[b] + pen[b]).                     */
enum { RMI_NORM_IDENTITY = 0, RMI_NORM_MEAN = 1, RMI_NORM_MEAN_STD = 2, RMI_NORM_ASYM_CLIP = 3 };
int rmi_group_normalize(const float* score, const float* pen, const int32_t* seg, int32_t G, int32_t B,
                        int32_t method, float* out, rmi_stream_t stream);

/* --------------------------------------------------------------- A12 rollout filter
 * Replaces: _filter_rollout (agent_trainer.py:461-500).  scores[G*gs] (row sums of
 * original_rm_scores).  Writes per-group std/max/mean, keep[G] (1 = selected) and
 * metrics[6] (f64: in_group_std/max/mean, chosen_in_group_std/max/mean means).
 * Selection = top int(ratio*G) by std ('std', type 0) or by -std ('std_rev', type 1);
 * ties broken by ascending group index (documented deviation: torch.topk's tie order is
 * implementation-defined).  ratio == 1 keeps everything.  n = number of scores: RMI_EINVAL
 * unless n == G*gs (the reference's rm_scores.view(num_groups, group_size) raises).
 * G <= 8192 sorts in LDS; larger G takes a radix-select path with the same result.       */
int rmi_filter_groups(const float* scores, int64_t n, int32_t G, int32_t gs, double ratio, int32_t type, float* g_std,
                      float* g_max, float* g_mean, uint8_t* keep, double* metrics, rmi_stream_t stream);

/* Row sum of a [B,L] f32 tensor (rm_scores.sum(-1), agent_trainer.py:467).              */
int rmi_row_sum(const float* x, int64_t B, int64_t L, float* out, rmi_stream_t stream);

/* ------------------------------------------------------ A11 token masks and scores
 * Replaces: get_masks_and_scores (ctx_manager.py:35-70).  ids i64[B,S] row-major.
 * turn = cumsum(ids == special_token); response_mask = turn odd and > 1; loss_mask =
 * response_mask (RMI_MS_RESPONSE_MASK) or turn > 1.  Scores: scores f64[T,B] turn-major
 * (EnvStatus.rewards, i.e. rmi_episode_t.turn_reward), n_scores i32[B] = len(all_scores[b]).
 *   - without RMI_MS_TURN_SCORES: f32(python sum of row b's scores) at the last column;
 *   - with it: for idx < n_slots (= zip_longest length = max len), the score (0 past the
 *     row's own scores) goes to the position with ids == reward_token and turn == 2*idx+3,
 *     or to the last column when there is none; RMI_MS_ROLL (Qwen) then rolls by +1.
 * Outputs (the reference's [:, 1:] / [:, :-1] slices): score_out f32[B,S-1], loss_mask
 * u8[B,S-1], response_mask u8[B,S-1].  err[b] = RMI_ERR_STATE where the reference raises
 * (a turn with more than one reward token position).  n_slots <= 64.                    */
enum { RMI_MS_TURN_SCORES = 1, RMI_MS_RESPONSE_MASK = 2, RMI_MS_ROLL = 4 };
int rmi_masks_and_scores(const int64_t* ids, int64_t B, int64_t S, int64_t special_token, int64_t reward_token,
                         const double* scores, const int32_t* n_scores, int32_t T, int32_t n_slots, int32_t flags,
                         float* score_out, uint8_t* loss_mask, uint8_t* response_mask, uint8_t* err,
                         rmi_stream_t stream);

/* ------------------------------------------ §8(f) rank 1: the training batch, assembled
 * Replaces: the batch of ContextManager.formulate_rollouts / get_lm_inputs(prepare_for_update)
 * (ctx_manager.py:278-306): the tokenizer's left padding (padding_side="left"), attention_mask,
 * position_ids = attention_mask.cumsum(-1), and get_masks_and_scores on the padded ids — in ONE
 * pass.  Row b is pad_id * (S - n_b) then tokens[row_off[b] .. row_off[b+1]) (n_b tokens,
 * ragged rows back to back; S >= max n_b, else the row is flagged RMI_ERR_UNSUP and keeps its
 * last S tokens; RMI_ERR_STATE as in rmi_masks_and_scores).  Outputs input_ids / attention_mask / position_ids i64[B,S] (responses =
 * input_ids[:, 1:] is a view) and the rmi_masks_and_scores outputs with the same arguments.  */
int rmi_assemble_batch(const int64_t* tokens, const int64_t* row_off, int64_t B, int64_t S, int64_t pad_id,
                       int64_t special_token, int64_t reward_token, const double* scores, const int32_t* n_scores,
                       int32_t T, int32_t n_slots, int32_t flags, int64_t* input_ids, int64_t* attention_mask,
                       int64_t* position_ids, float* score_out, uint8_t* loss_mask, uint8_t* response_mask,
                       uint8_t* err, rmi_stream_t stream);

/* rmi_assemble_batch with rows given by (start, length): row b = tokens[row_start[b] ..
 * row_start[b] + row_len[b]) — e.g. the per-env prompt arena of the device prompt path, one
 * row per env at a fixed stride (formulate_rollouts, ctx_manager.py:278-306).             */
int rmi_assemble_rows(const int64_t* tokens, const int64_t* row_start, const int32_t* row_len, int64_t B, int64_t S,
                      int64_t pad_id, int64_t special_token, int64_t reward_token, const double* scores,
                      const int32_t* n_scores, int32_t T, int32_t n_slots, int32_t flags, int64_t* input_ids,
                      int64_t* attention_mask, int64_t* position_ids, float* score_out, uint8_t* loss_mask,
                      uint8_t* response_mask, uint8_t* err, rmi_stream_t stream);

/* response_length's row sums (ctx_manager.py:305, response_mask.sum(-1)): out[i] = the number
 * of nonzero bytes of row i of mask u8[B, S] (a bool mask); one launch, no widening copy.   */
int rmi_row_counts(const uint8_t* mask, int64_t B, int64_t S, int32_t* out, rmi_stream_t stream);

/* ------------------------------------------------------------------- A13 advantages
 * Replaces: verl compute_gae_advantage_return (called agent_trainer.py:77-83; App. A.4).
 * variant 0 = legacy (RAGEN's snapshot), 1 = masked (newer verl).  Sequential f32
 * recurrence in the reference's op order: bit-exact advantages/returns BEFORE whitening.
 * row_stats [B,3] f64 (optional): per-row sum(adv*m), sum(adv^2*m), sum(m) for whitening.      */
int rmi_gae(const float* r, const float* v, const uint8_t* mask, int64_t B, int64_t L, double gamma,
            double lam, int32_t variant, float* adv, float* ret, double* row_stats, rmi_stream_t stream);

/* Replaces: compute_bi_level_gae_advantage_return (core_algos.py:4-92) without the final
 * whitening.  err[b] = RMI_ERR_INDEX where the reference raises IndexError (core_algos.py:79). */
int rmi_bilevel_gae(const float* r, const float* v, const uint8_t* mask, int64_t B, int64_t L, double gamma,
                    double lam, double high_level_gamma, float* adv, float* ret, double* row_stats,
                    uint8_t* err, rmi_stream_t stream);

/* Replaces: verl masked_whiten (core_algos.py:90; App. A.4), in place on x.
 * If row_stats is NULL they are computed here.  scratch: rmi_whiten_scratch_bytes(B).    */
size_t rmi_whiten_scratch_bytes(int64_t B);
int rmi_masked_whiten(float* x, const uint8_t* mask, int64_t B, int64_t L, const double* row_stats,
                      void* scratch, rmi_stream_t stream);

/* The per-row whitening partials alone: row_stats[B,3] f64 = (sum, sum_sq, count) of x over
 * the nonzero mask bytes of each row (what rmi_gae / rmi_bilevel_gae write as row_stats), for
 * masked_whiten of a tensor no estimator produced (verl masked_whiten, core_algos.py:90).  */
int rmi_whiten_row_stats(const float* x, const uint8_t* mask, int64_t B, int64_t L, double* row_stats,
                         rmi_stream_t stream);

/* masked_whiten with batch statistics gathered from several shards (the multi-GPU form of
 * verl masked_whiten): stats[n_stats,3] = every rank's per-row (sum, sum_sq,
 * count) in global row order (rmi_gae / rmi_bilevel_gae row_stats, all-gathered); x[B,L] =
 * this rank's rows, whitened in place.  scratch >= 64 bytes; on return (stream order) its
 * int32 at byte 8 = 0 ok, 1 mask sum 0, 2 mask sum 1 (verl raises ValueError for both). */
int rmi_masked_whiten_stats(float* x, int64_t B, int64_t L, const double* stats, int64_t n_stats, void* scratch,
                            rmi_stream_t stream);

/* Replaces: verl compute_grpo_outcome_advantage (agent_trainer.py:94-99; App. A.4) with
 * contiguous groups seg[G+1] (RAGEN passes unique uids => every group has size 1).       */
int rmi_grpo_outcome(const float* r, const uint8_t* mask, int64_t B, int64_t L, const int32_t* seg, int32_t G,
                     double eps, int32_t norm_by_std, float* adv, float* ret, rmi_stream_t stream);

/* Replaces: verl compute_reinforce_plus_plus_outcome_advantage (agent_trainer.py:110-117)
 * before its masked_whiten: ret[b,t] = running = r[b,t] + gamma * running, then
 * running *= mask[b,t], right to left in f32 (adv = ret).  row_stats (optional) gets the
 * per-row whitening partials of adv; the caller then whitens adv and applies rmi_mask_mul. */
int rmi_reinforce_pp_returns(const float* r, const uint8_t* mask, int64_t B, int64_t L, double gamma, float* adv,
                             float* ret, double* row_stats, rmi_stream_t stream);

/* Replaces: verl compute_remax_outcome_advantage (agent_trainer.py:118-126): ret = reverse
 * cumsum of r * mask (torch's CPU accumulator: double, each output rounded to f32);
 * adv = ret - baseline[b] * mask. */
int rmi_remax(const float* r, const uint8_t* mask, const float* baseline, int64_t B, int64_t L, float* adv,
              float* ret, rmi_stream_t stream);

/* Replaces: verl compute_rloo_outcome_advantage (agent_trainer.py:127-134) with contiguous
 * groups seg[G+1]: score s = sum_t r; for a group of n > 1, s * n / (n-1) - mean * n / (n-1),
 * else s; broadcast over the row's mask (adv = ret). */
int rmi_rloo_outcome(const float* r, const uint8_t* mask, int64_t B, int64_t L, const int32_t* seg, int32_t G,
                     float* adv, float* ret, rmi_stream_t stream);

/* x[i] *= (mask[i] != 0), in f32: the trailing `* response_mask` of verl's REINFORCE++ and
 * REINFORCE++-baseline estimators (agent_trainer.py:102-117) after their masked_whiten. */
int rmi_mask_mul(float* x, const uint8_t* mask, int64_t n, rmi_stream_t stream);

/* ------------------------------------------------ response -> action ids (§8(f) rank 2)
 * Replaces: ContextManager.get_env_inputs (ctx_manager.py:332-352): the tokenizer's
 *           batch_decode(responses, skip_special_tokens=True) (:334-337), the "<think>" /
 *           "<answer>" prefix (:338-339), _parse_response (:148-173); and
 *           EnvStateManager._extract_map_valid_actions (es_manager.py:230-240).
 *
 * rmi_detokenize: byte-level BPE decoding (the tokenizers ByteLevel decoder).  Token id t
 * contributes its bytes unless it is skipped (special tokens); the concatenation is UTF-8
 * decoded with U+FFFD replacing each maximal invalid subpart (String::from_utf8_lossy) and
 * written back as UTF-8: out[b, 0 .. out_len[b]) is exactly decoded_str.encode("utf-8").
 * ids [B,R] (n_ids[b] <= R ids used per row, NULL = R).  The vocabulary is the packed table
 * of rmi_vocab_pack (16-B aligned): one 16-byte gather per id.  err[b] is written for every
 * row (not OR-ed into): RMI_ERR_INDEX for an id outside [0, V), RMI_ERR_UNSUP when the text
 * exceeds `stride` bytes (truncated), else 0.
 * stride % 4 == 0, stride <= 16384.                                                         */
int rmi_detokenize(const int64_t* ids, int64_t B, int64_t R, const int32_t* n_ids, const uint32_t* vocab_packed,
                   const uint8_t* vocab_bytes, int64_t n_bytes, int64_t V, uint8_t* out, int32_t stride,
                   int32_t* out_len, uint8_t* err, rmi_stream_t stream);

/* rmi_gen_rows: the turn's generations onto the env batch, ahead of rmi_detok_parse (the
 * input side of ContextManager.get_env_inputs, ctx_manager.py:332-337, for the envs given).
 * resp [n_resp, R] token ids; src[e] = the resp row of env e (-1: none), or src = NULL when
 * resp holds every env's row in order (n_resp == n_envs; ids and n_ids are then not written).
 * With src: ids [n_envs, R] = the rows (zeros for envs without one), n_ids[e] = R or 0 and
 * has[e] = 1 or 0 (the step kernels' has_input; each may be NULL).  raw_max[0] = the most bytes any given row decodes to before U+FFFD replacement (the
 * sum of its ids' byte lengths, skipped tokens 0, ids clamped to [0, V)); it sizes the decoded
 * rows.  The entry point zeroes raw_max on the stream first.                              */
int rmi_gen_rows(const int64_t* resp, int64_t n_resp, int64_t R, const int64_t* src, int64_t n_envs,
                 const uint32_t* vocab_packed, int64_t V, int64_t* ids, int32_t* n_ids, uint8_t* has,
                 int32_t* raw_max, rmi_stream_t stream);

/* rmi_gen_rows without the zeroing launch, for a caller that alternates two raw_max slots
 * across turns: raw_max must be 0 on entry (zeroed by the previous call's raw_next, or by the
 * caller), and the launch sets raw_next[0] = 0 (NULL: not written; must not alias raw_max). */
int rmi_gen_rows_chained(const int64_t* resp, int64_t n_resp, int64_t R, const int64_t* src, int64_t n_envs,
                         const uint32_t* vocab_packed, int64_t V, int64_t* ids, int32_t* n_ids, uint8_t* has,
                         int32_t* raw_max, int32_t* raw_next, rmi_stream_t stream);

/* HOST function (CPU memory): the packed vocabulary of rmi_detokenize from the byte table
 * vocab_bytes[vocab_off[t] .. vocab_off[t+1]) and skip[t] (NULL = none skipped).
 * packed u32[V,4]: entry t = (w0, w1, w2, meta); meta bits 0-23 = the token's byte length,
 * bit 31 = skip; a token of <= 12 bytes holds them in w0..w2 (byte k in bits 8(k%4) of
 * w[k/4]), a longer one its offset into vocab_bytes in w0.  RMI_EUNSUP for a token longer
 * than 2^24 - 1 bytes or a blob past 4 GiB.                                                 */
int rmi_vocab_pack(const int64_t* vocab_off, const uint8_t* vocab_bytes, int64_t n_bytes, int64_t V,
                   const uint8_t* skip, uint32_t* packed);

/* Parse configuration (agent_proxy.* and the env's action_lookup).  Strings are packed
 * little-endian into two u64 words (byte k of the string = byte k of lo|hi).             */
#define RMI_PARSE_MAX_NAMES 8
typedef struct {
  int32_t enable_think;     /* agent_proxy.enable_think: <think>(.*?)</think>\s*<answer>(.*?)</answer>
                               else <answer>(.*?)</answer>  (re.DOTALL, re.search)          */
  int32_t prepend;          /* 1: the text lacks the "<think>"/"<answer>" tag that
                               get_env_inputs prepends (ctx_manager.py:338-339)            */
  int32_t K;                /* agent_proxy.max_actions_per_turn (<= 8)                     */
  int32_t sep_len;          /* agent_proxy.action_sep, 1..16 bytes ("||")                  */
  uint64_t sep_lo, sep_hi;
  int32_t n_names;          /* 0: env has no action_lookup (actions pass through as text)  */
  uint8_t name_len[RMI_PARSE_MAX_NAMES];   /* lowercased ASCII names, <= 16 bytes         */
  uint64_t name_lo[RMI_PARSE_MAX_NAMES], name_hi[RMI_PARSE_MAX_NAMES];
  int8_t name_id[2][RMI_PARSE_MAX_NAMES];  /* action id of each name; column sel[b]       */
} rmi_parse_cfg_t;

/* One response per row: text[b, 0 .. text_len[b]) (UTF-8, row stride `stride`).
 * Outputs: actions[b,k] = action_lookup id of action k (0 = name not in the lookup, dropped
 * by the step kernels) and n_actions[b] = len(actions) after the max_actions_per_turn cap —
 * exactly the rmi_turn_t inputs.  Optional: sel[b] picks the id column (Bandit's per-env
 * lookup, bandit/env.py:25-39); spans[b,4] = think [start, end), answer [start, end) in the
 * prefixed text (all -1: no match); action_text [B,K,Lact] / action_len [B,K] = the stripped
 * action strings (Countdown's answers).  err[b] (optional) is WRITTEN for every row (not
 * OR-ed into: a caller's bits already there are overwritten): RMI_ERR_UNSUP when an action is
 * longer than Lact, RMI_ERR_STATE when text_len[b] is outside [0, stride], else 0.
 * stride % 4 == 0, stride <= 8192.                                                         */
int rmi_parse_actions(const rmi_parse_cfg_t* cfg, const uint8_t* text, const int32_t* text_len, int64_t B,
                      int32_t stride, const uint8_t* sel, int8_t* actions, uint8_t* n_actions, int32_t* spans,
                      uint8_t* action_text, int32_t* action_len, int32_t Lact, uint8_t* err, rmi_stream_t stream);

/* rmi_detok_parse: rmi_detokenize then rmi_parse_actions on the decoded rows, fused in one
 * launch (the per-turn boundary of a device-resident generation: ContextManager.get_env_inputs
 * ctx_manager.py:332-352 = batch_decode + the "<think>"/"<answer>" prefix + _parse_response,
 * then es_manager.py:230-240's name map).  The decoded rows are written to text / text_len
 * exactly as rmi_detokenize writes them (decode_err: its error bits) and parsed exactly as
 * rmi_parse_actions parses text (parse_err: its error bits); stride <= 8192.                */
int rmi_detok_parse(const int64_t* ids, int64_t B, int64_t R, const int32_t* n_ids, const uint32_t* vocab_packed,
                    const uint8_t* vocab_bytes, int64_t n_bytes, int64_t V, uint8_t* text, int32_t stride,
                    int32_t* text_len, uint8_t* decode_err, const rmi_parse_cfg_t* cfg, const uint8_t* sel,
                    int8_t* actions, uint8_t* n_actions, int32_t* spans, uint8_t* action_text, int32_t* action_len,
                    int32_t Lact, uint8_t* parse_err, rmi_stream_t stream);

/* rmi_sokoban_token_turn: one Sokoban turn from the generations' token ids in ONE launch — the
 * decode + parse of rmi_detok_parse (ContextManager.get_env_inputs, ctx_manager.py:332-352, and
 * es_manager.py:230-240), then the turn and the next observation of rmi_sokoban_step_turn_render
 * (EnvStateManager.step es_manager.py:105-171, SokobanEnv.render sokoban/env.py:53-61).  Outputs:
 * exactly those of rmi_detok_parse(tok..., B = ep->B, actions = in->actions, n_actions =
 * in->n_actions, action_text = NULL) followed by rmi_sokoban_step_turn_render(env, ep, in, err,
 * fin, init_state, init_player, obs); tok->cfg->K == in->K.  A workgroup holds 16 envs: each wave
 * decodes and parses one env's generation, the group's turn then runs on one wave (a lane per env),
 * and each wave renders its env.  Fused for 36-cell rooms whose board window fits 32 bits and
 * H*(W+1)-1 <= 64, fin == NULL or fin->group_size dividing 16, and rows whose LDS fits (16 rows of
 * the parse's per-wave LDS within 56 KB); anything else runs the two calls (same outputs).        */
typedef struct {
  const int64_t* ids;           /* [B, R] generated ids                                        */
  int64_t R;
  const int32_t* n_ids;         /* [B] ids per row, or NULL (R each)                            */
  const uint32_t* vocab_packed; /* rmi_vocab_pack's 16-B entries (16-B aligned)                 */
  const uint8_t* vocab_bytes;   /* the blob of tokens longer than 12 bytes                     */
  int64_t n_bytes, V;
  uint8_t* text;                /* [B, stride] decoded rows (4-B aligned)                      */
  int32_t stride;
  int32_t* text_len;
  uint8_t* decode_err;          /* [B] or NULL                                                  */
  const rmi_parse_cfg_t* cfg;
  const uint8_t* sel;           /* [B] name-id column, or NULL                                  */
  int32_t* spans;               /* [B, 4] or NULL                                               */
  uint8_t* parse_err;           /* [B] or NULL                                                  */
  /* has != NULL: rmi_turn_inputs between the decode and the turn (the turn chain's step 3): has[b]
   * = (has_t == NULL || has_t[b]) && decode_err[b] == 0, err[b] zeroed; in->has_input must be
   * has and decode_err non-NULL.                                                                */
  const uint8_t* has_t;
  uint8_t* has;
} rmi_token_rows_t;
int rmi_sokoban_token_turn(const rmi_token_rows_t* tok, const rmi_sokoban_t* env, const rmi_episode_t* ep,
                           const rmi_turn_t* in, uint8_t* err, const rmi_finalize_t* fin, const uint8_t* init_state,
                           const int8_t* init_player, const rmi_render_t* obs, rmi_stream_t stream);


/* ---------------------------------------------- prompt token ids (§8(f) ranks 1-2)
 * Replaces: the tokenizer call of ContextManager.get_lm_inputs (ctx_manager.py:265-278,
 *           tokenizer(llm_input_texts, ...)) for a byte-level BPE tokenizer (HF `tokenizers`
 *           model "BPE", the Qwen2 pre-tokenizer Split(regex) + ByteLevel(use_regex=False),
 *           normalizer NFC or none, added tokens matched leftmost-longest).
 *
 * Tables (built on the host from the tokenizer's JSON, ragen_amd/tokenizer.py):
 *   cp_block[cp >> 8] -> block, cp_class[block * 256 + (cp & 255)] = RMI_CP_* bits of code
 *   point cp; byte_id[256] = id of each byte's byte-level symbol; merges = open-addressed
 *   (key, value) u64 pairs, key = left << 32 | right (~0 = empty slot), value = rank << 32 |
 *   merged id, slot (key * 0x9E3779B97F4A7C15) >> merge_shift, linear probing (merge_mask =
 *   slots - 1); added tokens = bytes [added_off[i], added_off[i+1]) of added_bytes -> id.   */
#define RMI_CP_L 1u       /* \p{L}                                                          */
#define RMI_CP_N 2u       /* \p{N}                                                          */
#define RMI_CP_W 4u       /* \s (White_Space, as the pre-tokenizer's regex engine sees it)  */
#define RMI_CP_NL 8u      /* \r or \n                                                       */
#define RMI_CP_UNSAFE 16u /* NFC may change text containing it (the row is left to the host) */
#define RMI_PRETOK_QWEN2 0 /* (?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}|
                              ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+            */
#define RMI_PRETOK_CHARS 1 /* every character is its own pre-token                           */
typedef struct {
  const uint16_t* cp_block; /* [0x1100]                                                      */
  const uint8_t* cp_class;  /* [n_blocks * 256]                                              */
  const int32_t* byte_id;   /* [256]                                                         */
  const uint64_t* merges;   /* [2 * (merge_mask + 1)]                                        */
  uint32_t merge_mask, merge_shift;
  int32_t pretok;           /* RMI_PRETOK_*                                                  */
  int32_t nfc;              /* 1: the tokenizer normalises NFC (rows holding RMI_CP_UNSAFE
                               code points are flagged RMI_ERR_UNSUP, not encoded)           */
  int32_t n_added;
  const uint8_t* added_bytes;
  const int32_t* added_off; /* [n_added + 1]                                                 */
  const int32_t* added_id;  /* [n_added]                                                     */
  uint32_t added_first[8];  /* bitmap of the added tokens' first bytes                       */
  /* Word cache (NULL: off): (word_cache_mask + 1) entries of 16 u32 in HBM, zero-initialised
   * once and kept across calls for this tokenizer's tables — a pre-token's bytes (2..16) ->
   * its BPE ids (<= 9).  A pre-token's merges depend on its bytes alone (the tokenizers
   * crate caches words the same way), so a hit skips its pair lookups and merges.  Entries
   * are claimed with an atomic compare-and-swap after a plain read finds the slot empty and
   * written once; every dword goes from zero to its final value once, ids are stored plus
   * one, and only words with no all-zero key dword are cached, so a reader (no acquire /
   * release across the XCDs' L2s inside a launch) that sees the key, the ready meta and
   * nonzero ids holds exactly the writer's entry; any other state is a miss.              */
  uint32_t* word_cache;
  uint32_t word_cache_mask; /* entries - 1 (a power of two minus one)                        */
  /* Expansions (n_exp 0: none): added tokens whose id in added_id is -(e + 1) stand for the
   * id sequence exp_ids[exp_off[e] .. exp_off[e+1]) instead of one id.  Their bytes are
   * (0xFF, 0x80 + e): never valid UTF-8, so no text holds them; the prompt programs write them
   * in place of a constant stretch whose tokenization the host has checked context-free at both
   * ends (llm_agent/prompts.py), so the kernel skips that stretch's bytes.  n_exp <= 64.       */
  int32_t n_exp;
  const int32_t* exp_off;   /* [n_exp + 1]                                                   */
  const int32_t* exp_ids;
  /* Staging tables (each NULL: derived in the kernel from the tables above): the added tokens
   * as zero-padded 32-byte words [n_added][4] (given only when every added token is <= 32
   * bytes and n_added <= 64), and the classes of the code points 0..127
   * (= cp_class[cp_block[0] * 256 + cp], [128]).  They take the staging's dependent loads off
   * every row's critical path.                                                               */
  const uint64_t* added_words;
  const uint8_t* ascii_class;
  /* exp_off[n_exp] when the caller knows it (0: unknown); <= 512 -> the kernel stages the
   * expansion tables in LDS with each row (one dependent HBM load per copied id otherwise).   */
  int32_t n_exp_ids;
  /* Two-pass scratch (all NULL, or pre_cap < rows * stride: one kernel per call).  With it the
   * call is three launches: the pre-tokenizer pass (its LDS is 6 B per text byte, so more rows
   * are in flight) writes each row's pre-token list (pre[row * stride + j] = start | length << 12
   * | added << 24, pre_np[row] entries; pre_gid[row * stride + start] = an added token's id);
   * the word pass looks each pre-token up in the word cache and merges the misses in a small
   * per-wave scratch; a row whose misses outgrow that scratch is flagged in pre_retry and
   * encoded again by the one-kernel algorithm.  Same outputs either way, except that a row
   * flagged for passing out_stride may have had ids written past out_len[b] (out_len[b], n_tok
   * and mark_tok are as for any flagged row).                                                 */
  uint32_t* pre;            /* [pre_cap]                                                     */
  int32_t* pre_gid;         /* [pre_cap]                                                     */
  int32_t* pre_np;          /* [pre_cap / 4]                                                 */
  uint8_t* pre_retry;       /* [pre_cap / 4]                                                 */
  int64_t pre_cap;          /* taken when rows * stride <= pre_cap (then rows <= pre_cap / 4) */
} rmi_bpe_t;

/* Row b: text[b * pitch .. + text_len[b]) (UTF-8; pitch % 4 == 0); `stride` (% 4 == 0,
 * <= 3072) bounds the row length and sizes the kernel's LDS (rows longer: RMI_ERR_STATE).
 * Its token ids are appended to out row b (i64, row stride out_stride) at position
 * out_len[b] (NULL: 0), and out_len[b] (if given) advances by their count; n_tok[b]
 * (optional) = the count.  mark_byte[b] (optional, a pre-token boundary, e.g. the start of a
 * chat-template block) -> mark_tok[b] = the row position of the first token at or after it.
 * err[b]: RMI_ERR_STATE for invalid UTF-8 or text_len outside [0, stride]; RMI_ERR_UNSUP for
 * a code point NFC may change (nfc = 1) or a row that would pass out_stride.  A flagged row
 * writes no token and leaves out_len[b] as it was.                                         */
int rmi_bpe_encode(const rmi_bpe_t* tok, const uint8_t* text, int64_t pitch, int32_t stride, const int32_t* text_len,
                   int64_t B, int64_t* out, int64_t out_stride, int32_t* out_len, int32_t* n_tok,
                   const int32_t* mark_byte, int32_t* mark_tok, uint8_t* err, rmi_stream_t stream);

/* Replaces: the prompt text of ContextManager.get_lm_inputs (ctx_manager.py:248-263) — the
 *           chat messages of each env's history under the tokenizer's chat template — for
 *           the part of it one turn adds, built on the device from the turn's own results.
 * Row b = the concatenation of a small program of pieces (the same program for every row):
 *   RMI_PT_CONST      pool[a .. a+b)
 *   RMI_PT_TAG_CONST  pool bytes of the row's tag: (offset, length) = tag_const[2*(a*n_tags + tag[b])]
 *   RMI_PT_OBS        obs[b, 0 .. obs_len[b])                    the env's rendered state
 *   RMI_PT_INT        str(ints[a*B + b])                         e.g. actions_left
 *   RMI_PT_REWARD     str(reward[b]): an int when reward_int[b], else repr(float) (CPython's
 *                     shortest round-trip form; rows with |reward| outside [1e-5, 2^53) are
 *                     flagged RMI_ERR_UNSUP)
 *   RMI_PT_RESPONSE   the llm_response _parse_response builds (ctx_manager.py:148-173) from
 *                     the decoded generation resp[b, 0 .. resp_len[b]) prefixed with
 *                     "<think>" / "<answer>" (ctx_manager.py:338-339) and the parse's spans
 *                     (rmi_parse_actions): no match -> the raw text; else the contents with the
 *                     special-token replace / strip cascade, and the answer re-joined with
 *                     " " + sep + " " when it holds more than K actions
 *   RMI_PT_MARK       mark[b] = the row length so far
 *   RMI_PT_IF         the row ends here unless cond[b]
 * Rows with active[b] == 0 (active may be NULL) get length 0.  err[b] = RMI_ERR_UNSUP for a
 * row past `stride` bytes (length 0) or an unsupported reward.  stride % 4 == 0, <= 3072.   */
enum { RMI_PT_CONST = 0, RMI_PT_TAG_CONST, RMI_PT_OBS, RMI_PT_INT, RMI_PT_REWARD, RMI_PT_RESPONSE, RMI_PT_MARK,
       RMI_PT_IF };
#define RMI_PROMPT_MAX_PIECES 32
typedef struct {
  int32_t kind, a, b;
} rmi_piece_t;
typedef struct {
  int32_t n_pieces;
  rmi_piece_t pieces[RMI_PROMPT_MAX_PIECES];
  const uint8_t* pool;
  const int32_t* tag_const;
  int32_t n_tags;
  const uint8_t* tag;        /* [B] (NULL: tag 0)                                               */
  const uint8_t* obs;        /* [B, obs_stride]                                                 */
  int32_t obs_stride;
  const int32_t* obs_len;
  const int32_t* ints;       /* [n][B]                                                          */
  const double* reward;      /* [B]                                                             */
  const uint8_t* reward_int; /* [B]                                                             */
  const uint8_t* resp;       /* [B, resp_stride] decoded generations (no prefix)                */
  int32_t resp_stride;
  const int32_t* resp_len;
  const int32_t* spans;      /* [B, 4] think [s, e), answer [s, e) in the prefixed text, -1 none */
  int32_t enable_think, K, sep_len;
  uint8_t sep[16];
  const uint8_t* cond;       /* [B]                                                             */
  const uint8_t* active;     /* [B] (NULL: every row)                                           */
  int32_t pool_len;          /* readable bytes at pool (0: unknown); <= 1024 the wave stages
                                the pool in LDS with the row's other loads                     */
  /* The turn form (turn_exec != NULL; reward_int and cond are then not read): both derived
   * from the turn record as ContextManager._build_messages prints a turn (ctx_manager.py:
   * 248-263, es_manager.py:148-160) — the reward is an int when the turn executed no action
   * (step() recorded the int 0) or, for a tag whose bit is set in int_reward_tags (Countdown's
   * 0 / 1 integer rewards), when it is 0.0 or 1.0; the next user block follows unless
   * flags[b] has RMI_FLAG_DONE or last_turn (the rollout's final turn).                     */
  const uint8_t* turn_exec;  /* [B] actions executed this turn                                  */
  const uint8_t* flags;      /* [B] episode flags after the turn                                */
  uint32_t int_reward_tags;  /* bit t: tag t's 0 / 1 rewards print as ints (tags < 32)          */
  int32_t last_turn;
  /* Reward text cache (NULL: off): (num_cache_mask + 1) entries of 16 u32, zero-initialised and
   * kept across calls — a reward's float bits -> its CPython repr (<= 24 bytes).  An entry is
   * written once: its writer claims the empty slot by a 64-bit compare-and-swap of the key word,
   * then stores the text and the ready | length word, and no one writes the slot again.  Every
   * word of an entry therefore goes from zero to its final value exactly once, and a reader
   * takes an entry only when its key matches, it is ready and every text byte below the length
   * is nonzero (a repr has no zero byte): a word not yet visible reads as zero and is a miss.
   * A turn's rewards take a handful of values; a hit replaces the row's shortest-repr search
   * on one lane.                                                                             */
  uint32_t* num_cache;
  uint32_t num_cache_mask;  /* entries - 1 (a power of two minus one)                          */
} rmi_prompt_t;
int rmi_prompt_text(const rmi_prompt_t* prog, int64_t B, uint8_t* out, int32_t stride, int32_t* out_len,
                    int32_t* mark, uint8_t* err, rmi_stream_t stream);

/* The generation batch of get_lm_inputs (ctx_manager.py:265-278: the tokenizer's left padding,
 * attention_mask, position_ids = attention_mask.cumsum(-1)) from the prompt arena: row i =
 * pad_id * (S - n) then arena[rows[i], 0 .. arena_len[rows[i]]) then tail[0 .. n_tail) (the
 * generation prompt), n = arena_len + n_tail.  i64[n_rows, S] outputs; err[i] = RMI_ERR_UNSUP
 * when n > S (the row keeps its last S tokens).                                             */
int rmi_pad_rows(const int64_t* arena, int64_t arena_stride, const int32_t* arena_len, const int64_t* rows,
                 int64_t n_rows, const int64_t* tail, int32_t n_tail, int64_t S, int64_t pad_id, int64_t* input_ids,
                 int64_t* attention_mask, int64_t* position_ids, uint8_t* err, rmi_stream_t stream);

/* ------------------------------------------------------------ turn-loop glue */
/* The small per-turn steps of the device turn loop around the kernels above, one launch each
 * (each replaced several torch elementwise / reduction launches of the Python host side):
 *
 * rmi_turn_inputs (EnvStateManager.step's device turn, es_manager.py:105-171, before the step
 * kernels): has[e] = (has_t ? has_t[e] : 1) && dec_err[e] == 0 — the envs stepped this turn
 * (a generation, decoded without error) — and err[e] = 0 (the step kernels OR into it).
 *
 * rmi_turn_readback (after the turn and the render): flags_copy = flags (the turn record),
 * left[e] = max_actions[e] - num_actions[e] (the next prompt's "You have N actions left"), and
 * pack = flags [B] | err [B] | dec_err [B] | zero pad to 4 | int32 max text_len | int32 max
 * obs_len (NULL lengths: 0) — the one buffer the host reads back per turn (the active set, the
 * errors es_manager raises, the sizes that bound the next prompt's text).  pack holds
 * ((3B + 3) & ~3) + 8 bytes, 4-byte aligned.
 *
 * rmi_prompt_commit (after rmi_bpe_encode of a turn's prompt text): bad[e] = the row takes
 * part (active NULL or active[e]) and bpe_err[e] or text_err[e] is set (the host rebuilds it);
 * with mark_tok, len_upd[e] = mark_tok[e] for the rows that take part (the update batch's row
 * end, ctx_manager.py:240-241).
 *
 * rmi_rows_stats (the generation batch, ctx_manager.py:265-278): stats[0] = max len[rows[i]]
 * over the n_rows rows (rows NULL: rows 0 .. n_rows-1; 0 when none; rows outside [0, B) are
 * skipped), stats[1] = 1 if any bad[e] (bad NULL: 0); len and bad hold B entries.           */
int rmi_turn_inputs(const uint8_t* has_t, const uint8_t* dec_err, int64_t B, uint8_t* has, uint8_t* err,
                    rmi_stream_t stream);
int rmi_turn_readback(const uint8_t* flags, const uint8_t* err, const uint8_t* dec_err, const uint8_t* num_actions,
                      const int32_t* max_actions, const int32_t* text_len, const int32_t* obs_len, int64_t B,
                      uint8_t* flags_copy, int32_t* left, uint8_t* pack, rmi_stream_t stream);
/* rmi_turn_readback with a longer tail: the pack's int32s after byte ((3B + 3) & ~3) get
 * [6] = the generation batch's rows rmi_pad_rows flagged (left-cut: pad_err u8[n_pad] nonzero;
 * pad_err NULL: 0), [7] = the OR of the err bytes | the OR of the dec_err bytes << 8, [8] = the
 * envs whose flags have RMI_FLAG_DONE ([2..5] are left to other writers): pack holds
 * ((3B + 3) & ~3) + 36 bytes.                                                                  */
int rmi_turn_readback_pad(const uint8_t* flags, const uint8_t* err, const uint8_t* dec_err, const uint8_t* num_actions,
                          const int32_t* max_actions, const int32_t* text_len, const int32_t* obs_len, int64_t B,
                          uint8_t* flags_copy, int32_t* left, uint8_t* pack, const uint8_t* pad_err, int64_t n_pad,
                          rmi_stream_t stream);
int rmi_prompt_commit(const uint8_t* bpe_err, const uint8_t* text_err, const uint8_t* active, const int32_t* mark_tok,
                      int32_t* len_upd, int64_t B, uint8_t* bad, rmi_stream_t stream);
int rmi_rows_stats(const int32_t* len, const int64_t* rows, int64_t n_rows, const uint8_t* bad, int64_t B,
                   int32_t* stats, rmi_stream_t stream);
/* rmi_rows_stats over the envs that go on after a turn -- the next generation batch of
 * get_lm_inputs (the env outputs es_manager.py:168-171 returns: an input this turn, not done):
 * e with (has == NULL || has[e]) and !(flags[e] & RMI_FLAG_DONE).  stats i32[3] = (longest
 * len[e] among them, any bad[e] over all B (0 without bad), their count).  Launched after the
 * next prompt's encode, into the turn's readback buffer: one readback per turn.              */
int rmi_next_rows_stats(const int32_t* len, const uint8_t* has, const uint8_t* flags, const uint8_t* bad, int64_t B,
                        int32_t* stats, rmi_stream_t stream);

/* rmi_prompt_commit then rmi_next_rows_stats with bad = the rows the commit flags, in one
 * launch: bad / len_upd exactly as rmi_prompt_commit; stats = (the longest len over the envs
 * with has (NULL: every env) and flags without FLAG_DONE, any bad row, their count).       */
int rmi_prompt_commit_stats(const uint8_t* bpe_err, const uint8_t* text_err, const uint8_t* active,
                            const int32_t* mark_tok, int32_t* len_upd, int64_t B, uint8_t* bad, const int32_t* len,
                            const uint8_t* has, const uint8_t* flags, int32_t* stats, rmi_stream_t stream);

/* The next generation batch's rows (es_manager.py:168-169 for a turn whose envs came in ascending
 * order, ctx_manager.py:265-278's batch order): rows i64[count] = the envs e, ascending, with
 * has[e] (NULL: every env) and no RMI_FLAG_DONE in flags[e]; src i64[B]: src[e] = e's index in
 * rows, or -1 (the next turn's rmi_gen_rows map).  count = rmi_next_rows_stats' stats[2].    */
int rmi_next_rows_list(const uint8_t* has, const uint8_t* flags, int64_t B, int64_t* rows, int64_t* src,
                       rmi_stream_t stream);

/* [host] The env ids that go on, from a turn's read-back flags (es_manager.py:168-169 over a
 * turn whose inputs were the previous turn's survivors): out[k] = lo + i for every i < n with
 * no bit of done_bits in flags[i], ascending -> their count, or -1 when more than cap (or a NULL
 * argument).  Host memory only: the turn loop's survivor list without a numpy pass.          */
int64_t rmi_host_live_ids(const uint8_t* flags, int64_t n, uint32_t done_bits, int64_t lo, int64_t* out,
                          int64_t cap);

/* ------------------------------------------------------------ the turn chain
 * Replaces: one turn of LLMAgentProxy.rollout's loop (agent_proxy.py:150-155) from the actor's
 *           output to the next generation batch's shape -- ContextManager.get_env_inputs
 *           (ctx_manager.py:332-352), EnvStateManager.step (es_manager.py:105-171) with the
 *           env's render (sokoban/env.py:53-61, frozen_lake/env.py:47-61), and the part of the
 *           next get_lm_inputs (ctx_manager.py:228-278) that one turn adds to each prompt --
 *           as ONE host call that enqueues every launch of the turn on `stream`, copies the
 *           turn's packed readback to host memory and waits for it.  [host] struct; every
 *           pointer in it is a device pointer unless marked [host].
 *
 * In order (each step exactly the entry point named; see there):
 *   1. rmi_gen_rows_chained(resp, n_resp, R, src, n_envs, vocab_packed, V, ids, n_ids, has_t,
 *      raw_max, raw_next) with ids / n_ids / has_t passed only when src != NULL -- skipped when
 *      resp == NULL (the rows are on the device already)
 *   2. rmi_detok_parse(ids, n_envs, R, n_ids, vocab, text, stride, text_len, dec_err, parse, sel,
 *      actions, n_actions, spans, -, -, 0, parse_err): ids [n_envs, R] are every env's row (= resp
 *      when src == NULL), n_ids NULL = R ids each
 *   3. rmi_turn_inputs(has_t, dec_err, n_envs, has, err): has_t NULL = every env has a generation
 *   4. the env's turn on {turn, K, actions, n_actions, has, max_actions_per_traj,
 *      format_penalty} with its render into obs: rmi_sokoban_step_turn_render (env_kind 0), or
 *      rmi_frozenlake_step_turn then rmi_frozenlake_render (env_kind 1)
 *   5. rmi_turn_readback_pad(ep->flags, err, dec_err, ep->num_actions, max_actions, text_len,
 *      obs->len, n_envs, flags_copy, left, pack, pad_err, n_pad): pad_err (NULL: not counted) =
 *      the generation batch's error bytes
 *   6. (prompt != NULL) rmi_prompt_text(prompt, n_envs, ptext, pstride, ptext_len, pmark, pterr),
 *      rmi_bpe_encode(bpe, ptext, pstride, bpe_stride, ptext_len, n_envs, arena, arena_stride,
 *      arena_len, NULL, pmark, mark_tok, bpe_err) and rmi_prompt_commit_stats(bpe_err, pterr,
 *      has, mark_tok, len_upd, n_envs, bad, arena_len, has, flags_copy, stats)
 *   7. rmi_readback(host, pack, pack_bytes): the copy, then the stream waited on; with next_rows
 *      the copy, then rmi_next_rows_list(has, flags_copy, n_envs, next_rows, next_src) enqueued
 *      behind it, then the copy alone waited on (the list is done in stream order before any
 *      later work on the stream).
 *   8. (pad_block and next_rows != NULL) with the readback's stats (longest, any_bad, count) =
 *      pack's int32 [2..4] after the tail offset: when any_bad == 0, count > 0 and
 *      3 * count * S <= pad_cap for S = longest + pad_tail_n, rmi_pad_rows(arena, arena_stride,
 *      arena_len, next_rows, count, pad_tail, pad_tail_n, S, pad_id, pad_block,
 *      pad_block + count * S, pad_block + 2 * count * S, pad_err_next) is enqueued (the
 *      next get_lm_inputs' batch, ctx_manager.py:265-278, built while the host reads the
 *      readback) and *pad_S_out = S; else *pad_S_out = 0 and nothing is launched.
 * One env tag (one env batch) per chain.  A step that fails returns its code at once (the
 * steps before it are enqueued; nothing after it is).  next_rows or pad_block set without
 * prompt and stats is RMI_EINVAL before anything is enqueued: steps 7-8 read the stats that
 * only step 6 writes.  The readback's host buffer is looked up (pinned or pageable) on every
 * call; nothing about it is remembered between calls.                                      */
enum { RMI_CHAIN_SOKOBAN = 0, RMI_CHAIN_FROZENLAKE = 1 };
typedef struct {
  int64_t n_envs;
  /* 5. the generation batch's error bytes (pad_err NULL: not counted) */
  const uint8_t* pad_err;
  int64_t n_pad;
  /* 1. the generations */
  const int64_t* resp;
  int64_t n_resp, R;
  const int64_t* src;               /* [n_envs] row of each env (-1: none); NULL: every env in order */
  const uint32_t* vocab_packed;
  const uint8_t* vocab_bytes;
  int64_t vocab_n_bytes, V;
  int64_t* ids;                     /* [n_envs, R] every env's row (written by step 1 when src)    */
  int32_t* n_ids;                   /* [n_envs] or NULL (R each)                                   */
  uint8_t* has_t;                   /* [n_envs] or NULL (every env)                                */
  int32_t* raw_max, *raw_next;
  /* 2. decode + parse */
  const rmi_parse_cfg_t* parse;
  const uint8_t* sel;
  uint8_t* text;
  int32_t stride;
  int32_t* text_len;
  uint8_t* dec_err;
  int8_t* actions;                  /* [n_envs, K]                                                  */
  uint8_t* n_actions;
  int32_t* spans;                   /* [n_envs, 4]                                                  */
  uint8_t* parse_err;
  /* 3-4. the turn and its render */
  uint8_t* has, *err;
  int32_t env_kind;                 /* RMI_CHAIN_*                                                  */
  const rmi_sokoban_t* sokoban;
  const rmi_frozenlake_t* frozenlake;
  const rmi_episode_t* ep;
  int32_t turn, K, max_actions_per_traj;
  double format_penalty;
  const rmi_render_t* obs;
  /* 5. the record's columns and the packed readback */
  const int32_t* max_actions;
  uint8_t* flags_copy;
  int32_t* left;
  uint8_t* pack;
  /* 6. the next prompt's append (prompt NULL: none) */
  const rmi_prompt_t* prompt;
  uint8_t* ptext;
  int32_t pstride;
  int32_t* ptext_len, *pmark;
  uint8_t* pterr;
  const rmi_bpe_t* bpe;
  int32_t bpe_stride;
  int64_t* arena;
  int64_t arena_stride;
  int32_t* arena_len, *mark_tok;
  uint8_t* bpe_err;
  int32_t* len_upd;
  uint8_t* bad;
  int32_t* stats;                   /* i32[3], inside pack                                          */
  /* 7. the readback; the next generation batch's rows and gen_rows map (NULL: not written) */
  int64_t* next_rows, *next_src;    /* [n_envs] each                                                */
  void* host;                       /* [host] pinned, >= pack_bytes                                 */
  int64_t pack_bytes;
  /* 8. the next generation batch padded in the same call (pad_block NULL or next_rows NULL: not) */
  int64_t* pad_block;               /* i64[pad_cap]: input_ids | attention_mask | position_ids      */
  int64_t pad_cap;
  const int64_t* pad_tail;          /* [pad_tail_n] the generation prompt's ids                     */
  int32_t pad_tail_n;
  int64_t pad_id;
  uint8_t* pad_err_next;            /* [n_envs] rmi_pad_rows' err                                   */
  int64_t* pad_S_out;               /* [host] the batch width padded to, 0: not padded              */
} rmi_turn_chain_t;
int rmi_turn_chain(const rmi_turn_chain_t* chain, rmi_stream_t stream);

/* ------------------------------------------------------- formulate_rollouts, chained
 * Replaces: ContextManager.formulate_rollouts (ctx_manager.py:354-356 -> get_lm_inputs with
 *           prepare_for_update, :228-330) over the device prompt arena and episode record.
 *
 * rmi_formulate_stats: stats i32[3] = (max len[e], any bad[e] (bad NULL: 0), max n_turns[e]) --
 * the batch width, whether a row waits for the host, zip_longest's length (:52-62) -- and
 * n_sc[e] = n_turns[e] widened (the assembly's n_scores).  One workgroup.
 * rmi_assemble_rows_ex: rmi_assemble_rows, plus resp_count[b] (optional) = the ones of row b's
 * response_mask (response_mask.sum(-1), :305) and, with last_score (flags without
 * RMI_MS_TURN_SCORES), score[b, S-2] = last_score[b] -- the normalised score
 * _normalize_score_tensor writes there in place (:175-226) -- instead of the raw sum.
 * rmi_formulate_tail: out i64[2] = (sum of resp_count, OR of err): response_length's exact
 * numerator and the assembly's error bits.  One workgroup.                                   */
int rmi_formulate_stats(const int32_t* len, const uint8_t* bad, const uint8_t* n_turns, int64_t B, int32_t* n_sc,
                        int32_t* stats, rmi_stream_t stream);
int rmi_assemble_rows_ex(const int64_t* tokens, const int64_t* row_start, const int32_t* row_len, int64_t B,
                         int64_t S, int64_t pad_id, int64_t special_token, int64_t reward_token, const double* scores,
                         const int32_t* n_scores, int32_t T, int32_t n_slots, int32_t flags, const float* last_score,
                         int64_t* input_ids, int64_t* attention_mask, int64_t* position_ids, float* score_out,
                         uint8_t* loss_mask, uint8_t* response_mask, int32_t* resp_count, uint8_t* err,
                         rmi_stream_t stream);
int rmi_formulate_tail(const int32_t* resp_count, const uint8_t* err, int64_t B, int64_t* out, rmi_stream_t stream);

/* rmi_formulate_chain: the update batch after its width is known, as one host call --
 *   1. rmi_rollout_finalize(ep, seg, G, method, metrics, NULL, NULL, norm): get_rollout_states'
 *      per-env metrics (es_manager.py:173-207) and the normalised trajectory scores
 *   2. rmi_assemble_rows_ex(..., last_score = norm, ...): the left-padded batch, masks, scores
 *   3. rmi_formulate_tail(resp_count, err, B, tail)
 *   4. the n_copies device -> host copies (host[i] pinned), then the stream waited on.        */
typedef struct {
  const rmi_episode_t* ep;
  const int32_t* seg;
  int32_t G, method;
  double* metrics;
  float* norm;
  const int64_t* tokens;
  const int64_t* row_start;
  const int32_t* row_len;
  int64_t B, S, pad_id, special_token, reward_token;
  const double* scores;
  const int32_t* n_scores;
  int32_t T, n_slots, flags;
  int64_t* input_ids, *attention_mask, *position_ids;
  float* score_out;
  uint8_t* loss_mask, *response_mask;
  int32_t* resp_count;
  uint8_t* err;
  int64_t* tail;
  int32_t n_copies;                 /* <= 4                                                         */
  void* host[4];                    /* [host] pinned                                                */
  const void* dev[4];
  int64_t bytes[4];
} rmi_formulate_chain_t;
int rmi_formulate_chain(const rmi_formulate_chain_t* chain, rmi_stream_t stream);
/* rmi_formulate_chain_part: the same launches and copies in two calls that do not wait -- part 1:
 * step 1 (the finalize) and copies [0, n_early), which may read only what the finalize or earlier
 * work wrote (the metric rows, turn_info, rmi_formulate_stats' stats launched just before);
 * part 2: steps 2-3 (the assembly, the tail) and copies [n_early, n_copies).  A caller waits after
 * part 1 for the batch width (rmi_formulate_chain_wait), launches part 2 with it, and reduces the
 * metric rows on the host while the assembly runs.  rmi_formulate_chain_wait: the stream waited on. */
int rmi_formulate_chain_part(const rmi_formulate_chain_t* chain, int32_t part, int32_t n_early, rmi_stream_t stream);
int rmi_formulate_chain_wait(rmi_stream_t stream);

/* --------------------------------------------------------------- reset seeding */
/* Replaces the per-env numpy seeding of BanditEnv.reset (bandit/env.py:25-39) and
 * FrozenLakeEnv.reset's env RNG (frozen_lake/env.py:28-37), both via gymnasium
 * seeding.np_random = Generator(PCG64(SeedSequence(seed))): per seed the PCG64 state after
 * seeding and `draws` Generator.random() calls, written as rng[4][ld] (state hi, state lo,
 * inc hi, inc lo — the layout every rmi_*_t rng pointer uses); last_draw[n] (optional) = the
 * last draw (0.0 if draws == 0).  err[n] (optional): RMI_ERR_STATE for a negative seed
 * (SeedSequence raises ValueError), else 0.                                               */
int rmi_pcg64_seed(const int64_t* seeds, int64_t n, int32_t draws, uint64_t* rng, int64_t ld,
                   double* last_draw, uint8_t* err, rmi_stream_t stream);

/* ------------------------------------------------------------------------- misc */
const char* rmi_version(void);
/* Stream-ordered device-to-device copy: a 16-B-per-lane grid-stride streaming kernel (the
 * achievable-HBM-bandwidth probe bench.py reports as roofline.achievable_peak).            */
int rmi_device_copy(void* dst, const void* src, size_t bytes, rmi_stream_t stream);
/* [host] Wait until every launch enqueued on the stream has finished: the turn loop's one
 * readback (a small async device -> pinned-host copy, then this) with no Stream object.     */
int rmi_stream_synchronize(rmi_stream_t stream);
/* [host] The turn loop's readback: bytes from device src to host dst (pinned), enqueued on the
 * stream after its launches, then the stream waited on.                                      */
int rmi_readback(void* dst /*[host]*/, const void* src, size_t bytes, rmi_stream_t stream);
/* [host] Enqueue a host (pinned) -> device copy on the stream, no wait (the turn loop's small
 * index uploads).                                                                            */
int rmi_upload(void* dst, const void* src /*[host]*/, size_t bytes, rmi_stream_t stream);

/* ------------------------------------------------------------ the one-shot arena exchange
 * Replaces: the reassembly of every rank's rollout record before compute_advantage and the
 *           update (agent_trainer.py:514-515 rollout + filter, :623-655 advantage + update
 *           consume the WHOLE batch) -- in the build's N>1 path an RCCL ring
 *           all-gather (torch.distributed.all_gather_into_tensor) of the per-rank episode
 *           arena, W-1 serial hops over one xGMI link per hop.  Here every rank STORES its
 *           nbytes into all W ranks' receive regions at once (one direct hop, the W-1 peers'
 *           links in parallel), then publishes a per-(sender) arrival count with a
 *           system-scope release; a rank's gather is complete when all W senders' counts
 *           reached the epoch's.  Receive regions are allocated here (fine-grained device
 *           memory: its L2 lines are invalidated at every kernel boundary and by a system-scope
 *           acquire, so stores arriving over xGMI are never shadowed by a stale L2 line)
 *           and mapped into the peers' processes once, through HIP IPC handles the caller
 *           exchanges over its process group.
 *
 * Region layout (one per rank, rmi_xgather_region_bytes): a 4096-B header -- u64 consumed at
 * byte 0 (the last epoch whose slot this rank has finished reading), u64 arrivals[W] at byte
 * 64 (sender q's arrivals at 64 + 8q) -- then two slots of W rows of nbp =
 * round_up(nbytes, 4096) bytes; epoch e (1, 2, ...) lands in slot e & 1, sender q's bytes at
 * row q (rmi_xgather_slot_offset + q * nbp).  Two slots let epoch e+1's stores land while the
 * consumer still reads epoch e; a sender stores epoch e into peer p's slot only after p's
 * consumed >= e - 2 (p is done with the slot's previous epoch).
 *
 * rmi_xgather(x, src, flags) enqueues ONE kernel on `stream`:
 *   RMI_XG_PUBLISH: e = state[0] + 1; marks this rank's consumed = e - 1 (everything enqueued
 *     before on the stream has finished with the slot of e - 1); for each rank p, waits for
 *     p's consumed >= e - 2, stores src[0, nbytes) into p's slot e & 1, row `rank`, then adds
 *     the storing blocks' arrivals to p's arrivals[rank] (release, system scope).
 *   RMI_XG_WAIT: waits until every sender's arrivals in this rank's region reached e *
 *     blocks_per_peer and this rank's own storing blocks all finished, then sets state[0] = e.
 *   Both (the default use): one launch that returns when the whole gather has landed.
 * PUBLISH alone followed later by WAIT alone splits the exchange (each rank's halves in stream
 * order; several ranks may share one stream, every rank's PUBLISH before any WAIT).  Every
 * wait is bounded by timeout_us (0: 2 s) of the GPU's constant 100-MHz clock: on expiry the
 * kernel sets RMI_XG_ERR_* in *err (sticky) and returns, so a missing peer never hangs the
 * device.  nbytes % 16 == 0, src 16-B aligned, 1 <= world <= RMI_XG_MAX_RANKS.             */
#define RMI_XG_MAX_RANKS 16
enum { RMI_XG_PUBLISH = 1, RMI_XG_WAIT = 2 };
enum { RMI_XG_ERR_PEER_BUSY = 1, RMI_XG_ERR_ARRIVALS = 2 };
/* RMI_XG_MEM_FINEGRAINED is the one to use.  RMI_XG_MEM_UNCACHED (hipDeviceMallocUncached) is
 * kept for measurement only: in one process, after earlier exchanges' uncached regions were
 * freed, it read stale slot rows in 2 of 5 runs on MI355X.                     */
enum { RMI_XG_MEM_UNCACHED = 0, RMI_XG_MEM_FINEGRAINED = 1 };
typedef struct {
  int32_t world, rank;
  int64_t nbytes;                      /* each rank's contribution                              */
  void* region[RMI_XG_MAX_RANKS];      /* every rank's region as mapped here (own at [rank])    */
  uint64_t* state;                     /* u64[2] this rank's, zeroed: epoch, own blocks finished */
  uint32_t* err;                       /* u32[1]: RMI_XG_ERR_* bits, OR-ed in                    */
  uint64_t timeout_us;                 /* bound on every wait (0: 2 000 000)                     */
  int32_t blocks_per_peer;             /* 0: by size (rmi_xgather_blocks_per_peer)               */
} rmi_xgather_t;
/* [host] bytes of one rank's region; -1 for a bad world / nbytes                              */
int64_t rmi_xgather_region_bytes(int32_t world, int64_t nbytes);
/* [host] byte offset, in a region, of the slot epoch e (>= 1) lands in; -1 if invalid         */
int64_t rmi_xgather_slot_offset(int32_t world, int64_t nbytes, int64_t epoch);
/* [host] the storing blocks per peer rmi_xgather launches for nbytes (0 asked)                */
int32_t rmi_xgather_blocks_per_peer(int64_t nbytes);
/* [host] allocate + zero a region of `bytes` on the current device (mode RMI_XG_MEM_*) and
 * write its IPC handle (64 B) to handle [host]; free with rmi_xgather_free                     */
int rmi_xgather_alloc(int64_t bytes, int32_t mode, void** region /*[host]*/, uint8_t* handle /*[host] 64 B*/);
/* [host] map a peer's region from its handle into this process / unmap it                     */
int rmi_xgather_open(const uint8_t* handle /*[host] 64 B*/, void** region /*[host]*/);
int rmi_xgather_close(void* region);
int rmi_xgather_free(void* region);
int rmi_xgather(const rmi_xgather_t* x /*[host]*/, const void* src, int32_t flags, rmi_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* RAGEN_AMD_H */
