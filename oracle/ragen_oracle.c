/*
 * ragen_oracle.c — CPU restatement of RAGEN's hot path.  TEST INFRASTRUCTURE (see header).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fno-fast-math) -> oracle/_build/libragen_oracle.so
 */
#include "ragen_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

enum { F_TERM = 1, F_TRUNC = 2, F_DONE = 4 };
enum { I_PRESENT = 1, I_EFF = 2, I_VALID = 4, I_SUCC = 8 };

/* ------------------------------------------------------------------ PCG64 (numpy)
 * numpy/random/src/pcg64: state = state * M + inc (mod 2^128), output = XSL-RR(new state);
 * Generator.random() = (next64 >> 11) * 2^-53.                          */
static uint64_t pcg64_next(uint64_t st[4]) {
  unsigned __int128 s = ((unsigned __int128)st[0] << 64) | st[1];
  const unsigned __int128 inc = ((unsigned __int128)st[2] << 64) | st[3];
  const unsigned __int128 mul = ((unsigned __int128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
  s = s * mul + inc;
  st[0] = (uint64_t)(s >> 64);
  st[1] = (uint64_t)s;
  const uint64_t x = st[0] ^ st[1];
  const unsigned rot = (unsigned)(st[0] >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}
double orc_pcg64_random(uint64_t st[4]) { return (double)(pcg64_next(st) >> 11) * (1.0 / 9007199254740992.0); }

/* ------------------------------------------------------------- EnvStateManager.step
 * es_manager.py:149-169 for one env; step_fn executes one env.step(action).             */
typedef int (*step_fn)(void* ctx, int a, double* r, int* done, int* eff, int* succ);

static void run_env_turn(void* ctx, step_fn fn, orc_episode_t* ep, const orc_turn_t* in, int64_t b, uint8_t* err) {
  const int8_t* acts = in->actions + b * in->K;
  int n_act = in->n_actions[b];
  if (n_act > in->K) n_act = in->K;
  /* valid_actions = [lookup[a] for a in actions if a in lookup]  (:230-240) */
  int valid[64], nv = 0;
  for (int k = 0; k < n_act; ++k)
    if (acts[k] != 0) valid[nv++] = acts[k];
  int left = in->max_actions_per_traj - ep->num_actions[b];
  int n_try = nv < left ? nv : (left > 0 ? left : 0);
  /* _execute_actions (:116-128) */
  double acc = 0.0;
  int exec = 0, turn_done = 0, have_info = 0, eff = 0, succ = 0;
  for (int i = 0; i < n_try; ++i) {
    double r;
    int done, e, s;
    if (!fn(ctx, valid[i], &r, &done, &e, &s)) {
      if (err) err[b] |= 1;
      break;
    }
    acc += r;
    exec++;
    have_info = 1;
    eff = e;
    succ = s;
    if (done) {
      turn_done = 1;
      break;
    }
  }
  /* penalty (:158-159) */
  if (nv != n_act || nv == 0) ep->penalty[b] += in->format_penalty;
  /* _log_env_state (:130-144) */
  ep->num_actions[b] += exec;
  ep->n_turns[b] += 1;
  const int64_t tb = (int64_t)in->turn * ep->B + b;
  ep->turn_reward[tb] = acc;
  ep->turn_exec[tb] = (uint8_t)exec;
  ep->turn_info[tb] = have_info ? (uint8_t)(I_PRESENT | (eff ? I_EFF : 0) | I_VALID | (succ ? I_SUCC : 0)) : 0;
  uint8_t f = ep->flags[b] & (uint8_t)~F_DONE;
  if (turn_done) {
    f |= F_TERM;
    if (succ) f &= (uint8_t)~F_TRUNC;
    else f |= F_TRUNC;
  }
  /* cap (:163-166) */
  if (ep->num_actions[b] >= in->max_actions_per_traj && !turn_done) {
    f |= F_TERM | F_TRUNC;
    turn_done = 1;
  }
  if (turn_done) f |= F_DONE;
  ep->flags[b] = f;
}

static int has_input(const orc_episode_t* ep, const orc_turn_t* in, int64_t b) {
  return in->has_input ? in->has_input[b] != 0 : !(ep->flags[b] & F_DONE);
}

/* ----------------------------------------------------------------------- Sokoban
 * SokobanEnv.step (sokoban/env.py:44-51) over gym_sokoban step/_push/_move/_calc_reward
 * (App. A.1), on the byte grid exactly as numpy indexes it.                              */
typedef struct {
  int H, W, num_boxes, max_steps;
  const uint8_t* fixed;
  uint8_t* state;
  int pr, pc, nes, bot;
  uint8_t err;
} sok_t;

static int sok_idx(const sok_t* e, int r, int c, int* idx) {
  if (r < -e->H || r >= e->H || c < -e->W || c >= e->W) return 0;
  *idx = (r < 0 ? r + e->H : r) * e->W + (c < 0 ? c + e->W : c);
  return 1;
}

static const int CHG[4][2] = {{-1, 0}, {1, 0}, {0, -1}, {0, 1}};

static int sok_move(sok_t* e, int a, int* moved) {
  const int dr = CHG[(a - 1) % 4][0], dc = CHG[(a - 1) % 4][1];
  int ni, oi;
  *moved = 0;
  if (!sok_idx(e, e->pr + dr, e->pc + dc, &ni)) return 0;
  if (e->state[ni] == 1 || e->state[ni] == 2) {
    /* current_position is indexed only once the move happens (after state[new] = 5) */
    if (!sok_idx(e, e->pr, e->pc, &oi)) return 0;
    e->pr += dr;
    e->pc += dc;
    e->state[ni] = 5;
    e->state[oi] = e->fixed[oi];
    *moved = 1;
  }
  return 1;
}

static int sok_step(void* ctx, int a, double* r, int* done, int* eff, int* succ) {
  sok_t* e = (sok_t*)ctx;
  if (a < 1 || a > 8) return 0;
  const int pr0 = e->pr, pc0 = e->pc;
  e->nes += 1;
  int moved = 0;
  if (a < 5) { /* _push */
    const int dr = CHG[(a - 1) % 4][0], dc = CHG[(a - 1) % 4][1];
    const int nr = e->pr + dr, nc = e->pc + dc, br = nr + dr, bc = nc + dc;
    if (!(br >= e->H || bc >= e->W)) {
      int ni, bi, oi;
      /* can_push_box = state[new] in [3, 4]; can_push_box &= state[new_box] in [1, 2]:
       * both cells are indexed whatever the first test gave */
      if (!sok_idx(e, nr, nc, &ni) || !sok_idx(e, br, bc, &bi)) {
        e->err |= 2;
        return 0;
      }
      if ((e->state[ni] == 3 || e->state[ni] == 4) && (e->state[bi] == 1 || e->state[bi] == 2)) {
        if (!sok_idx(e, e->pr, e->pc, &oi)) {
          e->err |= 2;
          return 0;
        }
        e->pr = nr;
        e->pc = nc;
        e->state[ni] = 5;
        e->state[oi] = e->fixed[oi];
        e->state[bi] = e->fixed[bi] == 2 ? 3 : 4;
      } else if (!sok_move(e, a, &moved)) {
        e->err |= 2;
        return 0;
      }
    }
  } else if (!sok_move(e, a, &moved)) {
    e->err |= 2;
    return 0;
  }
  /* _calc_reward */
  int n_open = 0;
  for (int i = 0; i < e->H * e->W; ++i)
    if (e->state[i] == 2 || (e->fixed[i] == 2 && e->state[i] == 5)) n_open++;
  const int cur = e->num_boxes - n_open;
  double rw = -0.1;
  if (cur > e->bot) rw += 1;
  else if (cur < e->bot) rw += -1;
  if (n_open == 0) rw += 10;
  e->bot = cur;
  *r = rw;
  *done = (n_open == 0) || (e->max_steps == e->nes);
  *eff = !(pr0 == e->pr && pc0 == e->pc);
  *succ = e->bot == e->num_boxes;
  return 1;
}

int orc_sokoban_turn(int32_t H, int32_t W, int32_t num_boxes, int32_t max_steps, const uint8_t* room_fixed,
                     uint8_t* room_state, int8_t* player, int32_t* num_env_steps, int32_t* boxes_on_target,
                     orc_episode_t* ep, const orc_turn_t* in, uint8_t* err) {
  const int hw = H * W;
  for (int64_t b = 0; b < ep->B; ++b) {
    if (!has_input(ep, in, b)) continue;
    sok_t e = {H, W, num_boxes, max_steps, room_fixed + b * hw, room_state + b * hw, player[2 * b],
               player[2 * b + 1], num_env_steps[b], boxes_on_target[b], 0};
    run_env_turn(&e, sok_step, ep, in, b, err);
    if (err && e.err) err[b] |= e.err;
    player[2 * b] = (int8_t)e.pr;
    player[2 * b + 1] = (int8_t)e.pc;
    num_env_steps[b] = e.nes;
    boxes_on_target[b] = e.bot;
  }
  return 0;
}

/* -------------------------------------------------------------------- FrozenLake
 * frozen_lake/env.py:39-45 -> gymnasium FrozenLakeEnv.step + categorical_sample (App. A.2). */
typedef struct {
  int nrow, ncol, slip;
  double cs[3];
  const uint8_t* desc;
  int s;
  uint64_t st[4];
} fl_t;

static int fl_inc(const fl_t* e, int s, int a) {
  int row = s / e->ncol, col = s % e->ncol;
  if (a == 0) col = col - 1 > 0 ? col - 1 : 0;
  else if (a == 1) row = row + 1 < e->nrow - 1 ? row + 1 : e->nrow - 1;
  else if (a == 2) col = col + 1 < e->ncol - 1 ? col + 1 : e->ncol - 1;
  else if (a == 3) row = row - 1 > 0 ? row - 1 : 0;
  return row * e->ncol + col;
}

static int fl_step(void* ctx, int a, double* r, int* done, int* eff, int* succ) {
  fl_t* e = (fl_t*)ctx;
  if (a < 1 || a > 4) return 0; /* action_map[action] */
  const int ga = a - 1, prev = e->s;
  const double u = orc_pcg64_random(e->st);
  const uint8_t L = e->desc[e->s];
  if (L == 'G' || L == 'H') {
    *r = 0;
    *done = 1;
  } else {
    /* transitions for b in [(a-1)%4, a, (a+1)%4]; i = argmax(cumsum(p) > u) */
    int i = 0;
    if (e->slip) {
      i = 0;
      int found = 0;
      for (int k = 0; k < 3 && !found; ++k)
        if (e->cs[k] > u) {
          i = k;
          found = 1;
        }
      if (!found) i = 0;
    }
    const int bdir = e->slip ? (ga + 3 + i) % 4 : ga;
    e->s = fl_inc(e, e->s, bdir);
    const uint8_t nl = e->desc[e->s];
    *r = nl == 'G' ? 1.0 : 0.0;
    *done = nl == 'G' || nl == 'H';
  }
  *eff = prev != e->s;
  *succ = e->desc[e->s] == 'G';
  return 1;
}

int orc_frozenlake_turn(int32_t nrow, int32_t ncol, int32_t is_slippery, double cs0, double cs1, double cs2,
                        const uint8_t* desc, int32_t* s, uint64_t* rng, orc_episode_t* ep, const orc_turn_t* in,
                        uint8_t* err) {
  const int64_t B = ep->B;
  for (int64_t b = 0; b < B; ++b) {
    if (!has_input(ep, in, b)) continue;
    fl_t e;
    e.nrow = nrow;
    e.ncol = ncol;
    e.slip = is_slippery;
    e.cs[0] = cs0;
    e.cs[1] = cs1;
    e.cs[2] = cs2;
    e.desc = desc + b * nrow * ncol;
    e.s = s[b];
    for (int k = 0; k < 4; ++k) e.st[k] = rng[k * B + b];
    run_env_turn(&e, fl_step, ep, in, b, err);
    s[b] = e.s;
    rng[b] = e.st[0];
    rng[B + b] = e.st[1];
  }
  return 0;
}

/* ------------------------------------------------------------------------ Bandit
 * bandit/env.py:62-76                                                                   */
typedef struct {
  int start, hi_first;
  double lo, hl, hh, hp;
  uint64_t st[4];
} bd_t;

static int bd_step(void* ctx, int a, double* r, int* done, int* eff, int* succ) {
  bd_t* e = (bd_t*)ctx;
  if (a != e->start && a != e->start + 1) return 0;
  const int hi = (a == e->start) ? e->hi_first : !e->hi_first;
  if (hi) *r = orc_pcg64_random(e->st) < e->hp ? e->hh : e->hl;
  else *r = e->lo;
  *done = 1;
  *eff = 1;
  *succ = hi;
  return 1;
}

int orc_bandit_turn(int32_t start, double lo, double hi_lo, double hi_hi, double hi_prob, const uint8_t* hi_is_first,
                    uint64_t* rng, orc_episode_t* ep, const orc_turn_t* in, uint8_t* err) {
  const int64_t B = ep->B;
  for (int64_t b = 0; b < B; ++b) {
    if (!has_input(ep, in, b)) continue;
    bd_t e = {start, hi_is_first[b] != 0, lo, hi_lo, hi_hi, hi_prob, {0, 0, 0, 0}};
    for (int k = 0; k < 4; ++k) e.st[k] = rng[k * B + b];
    run_env_turn(&e, bd_step, ep, in, b, err);
    rng[b] = e.st[0];
    rng[B + b] = e.st[1];
  }
  return 0;
}

/* ------------------------------------------------------- get_rollout_states (:173-207) */
void orc_rollout_metrics(const orc_episode_t* ep, double* out) {
  for (int64_t b = 0; b < ep->B; ++b) {
    double eff = 0, val = 0;
    int present = 0;
    for (int t = 0; t < ep->T; ++t) {
      const uint8_t i = ep->turn_info[(int64_t)t * ep->B + b];
      if (i & I_PRESENT) {
        present = 1;
        eff += (i & I_EFF) ? 1.0 : 0.0;
        val += (i & I_VALID) ? 1.0 : 0.0;
      }
    }
    const uint8_t f = ep->flags[b];
    out[4 * b] = ((f & F_TERM) && !(f & F_TRUNC)) ? 1.0 : 0.0;
    out[4 * b + 1] = ep->num_actions[b];
    out[4 * b + 2] = present ? eff / ep->n_turns[b] : NAN;
    out[4 * b + 3] = present ? val / ep->n_turns[b] : NAN;
  }
}

/* scores = [sum(turn rewards)] -> float32 (ctx_manager.py:282, :64-65); penalty -> float32 (:217) */
void orc_trajectory_scores(const orc_episode_t* ep, float* score, float* pen) {
  for (int64_t b = 0; b < ep->B; ++b) {
    double s = 0;
    for (int t = 0; t < ep->T; ++t) s += ep->turn_reward[(int64_t)t * ep->B + b];
    score[b] = (float)s;
    if (pen) pen[b] = (float)ep->penalty[b];
  }
}

/* _normalize_score_tensor (ctx_manager.py:175-226); methods 0 identity 1 mean 2 mean_std 3 asym_clip */
void orc_group_normalize(const float* score, const float* pen, const int32_t* seg, int32_t G, int32_t B, int32_t method,
                         float* out) {
  if (G >= B) method = 0;
  for (int g = 0; g < G; ++g) {
    const int lo = seg[g], hi = seg[g + 1], n = hi - lo;
    double s = 0;
    for (int i = lo; i < hi; ++i) s += (double)(score[i] + (pen ? pen[i] : 0.0f));
    const double md = n ? s / n : 0;
    const float mean = (float)md;
    double q = 0;
    for (int i = lo; i < hi; ++i) {
      const double d = (double)(score[i] + (pen ? pen[i] : 0.0f)) - md;
      q += d * d;
    }
    const float sd = n > 1 ? (float)sqrt(q / (n - 1)) : NAN;
    for (int i = lo; i < hi; ++i) {
      const float x = score[i] + (pen ? pen[i] : 0.0f);
      float y = x;
      if (method == 1) y = x - mean;
      else if (method >= 2) {
        y = (sd > 1e-6f) ? (x - mean) / (sd + 1e-6f) : 0.0f;
        if (method == 3) y = y < -1.0f ? -1.0f : (y > 3.0f ? 3.0f : y);
      }
      out[i] = y;
    }
  }
}

/* ---------------------------------------------------- verl GAE (App. A.4), per row */
void orc_gae(const float* r, const float* v, const uint8_t* mask, int64_t B, int64_t L, double gamma, double lam,
             int32_t variant, float* adv, float* ret) {
  const float g = (float)gamma, gl = (float)(gamma * lam);
  for (int64_t b = 0; b < B; ++b) {
    float last = 0.0f, nv = 0.0f;
    for (int64_t t = L - 1; t >= 0; --t) {
      const int64_t i = b * L + t;
      if (variant == 0) {
        const float next = t < L - 1 ? v[i + 1] : 0.0f;
        const float delta = (r[i] + g * next) - v[i];
        last = delta + gl * last;
      } else {
        const float m = mask[i] ? 1.0f : 0.0f;
        const float delta = (r[i] + g * nv) - v[i];
        const float l2 = delta + gl * last;
        nv = v[i] * m + (1.0f - m) * nv;
        last = l2 * m + (1.0f - m) * last;
      }
      adv[i] = last;
      ret[i] = last + v[i];
    }
  }
}

/* compute_bi_level_gae_advantage_return (core_algos.py:36-88), literal two-pass form */
int orc_bilevel_gae(const float* r, const float* v, const uint8_t* mask, int64_t B, int64_t L, double gamma,
                    double lam, double hlg, float* adv, float* ret, uint8_t* err) {
  const float g = (float)gamma, gl = (float)(gamma * lam), hg = (float)hlg, hgl = (float)(hlg * lam);
  int64_t* eos = (int64_t*)malloc(sizeof(int64_t) * (L ? L : 1));
  int64_t* val = (int64_t*)malloc(sizeof(int64_t) * (L ? L : 1));
  float* upd = (float*)malloc(sizeof(float) * (L ? L : 1));
  int any_err = 0;
  for (int64_t b = 0; b < B; ++b) {
    const float* rr = r + b * L;
    const float* vv = v + b * L;
    float* aa = adv + b * L;
    float* qq = ret + b * L;
    int64_t ne = 0, nvl = 0;
    for (int64_t t = 0; t < L; ++t) {
      aa[t] = 0.0f;
      qq[t] = 0.0f;
      upd[t] = rr[t];
      if (rr[t] != 0.0f || rr[t] != rr[t]) eos[ne++] = t;
      if (mask[b * L + t]) val[nvl++] = t;
    }
    float last = 0.0f;
    for (int64_t i = ne - 1; i >= 0; --i) {
      const int64_t p = eos[i];
      const float delta = i < ne - 1 ? (upd[p] + hg * vv[eos[i + 1]]) - vv[p] : (upd[p] + 0.0f) - vv[p];
      last = delta + hgl * last;
      aa[p] = last;
    }
    for (int64_t i = 0; i < ne; ++i) {
      const int64_t p = eos[i];
      qq[p] = aa[p] + vv[p];
      upd[p] = aa[p] + vv[p];
    }
    last = 0.0f;
    if (err) err[b] = 0;
    for (int64_t i = nvl - 1; i >= 0; --i) {
      const int64_t p = val[i];
      const int is_eos = rr[p] != 0.0f || rr[p] != rr[p];
      float nextv;
      if (!is_eos) {
        if (i + 1 >= nvl) {
          if (err) err[b] = 2;
          any_err = 1;
          break;
        }
        nextv = vv[val[i + 1]];
      } else {
        nextv = 0.0f;
        last = 0.0f;
      }
      const float delta = (upd[p] + g * nextv) - vv[p];
      last = delta + gl * last;
      aa[p] = last;
      qq[p] = last + vv[p];
    }
  }
  free(eos);
  free(val);
  free(upd);
  return any_err;
}

/* verl masked_whiten; stats in double (torch sums in f32 with its own order: tolerance) */
int orc_masked_whiten(float* x, const uint8_t* mask, int64_t B, int64_t L) {
  double s = 0, c = 0;
  const int64_t n = B * L;
  for (int64_t i = 0; i < n; ++i)
    if (mask[i]) {
      s += x[i];
      c += 1;
    }
  if (c < 2) return c == 0 ? 1 : 2;
  const double mean = s / c;
  double q = 0;
  for (int64_t i = 0; i < n; ++i)
    if (mask[i]) q += (x[i] - mean) * (x[i] - mean);
  const double var = q / c * (c / (c - 1));
  const float mf = (float)mean;
  const float sc = 1.0f / sqrtf((float)var + 1e-8f);
  for (int64_t i = 0; i < n; ++i) x[i] = (x[i] - mf) * sc;
  return 0;
}

/* verl compute_grpo_outcome_advantage with contiguous groups */
void orc_grpo(const float* r, const uint8_t* mask, int64_t B, int64_t L, const int32_t* seg, int32_t G, double eps,
              int32_t norm_by_std, float* adv, float* ret) {
  float* sc = (float*)malloc(sizeof(float) * (B ? B : 1));
  for (int64_t b = 0; b < B; ++b) {
    double s = 0;
    for (int64_t t = 0; t < L; ++t) s += r[b * L + t];
    sc[b] = (float)s;
  }
  for (int g = 0; g < G; ++g) {
    const int lo = seg[g], hi = seg[g + 1], n = hi - lo;
    float mean = 0.0f, sd = 1.0f;
    if (n > 1) {
      double s = 0;
      for (int i = lo; i < hi; ++i) s += sc[i];
      const double m = s / n;
      double q = 0;
      for (int i = lo; i < hi; ++i) q += (sc[i] - m) * (sc[i] - m);
      mean = (float)m;
      sd = (float)sqrt(q / (n - 1));
    }
    for (int i = lo; i < hi; ++i) {
      float y = sc[i] - mean;
      if (norm_by_std) y = y / (sd + (float)eps);
      for (int64_t t = 0; t < L; ++t) {
        const float o = y * (mask[(int64_t)i * L + t] ? 1.0f : 0.0f);
        adv[(int64_t)i * L + t] = o;
        ret[(int64_t)i * L + t] = o;
      }
    }
  }
  free(sc);
}

/* _filter_rollout (agent_trainer.py:461-500) with the deterministic tie order (-key, index) */
typedef struct {
  float key;
  int g;
} kv_t;
static int kv_cmp(const void* a, const void* b) {
  const kv_t *x = (const kv_t*)a, *y = (const kv_t*)b;
  const int xn = x->key != x->key, yn = y->key != y->key;
  if (xn != yn) return xn ? -1 : 1; /* NaN first (largest), as torch.topk */
  if (!xn && x->key != y->key) return x->key > y->key ? -1 : 1;
  return x->g - y->g;
}
/* verl compute_reinforce_plus_plus_outcome_advantage, before its whitening (agent_trainer.py:110-117):
 * for t from L-1 down: running = r_t + gamma * running; ret_t = running; running *= mask_t (f32). */
void orc_reinforce_pp(const float* r, const uint8_t* mask, int64_t B, int64_t L, double gamma, float* ret) {
  const float g = (float)gamma;
  for (int64_t b = 0; b < B; ++b) {
    float run = 0.0f;
    for (int64_t t = L - 1; t >= 0; --t) {
      run = r[b * L + t] + g * run;
      ret[b * L + t] = run;
      run = run * (mask[b * L + t] ? 1.0f : 0.0f);
    }
  }
}

/* verl compute_remax_outcome_advantage (agent_trainer.py:118-126): ret = flip(cumsum(flip(r * m)))
 * with torch's CPU cumsum accumulator (double, each output cast to f32); adv = ret - base * m. */
void orc_remax(const float* r, const uint8_t* mask, const float* base, int64_t B, int64_t L, float* adv, float* ret) {
  for (int64_t b = 0; b < B; ++b) {
    double acc = 0.0;
    for (int64_t t = L - 1; t >= 0; --t) {
      const float m = mask[b * L + t] ? 1.0f : 0.0f;
      acc += (double)(r[b * L + t] * m);
      ret[b * L + t] = (float)acc;
      adv[b * L + t] = ret[b * L + t] - base[b] * m;
    }
  }
}

/* verl compute_rloo_outcome_advantage (agent_trainer.py:127-134), contiguous groups seg[G+1]:
 * s = sum_t r (f32 result); n > 1: s * n / (n-1) - mean * n / (n-1), else s; times the mask. */
void orc_rloo(const float* r, const uint8_t* mask, int64_t B, int64_t L, const int32_t* seg, int32_t G, float* adv) {
  float* sc = (float*)malloc(sizeof(float) * (B ? B : 1));
  for (int64_t b = 0; b < B; ++b) {
    double s = 0;
    for (int64_t t = 0; t < L; ++t) s += r[b * L + t];
    sc[b] = (float)s;
  }
  for (int g = 0; g < G; ++g) {
    const int lo = seg[g], hi = seg[g + 1], n = hi - lo;
    double s = 0;
    for (int i = lo; i < hi; ++i) s += sc[i];
    const float mean = n > 0 ? (float)(s / n) : 0.0f, fn = (float)n, fd = (float)(n - 1);
    for (int i = lo; i < hi; ++i) {
      const float y = n > 1 ? (sc[i] * fn) / fd - (mean * fn) / fd : sc[i];
      for (int64_t t = 0; t < L; ++t) adv[(int64_t)i * L + t] = y * (mask[(int64_t)i * L + t] ? 1.0f : 0.0f);
    }
  }
  free(sc);
}

void orc_filter(const float* scores, int32_t G, int32_t gs, double ratio, int32_t type, float* g_std, float* g_max,
                float* g_mean, uint8_t* keep, double* metrics) {
  kv_t* kv = (kv_t*)malloc(sizeof(kv_t) * G);
  double a[3] = {0, 0, 0};
  for (int g = 0; g < G; ++g) {
    const float* x = scores + (int64_t)g * gs;
    double s = 0;
    float mx = -INFINITY;
    for (int i = 0; i < gs; ++i) {
      s += x[i];
      mx = x[i] > mx ? x[i] : mx;
    }
    const double m = s / gs;
    double q = 0;
    for (int i = 0; i < gs; ++i) q += (x[i] - m) * (x[i] - m);
    g_std[g] = gs > 1 ? (float)sqrt(q / (gs - 1)) : NAN;
    g_max[g] = mx;
    g_mean[g] = (float)m;
    a[0] += g_std[g];
    a[1] += g_max[g];
    a[2] += g_mean[g];
    kv[g].key = type == 1 ? -g_std[g] : g_std[g];
    kv[g].g = g;
  }
  int k = ratio == 1.0 ? G : (int)(ratio * (double)G);
  qsort(kv, G, sizeof(kv_t), kv_cmp);
  double c[3] = {0, 0, 0};
  memset(keep, 0, G);
  for (int i = 0; i < k; ++i) {
    keep[kv[i].g] = 1;
    c[0] += g_std[kv[i].g];
    c[1] += g_max[kv[i].g];
    c[2] += g_mean[kv[i].g];
  }
  for (int j = 0; j < 3; ++j) {
    metrics[j] = (float)(a[j] / G);
    metrics[3 + j] = k ? (float)(c[j] / k) : NAN;
  }
  free(kv);
}

/* ------------------------------------------------------------------ A11 masks / scores
 * get_masks_and_scores (ctx_manager.py:35-70), literally: turn_indicators = cumsum(ids ==
 * special) (:43-44); masks (:45-49); with turn scores, for idx over zip_longest(*all_scores,
 * fillvalue=0) (:52) the boolean-mask assignment score_tensor[reward_position] = scores with
 * the "no position -> last column" rule (:54-57), then the Qwen roll(+1) (:58-60); without,
 * python sum at the last column (:62-63); then [:, 1:] and [:, :-1] (:64-66).  A row whose
 * turn has several reward positions makes the reference raise: err[b] = 1.              */
int orc_masks_and_scores(const int64_t* ids, int64_t B, int64_t S, int64_t sp, int64_t rt, const double* scores,
                         const int32_t* n_scores, int32_t T, int32_t n_slots, int32_t flags, float* score_out,
                         uint8_t* loss_mask, uint8_t* response_mask, uint8_t* err) {
  if (S <= 1) return 0;
  int64_t* turn = (int64_t*)malloc(sizeof(int64_t) * S);
  float* full = (float*)malloc(sizeof(float) * S);
  int bad = 0;
  for (int64_t b = 0; b < B; ++b) {
    const int64_t* row = ids + b * S;
    int64_t c = 0;
    for (int64_t p = 0; p < S; ++p) {
      c += row[p] == sp;
      turn[p] = c;
    }
    err[b] = 0;
    for (int64_t p = 0; p < S; ++p) full[p] = 0.0f;
    if (flags & 1) {
      for (int idx = 0; idx < n_slots; ++idx) {
        const float s = (idx < n_scores[b] && idx < T) ? (float)scores[(int64_t)idx * B + b] : 0.0f;
        const int64_t want = 2 * (int64_t)idx + 3;
        int64_t count = 0;
        for (int64_t p = 0; p < S; ++p)
          if (row[p] == rt && turn[p] == want) {
            full[p] = s;
            count++;
          }
        if (count == 0) full[S - 1] = s;
        if (count > 1) err[b] = 1;
      }
      if (flags & 4) { /* roll(shifts=1): new[p] = old[p-1], new[0] = old[S-1] */
        const float lastv = full[S - 1];
        for (int64_t p = S - 1; p >= 1; --p) full[p] = full[p - 1];
        full[0] = lastv;
      }
    } else {
      double sum = 0.0;
      for (int i = 0; i < n_scores[b]; ++i) sum += scores[(int64_t)i * B + b];
      full[S - 1] = (float)sum;
    }
    for (int64_t p = 0; p + 1 < S; ++p) {
      const int64_t t = turn[p];
      const uint8_t r = (t % 2 == 1) && t > 1;
      response_mask[b * (S - 1) + p] = r;
      loss_mask[b * (S - 1) + p] = (flags & 2) ? r : (uint8_t)(t > 1);
      score_out[b * (S - 1) + p] = full[p + 1];
    }
    bad |= err[b];
  }
  free(turn);
  free(full);
  return bad;
}
