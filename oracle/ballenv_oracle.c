/*
 * ballenv_oracle.c -- CPU restatement of the reference's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this (oracle/liboracle.so); the
 * product path (gym-ballenv_amd/, libballenv.so) never links or calls it.
 *
 * Pinned: tests/test_oracle_golden.py checks every function below against the
 * golden vectors in tests/golden/ (*.npz), which tests/golden/make_golden.py
 * produced by running the reference itself (BallEnv + prep_state4).
 *
 * Plain scalar C, one env at a time, written from the reference:
 *   orc_reset   <- BallEnv.reset            gym_ballenv/envs/ballenv_env.py:113-167
 *                  obstacles.__init__       ballenv_env.py:19-33
 *                  check_overlap_rect       ballenv_env.py:193-197
 *   orc_step    <- BallEnv.step             ballenv_env.py:232-289
 *                  move_obstacles           ballenv_env.py:323-353
 *                  calculate_reward         ballenv_env.py:200-229
 *                  check_overlap            ballenv_env.py:185-191
 *                  gym TimeLimit(1000)      gym_ballenv/__init__.py:4-11 (gym 0.10.9
 *                                           semantics, not in the image: unpinned)
 *   orc_observe <- prep_state4 / prep_state2 examples/ball_cnn_ac3.py:330-352, 384-412
 *
 * Random draws: the reference calls numpy's global randint.  Here every draw
 * comes either from a tape (the values the reference drew, recorded by
 * make_golden.py) or from the engine's Philox4x32-10 stream, restated from
 * Salmon et al., "Parallel random numbers: as easy as 1, 2, 3" (SC'11) with
 * the same counter layout the HIP kernels use, so perf mode is checkable too.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ballenv.h"

/* ------------------------------------------------------------------ Philox */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

/* counter = (global env id, c1, c2, purpose << 24 | sub):
 *   obstacle moves  c1 = episode, c2 = ep_len before the step: obstacle k uses the 24-bit
 *                   field f = bits [24j, 24j+24) of block sub = k / 5 (j = k % 5, the block
 *                   read as x | y<<32 | z<<64 | w<<96); its draws are randint(n0) = (f*n0)>>24,
 *                   then randint(n1) = (((f*n0) mod 2^24)*n1)>>24  (n0, n1 <= 128)
 *   sampled action  c1 = episode, c2 = ep_len before the step, sub = 0
 *   reset (Philox)  c1 = the new episode number, c2 = 0, one block per quantity:
 *                   sub = 0: gx, gy, ax, ay | sub = 1 + r: agent re-sample r (ax, ay)
 *                   sub = 1<<22 | k<<12 | a: static k attempt a (x, y) | sub = 2<<22 | k<<12: dynamic k
 *   reset (tape)    the reference's single sequential stream
 *   be_sample_actions: c1 = t, c2 = 0                                              */
enum { PURPOSE_STEP_OBS = 1, PURPOSE_ACTION = 2, PURPOSE_RESET = 3, PURPOSE_SAMPLE = 4, PURPOSE_POLICY = 5 };

static void philox4x32_10(const uint32_t ctr_in[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
    uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += PHILOX_W0; k1 += PHILOX_W1;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* word w of the Philox block for (env gid, c1, c2, purpose, sub) */
static uint32_t philox_word(uint64_t seed, uint32_t gid, uint32_t c1, uint32_t c2, uint32_t purpose,
                            uint32_t sub, int w) {
  uint32_t ctr[4] = {gid, c1, c2, (purpose << 24) | (sub & 0xFFFFFFu)};
  uint32_t out[4];
  philox4x32_10(ctr, (uint32_t)seed, (uint32_t)(seed >> 32), out);
  return out[w & 3];
}

/* 24-bit field j (0..4) of the Philox block for (env gid, c1, c2, purpose, sub) */
static uint32_t philox_field(uint64_t seed, uint32_t gid, uint32_t c1, uint32_t c2, uint32_t purpose,
                             uint32_t sub, int j) {
  uint32_t ctr[4] = {gid, c1, c2, (purpose << 24) | (sub & 0xFFFFFFu)};
  uint32_t o[4];
  philox4x32_10(ctr, (uint32_t)seed, (uint32_t)(seed >> 32), o);
  const int bit = 24 * j, w = bit >> 5, sh = bit & 31;
  uint64_t two = (uint64_t)o[w] | (w < 3 ? (uint64_t)o[w + 1] << 32 : 0);
  return (uint32_t)(two >> sh) & 0xFFFFFFu;
}

/* uniform integer in [lo, hi) from one 32-bit word (multiply-shift) */
static int32_t map_range(uint32_t r, int32_t lo, int32_t hi) {
  return lo + (int32_t)(((uint64_t)r * (uint64_t)(uint32_t)(hi - lo)) >> 32);
}

/* ------------------------------------------------------------------ helpers */
static inline int32_t pk_x(int32_t p) { return (int16_t)(p & 0xFFFF); }
static inline int32_t pk_y(int32_t p) { return (int16_t)((uint32_t)p >> 16); }
static inline int32_t pk(int32_t x, int32_t y) { return (int32_t)(((uint32_t)(uint16_t)x) | ((uint32_t)(uint16_t)y << 16)); }

/* calculate_distance, ballenv_env.py:179-183: sqrt(pow(dx,2)+pow(dy,2)) in f64 */
static double calc_dist(int32_t x1, int32_t y1, int32_t x2, int32_t y2) {
  double dx = (double)(x1 - x2), dy = (double)(y1 - y2);
  return sqrt(pow(dx, 2.0) + pow(dy, 2.0));
}

/* check_overlap, ballenv_env.py:185-191: overlap unless dist > r_obs + r_agent */
static int check_overlap(const be_config* c, int32_t x1, int32_t y1, int32_t x2, int32_t y2) {
  double d = calc_dist(x1, y1, x2, y2);
  return !(d > (double)(c->radius_obstacle + c->radius_agent));
}

/* check_overlap_rect, ballenv_env.py:193-197 (rad/2 is true division in Py3) */
static int check_overlap_rect(const be_config* c, int32_t x1, int32_t y1, int32_t x2, int32_t y2) {
  double rad = (double)c->radius_obstacle;
  return fabs((double)(x1 - x2)) < rad + c->radius_agent &&
         fabs((double)(y1 - y2)) < rad / 2.0 + c->radius_agent;
}

typedef struct {
  const be_config* c;
  const int16_t* tape; int32_t tape_len; int32_t n; int32_t env; int32_t cursor;
  int32_t word_mode; uint32_t frac;   /* step draws: successive multiply-shifts of one 24-bit field */
  uint64_t seed; uint32_t gid; uint32_t c1, c2; uint32_t purpose;
  int32_t* status;
} draw_src;

/* np.random.randint(lo, hi) stand-in */
static int32_t draw(draw_src* s, int32_t lo, int32_t hi) {
  int32_t k = s->cursor++;
  if (s->word_mode) {
    uint32_t prod = s->frac * (uint32_t)(hi - lo);   /* < 2^31 for hi - lo <= 128 */
    s->frac = prod & 0xFFFFFFu;
    return lo + (int32_t)(prod >> 24);
  }
  if (s->tape) {
    if (k >= s->tape_len) { *s->status |= BE_STATUS_RESET_TAPE_EXHAUSTED; return lo; }
    return s->tape[(int64_t)k * s->n + s->env];
  }
  return map_range(philox_word(s->seed, s->gid, s->c1, s->c2, s->purpose, (uint32_t)k >> 2, k & 3), lo, hi);
}

#define REJECT_LIMIT 4096

/* BallEnv.reset for env i, ballenv_env.py:113-167 */
static void reset_env(const be_config* c, const be_state* st, int32_t i, draw_src* ds) {
  const int32_t N = c->num_envs;
  int32_t W = c->screen_width, H = c->screen_height;
  int32_t gx = draw(ds, W - c->strip_goal_x, W);                       /* :115 */
  int32_t gy = draw(ds, H - c->strip_goal_y, H);                       /* :116 */
  int32_t ax = draw(ds, 0, c->strip_agent_x);                          /* :117 */
  int32_t ay = draw(ds, 0, c->strip_agent_y);                          /* :118 */
  double dist = sqrt(pow((double)(gx - ax), 2.0) + pow((double)(gy - ay), 2.0)); /* :119 */
  int guard = 0;
  while (calc_dist(gx, gy, ax, ay) < c->min_spawn_dist) {             /* :121-126 */
    if (++guard > REJECT_LIMIT) { *ds->status |= BE_STATUS_REJECTION_LIMIT; break; }
    ax = draw(ds, 0, c->strip_agent_x);
    ay = draw(ds, 0, c->strip_agent_y);
  }
  st->agent[i] = pk(ax, ay);
  st->goal[i] = pk(gx, gy);
  st->prev_dist[i] = dist;                                             /* state[2] = pre-resample dist (Q9) */
  st->ep_return[i] = 0.0;                                              /* :129 */
  st->ep_len[i] = 0;
  st->episode[i] = ds->c1;                                             /* new episode number */
  for (int32_t k = 0; k < c->num_static; ++k) {                        /* :131-149 */
    int32_t ox = 0, oy = 0; guard = 0;
    for (;;) {
      ox = draw(ds, c->strip_obs_x, W - c->strip_obs_x);               /* obstacles.__init__ :24-25 */
      oy = draw(ds, c->strip_obs_y, H - c->strip_obs_y);
      if (!check_overlap_rect(c, ox, oy, ax, ay) && !check_overlap_rect(c, ox, oy, gx, gy)) break;
      if (++guard > REJECT_LIMIT) { *ds->status |= BE_STATUS_REJECTION_LIMIT; break; }
    }
    st->static_obs[(int64_t)k * N + i] = pk(ox, oy);
  }
  for (int32_t k = 0; k < c->num_dynamic; ++k) {                       /* :153-164 */
    int32_t ox = draw(ds, c->strip_obs_x, W - c->strip_obs_x);
    int32_t oy = draw(ds, c->strip_obs_y, H - c->strip_obs_y);
    st->dyn_obs[(int64_t)k * N + i] = pk(ox, oy);
    st->dyn_goal[(int64_t)k * N + i] = (uint8_t)k;                    /* curr_goal = goal list[k] */
  }
  st->total_dist[i] = calc_dist(ax, ay, gx, gy);                       /* :166 */
}

/* Perf-mode reset: same rules as reset_env, one Philox block per quantity (see the header comment). */
static void reset_env_philox(const be_config* c, const be_state* st, int32_t i, uint32_t gid, uint32_t episode,
                             int32_t* status) {
  const int32_t N = c->num_envs, W = c->screen_width, H = c->screen_height;
  uint32_t o[4];
  uint32_t ctr[4] = {gid, episode, 0u, (uint32_t)PURPOSE_RESET << 24};
  philox4x32_10(ctr, (uint32_t)c->seed, (uint32_t)(c->seed >> 32), o);
  int32_t gx = map_range(o[0], W - c->strip_goal_x, W), gy = map_range(o[1], H - c->strip_goal_y, H);
  int32_t ax = map_range(o[2], 0, c->strip_agent_x), ay = map_range(o[3], 0, c->strip_agent_y);
  double dist = sqrt(pow((double)(gx - ax), 2.0) + pow((double)(gy - ay), 2.0));
  for (int32_t r = 0; calc_dist(gx, gy, ax, ay) < c->min_spawn_dist; ++r) {
    if (r >= REJECT_LIMIT - 1) { *status |= BE_STATUS_REJECTION_LIMIT; break; }
    ctr[3] = ((uint32_t)PURPOSE_RESET << 24) | (uint32_t)(1 + r);
    philox4x32_10(ctr, (uint32_t)c->seed, (uint32_t)(c->seed >> 32), o);
    ax = map_range(o[0], 0, c->strip_agent_x);
    ay = map_range(o[1], 0, c->strip_agent_y);
  }
  st->agent[i] = pk(ax, ay);
  st->goal[i] = pk(gx, gy);
  st->prev_dist[i] = dist;
  st->total_dist[i] = calc_dist(ax, ay, gx, gy);
  st->ep_return[i] = 0.0;
  st->ep_len[i] = 0;
  st->episode[i] = episode;
  for (int32_t k = 0; k < c->num_static; ++k) {
    int32_t ox = 0, oy = 0;
    for (int32_t a = 0;; ++a) {
      ctr[3] = ((uint32_t)PURPOSE_RESET << 24) | (1u << 22) | ((uint32_t)k << 12) | (uint32_t)a;
      philox4x32_10(ctr, (uint32_t)c->seed, (uint32_t)(c->seed >> 32), o);
      ox = map_range(o[0], c->strip_obs_x, W - c->strip_obs_x);
      oy = map_range(o[1], c->strip_obs_y, H - c->strip_obs_y);
      if (!check_overlap_rect(c, ox, oy, ax, ay) && !check_overlap_rect(c, ox, oy, gx, gy)) break;
      if (a >= REJECT_LIMIT - 1) { *status |= BE_STATUS_REJECTION_LIMIT; break; }
    }
    st->static_obs[(int64_t)k * N + i] = pk(ox, oy);
  }
  for (int32_t k = 0; k < c->num_dynamic; ++k) {
    ctr[3] = ((uint32_t)PURPOSE_RESET << 24) | (2u << 22) | ((uint32_t)k << 12);
    philox4x32_10(ctr, (uint32_t)c->seed, (uint32_t)(c->seed >> 32), o);
    st->dyn_obs[(int64_t)k * N + i] = pk(map_range(o[0], c->strip_obs_x, W - c->strip_obs_x),
                                        map_range(o[1], c->strip_obs_y, H - c->strip_obs_y));
    st->dyn_goal[(int64_t)k * N + i] = (uint8_t)k;
  }
}

/* prep_state2 + prep_state4 for env i, examples/ball_cnn_ac3.py:330-352, 384-412 */
static void observe_env(const be_config* c, const be_state* st, int32_t i, uint8_t* row) {
  const int32_t N = c->num_envs, Wn = c->window, F = 4 + Wn * Wn;
  int32_t ax = pk_x(st->agent[i]), ay = pk_y(st->agent[i]);
  int32_t gx = pk_x(st->goal[i]), gy = pk_y(st->goal[i]);
  memset(row, 0, (size_t)F);
  int32_t dx = gx - ax, dy = gy - ay;                                  /* prep_state2 :343-351 */
  if (dx >= 0 && dy >= 0) row[1] = 1;
  else if (dx < 0 && dy >= 0) row[0] = 1;
  else if (dx < 0 && dy < 0) row[3] = 1;
  else row[2] = 1;
  int32_t h = Wn / 2;                                                  /* int(window/2) */
  int32_t start_x = ax - c->speed_x * h, start_y = ay - c->speed_y * h;
  int32_t cur_y = start_y, counter = 4;
  for (int32_t r = 0; r < Wn; ++r) {
    for (int32_t cc = 0; cc < Wn; ++cc) {
      int32_t cur_x = start_x + c->speed_x * cc;
      int hit = 0;
      for (int32_t k = 0; k < c->num_static && !hit; ++k) {
        int32_t p = st->static_obs[(int64_t)k * N + i];
        hit = check_overlap(c, cur_x, cur_y, pk_x(p), pk_y(p));
      }
      for (int32_t k = 0; k < c->num_dynamic && !hit; ++k) {
        int32_t p = st->dyn_obs[(int64_t)k * N + i];
        hit = check_overlap(c, cur_x, cur_y, pk_x(p), pk_y(p));
      }
      if (hit) row[counter] = 1;
      counter++;
    }
    cur_y = start_y + c->speed_y * r;                                  /* row-update quirk Q1 (:409) */
  }
}

static const int32_t OBS_MOVES[9][2] = {{1, 1}, {1, -1}, {1, 0}, {0, 1}, {0, -1}, {0, 0},
                                        {-1, 1}, {-1, -1}, {-1, -1}};  /* ballenv_env.py:324 (Q4) */

/* move_obstacles for dynamic obstacle k of env i, ballenv_env.py:323-353 */
static void move_obstacle(const be_config* c, const be_state* st, int32_t i, int32_t k,
                          int32_t counter, draw_src* ds) {
  const int32_t N = c->num_envs;
  int64_t a = (int64_t)k * N + i;
  int32_t ox = pk_x(st->dyn_obs[a]), oy = pk_y(st->dyn_obs[a]);
  int32_t g = st->dyn_goal[a];
  int32_t speed = c->obstacle_speed[k];
  if (counter < c->goal_change_step) {
    int32_t tx = c->goals[g][0] - ox, ty = c->goals[g][1] - oy;
    if (tx != 0 && ty != 0) {
      if (draw(ds, 0, 100) < c->obs_certainty) {
        ox += (tx > 0 ? 1 : -1) * speed;
        oy += (ty > 0 ? 1 : -1) * speed;
      } else {
        int32_t m = draw(ds, 0, 9);
        ox += OBS_MOVES[m][0] * speed; oy += OBS_MOVES[m][1] * speed;
      }
    } else {
      int32_t m = draw(ds, 0, 9);
      ox += OBS_MOVES[m][0] * speed; oy += OBS_MOVES[m][1] * speed;
    }
    if (ox < -32768 || ox > 32767 || oy < -32768 || oy > 32767) *ds->status |= BE_STATUS_COORD_RANGE;
    st->dyn_obs[a] = pk(ox, oy);
  } else {
    int32_t n_other = 0;
    for (int32_t q = 0; q < c->num_goals; ++q)
      n_other += (c->goals[q][0] != c->goals[g][0] || c->goals[q][1] != c->goals[g][1]);
    if (n_other == 0) { *ds->status |= BE_STATUS_NO_GOAL; return; }
    int32_t pick = draw(ds, 0, n_other);
    for (int32_t q = 0; q < c->num_goals; ++q) {
      if (c->goals[q][0] != c->goals[g][0] || c->goals[q][1] != c->goals[g][1]) {
        if (pick-- == 0) { st->dyn_goal[a] = (uint8_t)q; break; }
      }
    }
  }
}

/* ------------------------------------------------------------------ public */
int orc_observe(const be_config* c, const be_state* st, const be_out* out) {
  const int32_t N = c->num_envs, F = 4 + c->window * c->window;
  for (int32_t i = 0; i < N; ++i) {
    uint8_t* row = out->obs + (int64_t)i * F;
    observe_env(c, st, i, row);
    if (out->obs_f32)
      for (int32_t f = 0; f < F; ++f) out->obs_f32[(int64_t)i * F + f] = (float)row[f];
  }
  return 0;
}

int orc_reset(const be_config* c, const be_state* st, const uint8_t* mask, const int16_t* tape,
              int32_t tape_len, const be_out* out, int32_t* status) {
  for (int32_t i = 0; i < c->num_envs; ++i) {
    if (mask && !mask[i]) continue;
    if (!tape) {
      reset_env_philox(c, st, i, (uint32_t)(c->env_offset + i), st->episode[i] + 1u, status);
      continue;
    }
    draw_src ds = {c, tape, tape_len, c->num_envs, i, 0, 0, 0u, c->seed,
                   (uint32_t)(c->env_offset + i), st->episode[i] + 1u, 0u, PURPOSE_RESET, status};
    reset_env(c, st, i, &ds);
  }
  if (out && out->obs) orc_observe(c, st, out);
  return 0;
}

static void stats_add(double* s, double ret, int32_t len) {
  s[0] += 1.0; s[1] += ret; s[2] += ret * ret; s[3] += (double)len;
  if (ret < s[4]) s[4] = ret;
  if (ret > s[5]) s[5] = ret;
}

int orc_step(const be_config* c, const be_state* st, const uint8_t* actions,
             const int16_t* deltas, const int16_t* tape, const be_out* out, int32_t* status) {
  const int32_t N = c->num_envs, F = 4 + c->window * c->window;
  for (int32_t i = 0; i < N; ++i) {
    uint32_t gid = (uint32_t)(c->env_offset + i);
    uint32_t episode = st->episode[i], len0 = (uint32_t)st->ep_len[i];
    int32_t dx, dy;
    if (actions) {
      int32_t a = actions[i];
      if (a >= c->num_actions) { *status |= BE_STATUS_BAD_ACTION; a = 0; }
      dx = c->actions[a][0]; dy = c->actions[a][1];
    } else if (deltas) {
      dx = deltas[2 * (int64_t)i]; dy = deltas[2 * (int64_t)i + 1];
    } else {
      int32_t a = map_range(philox_word(c->seed, gid, episode, len0, PURPOSE_ACTION, 0, 0), 0, c->num_actions);
      dx = c->actions[a][0]; dy = c->actions[a][1];
    }
    double old_dist = st->prev_dist[i];                                /* :236 */
    int32_t ax = pk_x(st->agent[i]), ay = pk_y(st->agent[i]);
    int32_t nx = ax + c->speed_x * dx, ny = ay + c->speed_y * dy;      /* :247-250 */
    if (nx < 0) nx = 0;
    if (ny < 0) ny = 0;
    if (nx > c->screen_width) nx = c->screen_width;
    if (ny > c->screen_height) ny = c->screen_height;
    /* dynamic obstacles, :262-264; curr_counter == ep_len mod (G+1) (all start at 0 on reset) */
    int32_t counter = st->ep_len[i] % (c->goal_change_step + 1);
    for (int32_t k = 0; k < c->num_dynamic; ++k) {
      /* tape: rows (k*2 + d, N) of this step's (Nd, 2, N) tape.
       * Philox: both draws from 24-bit field k%5 of block k/5 (successive multiply-shifts). */
      draw_src ds = {c, tape ? tape + (int64_t)k * 2 * N : NULL, 2, N, i, 0, tape ? 0 : 1,
                     tape ? 0u : philox_field(c->seed, gid, episode, len0, PURPOSE_STEP_OBS, (uint32_t)k / 5, k % 5),
                     c->seed, gid, episode, len0, PURPOSE_STEP_OBS, status};
      move_obstacle(c, st, i, k, counter, &ds);
    }
    int32_t gx = pk_x(st->goal[i]), gy = pk_y(st->goal[i]);
    double dist = sqrt(pow((double)(gx - nx), 2.0) + pow((double)(gy - ny), 2.0)); /* :268 */
    st->agent[i] = pk(nx, ny);
    int goal_flag = dist < c->threshold_goal;                          /* :276 */
    /* calculate_reward, :200-229 */
    double reward = 0.0 - c->time_penalty;
    reward += (old_dist - dist) / st->total_dist[i];
    int hit = 0;
    for (int32_t k = 0; k < c->num_static && !hit; ++k) {
      int32_t p = st->static_obs[(int64_t)k * N + i];
      if (check_overlap(c, nx, ny, pk_x(p), pk_y(p))) { reward -= c->static_penalty; hit = 1; }
    }
    for (int32_t k = 0; k < c->num_dynamic && !hit; ++k) {
      int32_t p = st->dyn_obs[(int64_t)k * N + i];
      if (check_overlap(c, nx, ny, pk_x(p), pk_y(p))) { reward -= c->dynamic_penalty; hit = 1; }
    }
    st->ep_return[i] += reward;                                        /* :280 */
    st->prev_dist[i] = dist;                                           /* next step's state[2] */
    int32_t len = st->ep_len[i] + 1;
    st->ep_len[i] = len;
    int env_done = goal_flag || hit;                                   /* :286 */
    int trunc = c->time_limit > 0 && len >= c->time_limit;             /* TimeLimit */
    int done = env_done || trunc;
    if (out->reward) out->reward[i] = reward;
    if (out->done) out->done[i] = (uint8_t)done;
    if (out->truncated) out->truncated[i] = (uint8_t)(trunc && !env_done);
    if (done) {
      if (out->final_return) out->final_return[i] = st->ep_return[i];
      if (out->final_len) out->final_len[i] = len;
      if (out->stats) stats_add(out->stats, st->ep_return[i], len);
      if (c->autoreset) {
        if (out->terminal_obs) observe_env(c, st, i, out->terminal_obs + (int64_t)i * F);
        reset_env_philox(c, st, i, gid, episode + 1u, status);
      }
    }
    if (out->obs) {
      uint8_t* row = out->obs + (int64_t)i * F;
      observe_env(c, st, i, row);
      if (out->obs_f32)
        for (int32_t f = 0; f < F; ++f) out->obs_f32[(int64_t)i * F + f] = (float)row[f];
    }
  }
  return 0;
}

int orc_sample_actions(const be_config* c, uint8_t* out, int32_t steps, uint64_t seed) {
  for (int32_t t = 0; t < steps; ++t)
    for (int32_t i = 0; i < c->num_envs; ++i)
      out[(int64_t)t * c->num_envs + i] = (uint8_t)map_range(
          philox_word(seed, (uint32_t)(c->env_offset + i), (uint32_t)t, 0u, PURPOSE_SAMPLE, 0, 0), 0,
          c->num_actions);
  return 0;
}

/* exposed for the exhaustive Philox/known-answer tests */
void orc_philox4x32_10(const uint32_t ctr[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
  philox4x32_10(ctr, k0, k1, out);
}

/* The uniform behind be_policy_act's Categorical draw for env i (select_action,
 * examples/ball_cnn_ac3.py:210-220): word 0 of Philox(seed; gid, episode, ep_len,
 * POLICY<<24), top 24 bits / 2^24, in [0, 1).  The draw itself (inverse CDF of
 * the fp32 probs) is restated in torch by gym_ballenv_amd.policy.torch_select_action. */
int orc_policy_uniforms(const be_config* c, const uint32_t* episode, const int32_t* ep_len, uint64_t seed,
                        float* u_out) {
  for (int32_t i = 0; i < c->num_envs; ++i)
    u_out[i] = (float)(philox_word(seed, (uint32_t)(c->env_offset + i), episode[i], (uint32_t)ep_len[i],
                                   PURPOSE_POLICY, 0, 0) >> 8) * (1.0f / 16777216.0f);
  return 0;
}

/* prep_state2 of examples/ball_env_reinforce.py:130-172 (with block_to_arrpos :169-172):
 * the 29-input block-count encoding.  out[0:4] = quadrant one-hot (as prep_state4's),
 * out[16] = 1 (the agent's own cell), then per obstacle (statics, then dynamics, i.e.
 * state[3:]) with x_dist = ax - ox, y_dist = ay - oy: if both are non-zero,
 * x_block = sign(x_dist) * (x_dist - 10) // 20 (floor division; likewise y), else both
 * blocks are 0; if |x_block| < 3 and |y_block| < 3: out[4 + 12 + 5*y_block + x_block] += 1. */
static int32_t floordiv20(int32_t a) { return a >= 0 ? a / 20 : -((-a + 19) / 20); }

int orc_observe_blocks(const be_config* c, const be_state* st, uint8_t* out) {
  const int32_t N = c->num_envs;
  for (int32_t i = 0; i < N; ++i) {
    uint8_t* row = out + (int64_t)i * 29;
    memset(row, 0, 29);
    const int32_t ax = pk_x(st->agent[i]), ay = pk_y(st->agent[i]);
    const int32_t gx = pk_x(st->goal[i]), gy = pk_y(st->goal[i]);
    const int32_t dx = gx - ax, dy = gy - ay;                          /* :139-150 */
    if (dx >= 0 && dy >= 0) row[1] = 1;
    else if (dx < 0 && dy >= 0) row[0] = 1;
    else if (dx < 0 && dy < 0) row[3] = 1;
    else row[2] = 1;
    row[16] = 1;                                                       /* :138 */
    const int32_t nobs = c->num_static + c->num_dynamic;
    for (int32_t k = 0; k < nobs; ++k) {                               /* :152-165 */
      const int32_t p = k < c->num_static ? st->static_obs[(int64_t)k * N + i]
                                          : st->dyn_obs[(int64_t)(k - c->num_static) * N + i];
      const int32_t xd = ax - pk_x(p), yd = ay - pk_y(p);
      int32_t xb = 0, yb = 0;
      if (xd != 0 && yd != 0) {
        xb = floordiv20(xd > 0 ? xd - 10 : 10 - xd);
        yb = floordiv20(yd > 0 ? yd - 10 : 10 - yd);
      }
      if (abs(xb) < 3 && abs(yb) < 3) row[4 + 12 + 5 * yb + xb] += 1;
    }
  }
  return 0;
}
