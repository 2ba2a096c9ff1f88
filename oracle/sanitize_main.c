/* Test infrastructure only: drives the C oracle (ballenv_oracle.c, board_oracle.c) under
 * AddressSanitizer + UndefinedBehaviorSanitizer on the host (`make -C oracle sanitize`).
 * Covers tape and Philox resets, caller actions / deltas / sampled actions, W = 1, 5, 10, 21,
 * the default and a custom obstacle config, mass TimeLimit truncation with terminal obs and
 * stats, prep_state2 blocks, and the createBoard profile (tape and Philox resets) -- every public
 * orc_* entry point. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ballenv.h"

int orc_observe(const be_config* c, const be_state* st, const be_out* out);
int orc_reset(const be_config* c, const be_state* st, const uint8_t* mask, const int16_t* tape, int32_t tape_len,
              const be_out* out, int32_t* status);
int orc_step(const be_config* c, const be_state* st, const uint8_t* actions, const int16_t* deltas,
             const int16_t* tape, const be_out* out, int32_t* status);
int orc_sample_actions(const be_config* c, uint8_t* out, int32_t steps, uint64_t seed);
int orc_policy_uniforms(const be_config* c, const uint32_t* episode, const int32_t* ep_len, uint64_t seed,
                        float* out);
int orc_observe_blocks(const be_config* c, const be_state* st, uint8_t* out);
int orc_board_reset(const be_board_config* c, const be_board_state* st, const double* tape, int32_t len,
                    float* features);
int orc_board_step(const be_board_config* c, const be_board_state* st, const uint8_t* actions, const double* deltas,
                   double* reward, uint8_t* done, float* features);
int orc_board_reset_philox(const be_board_config* c, const be_board_state* st, const uint8_t* mask, float* features);

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return (uint32_t)(rng >> 16); }

static void defaults(be_config* c, int32_t n, int32_t w) {
  static const int32_t goals[5][2] = {{12, 122}, {123, 93}, {87, 150}, {430, 440}, {230, 11}};
  static const int32_t moves[9][2] = {{1, 1}, {1, -1}, {1, 0}, {0, 1}, {0, -1}, {0, 0}, {-1, 1}, {-1, 0}, {-1, -1}};
  memset(c, 0, sizeof *c);
  c->num_envs = n; c->window = w; c->env_offset = 3; c->seed = 0xBA11;
  c->screen_width = c->screen_height = 500;
  c->strip_obs_x = 0; c->strip_obs_y = 20; c->strip_goal_x = 500; c->strip_goal_y = 20;
  c->strip_agent_x = 500; c->strip_agent_y = 10;
  c->radius_obstacle = 20; c->radius_agent = 5; c->speed_x = c->speed_y = 1;
  c->threshold_goal = 10.0; c->time_penalty = 0.0; c->min_spawn_dist = 50.0;
  c->num_static = 13; c->num_dynamic = 5; c->static_penalty = 1.0; c->dynamic_penalty = 8000.0;
  c->goal_change_step = 50; c->obs_certainty = 60; c->num_goals = 5;
  for (int g = 0; g < 5; ++g) { c->goals[g][0] = goals[g][0]; c->goals[g][1] = goals[g][1]; }
  for (int k = 0; k < BE_MAX_DYNAMIC; ++k) c->obstacle_speed[k] = 1;
  c->num_actions = 9;
  for (int a = 0; a < 9; ++a) { c->actions[a][0] = moves[a][0]; c->actions[a][1] = moves[a][1]; }
  c->time_limit = 1000; c->autoreset = 1;
}

static int run(const be_config* c, int steps, int tape_mode) {
  const int32_t N = c->num_envs, F = 4 + c->window * c->window, NS = c->num_static, ND = c->num_dynamic;
  be_state st;
  be_out out;
  st.agent = calloc(N, 4); st.goal = calloc(N, 4); st.prev_dist = calloc(N, 8); st.total_dist = calloc(N, 8);
  st.ep_return = calloc(N, 8); st.ep_len = calloc(N, 4); st.episode = calloc(N, 4);
  st.static_obs = calloc((size_t)(NS ? NS : 1) * N, 4); st.dyn_obs = calloc((size_t)(ND ? ND : 1) * N, 4);
  st.dyn_goal = calloc((size_t)(ND ? ND : 1) * N, 1);
  memset(&out, 0, sizeof out);
  out.obs = calloc((size_t)N * F, 1); out.obs_f32 = calloc((size_t)N * F, 4);
  out.reward = calloc(N, 8); out.done = calloc(N, 1); out.truncated = calloc(N, 1);
  out.terminal_obs = calloc((size_t)N * F, 1); out.final_return = calloc(N, 8); out.final_len = calloc(N, 4);
  double stats[8] = {0, 0, 0, 0, INFINITY, -INFINITY, 0, 0};
  out.stats = stats;
  int32_t status = 0;
  /* reset tapes: a reset reads a sequential stream per env; hand it plenty (tape_len, N) */
  const int32_t TL = 4 + 2 * 8 + 2 * 8 * NS + 2 * ND + 64;
  int16_t* rtape = malloc((size_t)TL * N * 2);
  /* a tape holds the reference's randint outputs: positions in [0, 500) */
  for (int64_t k = 0; k < (int64_t)TL * N; ++k) rtape[k] = (int16_t)(rnd() % 500);
  orc_reset(c, &st, NULL, tape_mode ? rtape : NULL, TL, &out, &status);
  uint8_t* acts = malloc((size_t)N * steps);
  orc_sample_actions(c, acts, steps, 7);
  int16_t* deltas = malloc((size_t)N * 4);
  int16_t* stape = malloc((size_t)(ND ? ND : 1) * 2 * N * 2);
  uint8_t* mask = malloc(N);
  for (int t = 0; t < steps; ++t) {
    for (int32_t i = 0; i < N; ++i) { deltas[2 * i] = (int16_t)(rnd() % 3) - 1; deltas[2 * i + 1] = (int16_t)(rnd() % 3) - 1; }
    /* rows (k*2 + d, N) hold the draws in the order made: randint(100) then randint(9), or a lone
     * randint(9) (obstacle level with its goal), or randint(n_other) on a goal change -- values
     * valid for every draw a slot can be */
    const int32_t n2 = c->num_goals - 1 < 9 ? c->num_goals - 1 : 9;
    for (int64_t k = 0; k < (int64_t)(ND ? ND : 1) * 2 * N; ++k) stape[k] = (int16_t)(rnd() % (uint32_t)n2);
    const int mode = t % 3;   /* caller actions / caller deltas / in-library sampled actions */
    orc_step(c, &st, mode == 0 ? acts + (size_t)t * N : NULL, mode == 1 ? deltas : NULL, tape_mode ? stape : NULL,
             &out, &status);
    if (t % 37 == 5) {   /* a masked reset mid-episode */
      for (int32_t i = 0; i < N; ++i) mask[i] = (uint8_t)(rnd() & 1);
      orc_reset(c, &st, mask, tape_mode ? rtape : NULL, TL, &out, &status);
    }
  }
  uint8_t* blocks = malloc((size_t)N * 29);
  orc_observe_blocks(c, &st, blocks);
  orc_observe(c, &st, &out);
  float* u = malloc((size_t)N * 4);
  orc_policy_uniforms(c, st.episode, st.ep_len, 5, u);
  long lit = 0;
  for (int64_t k = 0; k < (int64_t)N * F; ++k) lit += out.obs[k];
  printf("W=%d N=%d tape=%d: episodes %.0f, lit cells %ld, status %d\n", c->window, N, tape_mode, stats[0], lit, status);
  free(u); free(blocks); free(mask); free(stape); free(deltas); free(acts); free(rtape);
  free(out.obs); free(out.obs_f32); free(out.reward); free(out.done); free(out.truncated); free(out.terminal_obs);
  free(out.final_return); free(out.final_len);
  free(st.agent); free(st.goal); free(st.prev_dist); free(st.total_dist); free(st.ep_return); free(st.ep_len);
  free(st.episode); free(st.static_obs); free(st.dyn_obs); free(st.dyn_goal);
  return 0;
}

static int run_board(int32_t N, int32_t ns, int steps) {
  be_board_config c;
  memset(&c, 0, sizeof c);
  c.num_envs = N; c.num_static = ns; c.seed = 0xB0A2D;
  c.screen_width = c.screen_height = 100; c.strip_goal_x = c.strip_goal_y = 100;
  c.strip_agent_x = c.strip_agent_y = 100;
  c.agent_radius = 10; c.static_radius = 10; c.obstacle_feature_radius = 20; c.goal_threshold = 15;
  c.min_spawn_dist = 50; c.spawn_thresh_agent = 15; c.spawn_thresh_goal = 5;
  static const double acts[4][2] = {{0, -1}, {1, 0}, {0, 1}, {-1, 0}};
  c.num_actions = 4;
  for (int a = 0; a < 4; ++a) { c.actions[a][0] = acts[a][0]; c.actions[a][1] = acts[a][1]; }
  be_board_state st;
  st.agent = calloc((size_t)N * 2, 8); st.goal = calloc((size_t)N * 2, 8); st.dist = calloc(N, 8);
  st.total_dist = calloc(N, 8); st.ep_return = calloc(N, 8); st.ep_len = calloc(N, 4); st.episode = calloc(N, 4);
  st.static_obs = calloc((size_t)(ns ? ns : 1) * N, 4);
  const int32_t TL = 4 + 2 * 64 + 2 * 64 * ns;
  double* tape = malloc((size_t)TL * N * 8);
  for (int64_t k = 0; k < (int64_t)TL * N; ++k) tape[k] = (double)(rnd() % 10000) / 100.0;   /* ranf() * 100-ish */
  float* feats = calloc((size_t)N * 20, 4);
  double* rew = calloc(N, 8);
  uint8_t* done = calloc(N, 1);
  uint8_t* a = malloc(N);
  double* d = malloc((size_t)N * 16);
  int status = orc_board_reset(&c, &st, tape, TL, feats);
  for (int t = 0; t < steps; ++t) {
    for (int32_t i = 0; i < N; ++i) { a[i] = (uint8_t)(rnd() % 4); d[2 * i] = (rnd() % 7) - 3.0; d[2 * i + 1] = (rnd() % 7) - 3.0; }
    orc_board_step(&c, &st, (t & 1) ? a : NULL, (t & 1) ? NULL : d, rew, done, feats);
    if (t % 5 == 4) status |= orc_board_reset_philox(&c, &st, done, feats);   /* Philox autoreset of the done envs */
  }
  double s = 0;
  for (int64_t k = 0; k < (int64_t)N * 20; ++k) s += feats[k];
  printf("board N=%d ns=%d: reset status %d, feature sum %.3f\n", N, ns, status, s);
  free(a); free(d); free(done); free(rew); free(feats); free(tape);
  free(st.agent); free(st.goal); free(st.dist); free(st.total_dist); free(st.ep_return); free(st.ep_len);
  free(st.episode); free(st.static_obs);
  return 0;
}

int main(void) {
  const int ws[4] = {1, 5, 10, 21};
  for (int k = 0; k < 4; ++k) {
    be_config c;
    defaults(&c, 97, ws[k]);
    run(&c, 120, 0);
    run(&c, 60, 1);
    c.time_limit = 7;          /* mass truncation: terminal obs, stats, resets every few steps */
    run(&c, 40, 0);
  }
  be_config c;                 /* custom obstacle config: no statics, 12 dynamics, 2 goals, goal change 1 */
  defaults(&c, 64, 10);
  c.num_static = 0; c.num_dynamic = 12; c.num_goals = 2; c.goal_change_step = 1; c.obs_certainty = 100;
  run(&c, 80, 0);
  run(&c, 40, 1);
  run_board(53, 6, 200);
  run_board(17, 0, 50);
  printf("sanitize: OK\n");
  return 0;
}
