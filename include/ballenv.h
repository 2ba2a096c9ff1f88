/*
 * ballenv.h -- C ABI of the MI355X batched BallEnv step engine (libballenv.so).
 *
 * The reference (ranok92/gym-ballenv) is pure Python; the "FFI" this library
 * stands behind is the gym.Env protocol that examples/ball_cnn_ac3.py drives:
 *
 *   be_config            <- BallEnv.__init__ constants + customize_environment(args)
 *                           (gym_ballenv/envs/ballenv_env.py:11-18, 43-85, 87-109;
 *                            argparse defaults examples/ball_cnn_ac3.py:37-59)
 *   be_reset             <- BallEnv.reset()            (ballenv_env.py:113-167)
 *   be_step              <- BallEnv.step(action)       (ballenv_env.py:232-289, incl.
 *                           move_obstacles :323-353, calculate_reward :200-229,
 *                           check_overlap :185-191) followed by
 *                           prep_state4(state, W)      (examples/ball_cnn_ac3.py:384-412,
 *                           quadrant prep_state2 :330-352) and the gym TimeLimit
 *                           registered with timestep_limit=1000 (gym_ballenv/__init__.py:4-11)
 *   be_observe           <- prep_state4(state, W) on the current state
 *
 * Conventions
 *   - Plain C: no C++ types, no exceptions cross this boundary.  Every entry
 *     point returns BE_OK (0) or a negative BE_E* code; be_last_error() gives
 *     the message for the last failing call on that context (or, for a NULL
 *     context, the last process-wide failure).
 *   - All per-env device buffers are allocated and owned by the CALLER
 *     (PyTorch tensors); the library owns one word of device scratch (the
 *     status word).  Every compute call is asynchronous and
 *     ordered on the hipStream_t the caller passes (as void*).
 *   - Layout is struct-of-arrays with the env index as the unit-stride axis:
 *     an (x, y) position is two int16 in one 32-bit word (x low, y high),
 *     i.e. an (N, 2) int16 array; per-obstacle arrays are (K, N, 2) int16.
 *   - One context per (device, config).  No internal threads.  Every entry point
 *     makes the context's device current for the call and restores the calling
 *     thread's current device before it returns: no be_* call changes which GPU
 *     the caller's later HIP / torch calls use.
 *   - Randomness (perf mode): Philox4x32-10 keyed by cfg.seed with counter
 *     (global env id, episode, ep_len, purpose|sub).  Every draw is a pure
 *     function of per-env state, so results do not depend on launch order,
 *     graph replay, or how the batch is split across GPUs.
 */
#ifndef BALLENV_H
#define BALLENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BE_ABI_VERSION 7

#define BE_MAX_STATIC   64
#define BE_MAX_DYNAMIC  32
#define BE_MAX_GOALS    16
#define BE_MAX_ACTIONS  16
#define BE_MAX_WINDOW   64

enum {
  BE_OK = 0,
  BE_E_INVALID = -1,   /* bad argument / config */
  BE_E_HIP = -2,       /* HIP runtime error */
  BE_E_NOMEM = -3,
  BE_E_DEVICE = -4     /* device-side status word reported a failure */
};

/* Device-side status bits (be_status). */
enum {
  BE_STATUS_RESET_TAPE_EXHAUSTED = 1,  /* a reset consumed more draws than its tape held */
  BE_STATUS_REJECTION_LIMIT = 2,       /* a reset rejection loop hit its bound */
  BE_STATUS_BAD_ACTION = 4,            /* action index >= num_actions */
  BE_STATUS_COORD_RANGE = 8,           /* a dynamic obstacle left the int16 range; the stored
                                          coordinate wraps (two's complement int16).  The
                                          reference's obstacles are unbounded ints (ballenv_env.py
                                          :334-347).  be_config_check rejects configs that can get
                                          here within an episode (autoreset with a time limit);
                                          with time_limit 0 or autoreset 0 poll be_status. */
  BE_STATUS_NO_GOAL = 16               /* goal change with no other goal (reference raises) */
};

typedef struct be_config {
  int32_t num_envs;          /* N on this device */
  int32_t window;            /* W of prep_state4 (1..BE_MAX_WINDOW) */
  int64_t env_offset;        /* global id of local env 0 (rank * N); keys the Philox streams */
  uint64_t seed;             /* Philox key for resets / obstacle moves / sampled actions */

  /* field and spawn strips, ballenv_env.py:11-18 */
  int32_t screen_width, screen_height;                 /* 500, 500 */
  int32_t strip_obs_x, strip_obs_y;                    /* 0, 20 */
  int32_t strip_goal_x, strip_goal_y;                  /* 500, 20 */
  int32_t strip_agent_x, strip_agent_y;                /* 500, 10 */

  /* BallEnv.__init__ constants, ballenv_env.py:49-65 */
  int32_t radius_obstacle;   /* radius_rand_person = 20 */
  int32_t radius_agent;      /* radius_ctrl_person = 5 */
  int32_t speed_x, speed_y;  /* speedx/y_ctrl_person = 1 (also the window cell step) */
  double threshold_goal;     /* 10 (strict <) */
  double time_penalty;       /* timepenalty = 0 */
  double min_spawn_dist;     /* reset re-sample distance, ballenv_env.py:122 (50) */

  /* customize_environment(args), ballenv_env.py:87-109 */
  int32_t num_static;        /* args.static_obstacles (13) */
  int32_t num_dynamic;       /* args.dynamic_obstacles (5) */
  double static_penalty;     /* args.static_penalty[1]  (threshold_2_penalty, 1) */
  double dynamic_penalty;    /* args.dynamic_penalty[1] (8000) */
  int32_t goal_change_step;  /* args.time_step_for_change (50) */
  int32_t obs_certainty;     /* args.rd_th_obs (60): P(directed move) in percent */
  int32_t num_goals;         /* len(args.obs_goal_position) */
  int32_t goals[BE_MAX_GOALS][2];
  int32_t obstacle_speed[BE_MAX_DYNAMIC];

  /* action table: index -> (dx, dy); default = move_list of ball_cnn_ac3.py:530 */
  int32_t num_actions;
  int32_t actions[BE_MAX_ACTIONS][2];

  int32_t time_limit;        /* gym TimeLimit max_episode_steps (1000); 0 = none */
  int32_t autoreset;         /* 1: a done env is reset inside be_step (vector-env semantics) */
} be_config;

/* Per-env state, all device pointers owned by the caller. */
typedef struct be_state {
  int32_t* agent;       /* (N)  int16x2 packed (x, y)            state[0]          */
  int32_t* goal;        /* (N)  int16x2 packed                    state[1]          */
  double* prev_dist;    /* (N)  f64                               state[2] / old_dist */
  double* total_dist;   /* (N)  f64                               total_distance    */
  double* ep_return;    /* (N)  f64                               total_reward_accumulated */
  int32_t* ep_len;      /* (N)  steps since reset (TimeLimit elapsed; also the obstacles' curr_counter phase) */
  uint32_t* episode;    /* (N)  resets so far; with ep_len it keys this env's Philox draws */
  int32_t* static_obs;  /* (Ns, N) int16x2 packed                 static_obstacle_list */
  int32_t* dyn_obs;     /* (Nd, N) int16x2 packed                 dynamic_obstacle_list */
  uint8_t* dyn_goal;    /* (Nd, N) index into goals               obstacle.curr_goal */
} be_state;

/* Step / observe outputs (device pointers; NULL = not requested). */
typedef struct be_out {
  uint8_t* obs;           /* (N, 4+W*W) u8 0/1: quadrant one-hot ++ W*W window */
  float* obs_f32;         /* (N, 4+W*W) f32 copy of the same (what prep_state4 returns) */
  double* reward;         /* (N) f64 (be_step only) */
  uint8_t* done;          /* (N) 0/1 (be_step only) */
  uint8_t* truncated;     /* (N) 0/1: done came from the time limit alone */
  uint8_t* terminal_obs;  /* (N, 4+W*W): obs of the terminal state, rows of done envs only (autoreset) */
  double* final_return;   /* (N): episode return, written for done envs only */
  int32_t* final_len;     /* (N): episode length, written for done envs only */
  double* stats;          /* (be_stats_slots(cfg), 8) f64 accumulators, one slot per 32 envs of the step
                             kernel (no atomics): [0]=episodes, [1]=sum return, [2]=sum return^2,
                             [3]=sum length, [4]=min return, [5]=max return, [6..7] unused; the caller
                             initialises [4]=+inf, [5]=-inf, the rest 0, and reduces over slots */
} be_out;

typedef struct be_ctx be_ctx;

/* ---- pure host functions (no GPU needed) ---- */
int be_abi_version(void);
/* Fill cfg with the ball_cnn_ac3.py / BallEnv defaults for N envs and window W. */
int be_config_default(be_config* cfg, int32_t num_envs, int32_t window);
/* Validate cfg; on failure returns BE_E_INVALID and writes a message into msg.
 * Besides the ranges, with autoreset and time_limit > 0 it requires
 *   max spawn extent + max|obstacle_speed| * time_limit <= 32767
 * (spawn extent: max(|strip_obs|, |screen - strip_obs|) per axis), so no dynamic obstacle can
 * leave the int16 coordinates within an episode (BE_STATUS_COORD_RANGE).                    */
int be_config_check(const be_config* cfg, char* msg, int32_t msg_len);
/* Bytes of HBM traffic per env-step the step kernel is designed to move (u8 obs). */
int64_t be_step_bytes(const be_config* cfg);
/* Number of 8-double slots the be_out.stats buffer must hold for this config. */
int64_t be_stats_slots(const be_config* cfg);
const char* be_last_error(const be_ctx* ctx);

/* Which kernel an entry point launches for this context (for profiles and bench lines: the
 * name matches rocprofv3's kernel name without the namespace/argument list), or NULL for a
 * bad ctx / entry.  No GPU work.  Diagnostics only; the reference has no counterpart. */
enum { BE_ENTRY_STEP_ACTIONS = 0,   /* be_step with caller action indices           */
       BE_ENTRY_STEP_SAMPLED = 1,   /* be_step with in-kernel sampled actions       */
       BE_ENTRY_ROLLOUT = 2,        /* be_rollout (NULL when it falls back to looping be_step) */
       BE_ENTRY_RESET = 3, BE_ENTRY_OBSERVE = 4 };
const char* be_kernel_name(const be_ctx* ctx, int32_t entry);

/* ---- device functions ---- */
int be_create(const be_config* cfg, int32_t device, be_ctx** out);
int be_destroy(be_ctx* ctx);

/* Reset envs (all, or those with mask[i] != 0) and write the obs of every env.
 * A reset env's episode counter is incremented first.
 * reset_tape == NULL: draws come from Philox(seed; global env id, new episode).
 * reset_tape != NULL: (tape_len, N) int16, the randint values the reference's
 * reset() would consume, in call order (parity mode).                           */
int be_reset(be_ctx* ctx, const be_state* st, const uint8_t* mask,
             const int16_t* reset_tape, int32_t tape_len, const be_out* out, void* stream);

/* One step of every env.
 * actions:       (N) u8 index into cfg.actions, or NULL to use action_deltas.
 * action_deltas: (N, 2) int16 raw (dx, dy) as BallEnv.step accepts, or NULL
 *                (both NULL: actions are sampled uniformly from Philox).
 * draw_tape:     (Nd, 2, N) int16: the move_obstacles randint values of this
 *                step per obstacle in call order (parity mode), or NULL (Philox). */
int be_step(be_ctx* ctx, const be_state* st, const uint8_t* actions, const int16_t* action_deltas,
            const int16_t* draw_tape, const be_out* out, void* stream);

/* `steps` consecutive be_step calls in one launch (a fused rollout), for an action tape.
 * actions: (steps, N) u8 indices into cfg.actions.  Outputs are per step: out->obs
 * (steps, N, 4+W*W) u8, out->reward (steps, N) f64, out->done / truncated (steps, N) u8,
 * out->final_return / final_len (steps, N) and out->terminal_obs (steps, N, 4+W*W) (rows of
 * reset envs only), or NULL; out->stats accumulates as for be_step.  out->obs_f32 must be
 * NULL; N*(4+W*W) must be a multiple of 16.
 * Results are bit-identical to `steps` be_step calls with actions + s*N (same state, same
 * Philox draws).  The reference has no batched counterpart: it is the caller's loop
 *   for t: state, reward, done, _ = env.step(move_list[a_t]); prep_state4(state)
 * (examples/ball_cnn_ac3.py:573-600 over ballenv_env.py:232-289), run for every env.
 * The default shape (13 static + 5 dynamic obstacles, W 5 or 10, unit moves) runs one kernel
 * that keeps each env's state in registers; other configs loop be_step.             */
int be_rollout(be_ctx* ctx, const be_state* st, const uint8_t* actions, int32_t steps, const be_out* out,
               void* stream);

/* `steps` be_step launches (one kernel per step, caller actions + s*N) queued from a host loop
 * in the library, with the same `out` every step: out holds the last step's outputs (and
 * stats accumulate) exactly as after `steps` be_step calls.  The reference's counterpart is
 * the caller's per-step loop (examples/ball_cnn_ac3.py:573-600): this is that loop for every
 * env, minus the per-call Python overhead.                                             */
int be_step_n(be_ctx* ctx, const be_state* st, const uint8_t* actions, int32_t steps, const be_out* out,
              void* stream);

/* prep_state4 of the current state of every env (no state change). */
int be_observe(be_ctx* ctx, const be_state* st, const be_out* out, void* stream);

/* Fill actions_out (steps, N) u8 with uniform action indices from Philox keyed
 * by (seed, global env id): identical per global env at any GPU count.         */
int be_sample_actions(be_ctx* ctx, uint8_t* actions_out, int32_t steps, uint64_t seed, void* stream);

/* Synchronise the stream and read (then clear) the device status word. */
int be_status(be_ctx* ctx, int32_t* status_out, void* stream);

/* ---- env-state checkpoint (SURVEY 8(b) be_save_state / be_load_state; the reference keeps no
 * env checkpoint, only torch.save of the policy, examples/ball_cnn_ac3.py:637-639) ----
 * The be_state arrays of every env packed into ONE contiguous blob of be_state_blob_bytes(cfg)
 * bytes, in device or host memory: a 64-byte header (magic "BALLENV1", ABI version, N, Ns, Nd,
 * blob bytes) then agent, goal, prev_dist, total_dist, ep_return, ep_len, episode, static_obs,
 * dyn_obs, dyn_goal in be_state order, each array at a 16-byte aligned offset.
 * be_save_state: asynchronous copies on the stream (graph-capturable).  be_load_state:
 * SYNCHRONISES the stream to read and check the header (BE_E_INVALID when it does not match this
 * context's N / Ns / Nd), then copies asynchronously -- it cannot be captured in a HIP graph.  A saved blob restores the envs bit for bit, Philox positions included
 * (episode / ep_len key every draw).                                                        */
int64_t be_state_blob_bytes(const be_config* cfg);
int be_save_state(be_ctx* ctx, const be_state* st, void* blob, void* stream);
int be_load_state(be_ctx* ctx, const be_state* st, const void* blob, void* stream);

/* ---- the autoreset pool (a cache inside the context; no reference counterpart) ----
 * In Philox mode BallEnv.reset (ballenv_env.py:113-167) of env i into episode e is a pure
 * function of (seed, global id, e) and the config.  When be_step's kernel is a fixed-shape one
 * that consumes it (step2_kernel at W=10, stepw_kernel at W=5, and the one-lane kernel up to
 * 128 x 4 x CUs envs -- two waves per SIMD; past that its waves hide the draws and the pool
 * measured slower -- all at the reference's 13 + 5 obstacles), the context holds, per env, the precomputed resets into episodes e+1 and e+2 (ep = the env's
 * episode); a finishing env copies its entry instead of drawing the reset on the step's critical
 * path, and draws it inline as before when the entry is stale.  Results are bit-identical either
 * way -- the pool changes timing only.  be_reset and be_load_state fill it after their own work,
 * and be_step queues a fill every `period` step launches (default 128; BALLENV_POOL_PERIOD, and
 * BALLENV_POOL=0 disables the pool, for A/B runs).  The pool serves one state: the one last
 * reset or loaded (or the first stepped); steps of any other state draw every reset inline, so
 * entries are only read and written by launches the caller already orders on one stream.
 * be_pool_fill: fill now (every env's stale entries) and make st the pool's state.
 * be_pool_invalidate: mark every entry unwritten (async on the stream): the inline path until the
 * next fill.  be_pool_set_period / be_pool_period: step launches per fill (0: only the explicit ones).
 * be_pool_bytes: the pool's device bytes (0: this context has no pool). */
int be_pool_fill(be_ctx* ctx, const be_state* st, void* stream);
int be_pool_invalidate(be_ctx* ctx, void* stream);
int be_pool_set_period(be_ctx* ctx, int32_t period);
int32_t be_pool_period(const be_ctx* ctx);
int64_t be_pool_bytes(const be_ctx* ctx);
/* Test hook (synchronous; device-wide sync first): read (write = 0) or overwrite (write = 1) env's
 * entry in slot (0 / 1: the slot of episode x is x & 1).  words: TAG, AGENT, GOAL, ROWS0..2, then
 * the NS + ND obstacles' packed xy (6 + 13 + 5 words); f64: PREV, TOTAL.  ROWS0 bit 30 marks a
 * written entry, bit 31 a rejection-limit hit (layout: csrc/ballenv.hip, "the autoreset pool"). */
int be_pool_entry(be_ctx* ctx, int32_t env, int32_t slot, uint32_t* words, double* f64, int32_t write);

/* ---- on-GPU select_action for batched rollouts (BASELINE config 5) ----
 * Replaces, for every env at once, the caller's per-step
 *   probs, value = Policy(W)(prep_state4(state))      examples/ball_cnn_ac3.py:109-146
 *   action ~ Categorical(probs); saved log_prob, value  ball_cnn_ac3.py:210-220
 * (the reference runs it per single env with a host round trip per step,
 * ball_cnn_ac3.py:573-600).  fc1 runs on the int8 matrix cores against a
 * 24-bit fixed-point image of the fp32 weights (see csrc/policy.hip); the heads,
 * softmax and log_prob are fp32.  The draw is an inverse-CDF of a Philox uniform
 * keyed by (seed; global env id, episode, ep_len), so it is reproducible and
 * independent of GPU count and graph replay.                                     */
typedef struct be_policy be_policy;

typedef struct be_act_out {
  uint8_t* action;   /* (N) u8 sampled action index (feeds be_step's actions) */
  float* log_prob;   /* (N) f32 log probs[action], or NULL */
  float* value;      /* (N) f32 value_head output, or NULL */
  float* probs;      /* (N, A) f32 softmax probabilities, or NULL */
} be_act_out;

/* A policy for ctx's window (inputs 4+W*W <= 128), hidden <= 256, actions <= 15. */
int be_policy_create(be_ctx* ctx, int32_t hidden, int32_t num_actions, be_policy** out);
int be_policy_destroy(be_policy* pol);
/* (Re)load weights from DEVICE f32 arrays in torch state_dict layout:
 * fc1_w (H, 4+W*W), fc1_b (H), act_w (A, H), act_b (A), val_w (1, H), val_b (1).
 * Asynchronous on stream (one packing kernel); graph-capturable.                  */
int be_policy_load(be_policy* pol, const float* fc1_w, const float* fc1_b, const float* act_w, const float* act_b,
                   const float* val_w, const float* val_b, void* stream);
/* Policy forward + draw for every env from obs (N, 4+W*W) u8; st supplies episode/ep_len (Philox key). */
int be_policy_act(be_policy* pol, const be_state* st, const uint8_t* obs, const be_act_out* out, uint64_t seed,
                  void* stream);

/* `steps` config-5 steps in one launch: for s in 0..steps-1
 *   act[s] = select_action(obs_s) (as be_policy_act, same Philox draw);  be_step(act[s]) -> obs_{s+1}
 * obs_in: (N, F) obs of the current state (obs_0, e.g. the env's obs buffer).  out: per-step
 * (steps, N, ...) outputs as for be_rollout; out->obs (steps, N, F) records obs_1..obs_steps or is
 * NULL; obs_last (N, F) receives obs_steps (may equal obs_in) or is NULL; one of the two is
 * required.  act: (steps, N) action / log_prob / value (probs must be NULL).  N*F % 16 == 0.
 * Bit-identical to the be_policy_act + be_step loop (ball_cnn_ac3.py:573-600 for every env).
 * The default env shape with the Policy(10) / Policy(5) shapes runs one kernel with the packed
 * weights in LDS and each env's state in registers; other shapes run that loop.          */
int be_policy_rollout(be_policy* pol, const be_state* st, const uint8_t* obs_in, uint8_t* obs_last, int32_t steps,
                      const be_out* out, const be_act_out* act, uint64_t seed, void* stream);
/* Bytes of the packed weight image (staged once per workgroup in LDS). */
int64_t be_policy_bytes(const be_policy* pol);

/* ---- sibling observation formats (the reference's other callers) ----
 * prep_state2 of examples/ball_env_reinforce.py:130-172 for every env's current state:
 * (N, 29) block counts -- quadrant one-hot, [16] = 1 (the agent's cell), +1 per obstacle
 * in its 20-px block of the 5x5 grid -- as u8 (out) and/or f32 (out_f32; NULL = skip). */
int be_observe_blocks(be_ctx* ctx, const be_state* st, uint8_t* out, float* out_f32, void* stream);

/* ---- the createBoard physics profile ----
 * N independent ballenv_pygame.createBoard worlds (reset :460-513, step :650-675,
 * calc_reward :680-706) with the 20 featureExtractor features (featureExtractor.py:247-265)
 * that step() computes.  f64 coordinates (ranf spawns), static obstacles only (the
 * reference's dynamic path is not runnable: createBoard never sets obstacle_goal_list). */
#define BE_BOARD_MAX_STATIC 32
#define BE_BOARD_MAX_ACTIONS 16
#define BE_BOARD_FEATURES 20

typedef struct be_board_config {
  int32_t num_envs;
  int32_t num_static;         /* createBoard(static_obstacles=) */
  int64_t env_offset;         /* global id of local env 0 (Philox key) */
  uint64_t seed;
  int32_t screen_width, screen_height;                /* _screen_width/_height = 100 (:8-9) */
  int32_t strip_obs_x, strip_obs_y;                   /* 0, 0 */
  int32_t strip_goal_x, strip_goal_y;                 /* 100, 100 */
  int32_t strip_agent_x, strip_agent_y;               /* 100, 100 */
  double agent_radius;        /* agent_radius = 10 (:316) */
  double static_radius;       /* static_obstacle_radius = 10: collisions at <= static + agent (:381-387) */
  double obstacle_feature_radius;  /* Obstacle.rad = 20 (:35-38): featureExtractor's calcDistance */
  double goal_threshold;      /* 15, strict < (:345, :690) */
  double min_spawn_dist;      /* 50: agent re-sampled while closer to the goal (:476-481) */
  double spawn_thresh_agent, spawn_thresh_goal;       /* 15, 5: static spawn rejection (:494) */
  int32_t num_actions;
  double actions[BE_BOARD_MAX_ACTIONS][2];            /* actionArray (:352-353): (0,-1),(1,0),(0,1),(-1,0) */
  int32_t time_limit;         /* 0 = none (createBoard has no TimeLimit) */
  int32_t autoreset;          /* 1: a done env is reset inside be_board_step */
} be_board_config;

typedef struct be_board_state {
  double* agent;        /* (N, 2) f64  state[0] */
  double* goal;         /* (N, 2) f64  state[1] */
  double* dist;         /* (N) f64     state[2] */
  double* total_dist;   /* (N) f64     total_distance */
  double* ep_return;    /* (N) f64     total_reward_accumulated */
  int32_t* ep_len;      /* (N) */
  uint32_t* episode;    /* (N) resets so far (Philox key) */
  int32_t* static_obs;  /* (Ns, N) int16x2 packed integer obstacle positions */
} be_board_state;

typedef struct be_board_out {
  float* features;      /* (N, 20) f32 featureExtractor output (sensor_readings), or NULL */
  double* reward;       /* (N) (step only) */
  uint8_t* done;        /* (N) (step only) */
  uint8_t* truncated;   /* (N) or NULL */
} be_board_out;

typedef struct be_board be_board;

int be_board_config_default(be_board_config* cfg, int32_t num_envs, int32_t num_static);
int be_board_create(const be_board_config* cfg, int32_t device, be_board** out);
int be_board_destroy(be_board* b);
const char* be_board_last_error(const be_board* b);
/* createBoard.reset for every env (or mask[i] != 0).  reset_tape: (tape_len, N) f64, the
 * reference's np.random.ranf / randint values in call order (parity); NULL: Philox. */
int be_board_reset(be_board* b, const be_board_state* st, const uint8_t* mask, const double* reset_tape,
                   int32_t tape_len, const be_board_out* out, void* stream);
/* createBoard.step + featureExtractor for every env: actions (N) u8 indices into cfg.actions,
 * or deltas (N, 2) f64 (take_action_from_user's float moves). */
int be_board_step(be_board* b, const be_board_state* st, const uint8_t* actions, const double* deltas,
                  const be_board_out* out, void* stream);
/* featureExtractor of the current state (no state change). */
/* `steps` consecutive be_board_step calls in one launch, each env's state in registers:
 * actions (steps, N) u8 or deltas (steps, N, 2) f64; out->reward / done / truncated
 * (steps, N) and out->features (steps, N, 20) or NULL.  Philox resets only (no tape).
 * Bit-identical to `steps` be_board_step calls (the caller's per-step loop over
 * createBoard.step, ballenv_pygame.py:650-675, for every env).                      */
int be_board_rollout(be_board* b, const be_board_state* st, const uint8_t* actions, const double* deltas,
                     int32_t steps, const be_board_out* out, void* stream);
int be_board_observe(be_board* b, const be_board_state* st, const be_board_out* out, void* stream);
int be_board_status(be_board* b, int32_t* status_out, void* stream);
/* The board's autoreset pool (as be_pool_* above): with Philox autoreset and one lane
 * per env, be_board_reset queues a fill of every env's next two episodes' resets and be_board_step
 * one every 128 steps (BALLENV_POOL_PERIOD), and the steps of the state last reset copy a current
 * entry where they would draw the reset inline -- the same bits either way.  BALLENV_POOL=0 at
 * create disables it.  Bytes held (0: no pool). */
int64_t be_board_pool_bytes(const be_board* b);

#ifdef __cplusplus
}
#endif
#endif /* BALLENV_H */
