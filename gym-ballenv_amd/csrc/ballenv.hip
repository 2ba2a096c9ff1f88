// ballenv.hip -- MI355X (gfx950) batched BallEnv step engine + its C ABI.
//
// One thread per env; the env index is the unit-stride (coalesced) HBM axis of
// every state array (include/ballenv.h).  One launch of be_kernel<W, STEP>
// does, for every env, what the reference does per call of
//   BallEnv.step(action)              gym_ballenv/envs/ballenv_env.py:232-289
//     move_obstacles                  ballenv_env.py:323-353
//     calculate_reward/check_overlap  ballenv_env.py:200-229, 185-191
//   gym TimeLimit(1000)               gym_ballenv/__init__.py:4-11
//   prep_state4(state, W)             examples/ball_cnn_ac3.py:384-412 (+ prep_state2 :330-352)
// and, with autoreset, BallEnv.reset  ballenv_env.py:113-167 for the envs that finished.
//
// Latency structure (at 65536 envs there is one wave per SIMD, so every
// dependent round trip is exposed):
//  * the kernel argument block is small and hot-first (KParams, 4 cache
//    lines): scalar loads from the kernarg segment that miss are each a full
//    round trip, and a big by-value config struct spread them over the kernel;
//  * everything indexed per lane or used only on cold paths (goal/action
//    tables, obstacle speeds, spawn strips) lives in a device buffer staged
//    into LDS once per block;
//  * every per-env word the step needs is loaded up front (obstacles in
//    register chunks of 16 static / 8 dynamic), so all of a wave's loads are in
//    flight together and one barrier covers them and the table staging;
//  * no cross-block communication: randomness is Philox keyed by per-env state
//    (global env id, episode, ep_len), so there is no global counter or atomic.
//
// Window ("feature extraction") stage: an obstacle can only light cells of a
// W x W window if its radius-R disk meets the window's cell box.  Pass 1 tests
// every obstacle once against that box (it is already in registers for the
// collision test) and appends the few that qualify to a per-thread list in
// LDS (the obstacle-occupancy tile).  Pass 2 rasterises only those: for each
// distinct window row (Q1 makes rows 0 and 1 identical) the lit cells of one
// obstacle are a contiguous span [f-hw, f+hw], hw = isqrt(R^2 - dy^2), OR-ed
// into a per-row bitmask.  The bitmasks are expanded to 0/1 bytes four cells
// at a time (nibble * 0x00204081 & 0x01010101), staged per block in LDS and
// written out with 16-byte coalesced stores.
//
// Everything is integer except the reward path, which is f64 with the same
// operation order as the reference (correctly rounded sqrt/div, no FMA
// contraction: built with -ffp-contract=off), so results are bit-exact.
#include <type_traits>
#include <hip/hip_runtime.h>

#include <math.h>
#include <algorithm>
#include <mutex>
#include <new>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ballenv.h"
#include "internal.h"
#include "philox.h"
#include "policy_core.h"

namespace {

// Philox purposes (counter word 3, high byte); oracle/ballenv_oracle.c uses the same.
constexpr uint32_t PURPOSE_STEP_OBS = 1, PURPOSE_ACTION = 2, PURPOSE_RESET = 3, PURPOSE_SAMPLE = 4;
constexpr int REJECT_LIMIT = 4096;
constexpr int CS = 16;  // static obstacles per register chunk
constexpr int CD = 8;   // dynamic obstacles per register chunk
constexpr int HW_MAX = 63;   // largest collision radius R with a half-width table

enum Mode { MODE_STEP = 0, MODE_RESET = 1, MODE_OBSERVE = 2 };

// Per-context tables: a device buffer staged into LDS once per block.
struct Tables {
  int32_t goal[BE_MAX_GOALS];                 // packed goal xy
  int32_t action[BE_MAX_ACTIONS];             // packed (dx, dy)
  int32_t speed[BE_MAX_DYNAMIC];              // obstacle_speed
  int32_t strip_obs_x, strip_obs_y, strip_goal_x, strip_goal_y, strip_agent_x, strip_agent_y;
  int32_t radius_obstacle, radius_agent;
  uint8_t n_other[BE_MAX_GOALS];              // goals with a different value than goal g
  uint8_t other[BE_MAX_GOALS][BE_MAX_GOALS];  // pick -> goal index, per current goal g (newGoalList)
  uint8_t hw[HW_MAX + 1];                     // floor(sqrt(R^2 - d^2)), d = 0..R (only when R <= HW_MAX)
};

// The fixed-shape step kernels' 64-bit row-span table (span_fits: W-1+2R <= 63): span[j] holds the cells an obstacle
// at window column C = W-1+R lights in a row at distance |j - J0| (J0 = R+K-1): bits C-hw .. C+hw,
// 0 past R.  A near entry at window (f, e) lights row k with span[e - k + J0] >> (C - f), clipped to
// W bits -- one LDS read, one shift and one OR per row (raster_rows_span).  It follows Tables in the
// same device buffer; only the fixed-shape step kernels stage it.
constexpr int SPAN_N = 72;
struct TablesX {
  Tables t;
  uint64_t span[SPAN_N];
};
static_assert(sizeof(Tables) % 16 == 0 && sizeof(TablesX) % 16 == 0, "16-byte table staging");
__host__ __device__ constexpr bool span_fits(int W, int R) {   // W >= 2: K = W-1 rows, J0 = R+W-2
  return W >= 2 && R >= 0 && W - 1 + 2 * R <= 63 && 2 * R + 2 * (W - 1) - 1 <= SPAN_N;
}

// Kernel arguments: hot fields first, 64-byte lines (see the latency notes above).
struct KParams {
  // line 0
  int32_t* agent; int32_t* goal; double* prev_dist; double* total_dist;
  double* ep_return; int32_t* ep_len; uint32_t* episode; int32_t* static_obs;
  // line 1
  int32_t* dyn_obs; uint8_t* dyn_goal; uint8_t* obs; float* obs_f32;
  double* reward; uint8_t* done; const uint8_t* actions; const Tables* tables;
  // line 2
  int32_t n, window, ns, nd, R, speed_x, speed_y, screen_w;
  int32_t screen_h, goal_change, certainty, time_limit, num_actions, autoreset, gid0, dbg;
  // line 3
  double threshold_goal, time_penalty, static_penalty, dynamic_penalty, min_spawn_dist;
  double inv_g1;               // 1 / (goal_change + 1): counter = ep_len mod (G+1) without an integer divide
  unsigned long long seed;
  int* status;
  // line 4 (cold)
  const int16_t* deltas; const int16_t* tape; const uint8_t* mask; const int16_t* reset_tape;
  uint8_t* truncated; uint8_t* terminal_obs; double* final_return; int32_t* final_len;
  // line 5 (cold)
  double* stats;               // (slots, 8): one slot per wave / block of the step kernel (be_stats_slots)
  int32_t reset_tape_len;
  int32_t min_spawn_d2;        // integer d2: sqrt(d2) < min_spawn_dist  <=>  d2 < min_spawn_d2
  // fixed-shape kernels only (pick_kernel checks the preconditions):
  uint32_t amx, amy;           // action a's (dx+1, dy+1) at bits 2a..2a+1 (every move in {-1,0,1})
  int32_t num_goals;           // goals pairwise distinct: newGoalList(g)[pick] = pick + (pick >= g)
  int32_t prev_read;           // 1: read prev_dist; 0 (A/B only, when no reset can re-sample the agent,
                               // Q9): prev_dist == calc_dist(goal, agent), recomputed
  int32_t steps;               // rollout_kernel: steps per launch (actions / outputs are (steps, N, ...))
  // fused policy rollouts (rollout_kernel with HT > 0, be_policy_rollout)
  int32_t pol_bytes, pol_actions;
  const uint8_t* pol_img;      // packed Policy(W) image (policy_core.h PolLayout)
  const uint8_t* obs_in;       // (N, F) obs of the current state: step 0's policy input
  uint8_t* obs_last;           // (N, F) obs after the last step, or NULL
  uint8_t* act_out; float* logp_out; float* value_out;   // (steps, N)
  unsigned long long pol_seed;
  // the autoreset pool (layout below; nullptr: every reset is drawn inline)
  uint32_t* pool;
};

// ------------------------------------------------------------------ the autoreset pool
// A reset in Philox mode is a pure function of (seed, global env id, new episode) and the context's
// config (reset_env_philox's counter layout), so it can be drawn before the env finishes.
// pool_fill_kernel draws, for every env at episode e, the resets into episodes e+1 and e+2; the step
// kernels (step2_kernel, stepw_kernel) copy the entry of episode e+1 when the env finishes, instead
// of running the reset's Philox chains on the wave's critical path, and fall back to the inline
// wave_resets pass when the entry is stale (its tag is not e+1: the env reset twice since the last
// fill, or no fill ran).  Two entries per env, slot = episode & 1 (entry index x = slot * N + env),
// everything addressed from the one base p.pool (a uniform pointer + a 32-bit byte offset + an
// immediate: no per-array base pointers to keep in SGPRs):
//   tags    uint2 [2N] at byte 0:      (the episode the entry resets into, flags: POOL_VALID written,
//                                      POOL_REJ a rejection loop hit its bound) -- the fill's scan
//                                      reads these 8 bytes per entry, coalesced
//   bodies  112 B [2N] at byte 16 N:   the entry itself, contiguous (a consuming lane reads it with
//                                      seven 16-byte loads):
//     w0..2  ROWS: the reset obs's distinct window rows, packed as the consuming kernel ORs them
//            (W = 10: three rows per word at bits 10 r; W = 5: four rows at bits 5 r, in w0)
//     w3 AGENT, w4 GOAL (packed xy), w5 unused, w6..7 PREV f64 (state[2], the pre-resample distance,
//     Q9), w8..9 TOTAL f64, w10.. the NS statics' then the ND dynamics' packed xy (a reset's dyn_goal
//     is k)
constexpr uint32_t POOL_VALID = 1u, POOL_REJ = 2u;
constexpr int PB_ROWS = 0, PB_AGENT = 3, PB_GOAL = 4, PB_PREV = 6, PB_TOTAL = 8, PB_OBS = 10;
__host__ __device__ constexpr int pool_body_words(int ns, int nd) { return (PB_OBS + ns + nd + 3) & ~3; }
__host__ __device__ constexpr int64_t pool_bytes_per_env(int ns, int nd) { return 2 * (8 + 4ll * pool_body_words(ns, nd)); }
static_assert(pool_body_words(13, 5) == 28, "the fixed-shape kernels' 112-byte entry body");
// byte offset of word w of entry x's body (N <= 2^22 keeps every offset below 2^32: pool_max_envs)
__device__ __forceinline__ uint32_t pool_body(uint32_t n, uint32_t x, int nbw) { return 16u * n + x * (4u * (uint32_t)nbw); }
// T at byte off + imm of the pool: the uniform base + zext(32-bit offset) + an immediate, so the
// access is one global load / store with the immediate in its offset field
template <class T>
__device__ __forceinline__ T pool_ld(const uint32_t* pool, uint32_t off, uint32_t imm = 0) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(pool) + (size_t)off + imm);
}
template <class T>
__device__ __forceinline__ void pool_st(uint32_t* pool, uint32_t off, T v, uint32_t imm = 0) {
  *reinterpret_cast<T*>(reinterpret_cast<char*>(pool) + (size_t)off + imm) = v;
}
// BE_POOL_MODE (A/B): where a step kernel loads the pool entries of its finished envs.
//   1: right after done is known, before the physics stores, waited for inside that (divergent)
//      branch -- only the waves with a finished env wait;
//   5: inside the reset section (the uniform `if (m)` of the waves with a finished env), after the
//      stores: the rest of the kernel is the pre-pool code.
// (Measured and dropped: the loads unwaited in the branch -- the waitcnt pass then drains every
// outstanding store at the merge before the reset loop, in every wave; branch-free buffer loads with
// an out-of-range offset for the lanes without a finished env; the loads after the stores outside the
// reset section.  profiles/r06_pool_ab.txt)
#ifndef BE_POOL_MODE
#define BE_POOL_MODE 1
#endif
__device__ __forceinline__ uint32_t u4w(const uint4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }
__device__ __forceinline__ double u2d(uint32_t lo, uint32_t hi) {
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
constexpr int64_t POOL_MAX_ENVS = 1ll << 22;

// Diagnostics hooks (DBG skip bits, DIAG / PH phase stamps): no-ops in the release build; a
// -DBE_DIAG_STAMPS / -DBE_DIAG_SKIP build (tools/build_diag.sh, tools/build_ab_lib.sh) defines them.
#define BE_DIAG_UNIT_STEP 1
#include "diag.h"

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ int px(int32_t p) { return (int)(int16_t)(p & 0xFFFF); }
__device__ __forceinline__ int py(int32_t p) { return p >> 16; }
__device__ __forceinline__ int32_t pk(int x, int y) {
  return (int32_t)(((uint32_t)x & 0xFFFFu) | ((uint32_t)y << 16));
}
__device__ __forceinline__ uint32_t d2u(int dx, int dy) {
  uint32_t ax = (uint32_t)abs(dx), ay = (uint32_t)abs(dy);
  return ax * ax + ay * ay;  // < 2^32 for int16 coordinates
}
__device__ __forceinline__ int d2i(int dx, int dy) { return dx * dx + dy * dy; }
// element idx of a uniform base pointer, as base + zext(32-bit byte offset)
template <class T>
__device__ __forceinline__ T ld_s(const T* base, uint32_t idx) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + (size_t)(idx * (uint32_t)sizeof(T)));
}
// Output / state stores of the fixed-shape step kernels: write-through (sc1, a relaxed agent-scope
// atomic store), so the stores drain while the wave runs instead of in the kernel-end L2 write-back.
#ifndef BE_S2_CT
#define BE_S2_CT 256        // step2_kernel: threads per block (A/B)
#endif
constexpr int S2_CT = BE_S2_CT;
// copy-out store kinds: the step kernels write through (sc1); the fused rollouts' per-step obs rows
// are plain stores (sc1 there measured no faster)
constexpr int ST_PLAIN = 0, ST_WT = 1;
template <class T>
__device__ __forceinline__ void st_wt(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T& ld_s_ptr(T* base, uint32_t idx) {   // (stores: the same addressing)
  return *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + (size_t)(idx * (uint32_t)sizeof(T)));
}
// write-through store at element idx of a uniform base, as base + zext(32-bit byte offset): the
// SGPR-base store form, one 32-bit offset per element size instead of a 64-bit address per store
template <class T>
__device__ __forceinline__ void st_ws(T* base, uint32_t idx, T v) {
  st_wt(&ld_s_ptr(base, idx), v);
}
__device__ __forceinline__ int isqrt_small(int n) {  // floor(sqrt(n)), 0 <= n < 2^22
  int s = (int)__builtin_amdgcn_sqrtf((float)n);
  if (s * s > n) --s;
  if ((s + 1) * (s + 1) <= n) ++s;
  return s;
}
__device__ __forceinline__ int floordiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

typedef short v2s __attribute__((ext_vector_type(2)));   // a packed (x, y) int16 position

__device__ __forceinline__ uint32_t pick_word(const u4& b, int w) {
  return w == 0 ? b.x : (w == 1 ? b.y : (w == 2 ? b.z : b.w));
}
// 24-bit field j (0..4) of a Philox block read as x | y<<32 | z<<64 | w<<96
__device__ __forceinline__ uint32_t pick_field(const u4& b, int j) {
  constexpr uint32_t M = 0xFFFFFFu;
  return j == 0 ? (b.x & M)
       : j == 1 ? (__builtin_amdgcn_alignbit(b.y, b.x, 24) & M)
       : j == 2 ? (__builtin_amdgcn_alignbit(b.z, b.y, 16) & M)
       : j == 3 ? (b.z >> 8) : (b.w & M);
}
// uniform integer in [lo, hi) from one 32-bit word (multiply-shift)
__device__ __forceinline__ int map_range(uint32_t r, int lo, int hi) {
  return lo + (int)__umulhi(r, (uint32_t)(hi - lo));
}

// Sequential randint source for a reset: a tape column or Philox(gid, episode, 0, RESET|block).
struct ResetDraws {
  const int16_t* tape; int32_t len; int32_t n; int32_t env; int32_t cursor;
  uint32_t gid; uint32_t episode; unsigned long long seed;
  int* status;
  __device__ int draw(int lo, int hi) {
    int k = cursor++;
    if (tape) {
      if (k >= len) { atomicOr(status, BE_STATUS_RESET_TAPE_EXHAUSTED); return lo; }
      return tape[(int64_t)k * n + env];
    }
    u4 b = philox(gid, episode, 0u, tag(PURPOSE_RESET, (uint32_t)k >> 2), seed);
    return map_range(pick_word(b, k & 3), lo, hi);
  }
};

// sqrt(x) for x = 0 or an integer >= 1 (< 2^53), bit-identical to the correctly rounded f64 sqrt:
// the compiler's own gfx950 sequence (v_rsq_f64 + two Goldschmidt / Newton rounds) without its
// tiny-input rescaling (x < 2^-767: ldexp by 0 and back here) and with the +-0 / inf class select
// reduced to x == 0 -- five dependent instructions fewer on the reward / done path.
__device__ __forceinline__ double sqrt_int(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  return x == 0.0 ? x : g;
}

__device__ __forceinline__ double calc_dist(int x1, int y1, int x2, int y2) {
  // math.sqrt(math.pow(dx,2)+math.pow(dy,2)): the squares are exact integers in f64
  double dx = (double)(x1 - x2), dy = (double)(y1 - y2);
  return sqrt_int(dx * dx + dy * dy);
}
// The same with the library sqrt (the same bits): the fused rollouts keep it -- sqrt_int measured
// within noise to slightly slower there (profiles/r05_rollout_sqrt_ab.txt)
__device__ __forceinline__ double calc_dist_lib(int x1, int y1, int x2, int y2) {
  double dx = (double)(x1 - x2), dy = (double)(y1 - y2);
  return sqrt(dx * dx + dy * dy);
}

// Window geometry shared by the near test and the rasteriser.
struct Win {
  int x0, y0;     // cell (0,0) position: agent - speed*h
  int sx, sy;     // cell step = agent speed
  int w;          // W
  int kr;         // distinct rows K = max(W-1, 1)
  int R, R2;
  __device__ Win(const KParams& p, int ax, int ay) {
    w = p.window; const int h = w / 2;
    sx = p.speed_x; sy = p.speed_y;
    x0 = ax - sx * h; y0 = ay - sy * h;
    kr = w > 1 ? w - 1 : 1;
    R = p.R; R2 = R * R;
  }
  // Can obstacle (ox,oy) light any cell?  (f, e) = its window-relative position.
  __device__ __forceinline__ bool near(int ox, int oy, int& f, int& e) const {
    f = ox - x0; e = oy - y0;
    const int cx = min(max(f, 0), sx * (w - 1));
    const int cy = min(max(e, 0), sy * (kr - 1));
    return d2u(f - cx, e - cy) <= (uint32_t)R2;
  }
};

__device__ __forceinline__ int quadrant(int ax, int ay, int gx, int gy) {
  // prep_state2, examples/ball_cnn_ac3.py:343-351
  const int dx = gx - ax, dy = gy - ay;
  if (dx >= 0 && dy >= 0) return 1;
  if (dx < 0 && dy >= 0) return 0;
  if (dx < 0 && dy < 0) return 3;
  return 2;
}

// Byte distance between two pointers into LDS, in 32 bits (a pointer difference goes through the
// 64-bit flat aperture: ~15 instructions with the signed-division fixup).
__device__ __forceinline__ uint32_t lds_bytes(const void* lo, const void* hi) {
  return (uint32_t)(uintptr_t)hi - (uint32_t)(uintptr_t)lo;
}

// Per-thread list of window-relevant obstacles in LDS, laid out [slot][BLOCK].
template <int BLOCK>
struct NearList {
  uint32_t* base; int cnt;
  __device__ __forceinline__ void push(int f, int e) {
    base[cnt * BLOCK] = (uint32_t)(f & 0xFFFF) | ((uint32_t)e << 16);
    ++cnt;
  }
  __device__ __forceinline__ void push_if(bool c, int f, int e) {
    if (c) push(f, e);   // (an unconditional write + predicated count measured no faster)
  }
  __device__ __forceinline__ void get(int n, int& f, int& e) const {
    const uint32_t v = base[n * BLOCK];
    f = (int)(int16_t)(v & 0xFFFF); e = (int)v >> 16;
  }
};

template <int WT> struct Geo {
  static constexpr int K = WT > 1 ? WT - 1 : 1;       // distinct rows
  static constexpr int NW = (WT * WT + 31) / 32 + 1;  // flat cell words (+1 spill word)
  static constexpr int F = 4 + WT * WT;
};

// Rasterise the near list into K row bitmasks (compile-time W).  HWT (fixed-shape kernels):
// unit cell step, R <= HW_MAX and agent-relative list entries; a row's half-width comes from
// the LDS table instead of an isqrt.
template <int WT, int BLOCK, bool HWT = false>
__device__ __forceinline__ void raster_rows(const NearList<BLOCK>& nl, const Win& g, uint32_t (&rows)[Geo<WT>::K],
                                            const uint8_t* hwt = nullptr) {
  constexpr int K = Geo<WT>::K;
#pragma unroll
  for (int k = 0; k < K; ++k) rows[k] = 0u;
  if constexpr (HWT) {   // entries are agent-relative (dx, dy); unit cell step, so f = dx + W/2
    for (int n = 0; n < nl.cnt; ++n) {
      int f, e;
      nl.get(n, f, e);
      f += WT / 2; e += WT / 2;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int ady = abs(e - k);
        const int hw = hwt[min(ady, HW_MAX)];
        const int lo = max(f - hw, 0), hi = min(f + hw, WT - 1);
        rows[k] |= (ady <= g.R && lo <= hi) ? (2u << hi) - (1u << lo) : 0u;
      }
    }
    return;
  }
  for (int n = 0; n < nl.cnt; ++n) {
    int f, e;
    nl.get(n, f, e);
    if (g.sx == 1) {  // branch-free span per row
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int ady = abs(e - g.sy * k);
        const bool in = ady <= g.R;
        const int hw = isqrt_small(in ? g.R2 - ady * ady : 0);
        const int lo = max(f - hw, 0), hi = min(f + hw, WT - 1);
        rows[k] |= (in && lo <= hi) ? (2u << hi) - (1u << lo) : 0u;
      }
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int ady = abs(e - g.sy * k);
        if (ady <= g.R) {
          const int hw = isqrt_small(g.R2 - ady * ady);
          const int lo = max(-floordiv(hw - f, g.sx), 0), hi = min(floordiv(f + hw, g.sx), WT - 1);
          if (lo <= hi) rows[k] |= (2u << hi) - (1u << lo);
        }
      }
    }
  }
}

// Row-span table of the fixed-shape kernels (unit cell step, agent-relative near entries, R <=
// HW_MAX): mt[(f + R) * (R + 2) + min(ady, R + 1)] is raster_rows' row mask for an obstacle at
// window column f (-R .. W-1+R: the near box's range) and row distance ady (0 past R), so a near
// entry costs one LDS read per row instead of the span arithmetic.  Same masks, bit for bit.
template <int WT>
__device__ void build_span_table(uint16_t* mt, int R, int tid, int nthreads) {
  const int RA = R + 2, n = (WT + 2 * R) * RA;
  for (int x = tid; x < n; x += nthreads) {
    const int f = x / RA - R, ady = x - (x / RA) * RA;
    uint16_t m = 0;
    if (ady <= R) {
      const int hw = isqrt_small(R * R - ady * ady);   // == Tables::hw[ady] (exact floor sqrt)
      const int lo = max(f - hw, 0), hi = min(f + hw, WT - 1);
      m = lo <= hi ? (uint16_t)((2u << hi) - (1u << lo)) : (uint16_t)0;
    }
    mt[x] = m;
  }
}
template <int WT, int BLOCK>
__device__ __forceinline__ void raster_rows_mt(const NearList<BLOCK>& nl, int R, uint32_t (&rows)[Geo<WT>::K],
                                               const uint16_t* mt) {
  constexpr int K = Geo<WT>::K;
  static_assert(WT <= 16, "16-bit row masks");
#pragma unroll
  for (int k = 0; k < K; ++k) rows[k] = 0u;
  const int RA = R + 2;
  for (int n = 0; n < nl.cnt; ++n) {
    int f, e;
    nl.get(n, f, e);
    const uint16_t* col = mt + (f + WT / 2 + R) * RA;
    e += WT / 2;
#pragma unroll
    for (int k = 0; k < K; ++k) rows[k] |= col[min(abs(e - k), R + 1)];
  }
}

// raster_rows<WT, BLOCK, true> from the 64-bit span table (TablesX; span_fits(WT, R)), bit for bit:
// an entry's rows cost one LDS read, one 64-bit shift and one OR each instead of the span arithmetic.
template <int WT, int BLOCK>
__device__ __forceinline__ void raster_rows_span(const NearList<BLOCK>& nl, int R, uint32_t (&rows)[Geo<WT>::K],
                                                 const uint64_t* span, const uint32_t* init = nullptr) {
  constexpr int K = Geo<WT>::K;
#pragma unroll
  for (int k = 0; k < K; ++k) rows[k] = init ? init[k] : 0u;   // (init: masks already within W bits)
  for (int n = 0; n < nl.cnt; ++n) {
    int f, e;
    nl.get(n, f, e);                                   // agent-relative: window (f + W/2, e + W/2)
    const uint64_t* col = span + (e + WT / 2 + R);    // row k: span[e + W/2 - k + J0] = col[K-1-k]
    const uint32_t sh = (uint32_t)(WT - 1 + R - (f + WT / 2));   // C - f, in [0, W-1+2R] for a near entry
#pragma unroll
    for (int k = 0; k < K; ++k) rows[k] |= (uint32_t)(col[K - 1 - k] >> sh);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) rows[k] &= (1u << WT) - 1u;
}

// dx^2 + dy^2 of a packed int16 pair as the VOP3P dot with an inline-zero accumulator (the compiler
// picks the VOP2 accumulate form, which costs a zeroing move per call)
__device__ __forceinline__ int dot2_sq(v2s d) {
  int r;
  asm("v_dot2_i32_i16 %0, %1, %1, 0" : "=v"(r) : "v"(d));
  return r;
}
// Flatten rows into prep_state4's cell order (window row r uses distinct row max(r-1,0): quirk Q1).
template <int WT>
__device__ __forceinline__ void flatten(const uint32_t (&rows)[Geo<WT>::K], uint32_t (&flat)[Geo<WT>::NW]) {
#pragma unroll
  for (int q = 0; q < Geo<WT>::NW; ++q) flat[q] = 0u;
#pragma unroll
  for (int r = 0; r < WT; ++r) {
    const uint32_t row = rows[r > 0 ? r - 1 : 0];
    const int off = r * WT;
    flat[off >> 5] |= row << (off & 31);
    if ((off & 31) + WT > 32) flat[(off >> 5) + 1] |= row >> (32 - (off & 31));
  }
}

template <int WT>
__device__ __forceinline__ uint32_t obs_byte(const uint32_t (&flat)[Geo<WT>::NW], int quad, int b) {
  return b < 4 ? (uint32_t)(b == quad) : (flat[(b - 4) >> 5] >> ((b - 4) & 31)) & 1u;
}

template <int WT>
__device__ void write_row_global(uint8_t* row, const uint32_t (&flat)[Geo<WT>::NW], int quad) {
#pragma unroll 4
  for (int b = 0; b < Geo<WT>::F; ++b) row[b] = (uint8_t)obs_byte<WT>(flat, quad, b);
}

// Write one thread's obs row into the block's LDS stage.
template <int WT>
__device__ __forceinline__ void stage_row(uint8_t* stage, int tid, const uint32_t (&flat)[Geo<WT>::NW], int quad) {
  constexpr int F = Geo<WT>::F;
  if constexpr ((F & 3) == 0) {
    uint32_t* dst = reinterpret_cast<uint32_t*>(stage + tid * F);
    dst[0] = 1u << (8 * quad);
#pragma unroll
    for (int w = 1; w < F / 4; ++w) {
      const int j = 4 * (w - 1);  // first cell of this word (nibble aligned)
      const uint32_t nib = (flat[j >> 5] >> (j & 31)) & 0xFu;
      dst[w] = (nib * 0x00204081u) & 0x01010101u;
    }
  } else {
    uint8_t* dst = stage + tid * F;
#pragma unroll
    for (int b = 0; b < F; ++b) dst[b] = (uint8_t)obs_byte<WT>(flat, quad, b);
  }
}

// Copy the block's staged rows to obs (u8) and/or obs_f32 with 16-byte stores.
// SF = ST_WT (default): sc1 write-through buffer stores -- the kernel-end L2 write-back then has
// little left to do (measured 7.8 -> 7.3 us per step at 65 536 envs; plain and nt stores slower);
// ST_PLAIN: plain stores (the fused rollouts).
constexpr int AUX_SC1 = 16;   // buffer-store cache-policy bits (gfx950: sc0 1, nt 2, sc1 16)
template <int BLOCK, int SF = ST_WT>
__device__ __forceinline__ void copy_out(const uint8_t* stage, int F, int nvalid, int64_t row0,
                                         uint8_t* obs, float* obs_f32, int tid = (int)threadIdx.x) {
  if constexpr (BLOCK == 64) {   // a wave's own rows: row0 / nvalid are wave-uniform -- say so, or the
    nvalid = __builtin_amdgcn_readfirstlane(nvalid);   // buffer descriptor lands in VGPRs and every
    row0 = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)row0 >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)row0));   // store runs a waterfall loop
  }
  const int bytes = nvalid * F;
  if (obs) {
    uint8_t* dst = obs + row0 * F;
    const int nv = bytes >> 4;
    if constexpr (SF == ST_WT) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, bytes, 0x00020000);
    for (int v = tid; v < nv; v += BLOCK) {
      const uint4 x = reinterpret_cast<const uint4*>(stage)[v];
      typedef int v4i_ __attribute__((ext_vector_type(4)));
      const v4i_ y = {(int)x.x, (int)x.y, (int)x.z, (int)x.w};
      __builtin_amdgcn_raw_buffer_store_b128(y, rsrc, v * 16, 0, AUX_SC1);
    }
    } else {
    for (int v = tid; v < nv; v += BLOCK)
      reinterpret_cast<uint4*>(dst)[v] = reinterpret_cast<const uint4*>(stage)[v];
    }
    for (int b = (nv << 4) + tid; b < bytes; b += BLOCK) dst[b] = stage[b];
  }
  if (obs_f32) {
    float* dst = obs_f32 + row0 * F;
    const int nv = bytes >> 2;
    for (int v = tid; v < nv; v += BLOCK) {
      const uint32_t q = reinterpret_cast<const uint32_t*>(stage)[v];
      reinterpret_cast<float4*>(dst)[v] =
          make_float4((float)(q & 0xFF), (float)((q >> 8) & 0xFF), (float)((q >> 16) & 0xFF), (float)(q >> 24));
    }
    for (int b = (nv << 2) + tid; b < bytes; b += BLOCK) dst[b] = (float)stage[b];
  }
}

// A wave's NV16 staged 16-byte words to dst (wave-uniform) in one unrolled pass: every LDS read
// is issued before the first store, so the copy pays one LDS latency instead of one per word.
template <int NV16, int SF = ST_WT>
__device__ __forceinline__ void copy_wave_full(const uint8_t* stage, uint8_t* dst, int lane) {
  constexpr int IT = (NV16 + 63) / 64;
  typedef int v4i_ __attribute__((ext_vector_type(4)));
  v4i_ x[IT];
#pragma unroll
  for (int j = 0; j < IT; ++j) x[j] = reinterpret_cast<const v4i_*>(stage)[min(lane + 64 * j, NV16 - 1)];
  // branch-free tail: the descriptor's size is NV16 * 16 bytes, so the buffer unit drops the
  // stores of lanes past the end (no divergent second copy of the store sequence)
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, NV16 * 16, 0x00020000);
#pragma unroll
  for (int j = 0; j < IT; ++j) __builtin_amdgcn_raw_buffer_store_b128(x[j], rsrc, (lane + 64 * j) * 16, 0, SF == ST_WT ? AUX_SC1 : 0);
}

// Generic-W (runtime W, no staging) obs writer: per cell over the near list.
template <int BLOCK>
__device__ void write_row_generic(const NearList<BLOCK>& nl, const Win& g, int quad, uint8_t* row, float* rowf) {
  for (int b = 0; b < 4; ++b) {
    if (row) row[b] = (uint8_t)(b == quad);
    if (rowf) rowf[b] = (float)(b == quad);
  }
  for (int r = 0; r < g.w; ++r) {
    const int k = r > 0 ? r - 1 : 0;
    for (int cc = 0; cc < g.w; ++cc) {
      int hit = 0;
      for (int n = 0; n < nl.cnt && !hit; ++n) {
        int f, e;
        nl.get(n, f, e);
        hit = d2u(f - g.sx * cc, e - g.sy * k) <= (uint32_t)g.R2;
      }
      const int b = 4 + r * g.w + cc;
      if (row) row[b] = (uint8_t)hit;
      if (rowf) rowf[b] = (float)hit;
    }
  }
}

// ------------------------------------------------------------------ reset
// BallEnv.reset for one env (ballenv_env.py:113-167); also rebuilds the near list.
template <int BLOCK>
__device__ void reset_env(const KParams& p, const Tables& t, int i, ResetDraws& ds, int& ax, int& ay, int& gx,
                          int& gy, NearList<BLOCK>& nl) {
  const int N = p.n, W = p.screen_w, H = p.screen_h;
  gx = ds.draw(W - t.strip_goal_x, W);                                  // :115
  gy = ds.draw(H - t.strip_goal_y, H);                                  // :116
  ax = ds.draw(0, t.strip_agent_x);                                     // :117
  ay = ds.draw(0, t.strip_agent_y);                                     // :118
  const double dist = calc_dist(gx, gy, ax, ay);                        // :119
  for (int guard = 0; calc_dist(gx, gy, ax, ay) < p.min_spawn_dist;) {  // :121-126
    if (++guard > REJECT_LIMIT) { atomicOr(p.status, BE_STATUS_REJECTION_LIMIT); break; }
    ax = ds.draw(0, t.strip_agent_x);
    ay = ds.draw(0, t.strip_agent_y);
  }
  p.agent[i] = pk(ax, ay);
  p.goal[i] = pk(gx, gy);
  p.prev_dist[i] = dist;  // state[2] keeps the pre-resample distance (Q9)
  p.total_dist[i] = calc_dist(ax, ay, gx, gy);                          // :166
  p.ep_return[i] = 0.0;
  p.ep_len[i] = 0;
  p.episode[i] = ds.episode;
  const Win g(p, ax, ay);
  nl.cnt = 0;
  // check_overlap_rect (:193-197): |dx| < rad + r_a and |dy| < rad/2 + r_a  <=>  2|dy| < rad + 2 r_a
  const int rx = t.radius_obstacle + t.radius_agent, ry2 = t.radius_obstacle + 2 * t.radius_agent;
  for (int k = 0; k < p.ns; ++k) {                                      // :131-149
    int ox = 0, oy = 0;
    for (int guard = 0;;) {
      ox = ds.draw(t.strip_obs_x, W - t.strip_obs_x);                   // obstacles.__init__ :24-25
      oy = ds.draw(t.strip_obs_y, H - t.strip_obs_y);
      const bool ra = abs(ox - ax) < rx && 2 * abs(oy - ay) < ry2;
      const bool rg = abs(ox - gx) < rx && 2 * abs(oy - gy) < ry2;
      if (!ra && !rg) break;
      if (++guard > REJECT_LIMIT) { atomicOr(p.status, BE_STATUS_REJECTION_LIMIT); break; }
    }
    p.static_obs[(int64_t)k * N + i] = pk(ox, oy);
    int f, e;
    if (g.near(ox, oy, f, e)) nl.push(f, e);
  }
  for (int k = 0; k < p.nd; ++k) {                                      // :153-164
    const int ox = ds.draw(t.strip_obs_x, W - t.strip_obs_x);
    const int oy = ds.draw(t.strip_obs_y, H - t.strip_obs_y);
    p.dyn_obs[(int64_t)k * N + i] = pk(ox, oy);
    p.dyn_goal[(int64_t)k * N + i] = (uint8_t)k;                       // curr_goal = goal list[k]
    int f, e;
    if (g.near(ox, oy, f, e)) nl.push(f, e);
  }
}

// Perf-mode (Philox) reset, split over the env's LPE lanes.  Each quantity has its
// own counter, so the lanes draw in parallel and nothing is serial but the
// (rare) agent re-sample loop:
//   sub = 0                         words gx, gy, ax, ay
//   sub = 1 + r                     agent re-sample r: words ax, ay
//   sub = 1<<22 | k<<12 | a         static obstacle k, attempt a: words x, y
//   sub = 2<<22 | k<<12             dynamic obstacle k: words x, y
// Distributions and rejection rules are the reference's (ballenv_env.py:113-167);
// only the order in which the random words are consumed differs from numpy's
// single stream, which the tape mode (reset_env) reproduces exactly.
template <int BLOCK, int LPE>
__device__ void reset_env_philox(const KParams& p, const Tables& t, int i, int q, uint32_t gid, uint32_t episode,
                                 int& ax, int& ay, int& gx, int& gy, NearList<BLOCK>& nl) {
  const int N = p.n, W = p.screen_w, H = p.screen_h;
  const u4 b0 = philox(gid, episode, 0u, tag(PURPOSE_RESET, 0), p.seed);
  gx = map_range(b0.x, W - t.strip_goal_x, W);
  gy = map_range(b0.y, H - t.strip_goal_y, H);
  ax = map_range(b0.z, 0, t.strip_agent_x);
  ay = map_range(b0.w, 0, t.strip_agent_y);
  const double dist = calc_dist(gx, gy, ax, ay);
  for (int r = 0; calc_dist(gx, gy, ax, ay) < p.min_spawn_dist; ++r) {
    if (r >= REJECT_LIMIT - 1) { if (q == 0) atomicOr(p.status, BE_STATUS_REJECTION_LIMIT); break; }
    const u4 b = philox(gid, episode, 0u, tag(PURPOSE_RESET, 1 + r), p.seed);
    ax = map_range(b.x, 0, t.strip_agent_x);
    ay = map_range(b.y, 0, t.strip_agent_y);
  }
  if (q == 0) {
    p.agent[i] = pk(ax, ay);
    p.goal[i] = pk(gx, gy);
    p.prev_dist[i] = dist;  // pre-resample distance (Q9)
    p.total_dist[i] = calc_dist(ax, ay, gx, gy);
    p.ep_return[i] = 0.0;
    p.ep_len[i] = 0;
    p.episode[i] = episode;
  }
  const Win g(p, ax, ay);
  nl.cnt = 0;
  const int rx = t.radius_obstacle + t.radius_agent, ry2 = t.radius_obstacle + 2 * t.radius_agent;
  for (int k = q; k < p.ns; k += LPE) {
    int ox = 0, oy = 0;
    for (int a = 0;; ++a) {
      const u4 b = philox(gid, episode, 0u, tag(PURPOSE_RESET, (1u << 22) | ((uint32_t)k << 12) | (uint32_t)a), p.seed);
      ox = map_range(b.x, t.strip_obs_x, W - t.strip_obs_x);
      oy = map_range(b.y, t.strip_obs_y, H - t.strip_obs_y);
      const bool ra = abs(ox - ax) < rx && 2 * abs(oy - ay) < ry2;
      const bool rg = abs(ox - gx) < rx && 2 * abs(oy - gy) < ry2;
      if (!ra && !rg) break;
      if (a >= REJECT_LIMIT - 1) { atomicOr(p.status, BE_STATUS_REJECTION_LIMIT); break; }
    }
    p.static_obs[(int64_t)k * N + i] = pk(ox, oy);
    int f, e;
    if (g.near(ox, oy, f, e)) nl.push(f, e);
  }
  for (int k = q; k < p.nd; k += LPE) {
    const u4 b = philox(gid, episode, 0u, tag(PURPOSE_RESET, (2u << 22) | ((uint32_t)k << 12)), p.seed);
    const int ox = map_range(b.x, t.strip_obs_x, W - t.strip_obs_x);
    const int oy = map_range(b.y, t.strip_obs_y, H - t.strip_obs_y);
    p.dyn_obs[(int64_t)k * N + i] = pk(ox, oy);
    p.dyn_goal[(int64_t)k * N + i] = (uint8_t)k;
    int f, e;
    if (g.near(ox, oy, f, e)) nl.push(f, e);
  }
}

// ------------------------------------------------------------------ statistics
// Finished-episode statistics go to per-block slots (slots, 8) f64:
// [count, sum return, sum return^2, sum length, min return, max return, 0, 0].
// A block's thread 0 read-modify-writes only its own slot, so there are no
// atomics and no contention; be_stats_slots() tells the caller how many slots.
struct WaveStats { double n, s1, s2, sl, mn, mx; };

__device__ __forceinline__ WaveStats wave_stats(bool done, double ret, int len,
                                                unsigned long long lanes = ~0ull) {
  WaveStats w{0.0, 0.0, 0.0, 0.0, INFINITY, -INFINITY};
  // wave-uniform loop over the finished lanes in lane order (deterministic; ~1 per wave per
  // step at the reference's episode lengths, so a few readlanes beat a 6-level shuffle tree)
  for (unsigned long long m = __ballot(done) & lanes; m; m &= m - 1) {
    const int l = __ffsll((long long)m) - 1;
    const unsigned long long bits = __double_as_longlong(ret);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bits, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bits >> 32), l);
    const double r = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
    const int n = __builtin_amdgcn_readlane(len, l);
    w.n += 1.0; w.s1 += r; w.s2 += r * r; w.sl += (double)n;
    w.mn = fmin(w.mn, r); w.mx = fmax(w.mx, r);
  }
  return w;
}

// Both half-waves' folds (slots of 32 envs) from ONE ballot loop: lanes 0..31 into lo, 32..63
// into hi, each in lane order from zero -- the same sums as two masked wave_stats calls.
__device__ __forceinline__ void wave_stats2(bool done, double ret, int len, WaveStats& lo, WaveStats& hi) {
  lo = WaveStats{0.0, 0.0, 0.0, 0.0, INFINITY, -INFINITY};
  hi = lo;
  for (unsigned long long m = __ballot(done); m; m &= m - 1) {
    const int l = __ffsll((long long)m) - 1;
    const unsigned long long bits = __double_as_longlong(ret);
    const uint32_t rl = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bits, l);
    const uint32_t rh = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bits >> 32), l);
    const double r = __longlong_as_double((long long)(((unsigned long long)rh << 32) | rl));
    const double dn = (double)__builtin_amdgcn_readlane(len, l);
    if (l < 32) {   // (uniform branch; no runtime-selected reference, which would go to scratch)
      lo.n += 1.0; lo.s1 += r; lo.s2 += r * r; lo.sl += dn; lo.mn = fmin(lo.mn, r); lo.mx = fmax(lo.mx, r);
    } else {
      hi.n += 1.0; hi.s1 += r; hi.s2 += r * r; hi.sl += dn; hi.mn = fmin(hi.mn, r); hi.mx = fmax(hi.mx, r);
    }
  }
}

// ------------------------------------------------------------------ lane groups
// LPE lanes cooperate on one env: obstacle k belongs to lane k % LPE, obs word w to lane w % LPE.
constexpr int BLOCK_THREADS = 256;
template <int LPE>
__device__ __forceinline__ uint32_t group_or(uint32_t x) {
  static_assert(LPE == 1 || LPE == 2 || LPE == 4, "LPE must be 1, 2 or 4");
  if constexpr (LPE >= 2) x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
  if constexpr (LPE >= 4) x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
  return x;
}
template <int LPE>
__device__ __forceinline__ int group_bcast(int x) {  // value of the group's lane 0
  if constexpr (LPE == 1) return x;
  else if constexpr (LPE == 2) return __builtin_amdgcn_update_dpp(0, x, 0xA0, 0xF, 0xF, false);  // quad_perm 0,0,2,2
  else return __builtin_amdgcn_update_dpp(0, x, 0x00, 0xF, 0xF, false);                          // quad_perm 0,0,0,0
}

constexpr int lanes_for(int) { return 1; }   // the generic kernel: one lane per env
constexpr int envs_per_block(int WT) { return BLOCK_THREADS / lanes_for(WT); }
constexpr int RCAP = 64;  // resets handled per cooperative pass (more loop)

// One dynamic obstacle's move_obstacles (ballenv_env.py:323-353), branch-free.
// Tape mode: t0/t1 are the values of its first/second randint call.  Philox mode:
// both draws come from one 24-bit field f -- randint(n0) = (f*n0) >> 24, then
// randint(n1) = (((f*n0) mod 2^24) * n1) >> 24 (the multiply-shift's fractional part;
// n0, n1 <= 128, so every product fits 32 bits and runs on the full-rate 24-bit multiplier).
// Returns the new goal index (== gi unless a goal change picked another one).
// move_list of ballenv_env.py:324, (dx+1, dy+1) packed 2 bits per entry:
// (1,1) (1,-1) (1,0) (0,1) (0,-1) (0,0) (-1,1) (-1,-1) (-1,-1) -- (-1,-1) twice, no (-1,0) (Q4)
constexpr uint32_t OBS_MX = (2u << 0) | (2u << 2) | (2u << 4) | (1u << 6) | (1u << 8) | (1u << 10) | (0u << 12) | (0u << 14) | (0u << 16);
constexpr uint32_t OBS_MY = (2u << 0) | (0u << 2) | (1u << 4) | (2u << 6) | (0u << 8) | (1u << 10) | (2u << 12) | (0u << 14) | (0u << 16);
__device__ __forceinline__ int dyn_move(const KParams& p, const Tables& t, int& ox, int& oy, int gi, int speed,
                                        bool change, bool tape, int t0, int t1, uint32_t w, uint32_t& flags) {
  const int32_t gp = t.goal[gi];
  const int tx = px(gp) - ox, ty = py(gp) - oy;
  const bool both = (tx != 0) & (ty != 0);
  const uint32_t p1 = __umul24(w, 100u);
  const int u = tape ? t0 : (int)(p1 >> 24);
  const int m = tape ? (both ? t1 : t0) : (int)(__umul24(both ? (p1 & 0xFFFFFFu) : w, 9u) >> 24);
  const bool directed = both & (u < p.certainty);
  const int mx = directed ? (tx > 0 ? 1 : -1) : (int)((OBS_MX >> (2 * m)) & 3u) - 1;
  const int my = directed ? (ty > 0 ? 1 : -1) : (int)((OBS_MY >> (2 * m)) & 3u) - 1;
  const int nx = ox + mx * speed, ny = oy + my * speed;
  // goal change (no move this step, Q5): newGoalList pick
  const int n_other = t.n_other[gi];
  const int pick = tape ? t0 : (int)(__umul24(w, (uint32_t)n_other) >> 24);
  const int ng = t.other[gi][min(pick, BE_MAX_GOALS - 1)];
  flags |= (change && n_other == 0) ? (uint32_t)BE_STATUS_NO_GOAL : 0u;
  flags |= (!change && (nx < -32768 || nx > 32767 || ny < -32768 || ny > 32767)) ? (uint32_t)BE_STATUS_COORD_RANGE : 0u;
  ox = change ? ox : nx;
  oy = change ? oy : ny;
  return (change && n_other > 0) ? ng : gi;
}

// Philox-mode dyn_move for the fixed-shape kernels, written as straight-line integer code so
// the scheduler can interleave the obstacles (select by mask, no divergent regions).
// Returns the goal index after the step; (ox, oy) is moved unless change.
__device__ __forceinline__ int dyn_move_philox(const KParams& p, const Tables& t, int& ox, int& oy, int gi, int speed,
                                               bool change, uint32_t f, uint32_t& flags) {
  const int32_t gp = t.goal[gi];
  const int n_other = t.n_other[gi];
  const int tx = px(gp) - ox, ty = py(gp) - oy;
  const bool both = (tx != 0) & (ty != 0);
  const uint32_t p1 = __umul24(f, 100u);
  const uint32_t src = both ? (p1 & 0xFFFFFFu) : f;
  const uint32_t m2 = 2u * (__umul24(src, 9u) >> 24);            // 2 * OBS_MOVES index
  const bool directed = both & ((int)(p1 >> 24) < p.certainty);
  const int sx = (tx > 0) - (tx < 0), sy = (ty > 0) - (ty < 0);
  const int rx = (int)((OBS_MX >> m2) & 3u) - 1, ry = (int)((OBS_MY >> m2) & 3u) - 1;
  const int mx = directed ? sx : rx, my = directed ? sy : ry;
  const int step = change ? 0 : speed;                             // goal change: no move (Q5)
  const int nx = ox + mx * step, ny = oy + my * step;
  const int pick = (int)(__umul24(f, (uint32_t)n_other) >> 24);
  const int ng = t.other[gi][min(pick, BE_MAX_GOALS - 1)];
  flags |= (change && n_other == 0) ? (uint32_t)BE_STATUS_NO_GOAL : 0u;
  flags |= ((uint32_t)(nx + 32768) > 65535u || (uint32_t)(ny + 32768) > 65535u) ? (uint32_t)BE_STATUS_COORD_RANGE : 0u;
  ox = nx; oy = ny;
  return (change && n_other > 0) ? ng : gi;
}

// dyn_move_philox for pairwise-distinct goals (the fixed-shape kernels): newGoalList(g) is
// every other goal in order, so the pick needs no table; n_other = num_goals - 1 >= 1.
__device__ __forceinline__ int dyn_move_fixed(const KParams& p, const Tables& t, int& ox, int& oy, int gi, int speed,
                                              bool change, uint32_t f, uint32_t& flags) {
  const int32_t gp = t.goal[gi];
  const int tx = px(gp) - ox, ty = py(gp) - oy;
  const bool both = (tx != 0) & (ty != 0);
  const uint32_t p1 = __umul24(f, 100u);
  const uint32_t src = both ? (p1 & 0xFFFFFFu) : f;
  const uint32_t m2 = 2u * (__umul24(src, 9u) >> 24);            // 2 * OBS_MOVES index
  const bool directed = both & ((int)(p1 >> 24) < p.certainty);
  const int sx = (tx > 0) - (tx < 0), sy = (ty > 0) - (ty < 0);
  const int rx = (int)((OBS_MX >> m2) & 3u) - 1, ry = (int)((OBS_MY >> m2) & 3u) - 1;
  const int mx = directed ? sx : rx, my = directed ? sy : ry;
  const int step = change ? 0 : speed;                             // goal change: no move (Q5)
  const int nx = ox + mx * step, ny = oy + my * step;
  const int pick = (int)(__umul24(f, (uint32_t)(p.num_goals - 1)) >> 24);
  flags |= ((uint32_t)(nx + 32768) > 65535u || (uint32_t)(ny + 32768) > 65535u) ? (uint32_t)BE_STATUS_COORD_RANGE : 0u;
  ox = nx; oy = ny;
  return change ? pick + (pick >= gi ? 1 : 0) : gi;
}

// Window-box pre-filter: an obstacle can light a cell only if it lies in the cell box grown by R.
struct NearBox {
  int bx0, by0; uint32_t bw, bh;
  __device__ explicit NearBox(const Win& g)
      : bx0(g.x0 - g.R), by0(g.y0 - g.R), bw((uint32_t)(g.sx * (g.w - 1) + 2 * g.R)),
        bh((uint32_t)(g.sy * (g.kr - 1) + 2 * g.R)) {}
  __device__ __forceinline__ bool maybe(int ox, int oy) const {
    return (uint32_t)(ox - bx0) <= bw && (uint32_t)(oy - by0) <= bh;
  }
};

__device__ __forceinline__ bool collides(int ox, int oy, int ax, int ay, uint32_t R2) {
  const int dx = ox - ax, dy = oy - ay;  // |d| < 2^17: 24-bit multiplies are exact
  return (uint32_t)__mul24(dx, dx) + (uint32_t)__mul24(dy, dy) <= R2;
}

// Rasterise ONE obstacle into row masks with LDS atomic OR (cooperative reset path).
template <int WT>
__device__ void raster_one_lds(uint32_t* rows, const Win& g, int f, int e) {
  constexpr int K = Geo<WT>::K;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int ady = abs(e - g.sy * k);
    if (ady <= g.R) {
      const int hw = isqrt_small(g.R2 - ady * ady);
      int lo, hi;
      if (g.sx == 1) { lo = f - hw; hi = f + hw; }
      else { lo = -floordiv(hw - f, g.sx); hi = floordiv(f + hw, g.sx); }
      lo = max(lo, 0); hi = min(hi, WT - 1);
      if (lo <= hi) atomicOr(&rows[k], (2u << hi) - (1u << lo));
    }
  }
}

// Write one env's obs row (all F bytes) into the LDS stage from row masks (one thread).
template <int WT>
__device__ void stage_full_row(uint8_t* dst, const uint32_t (&flat)[Geo<WT>::NW], int quad) {
  constexpr int F = Geo<WT>::F;
  if constexpr ((F & 3) == 0) {
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    d[0] = 1u << (8 * quad);
#pragma unroll
    for (int w = 1; w < F / 4; ++w) {
      const int jc = 4 * (w - 1);
      d[w] = (((flat[jc >> 5] >> (jc & 31)) & 0xFu) * 0x00204081u) & 0x01010101u;
    }
  } else {
#pragma unroll
    for (int b = 0; b < F; ++b) dst[b] = (uint8_t)obs_byte<WT>(flat, quad, b);
  }
}

// A reset env's distances: returns total_distance = |agent - goal| and sets prev to the
// pre-resample distance (Q9; equal to total unless the agent was re-drawn).
template <bool LIB = false>
__device__ __forceinline__ double reset_dists(int32_t ag, int32_t go, int32_t a0, double& prev) {
  const double td = LIB ? calc_dist_lib(px(ag), py(ag), px(go), py(go)) : calc_dist(px(ag), py(ag), px(go), py(go));
  prev = a0 == ag ? td : (LIB ? calc_dist_lib(px(go), py(go), px(a0), py(a0)) : calc_dist(px(go), py(go), px(a0), py(a0)));
  return td;
}

// Wave-cooperative autoreset (fixed-shape step kernels).  The finished envs of one wave are
// reset by the whole wave, P = 64 / (NS+ND) envs per pass: lane s*(NS+ND) + k draws obstacle k
// of the pass's env s (and, redundantly, that env's goal/agent) and ORs its window rows into a
// per-wave LDS buffer, so no other wave of the block waits on them (no block barrier).  Draws
// use reset_env_philox's counter layout, so results equal the block-cooperative path's.
// wl: per-wave LDS scratch, >= P*(K+8) words.  Where the new state goes is the caller's:
// osink(slot, k, il, packed xy) for obstacle k of env il (drawn by lane slot*G + k), then
// esink(own, agent, goal, pre-resample agent) on the env's own lane, after a wave barrier.
// LPE = 2 (step2_kernel): lanes 2e and 2e+1 share env e; m holds the even (owner) lanes, and
// both lanes of a reset env take the new agent / goal / window rows (esink runs on both).
// Ordering of a reset env's stores.  The physics stored the env's obstacles and scalars earlier
// in the same launch, from the env's own lane(s); the sinks store the new values again, from
// whichever lane drew them (osink: lane slot*G + k).  Both are vector stores of ONE wave, issued
// in program order (the sinks after a wave barrier, the physics before it).  A wave's vector
// memory instructions go through the CU's address / data path and the write-through L1 to the L2
// channel of the address in issue order, so the later instruction's bytes win whichever lanes
// issued the two: the same guarantee a lane relies on for its own two stores to one address
// (the stores are sc1, none is an atomic).  The rule is per-wave program order, not per lane.
// Rejection limits (ballenv_env.py:121-126, :145): with rej_own == nullptr the lane that hits the
// bound ORs BE_STATUS_REJECTION_LIMIT into the status word; otherwise each owner lane gets its env's
// flag in *rej_own and the status word is left alone (pool_fill_kernel stores it with the entry, and
// the step kernel that consumes the entry raises the status bit then).
template <int WT, int NSC, int NDC, int PMAX, class OSink, class ESink, int LPE = 1>
__device__ void wave_resets(const KParams& p, const Tables& t, unsigned long long m, int i, uint32_t gid,
                            uint32_t episode, int& ax, int& ay, int& gx, int& gy, int& ncnt,
                            uint32_t (&xrows)[Geo<WT>::K], uint32_t* wl, OSink&& osink, ESink&& esink,
                            const uint64_t* span = nullptr,   // span: the wave's row-span table (step2_kernel)
                            uint32_t* rej_own = nullptr) {
  // G + 1 lanes per env: lane k < G draws obstacle k, lane G the goal / agent block; every lane
  // runs ONE Philox chain, and the goal lane's four values reach the slot's lanes by readlane
  constexpr int K = Geo<WT>::K, G = NSC + NDC, GL = G + 1, P = (64 / GL < PMAX) ? 64 / GL : PMAX;
  static_assert(P >= 1, "one env's obstacles must fit a wave");
  const int lane = (int)(threadIdx.x & 63);
  const int W = p.screen_w, H = p.screen_h;
  const int rx = t.radius_obstacle + t.radius_agent, ry2 = t.radius_obstacle + 2 * t.radius_agent;
  const int slot = lane / GL, k = lane - slot * GL;
  uint32_t* wrows = wl;            // [P][K] row masks
  int* stash = reinterpret_cast<int*>(wl + P * K);   // [P][4]: agent xy, goal xy, pre-resample agent xy packed
  while (m) {
    int ls[P], n = 0;
#pragma unroll
    for (int s2 = 0; s2 < P; ++s2) {   // the next (up to) P finished lanes, uniform
      ls[s2] = m ? __ffsll((long long)m) - 1 : 0;
      n += m ? 1 : 0;
      m &= m - 1;
    }
    // this lane's env (slot), selected from uniform per-slot readlanes
    int il = 0; uint32_t u = 0, ep = 0;
#pragma unroll
    for (int s2 = 0; s2 < P; ++s2) {
      const int il2 = __builtin_amdgcn_readlane(i, ls[s2]);
      const uint32_t u2 = (uint32_t)__builtin_amdgcn_readlane((int)gid, ls[s2]);
      const uint32_t e2 = (uint32_t)__builtin_amdgcn_readlane((int)episode, ls[s2]) + 1u;
      il = slot == s2 ? il2 : il; u = slot == s2 ? u2 : u; ep = slot == s2 ? e2 : ep;
    }
    asm volatile("" : "+v"(il), "+v"(u), "+v"(ep));   // keep the Philox inputs in VGPRs
    const bool act = slot < n;
    bool rej = false;   // this lane's rejection loop hit its bound
    if (lane < P * K) wrows[lane] = 0u;
    // intra-wave LDS hand-offs: a wave's LDS operations execute in issue order, so only the
    // compiler must keep them in program order (a memory fence would also drain the stores)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // one Philox block per lane: obstacle k's first attempt (ballenv_env.py:131-164), or the
    // goal / agent block (:115-126) on the slot's lane G
    const bool is_goal = k == G, is_static = k < NSC;
    const uint32_t sub0 = is_goal ? 0u
                        : is_static ? ((1u << 22) | ((uint32_t)k << 12)) : ((2u << 22) | ((uint32_t)(k - NSC) << 12));
    u4 bo = philox(u, ep, 0u, tag(PURPOSE_RESET, sub0), p.seed);
    int rgx = 0, rgy = 0, rax = 0, ray = 0, ax0 = 0, ay0 = 0;
    if (act && is_goal) {
      rgx = map_range(bo.x, W - t.strip_goal_x, W); rgy = map_range(bo.y, H - t.strip_goal_y, H);
      rax = map_range(bo.z, 0, t.strip_agent_x); ray = map_range(bo.w, 0, t.strip_agent_y);
      ax0 = rax; ay0 = ray;
      for (int r = 0; d2i(rgx - rax, rgy - ray) < p.min_spawn_d2; ++r) {   // dist < 50 <=> d2 < 2500 (integers)
        if (r >= REJECT_LIMIT - 1) {
          if (!rej_own) atomicOr(p.status, BE_STATUS_REJECTION_LIMIT);
          rej = true; break;
        }
        const u4 b = philox(u, ep, 0u, tag(PURPOSE_RESET, 1 + r), p.seed);
        rax = map_range(b.x, 0, t.strip_agent_x); ray = map_range(b.y, 0, t.strip_agent_y);
      }
    }
    {   // the slot's goal / agent to all its lanes (uniform readlanes, one select per slot)
      const int32_t gp = pk(rgx, rgy), apk = pk(rax, ray);
      int32_t gsel = 0, asel = 0;
#pragma unroll
      for (int s2 = 0; s2 < P; ++s2) {
        const int32_t g2 = __builtin_amdgcn_readlane(gp, s2 * GL + G), a2 = __builtin_amdgcn_readlane(apk, s2 * GL + G);
        gsel = slot == s2 ? g2 : gsel; asel = slot == s2 ? a2 : asel;
      }
      if (is_goal && act) stash[slot * 4 + 2] = pk(ax0, ay0);
      rgx = px(gsel); rgy = py(gsel); rax = px(asel); ray = py(asel);
    }
    DIAG(12);
    if (act && !is_goal) {
      int ox = map_range(bo.x, t.strip_obs_x, W - t.strip_obs_x);
      int oy = map_range(bo.y, t.strip_obs_y, H - t.strip_obs_y);
      if (is_static) {        // rejection vs the agent / goal rectangles (:145, :193-197)
        for (int a = 1;; ++a) {
          const bool ra = abs(ox - rax) < rx && 2 * abs(oy - ray) < ry2;
          const bool rg = abs(ox - rgx) < rx && 2 * abs(oy - rgy) < ry2;
          if (!ra && !rg) break;
          if (a >= REJECT_LIMIT) {
            if (!rej_own) atomicOr(p.status, BE_STATUS_REJECTION_LIMIT);
            rej = true; break;
          }
          bo = philox(u, ep, 0u, tag(PURPOSE_RESET, sub0 | (uint32_t)a), p.seed);
          ox = map_range(bo.x, t.strip_obs_x, W - t.strip_obs_x);
          oy = map_range(bo.y, t.strip_obs_y, H - t.strip_obs_y);
        }
      }
      osink(slot, k, il, pk(ox, oy));
      if (k == 0) { stash[slot * 4 + 0] = pk(rax, ray); stash[slot * 4 + 1] = pk(rgx, rgy); }
      const int f = ox - (rax - WT / 2), e = oy - (ray - WT / 2);   // unit cell step (fixed-shape kernels)
      if ((uint32_t)(f + rx) <= (uint32_t)(WT - 1 + 2 * rx) && (uint32_t)(e + rx) <= (uint32_t)(K - 1 + 2 * rx)) {
        uint32_t mk[K];   // few lanes get here: the row masks branch-free, then same-address LDS atomics
        if (span) {       // raster_rows_span's rows (window-relative f, e here)
          const uint64_t* col = span + (e + rx);
          const uint32_t sh = (uint32_t)(WT - 1 + rx - f);
#pragma unroll
          for (int r = 0; r < K; ++r) mk[r] = (uint32_t)(col[K - 1 - r] >> sh) & ((1u << WT) - 1u);
        } else {
#pragma unroll
          for (int r = 0; r < K; ++r) {
            const int ady = abs(e - r);
            const int hw = t.hw[min(ady, HW_MAX)];
            const int lo = max(f - hw, 0), hi = min(f + hw, WT - 1);
            mk[r] = (ady <= rx && lo <= hi) ? (2u << hi) - (1u << lo) : 0u;
          }
        }
#pragma unroll
        for (int r = 0; r < K; ++r) atomicOr(&wrows[slot * K + r], mk[r]);
      }
    }
    // (the step kernels keep the status atomic at the loop's bound, as in round 5: one ballot and a
    // conditional atomic per pass instead measured 0.08 us slower per step, profiles/r06_pool_ab.txt)
    const unsigned long long rb = rej_own ? __ballot(rej) : 0ull;
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    DIAG(13);
    int own = -1;   // the slot whose env this lane owns
#pragma unroll
    for (int s2 = 0; s2 < P; ++s2) own = (s2 < n && lane / LPE == ls[s2] / LPE) ? s2 : own;
    if (own >= 0) {
      const int32_t ag = stash[own * 4 + 0], go = stash[own * 4 + 1], a0 = stash[own * 4 + 2];
      ax = px(ag); ay = py(ag); gx = px(go); gy = py(go);
      esink(own, ag, go, a0);
      if (rej_own) *rej_own = ((rb >> (own * GL)) & ((1ull << GL) - 1ull)) ? 1u : 0u;
      ncnt = 0;
#pragma unroll
      for (int r = 0; r < K; ++r) xrows[r] = wrows[own * K + r];
    }
    __builtin_amdgcn_wave_barrier();
    DIAG(14);
  }
}

// ------------------------------------------------------------------ the kernel
// MODE_STEP: physics + (autoreset) + obs.  MODE_RESET: reset masked envs + obs.
// MODE_OBSERVE: obs only.  WT = compile-time W (0 = runtime W: no LDS staging,
// sequential resets).  LPE = lanes per env.
//
// Resets (Philox mode) are block-cooperative: envs that must reset are compacted
// into an LDS list, then phase A draws each one's goal/agent (one thread per env)
// and phase B draws every obstacle of every listed env (one thread per obstacle),
// rasterising it straight into the env's LDS row masks.  A finishing env therefore
// costs the block ~2 Philox blocks of latency instead of a serial ~20 on one lane.
//
// NSC/NDC > 0: a step kernel specialised for exactly NSC static / NDC dynamic obstacles in
// Philox mode (no tape), one lane per env -- every obstacle loop is unrolled to its exact
// trip count (the dispatcher picks it only for a matching config).
__device__ __forceinline__ Tables& tab_of(TablesX& x) { return x.t; }
__device__ __forceinline__ Tables& tab_of(Tables& x) { return x; }
// be_kernel's rasteriser: FIXED from the wave's span table when it fits R (a uniform branch),
// the half-width table otherwise; the generic kernels their span arithmetic.
template <int WT, bool FIXED, class TT>
__device__ __forceinline__ void raster_fixed(const NearList<BLOCK_THREADS>& nl, const Win& g, int R,
                                             uint32_t (&rows)[Geo<WT>::K], TT& tb) {
  if constexpr (FIXED) {
    if (span_fits(WT, R)) raster_rows_span<WT, BLOCK_THREADS>(nl, R, rows, tb.span);
    else raster_rows<WT, BLOCK_THREADS, true>(nl, g, rows, tb.t.hw);
  } else {
    raster_rows<WT, BLOCK_THREADS, false>(nl, g, rows, tab_of(tb).hw);
  }
}

// POOL (the fixed-shape step only): a finishing env copies its autoreset-pool entry (§3.10) when it
// is current; the false instances are the code without the pool
template <int WT, int MODE, int NSC = 0, int NDC = 0, bool POOL = false>
__global__ __launch_bounds__(BLOCK_THREADS) void be_kernel(KParams p) {
  constexpr bool FIXED = NSC > 0 || NDC > 0;
  static_assert(!POOL || (FIXED && MODE == MODE_STEP && (WT == 10 || WT == 5)), "the pool: fixed-shape steps at W = 10 / 5");
  constexpr int LPE = FIXED ? 1 : lanes_for(WT);
  constexpr int EPB = BLOCK_THREADS / LPE;
  static_assert(!FIXED || (MODE == MODE_STEP && WT > 0 && NSC <= CS && NDC <= CD), "fixed-shape kernels: step only");
  constexpr int SPL = FIXED ? NSC : CS / LPE, DPL = FIXED ? NDC : CD / LPE;   // obstacle slots per lane
  constexpr bool COOP = WT > 0;                   // cooperative reset path (needs compile-time W)
  constexpr int KR = WT > 0 ? Geo<WT>::K : 1;
  extern __shared__ __align__(16) uint8_t smem[];
  // FIXED: one copy of the tables per wave, so the fixed-shape kernel has no block barrier (8.11-8.21
  // against 8.15-8.27 us at 131 072 envs, the same within noise at 262 144 and 2^20 envs:
  // profiles/r04_onelane_wave_tables_ab.txt)
  // (FIXED: TablesX, the row-span table included)
  __shared__ __align__(16) std::conditional_t<FIXED, TablesX, Tables> t_blk[FIXED ? BLOCK_THREADS / 64 : 1];
  // block-cooperative reset list and block stats: the generic kernels only.  FIXED never
  // initialises or reads them (it resets wave by wave through wave_resets and folds its stats per
  // half-wave), so they are sized 1 there: a FIXED change that needs them must size them again.
  constexpr int BLK_LIST = FIXED ? 1 : RCAP;
  __shared__ WaveStats s_ws[FIXED ? 1 : BLOCK_THREADS / 64];
  __shared__ int s_nreset;
  __shared__ int16_t s_slot_of[FIXED ? 1 : EPB];   // env -> reset slot (-1: none)
  __shared__ int16_t s_reset_el[BLK_LIST];
  __shared__ uint32_t s_reset_ep[BLK_LIST];
  __shared__ int32_t s_reset_agent[BLK_LIST], s_reset_goal[BLK_LIST];
  __shared__ uint32_t s_rows[RCAP][KR];            // FIXED too: 16 rows of wave_resets scratch per wave
  constexpr int TW = (int)(sizeof(Tables) / 4);
  static_assert(TW <= BLOCK_THREADS && sizeof(Tables) % 4 == 0, "table staging assumes <= 256 words");
  constexpr int TW4 = (int)(sizeof(TablesX) / 16);   // FIXED: 16-byte words of TablesX per wave copy

  DIAG(0);
  if (DBG(DBG_EXIT_ENTRY)) return;
  const int N = p.n, Ns = FIXED ? NSC : p.ns, Nd = FIXED ? NDC : p.nd;
  const int tid = threadIdx.x;
  Tables& t = tab_of(t_blk[FIXED ? (tid >> 6) : 0]);
  const int q = tid & (LPE - 1);                  // lane within the env's group
  const int el = tid / LPE;                        // env within the block
  const int blk0 = (int)blockIdx.x * EPB;
  const int i = blk0 + el;
  const bool valid = i < N;
  const bool lead = q == 0;                        // the group lane that owns per-env stores

  // LDS: [near lists: nobs+1 slots x 256 lanes x 4 B][obs stage: EPB x F bytes]
  NearList<BLOCK_THREADS> nl{reinterpret_cast<uint32_t*>(smem) + tid, 0};
  uint8_t* stage = smem + (size_t)(Ns + Nd + 1) * BLOCK_THREADS * 4;

  int ax = 0, ay = 0, gx = 0, gy = 0;
  bool done = false;
  double fin_ret = 0.0;
  int fin_len = 0;
  uint32_t episode = 0;
  uint32_t st_flags = 0;   // BE_STATUS_* raised by this lane, published once per wave
  // fixed-shape kernels defer the step's state / output stores to the very end of the wave
  // (a store still in flight makes later register reuse wait for vmcnt(0), on the critical path)
  const uint32_t gid = (uint32_t)p.gid0 + (uint32_t)i;

  // ---- phase 0: issue every load of this env (independent, coalesced across the wave)
  //      together with the block's table words; one barrier then covers them all.
  int a = 0, dx = 0, dy = 0, len0 = 0;
  int32_t agent0 = 0, goal0 = 0;
  double old_dist = 0.0, total = 1.0, ret = 0.0;
  const int ns0 = FIXED ? NSC : min(Ns, CS), nd0 = FIXED ? NDC : min(Nd, CD);
  int32_t so[SPL], dp[DPL];
  int dgi[DPL], t0[DPL], t1[DPL];
#pragma unroll
  for (int j = 0; j < SPL; ++j) so[j] = 0;
#pragma unroll
  for (int j = 0; j < DPL; ++j) { dp[j] = 0; dgi[j] = 0; t0[j] = 0; t1[j] = 0; }
  constexpr int TLW = FIXED ? (TW4 + 63) / 64 : 1;   // table words per lane (FIXED: 16-byte)
  uint4 tword[TLW];
#pragma unroll
  for (int j = 0; j < TLW; ++j) tword[j] = uint4{0u, 0u, 0u, 0u};
  if constexpr (FIXED) {
    // straight-line prologue (no branches around loads, clamped env index; invalid lanes
    // never store): the waitcnt pass can then retire the loads one by one -- tables
    // first, then in use order -- instead of draining everything at the first join
    // (32-bit unsigned element offsets from uniform bases: global_load's SGPR-base form)
    const uint32_t ic = (uint32_t)min(i, N - 1);
#pragma unroll
    for (int j = 0; j < TLW; ++j)
      tword[j] = ld_s(reinterpret_cast<const uint4*>(p.tables), (uint32_t)min((tid & 63) + j * 64, TW4 - 1));
    episode = ld_s(p.episode, ic);
    len0 = ld_s(p.ep_len, ic);
    a = ld_s(p.actions, ic);
    agent0 = ld_s(p.agent, ic);
    goal0 = ld_s(p.goal, ic);
#pragma unroll
    for (int j = 0; j < NDC; ++j) { dp[j] = ld_s(p.dyn_obs + (size_t)j * N, ic); dgi[j] = ld_s(p.dyn_goal + (size_t)j * N, ic); }
#pragma unroll
    for (int j = 0; j < NSC; ++j) so[j] = ld_s(p.static_obs + (size_t)j * N, ic);
    // prev_dist read even when prev_read = 0 recomputes it, the select after every load is issued
    // (a branch among the loads made the compiler wait for the agent / goal loads first)
    const double old_read = ld_s(p.prev_dist, ic);
    total = ld_s(p.total_dist, ic);
    ret = ld_s(p.ep_return, ic);
    __builtin_amdgcn_sched_barrier(0);
    old_dist = p.prev_read ? old_read : calc_dist(px(goal0), py(goal0), px(agent0), py(agent0));
  } else {
  tword[0].x = tid < TW ? reinterpret_cast<const uint32_t*>(p.tables)[tid] : 0u;
  if (valid) {
    // issue order = use order: vmcnt retires loads in order, so the Philox draws (keyed by
    // episode, ep_len) and the obstacle moves start while the statics and f64s are in flight
    if (MODE != MODE_OBSERVE) episode = p.episode[i];
    if (MODE == MODE_STEP) {
      len0 = p.ep_len[i];
      if (p.actions) a = p.actions[i];
      else if (p.deltas) { dx = p.deltas[2 * (int64_t)i]; dy = p.deltas[2 * (int64_t)i + 1]; }
    }
    agent0 = p.agent[i];
    goal0 = p.goal[i];
    if (MODE == MODE_STEP) {
      if (nd0 > 0) {
#pragma unroll
        for (int j = 0; j < DPL; ++j) {
          const int k = min(q + LPE * j, nd0 - 1);
          dp[j] = (p.dyn_obs + (size_t)k * N)[i];
          dgi[j] = (p.dyn_goal + (size_t)k * N)[i];
          if (!FIXED && p.tape) { t0[j] = (p.tape + (size_t)(2 * k) * N)[i]; t1[j] = (p.tape + (size_t)(2 * k + 1) * N)[i]; }
        }
      }
      // fixed slots: indices past the count re-read the last obstacle (same lines: no extra traffic)
      if (ns0 > 0) {
#pragma unroll
        for (int j = 0; j < SPL; ++j) so[j] = (p.static_obs + (size_t)min(q + LPE * j, ns0 - 1) * N)[i];
      }
      old_dist = p.prev_dist[i];
      total = p.total_dist[i];
      ret = p.ep_return[i];
    }
  }
  }
  if constexpr (FIXED) {   // this wave's copy of the tables; nothing else is block-shared here
#pragma unroll
    for (int j = 0; j < TLW; ++j) reinterpret_cast<uint4*>(&t_blk[tid >> 6])[min((tid & 63) + j * 64, TW4 - 1)] = tword[j];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    if (tid < TW) reinterpret_cast<uint32_t*>(&t)[tid] = tword[0].x;
    if (EPB == BLOCK_THREADS || tid < EPB) s_slot_of[tid] = -1;
    if (tid == 0) s_nreset = 0;
    __syncthreads();  // barrier 1: tables staged (the state loads retire in order as they are used)
  }
  DIAG(1);
  if (DBG(DBG_WAIT_LOADS)) {   // diagnostics: when has every load of this wave landed?
    __builtin_amdgcn_s_waitcnt(0);   // vmcnt(0) expcnt(0) lgkmcnt(0)
    DIAG(15);
  }
  if (DBG(DBG_EXIT_BARRIER)) {
    if (valid && (agent0 ^ goal0 ^ so[0] ^ dp[0] ^ (int)len0 ^ (int)old_dist) == 0x7fffffff) p.obs[i] = 1;
    return;
  }

  if (valid) {
    gx = px(goal0); gy = py(goal0);
    if (MODE == MODE_STEP) {
      // ---- action -> agent move + clamp (ballenv_env.py:247-259); every lane of the group
      if (FIXED) {   // unit moves from the packed kernel-argument table: no LDS round trip
        st_flags |= a >= p.num_actions ? (uint32_t)BE_STATUS_BAD_ACTION : 0u;
        const uint32_t sh = 2u * (uint32_t)(a < p.num_actions ? a : 0);
        dx = (int)((p.amx >> sh) & 3u) - 1; dy = (int)((p.amy >> sh) & 3u) - 1;
      } else if (p.actions) {
        st_flags |= a >= p.num_actions ? (uint32_t)BE_STATUS_BAD_ACTION : 0u;
        a = a < p.num_actions ? a : 0;
        const int32_t m = t.action[a]; dx = px(m); dy = py(m);
      } else if (!p.deltas) {  // sampled actions
        const u4 b = philox(gid, episode, (uint32_t)len0, tag(PURPOSE_ACTION, 0), p.seed);
        const int32_t m = t.action[map_range(b.x, 0, p.num_actions)]; dx = px(m); dy = py(m);
      }
      ax = min(max(px(agent0) + p.speed_x * dx, 0), p.screen_w);
      ay = min(max(py(agent0) + p.speed_y * dy, 0), p.screen_h);
      const Win g(p, ax, ay);
      const NearBox nb(g);
      const uint32_t R2 = (uint32_t)g.R2;
      bool hs = false, hd = false;
      DIAG(8);

      // ---- dynamic obstacles: move (counter == ep_len mod (G+1): all start at 0 on reset)
      int counter = (int)((double)len0 * p.inv_g1);
      counter = len0 - counter * (p.goal_change + 1);
      if (counter < 0) counter += p.goal_change + 1;
      if (counter > p.goal_change) counter -= p.goal_change + 1;
      const bool change = counter >= p.goal_change;
      const bool tape = !FIXED && p.tape != nullptr;
      // Philox fields: obstacle k uses 24-bit field k%5 of block k/5 (both of its draws).
      uint32_t wj[DPL];
#pragma unroll
      for (int j = 0; j < DPL; ++j) wj[j] = 0u;
      if (!tape && !DBG(DBG_NO_PHILOX)) {
        const u4 b0 = philox(gid, episode, (uint32_t)len0, tag(PURPOSE_STEP_OBS, 0u), p.seed);
        u4 b1{0u, 0u, 0u, 0u};
        if (nd0 > 5) b1 = philox(gid, episode, (uint32_t)len0, tag(PURPOSE_STEP_OBS, 1u), p.seed);
#pragma unroll
        for (int j = 0; j < DPL; ++j) {
          const int k = q + LPE * j;   // < CD = 8 <= 10: blocks 0 and 1 cover every slot
          wj[j] = k < 5 ? pick_field(b0, k) : pick_field(b1, k - 5);
        }
      }
      // FIXED: exact trip counts; one (dx, dy) per obstacle feeds both the collision test and
      // the window-box test (the box is a superset of the cells' R-neighbourhood; the
      // rasteriser is exact, so a box hit that lights nothing costs only raster work)
      const int bxo = p.speed_x * (p.window / 2) + g.R, byo = p.speed_y * (p.window / 2) + g.R;
      const uint32_t bw = nb.bw, bh = nb.bh;   // = NearBox's test, relative to the agent
      auto obstacle = [&](int ox, int oy, bool& hit) {
        const int dx = ox - ax, dy = oy - ay;
        hit |= (uint32_t)__mul24(dx, dx) + (uint32_t)__mul24(dy, dy) <= R2;
        // unconditional LDS write, predicated count: no divergent region per obstacle
        nl.base[nl.cnt * BLOCK_THREADS] = (uint32_t)((dx + bxo - g.R) & 0xFFFF) | ((uint32_t)(dy + byo - g.R) << 16);
        nl.cnt += ((uint32_t)(dx + bxo) <= bw && (uint32_t)(dy + byo) <= bh) ? 1 : 0;
      };
      // packed int16x2 form: saturating subtract (a saturated offset is out of reach either way,
      // as is the true one), dx^2 + dy^2 by one v_dot2 (compared unsigned: no overflow case)
      const v2s agv = __builtin_bit_cast(v2s, pk(ax, ay));
      typedef unsigned short v2u __attribute__((ext_vector_type(2)));
      const v2s boxo = {(short)bxo, (short)byo};
      const v2u boxw = {(unsigned short)bw, (unsigned short)bh};
      // near-list entries are agent-relative (dx, dy) here; the raster adds the window offset
      // (the near list's next slot as an LDS address advanced by sat(1 - over) slots, as in
      // step2_kernel: no compare / select / carry chain per obstacle; nl.cnt is set after the tests)
      uint32_t* nlp = nl.base;
      auto obstacle_pk = [&](int32_t opk, bool& hit) {
        const v2s d = __builtin_elementwise_sub_sat(__builtin_bit_cast(v2s, opk), agv);
        hit |= (uint32_t)__builtin_amdgcn_sdot2(d, d, 0, false) <= R2;   // (dot2_sq: neutral here, r05_dot2_vop3p_ab.txt)
        const v2u b = __builtin_bit_cast(v2u, __builtin_elementwise_add_sat(d, boxo));
        const v2u over = __builtin_elementwise_sub_sat(b, boxw);   // (0, 0) iff inside the box
        *nlp = __builtin_bit_cast(uint32_t, d);
        nlp += BLOCK_THREADS * __builtin_elementwise_sub_sat(1u, __builtin_bit_cast(uint32_t, over));
      };
      if constexpr (FIXED) {
        DIAG(7);
        int ngs[NDC];
#pragma unroll
        for (int j = 0; j < NDC; ++j) {
          int ox = px(dp[j]), oy = py(dp[j]);
          ngs[j] = dyn_move_fixed(p, t, ox, oy, dgi[j], t.speed[j], change, wj[j], st_flags);
          const int32_t npk = pk(ox, oy);
          if (valid) st_ws(p.dyn_obs + (size_t)j * N, (uint32_t)i, npk);
          obstacle_pk(npk, hd);
        }
        if (valid && change) {   // every obstacle re-picks its goal on the same step
#pragma unroll
          for (int j = 0; j < NDC; ++j) st_ws(p.dyn_goal + (size_t)j * N, (uint32_t)i, (uint8_t)ngs[j]);
        }
        DIAG(11);
#pragma unroll
        for (int j = 0; j < NSC; ++j) obstacle_pk(so[j], hs);
        nl.cnt = (int)(lds_bytes(nl.base, nlp) / (BLOCK_THREADS * 4u));
      }
      // generic slot loops: slots past the obstacle count hold a far-away sentinel, so the
      // collision / window tests are branch-free; only their stores are skipped
      constexpr int FAR = -30000;
#pragma unroll
      for (int j = 0; j < (FIXED ? 0 : DPL); ++j) {
        const int k = q + LPE * j;
        const bool real = k < nd0;
        int ox = real ? px(dp[j]) : FAR, oy = real ? py(dp[j]) : FAR;
        if (!DBG(DBG_NO_DYN) && real) {
          const int ng = dyn_move(p, t, ox, oy, dgi[j], t.speed[k], change, tape, t0[j], t1[j], wj[j], st_flags);
          (p.dyn_obs + (size_t)k * N)[i] = pk(ox, oy);
          if (ng != dgi[j]) (p.dyn_goal + (size_t)k * N)[i] = (uint8_t)ng;
        }
        hd |= collides(ox, oy, ax, ay, R2);
        int f, e;
        nl.push_if(nb.maybe(ox, oy) && g.near(ox, oy, f, e) && !DBG(DBG_NO_NEAR), f, e);
      }
      for (int kb = CD + q; !FIXED && kb < Nd; kb += LPE) {  // configs with more than CD dynamic obstacles
        int32_t* pos = p.dyn_obs + (size_t)kb * N + i;
        uint8_t* gp = p.dyn_goal + (size_t)kb * N + i;
        int ox = px(*pos), oy = py(*pos);
        const int gi = *gp;
        const u4 blk = tape ? u4{0, 0, 0, 0} : philox(gid, episode, (uint32_t)len0, tag(PURPOSE_STEP_OBS, (uint32_t)(kb / 5)), p.seed);
        const int tt0 = tape ? (p.tape + (size_t)(2 * kb) * N)[i] : 0, tt1 = tape ? (p.tape + (size_t)(2 * kb + 1) * N)[i] : 0;
        const int ng = dyn_move(p, t, ox, oy, gi, t.speed[kb], change, tape, tt0, tt1, pick_field(blk, kb % 5), st_flags);
        *pos = pk(ox, oy);
        if (ng != gi) *gp = (uint8_t)ng;
        hd |= collides(ox, oy, ax, ay, R2);
        int f, e;
        if (nb.maybe(ox, oy) && g.near(ox, oy, f, e)) nl.push(f, e);
      }
      DIAG(9);
      // ---- static obstacles: collision + near test
#pragma unroll
      for (int j = 0; j < (FIXED ? 0 : SPL); ++j) {
        const int k = q + LPE * j;
        const bool real = k < ns0;
        const int ox = real ? px(so[j]) : FAR, oy = real ? py(so[j]) : FAR;
        hs |= collides(ox, oy, ax, ay, R2);
        int f, e;
        nl.push_if(nb.maybe(ox, oy) && g.near(ox, oy, f, e) && !DBG(DBG_NO_NEAR), f, e);
      }
      for (int kb = CS + q; !FIXED && kb < Ns; kb += LPE) {
        const int32_t o = (p.static_obs + (size_t)kb * N)[i];
        const int ox = px(o), oy = py(o);
        hs |= collides(ox, oy, ax, ay, R2);
        int f, e;
        if (nb.maybe(ox, oy) && g.near(ox, oy, f, e)) nl.push(f, e);
      }
      // the group's collision flags (every lane of a valid group is active here)
      hs = group_or<LPE>((uint32_t)hs) != 0u;
      hd = group_or<LPE>((uint32_t)hd) != 0u;
      DIAG(10);

      // ---- distance, reward, done (ballenv_env.py:268-286, 200-229)
      const double dist = calc_dist(gx, gy, ax, ay);
      double reward = 0.0 - p.time_penalty;
      reward += (old_dist - dist) / total;
      if (hs) reward -= p.static_penalty;          // statics come first in obstacle_list (Q3)
      else if (hd) reward -= p.dynamic_penalty;
      ret += reward;
      const int len = len0 + 1;
      const bool env_done = (dist < p.threshold_goal) || hs || hd;
      const bool trunc = p.time_limit > 0 && len >= p.time_limit;
      done = env_done || trunc;
      if (lead) {
        // FIXED: SGPR-base stores with 32-bit offsets (FIX_MAX_ENVS); the generic kernels index in 64 bits
        auto sto = [&](auto* base, auto v) {
          if constexpr (FIXED) st_ws(base, (uint32_t)i, v);
          else st_wt(base + i, v);
        };
        sto(p.reward, reward);
        sto(p.done, (uint8_t)done);
        if (p.truncated) sto(p.truncated, (uint8_t)(trunc && !env_done));
        sto(p.agent, pk(ax, ay));
        sto(p.prev_dist, dist);
        sto(p.ep_return, ret);
        sto(p.ep_len, len);
        if (done) {
          if (p.final_return) st_wt(p.final_return + i, ret);
          if (p.final_len) st_wt(p.final_len + i, len);
        }
      }
      fin_ret = ret; fin_len = len;
    } else {
      ax = px(agent0); ay = py(agent0);
    }
  }
  DIAG(2);
  if (DBG(DBG_EXIT_PHYSICS)) return;
  if (MODE == MODE_STEP && __ballot(st_flags != 0u)) {   // rare: OR the wave's flags, one atomic
    uint32_t f = st_flags;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) f |= (uint32_t)__shfl_xor((int)f, o);
    if ((tid & 63) == 0) atomicOr(p.status, (int)f);
  }
  WaveStats ws{0.0, 0.0, 0.0, 0.0, INFINITY, -INFINITY}, ws_hi = ws;
  // (POOL: after the resets, below -- a reset leaves fin_ret / fin_len alone -- so that the two halves'
  // sums are not live across the pool's loads: 148 -> 107 VGPRs, four waves per SIMD again)
  if (!POOL && MODE == MODE_STEP && p.stats && !DBG(DBG_NO_STATS)) {   // all lanes converged here
    if constexpr (FIXED) {   // one slot per 32 envs (be_stats_slots): the wave's two halves
      wave_stats2(done && lead, fin_ret, fin_len, ws, ws_hi);
    } else {
      ws = wave_stats(done && lead, fin_ret, fin_len);
    }
  }

  // ---- episode boundary
  bool do_reset = false;
  if (valid) {
    if (MODE == MODE_STEP) do_reset = done && p.autoreset;
    if (MODE == MODE_RESET) do_reset = p.mask ? (p.mask[i] != 0) : true;
  }
  const bool tape_reset = MODE == MODE_RESET && p.reset_tape != nullptr;
  if (valid && do_reset) {
    if (MODE == MODE_STEP && p.terminal_obs) {  // obs of the terminal state (group-uniform branch)
      const int F = 4 + p.window * p.window;
      const Win g(p, ax, ay);
      const int quad = quadrant(ax, ay, gx, gy);
      if constexpr (WT > 0) {
        uint32_t rows[Geo<WT>::K], flat[Geo<WT>::NW];
        raster_fixed<WT, FIXED>(nl, g, p.R, rows, t_blk[FIXED ? (tid >> 6) : 0]);
#pragma unroll
        for (int k = 0; k < Geo<WT>::K; ++k) rows[k] = group_or<LPE>(rows[k]);
        flatten<WT>(rows, flat);
        if (lead) write_row_global<WT>(p.terminal_obs + (int64_t)i * F, flat, quad);
      } else {
        write_row_generic<BLOCK_THREADS>(nl, g, quad, p.terminal_obs + (int64_t)i * F, nullptr);
      }
    }
    if (!COOP || tape_reset) {
      // sequential reset on the lead lane: the reference's single draw stream (tape), or runtime-W kernels
      if (lead) {
        ResetDraws ds{tape_reset ? p.reset_tape : nullptr, p.reset_tape_len, N, i, 0, gid, episode + 1u, p.seed,
                      p.status};
        if (tape_reset) reset_env<BLOCK_THREADS>(p, t, i, ds, ax, ay, gx, gy, nl);
        else reset_env_philox<BLOCK_THREADS, 1>(p, t, i, 0, gid, episode + 1u, ax, ay, gx, gy, nl);
      } else {
        nl.cnt = 0;
      }
      ax = group_bcast<LPE>(ax); ay = group_bcast<LPE>(ay);
      gx = group_bcast<LPE>(gx); gy = group_bcast<LPE>(gy);
    } else if (!FIXED && lead) {
      const int slot = atomicAdd(&s_nreset, 1);   // LDS atomic: compact the block's resets
      s_slot_of[el] = (int16_t)slot;
      if (slot < RCAP) { s_reset_el[slot] = (int16_t)el; s_reset_ep[slot] = episode + 1u; }
    }
  } else if (valid && MODE != MODE_STEP) {
    // observe / reset of an unmasked env: near list of the current state, split over the group
    const Win g(p, ax, ay);
    for (int k = q; k < Ns; k += LPE) {
      const int32_t o = (p.static_obs + (size_t)k * N)[i];
      int f, e;
      if (g.near(px(o), py(o), f, e)) nl.push(f, e);
    }
    for (int k = q; k < Nd; k += LPE) {
      const int32_t o = (p.dyn_obs + (size_t)k * N)[i];
      int f, e;
      if (g.near(px(o), py(o), f, e)) nl.push(f, e);
    }
  }
  uint32_t xrows[KR];   // window rows of a wave-reset env (fixed-shape kernels)
#pragma unroll
  for (int k = 0; k < KR; ++k) xrows[k] = 0u;
  if constexpr (FIXED) {
    bool hit = false;
    if constexpr (POOL) {   // the entry for episode + 1 (its tag and 112-byte body), waited for in the branch
      constexpr int NBW = pool_body_words(NSC, NDC);
      static_assert(NBW == 28, "seven 16-byte body loads");
      const bool ptry = valid && do_reset && p.pool != nullptr;
      uint2 q_tv = make_uint2(0u, 0u);
      uint4 qb[7];
      if (ptry) {
        const uint32_t x = ((episode + 1u) & 1u) * (uint32_t)N + (uint32_t)i;
        q_tv = pool_ld<uint2>(p.pool, x * 8u);
        const uint32_t bo = pool_body((uint32_t)N, x, NBW);
#pragma unroll
        for (int j = 0; j < 7; ++j) qb[j] = pool_ld<uint4>(p.pool, bo, 16u * j);
        __builtin_amdgcn_s_waitcnt(0);   // here, in the branch: no pending pool load past its end
      }
      if (__ballot(ptry)) {
        hit = ptry && q_tv.x == episode + 1u && (q_tv.y & POOL_VALID) != 0u;
        if (hit) {   // the new state as esink / osink below store it, then the rows for the obs
          auto qw = [&](int k) -> uint32_t { return u4w(qb[k >> 2], k & 3); };   // body word k (compile-time k)
          const uint32_t iu = (uint32_t)i;
          const int32_t ag = (int32_t)qw(PB_AGENT), go = (int32_t)qw(PB_GOAL);
          st_ws(p.agent, iu, ag);
          st_ws(p.goal, iu, go);
          st_ws(p.prev_dist, iu, u2d(qw(PB_PREV), qw(PB_PREV + 1)));
          st_ws(p.total_dist, iu, u2d(qw(PB_TOTAL), qw(PB_TOTAL + 1)));
          st_ws(p.ep_return, iu, 0.0);
          st_ws(p.ep_len, iu, 0);
          st_ws(p.episode, iu, episode + 1u);
#pragma unroll
          for (int k = 0; k < NSC; ++k) st_ws(p.static_obs + (size_t)k * N, iu, (int32_t)qw(PB_OBS + k));
#pragma unroll
          for (int k = 0; k < NDC; ++k) {
            st_ws(p.dyn_obs + (size_t)k * N, iu, (int32_t)qw(PB_OBS + NSC + k));
            st_ws(p.dyn_goal + (size_t)k * N, iu, (uint8_t)k);
          }
          ax = px(ag); ay = py(ag); gx = px(go); gy = py(go);
#pragma unroll
          for (int k = 0; k < KR; ++k)
            xrows[k] = WT == 10 ? (qw(PB_ROWS + k / 3) >> (10 * (k % 3))) & 0x3FFu   // three rows per word
                                : (qw(PB_ROWS) >> (5 * k)) & 0x1Fu;                  // W = 5: four in one
          nl.cnt = 0;
        }
        if (__ballot(hit && (q_tv.y & POOL_REJ)) && (tid & 63) == 0) atomicOr(p.status, BE_STATUS_REJECTION_LIMIT);
      }
    }
    const unsigned long long m = __ballot(valid && do_reset && !hit);
    static_assert(!FIXED || (RCAP >= (BLOCK_THREADS / 64) * 16 && 16 * KR >= (64 / (NSC + NDC + !FIXED)) * (KR + 4)), "wave reset scratch");
    // one finished env (the common case): the lean single-env pass; several: up to 3 per pass
    // a reset env's new state goes straight to HBM
    auto osink = [&](int, int k, int il, int32_t o) {
      if (k < NSC) {
        st_wt(p.static_obs + (size_t)k * N + il, o);
      } else {
        st_wt(p.dyn_obs + (size_t)(k - NSC) * N + il, o);
        st_wt(p.dyn_goal + (size_t)(k - NSC) * N + il, (uint8_t)(k - NSC));
      }
    };
    auto esink = [&](int, int32_t ag, int32_t go, int32_t a0) {
      st_wt(p.agent + i, ag);
      st_wt(p.goal + i, go);
      double prev;
      const double td = reset_dists(ag, go, a0, prev);
      st_wt(p.prev_dist + i, prev);
      st_wt(p.total_dist + i, td);
      st_wt(p.ep_return + i, 0.0);
      st_wt(p.ep_len + i, 0);
      st_wt(p.episode + i, episode + 1u);
    };
    if (m && !(m & (m - 1)))
      wave_resets<WT, NSC, NDC, 1>(p, t, m, i, gid, episode, ax, ay, gx, gy, nl.cnt, xrows, &s_rows[(tid >> 6) * 16][0],
                                   osink, esink);
    else if (m)
      wave_resets<WT, NSC, NDC, 64>(p, t, m, i, gid, episode, ax, ay, gx, gy, nl.cnt, xrows, &s_rows[(tid >> 6) * 16][0],
                                    osink, esink);
  }
  if (POOL && p.stats && !DBG(DBG_NO_STATS)) wave_stats2(done && lead, fin_ret, fin_len, ws, ws_hi);   // (converged)
  DIAG(3);

  // ---- observation (prep_state4)
  if constexpr (WT > 0) {
    constexpr int F = Geo<WT>::F;
    // 1) envs that did not go through the cooperative reset: their own near lists
    uint32_t flat[Geo<WT>::NW];
    int quad = 0;
    if (valid) {
      const Win g(p, ax, ay);
      uint32_t rows[Geo<WT>::K];
      if (DBG(DBG_NO_RASTER)) nl.cnt = 0;
      raster_fixed<WT, FIXED>(nl, g, p.R, rows, t_blk[FIXED ? (tid >> 6) : 0]);
#pragma unroll
      for (int k = 0; k < Geo<WT>::K; ++k) rows[k] = group_or<LPE>(rows[k] | xrows[k]);
      flatten<WT>(rows, flat);
      quad = quadrant(ax, ay, gx, gy);
    }
    if (DBG(DBG_NO_OBS | DBG_EXIT_RASTER)) {
      if (valid && flat[0] == 0x12345u && quad == 7) p.obs[i] = 1;   // keep the rows live
      return;
    }
    if (valid) {  // lane q writes words (bytes, when F % 4 != 0) q, q+LPE, ... of its env's row
      auto word = [&](int w) -> uint32_t {
        const int jc = 4 * (w - 1);  // first cell of this word (nibble aligned)
        return w == 0 ? 1u << (8 * quad) : (((flat[jc >> 5] >> (jc & 31)) & 0xFu) * 0x00204081u) & 0x01010101u;
      };
      if constexpr (LPE == 1 && (F & 7) == 0) {   // 8-byte LDS stores (half the ds_write count)
        uint2* dst = reinterpret_cast<uint2*>(stage + el * F);
#pragma unroll
        for (int w = 0; w < F / 8; ++w) dst[w] = make_uint2(word(2 * w), word(2 * w + 1));
      } else if constexpr ((F & 3) == 0) {
        uint32_t* dst = reinterpret_cast<uint32_t*>(stage + el * F);
#pragma unroll
        for (int w0 = 0; w0 < F / 4; w0 += LPE) {
          const int w = w0 + q;
          if (w < F / 4) {
            uint32_t v;
            if (w == 0) v = 1u << (8 * quad);
            else {
              const int jc = 4 * (w - 1);  // first cell of this word (nibble aligned)
              v = (((flat[jc >> 5] >> (jc & 31)) & 0xFu) * 0x00204081u) & 0x01010101u;
            }
            dst[w] = v;
          }
        }
      } else {
        uint8_t* dst = stage + el * F;
#pragma unroll
        for (int b0 = 0; b0 < F; b0 += LPE) {
          const int b = b0 + q;
          if (b < F) dst[b] = (uint8_t)obs_byte<WT>(flat, quad, b);
        }
      }
    }
    DIAG(4);
    if constexpr (FIXED) {
      // each wave owns 64 contiguous obs rows: it copies them out and settles its own stats
      // slot -- no block barrier, so a wave that ran resets delays nobody else
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int w = tid >> 6, lane = tid & 63;
      const int e0 = blk0 + w * 64;
      DIAG(5);
      copy_out<64>(stage + w * 64 * F, F, max(0, min(64, N - e0)), (int64_t)e0, p.obs, p.obs_f32, lane);
      if (p.stats && (lane == 0 || lane == 32)) {
        const WaveStats& v = lane == 0 ? ws : ws_hi;
        if (v.n > 0.0) {
          double* slot = p.stats + (((size_t)blockIdx.x * (BLOCK_THREADS / 64) + w) * 2 + (lane >> 5)) * 8;
          slot[0] += v.n; slot[1] += v.s1; slot[2] += v.s2; slot[3] += v.sl;
          slot[4] = fmin(slot[4], v.mn); slot[5] = fmax(slot[5], v.mx);
        }
      }
      DIAG(6);
      return;
    }
    if (MODE == MODE_STEP && (tid & 63) == 0) s_ws[tid >> 6] = ws;
    __syncthreads();  // barrier 2: stage written; reset list complete

    // 2) cooperative resets (Philox): overwrite the stage rows of the listed envs
    if (COOP && !FIXED && !tape_reset) {
      const int nres = s_nreset;   // block-uniform
      for (int r0 = 0; r0 < nres; r0 += RCAP) {
        const int nr = min(RCAP, nres - r0);
        if (r0 > 0) {   // more than RCAP resets in this block (e.g. reset of every env): refill the list
          if (valid && lead && s_slot_of[el] >= r0 && s_slot_of[el] < r0 + RCAP) {
            const int s = s_slot_of[el] - r0;
            s_reset_el[s] = (int16_t)el; s_reset_ep[s] = episode + 1u;
          }
          __syncthreads();
        }
        // phase A: goal / agent (one thread per env), per-env scalars, clear row masks
        if (tid < nr) {
          const int e_l = s_reset_el[tid];
          const int ir = blk0 + e_l;
          const uint32_t ep = s_reset_ep[tid];
          const uint32_t g_id = (uint32_t)p.gid0 + (uint32_t)ir;
          const int W = p.screen_w, H = p.screen_h;
          const u4 b0 = philox(g_id, ep, 0u, tag(PURPOSE_RESET, 0), p.seed);
          const int rgx = map_range(b0.x, W - t.strip_goal_x, W), rgy = map_range(b0.y, H - t.strip_goal_y, H);
          int rax = map_range(b0.z, 0, t.strip_agent_x), ray = map_range(b0.w, 0, t.strip_agent_y);
          const double dist = calc_dist(rgx, rgy, rax, ray);
          for (int r = 0; calc_dist(rgx, rgy, rax, ray) < p.min_spawn_dist; ++r) {   // :121-126
            if (r >= REJECT_LIMIT - 1) { atomicOr(p.status, BE_STATUS_REJECTION_LIMIT); break; }
            const u4 b = philox(g_id, ep, 0u, tag(PURPOSE_RESET, 1 + r), p.seed);
            rax = map_range(b.x, 0, t.strip_agent_x); ray = map_range(b.y, 0, t.strip_agent_y);
          }
          p.agent[ir] = pk(rax, ray);
          p.goal[ir] = pk(rgx, rgy);
          p.prev_dist[ir] = dist;  // pre-resample distance (Q9)
          p.total_dist[ir] = calc_dist(rax, ray, rgx, rgy);
          p.ep_return[ir] = 0.0;
          p.ep_len[ir] = 0;
          p.episode[ir] = ep;
          s_reset_agent[tid] = pk(rax, ray);
          s_reset_goal[tid] = pk(rgx, rgy);
#pragma unroll
          for (int k = 0; k < KR; ++k) s_rows[tid][k] = 0u;
        }
        __syncthreads();
        DIAG(12);
        // phase B: every obstacle of every listed env, one per thread
        const int per = Ns + Nd;
        const int R = t.radius_obstacle + t.radius_agent;
        const int rx = R, ry2 = t.radius_obstacle + 2 * t.radius_agent;
        for (int it = tid; it < nr * per; it += BLOCK_THREADS) {
          const int s = it / per, k = it - s * per;
          const int ir = blk0 + s_reset_el[s];
          const uint32_t ep = s_reset_ep[s];
          const uint32_t g_id = (uint32_t)p.gid0 + (uint32_t)ir;
          const int rax = px(s_reset_agent[s]), ray = py(s_reset_agent[s]);
          const int rgx = px(s_reset_goal[s]), rgy = py(s_reset_goal[s]);
          const int W = p.screen_w, H = p.screen_h;
          int ox, oy;
          if (k < Ns) {   // static: rejection vs agent/goal rectangles (:131-149, :193-197)
            for (int at = 0;; ++at) {
              const u4 b = philox(g_id, ep, 0u, tag(PURPOSE_RESET, (1u << 22) | ((uint32_t)k << 12) | (uint32_t)at), p.seed);
              ox = map_range(b.x, t.strip_obs_x, W - t.strip_obs_x);
              oy = map_range(b.y, t.strip_obs_y, H - t.strip_obs_y);
              const bool ra = abs(ox - rax) < rx && 2 * abs(oy - ray) < ry2;
              const bool rg = abs(ox - rgx) < rx && 2 * abs(oy - rgy) < ry2;
              if (!ra && !rg) break;
              if (at >= REJECT_LIMIT - 1) { atomicOr(p.status, BE_STATUS_REJECTION_LIMIT); break; }
            }
            (p.static_obs + (size_t)k * N)[ir] = pk(ox, oy);
          } else {        // dynamic (:153-164)
            const int kd = k - Ns;
            const u4 b = philox(g_id, ep, 0u, tag(PURPOSE_RESET, (2u << 22) | ((uint32_t)kd << 12)), p.seed);
            ox = map_range(b.x, t.strip_obs_x, W - t.strip_obs_x);
            oy = map_range(b.y, t.strip_obs_y, H - t.strip_obs_y);
            (p.dyn_obs + (size_t)kd * N)[ir] = pk(ox, oy);
            (p.dyn_goal + (size_t)kd * N)[ir] = (uint8_t)kd;
          }
          const Win g(p, rax, ray);
          int f, e;
          if (g.near(ox, oy, f, e)) raster_one_lds<WT>(s_rows[s], g, f, e);
        }
        __syncthreads();
        DIAG(13);
        // phase C: the listed envs' obs rows into the stage
        if (tid < nr) {
          uint32_t rows[Geo<WT>::K], fl[Geo<WT>::NW];
#pragma unroll
          for (int k = 0; k < Geo<WT>::K; ++k) rows[k] = s_rows[tid][k];
          flatten<WT>(rows, fl);
          const int e_l = s_reset_el[tid];
          const int32_t ag = s_reset_agent[tid], go = s_reset_goal[tid];
          stage_full_row<WT>(stage + e_l * F, fl, quadrant(px(ag), py(ag), px(go), py(go)));
        }
        __syncthreads();
        DIAG(14);
      }
    }
    DIAG(5);
    const int nvalid = min(EPB, N - blk0);
    copy_out<BLOCK_THREADS>(stage, F, nvalid, (int64_t)blk0, p.obs, p.obs_f32);
  } else {
    if (valid && lead) {
      const int F = 4 + p.window * p.window;
      const Win g(p, ax, ay);
      write_row_generic<BLOCK_THREADS>(nl, g, quadrant(ax, ay, gx, gy), p.obs ? p.obs + (int64_t)i * F : nullptr,
                                       p.obs_f32 ? p.obs_f32 + (int64_t)i * F : nullptr);
    }
    if (MODE == MODE_STEP && (tid & 63) == 0) s_ws[tid >> 6] = ws;
    __syncthreads();
  }

  DIAG(6);
  // ---- the block's statistics slot (thread 0 only; no other block touches it)
  if (MODE == MODE_STEP && p.stats && tid == 0) {
    WaveStats b = s_ws[0];
#pragma unroll
    for (int w = 1; w < BLOCK_THREADS / 64; ++w) {
      const WaveStats& o = s_ws[w];
      b.n += o.n; b.s1 += o.s1; b.s2 += o.s2; b.sl += o.sl; b.mn = fmin(b.mn, o.mn); b.mx = fmax(b.mx, o.mx);
    }
    if (b.n > 0.0) {
      double* slot = p.stats + (size_t)blockIdx.x * 8;
      slot[0] += b.n; slot[1] += b.s1; slot[2] += b.s2; slot[3] += b.sl;
      slot[4] = fmin(slot[4], b.mn); slot[5] = fmax(slot[5], b.mx);
    }
  }
}

// ------------------------------------------------------------------ two lanes per env
// step2_kernel<W, NS, ND>: the fixed-shape step of be_kernel<W, MODE_STEP, NS, ND>, bit for bit,
// with TWO lanes per env: lanes 2e and 2e+1 of a wave hold env e of the wave's 32.
//
// At 65 536 envs one lane per env is one wave per SIMD, and a lone wave issues at most one
// vector instruction every ~4 cycles (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost')
// while the SIMD could take one every 2: the step is bound by the length of each wave's
// instruction chain, not by HBM.  Two lanes per env give two waves per SIMD and split the
// per-obstacle work, so each wave's chain is shorter:
//  * lane h of an env takes obstacles k = 2j + h (dynamic: 3 slots, static: 7; the slot past
//    the count re-reads a real obstacle and is masked out), moves / tests / stores them and
//    keeps its own near list;
//  * the pair's collision flags and window rows are OR-ed with one DPP op each;
//  * a near entry's rows come from the wave's copy of the 64-bit span table (raster_rows_span:
//    a read, a shift and an OR per row; 6.18 against 6.39 us at 65 536 envs, 5.09 against 5.24 at
//    32 768 -- profiles/r05_step2_span_raster_ab.txt), so pick_kernel takes this kernel only while
//    W-1+2R <= 63 (R <= 27; the defaults' R is 25), the one-lane kernel past it;
//  * lane h writes its half of the obs row (uint2 words [7h, 7h+7)) into the wave's stage; both
//    lanes store every per-env scalar (the same value to the same address: one full-wave store per
//    array, 5.98 -> 5.90 us against splitting the arrays over the pair by per-lane pointer selects,
//    profiles/r05_step2_dup_stores_ab.txt);
//  * the Philox block, the agent move, the f64 reward and done run on both lanes (the same
//    instruction stream, so no extra issue).
// Autoreset is wave_resets with the even lanes as owners; stats fold per wave (32 envs =
// one be_stats_slots slot) in env order, as be_kernel's half-wave folds do.
// byte sel of x times k (24-bit), as one SDWA multiply: the compiler folds a byte select back into a
// shift and a mask, which costs two more VALU per obs word
__device__ __forceinline__ uint32_t mul24_byte(uint32_t x, uint32_t k, int sel) {
  uint32_t r;
  switch (sel) {
    case 0: asm("v_mul_u32_u24_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD" : "=v"(r) : "v"(x), "v"(k)); break;
    case 1: asm("v_mul_u32_u24_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "=v"(r) : "v"(x), "v"(k)); break;
    case 2: asm("v_mul_u32_u24_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD" : "=v"(r) : "v"(x), "v"(k)); break;
    default: asm("v_mul_u32_u24_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD" : "=v"(r) : "v"(x), "v"(k)); break;
  }
  return r;
}
__device__ __forceinline__ uint32_t pair_or(uint32_t x) {   // OR with the other lane of the pair
  return x | (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
}

template <int WT, int NSC, int NDC, bool POOL = false>
__global__ __launch_bounds__(S2_CT, 2) void step2_kernel(KParams p) {
  constexpr int CT = S2_CT;
  constexpr int L = 2, EPW = 64 / L, EPB = CT / L, NWAVE = CT / 64;
  constexpr int SS = (NSC + L - 1) / L, SD = (NDC + L - 1) / L;   // obstacle slots per lane
  constexpr int KR = Geo<WT>::K, F = Geo<WT>::F, NW = Geo<WT>::NW;
  constexpr int NQ = F / 8, HQ = (NQ + 1) / 2;                     // uint2 words per row / per lane
  static_assert(WT == 10 && F == 104 && NW == 5, "the half-row word split below is laid out for W = 10");
  static_assert(NDC <= 5, "one Philox block of 24-bit fields");
  static_assert(16 * KR >= (64 / (NSC + NDC)) * (KR + 4), "wave reset scratch");
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ __align__(16) TablesX t_wave[NWAVE];   // one copy of the tables per wave (no block barrier)
  __shared__ uint32_t s_rows[NWAVE][16 * KR];    // wave_resets scratch (row masks + stash)
  constexpr int TW = (int)(sizeof(TablesX) / 16);   // 16-byte table words

  DIAG(0);
  if (DBG(DBG_EXIT_ENTRY)) return;
  const int N = p.n, tid = (int)threadIdx.x, w = tid >> 6, lane = tid & 63, h = lane & 1;
  const int blk0 = (int)blockIdx.x * EPB, i = blk0 + (tid >> 1), e0 = blk0 + w * EPW;
  uint8_t* stage_blk = smem + (size_t)(SS + SD + 1) * CT * 4;   // [EPB envs][F]
  const bool valid = i < N;
  const uint32_t ic = (uint32_t)min(i, N - 1), gid = (uint32_t)p.gid0 + (uint32_t)i;
  NearList<CT> nl{reinterpret_cast<uint32_t*>(smem) + tid, 0};
  Tables& t = t_wave[w].t;
  const uint64_t* span = t_wave[w].span;
  uint8_t* stage = stage_blk + (size_t)w * EPW * F;   // the wave's 32 rows
  constexpr int TB = 64;     // each wave stages its own copy of the tables
  const int tt0 = lane;

  // ---- every load, straight-line, in use order (32-bit element offsets from uniform bases;
  //      obstacle k of lane h at element k*N + env: pick_kernel keeps NS*N < 2^30)
  constexpr int TL = (TW + TB - 1) / TB;   // table words per lane (each wave stages its own copy)
  uint4 tword[TL];
#pragma unroll
  for (int j = 0; j < TL; ++j)
    tword[j] = ld_s(reinterpret_cast<const uint4*>(p.tables), (uint32_t)min(tt0 + j * TB, TW - 1));
  const uint32_t episode = ld_s(p.episode, ic);
  const int len0 = ld_s(p.ep_len, ic);
  const int32_t agent0 = ld_s(p.agent, ic), goal0 = ld_s(p.goal, ic);
  int32_t dp[SD], so[SS];
  int dgi[SD];
#pragma unroll
  for (int j = 0; j < SD; ++j) {
    const uint32_t e = (uint32_t)min(L * j + h, NDC - 1) * (uint32_t)N + ic;
    dp[j] = ld_s(p.dyn_obs, e);
    dgi[j] = ld_s(p.dyn_goal, e);
  }
#pragma unroll
  for (int j = 0; j < SS; ++j) so[j] = ld_s(p.static_obs, (uint32_t)min(L * j + h, NSC - 1) * (uint32_t)N + ic);
  // state[2] of the last step (prev_read = 0: recomputed, it is calc_dist(goal, agent) -- see KParams).
  // (Read unconditionally with the select after a scheduling barrier, so that the action is issued
  // with the other loads instead of after the goal load lands: 5.26-5.27 against 5.22-5.24 us at
  // 32 768 envs, the same within noise at 65 536 -- profiles/r05_prologue_ab.txt, not kept here; it
  // is kept in the one-lane kernel, 8.05 against 8.13-8.15 us at 131 072)
  const double old_dist = p.prev_read ? ld_s(p.prev_dist, ic) : calc_dist(px(goal0), py(goal0), px(agent0), py(agent0));
  const double total = ld_s(p.total_dist, ic);
  double ret = ld_s(p.ep_return, ic);
  // the action last: the obstacle draws and moves below need no action, so a row that misses the
  // caches (a pre-sampled action tape) delays only the work that needs it (6.46 -> 6.37 us with
  // cache-resident rows, 6.92 -> 6.79 us with rows from HBM)
  const int a = ld_s(p.actions, ic);
  // the wave's stats slot (one per 32 envs), read now: a wave with a finished env updates it at
  // the very end, and a dependent load there would lengthen exactly the waves that reset
  double* const slot = p.stats ? p.stats + (size_t)(e0 / 32) * 8 : nullptr;
  double2 sp0 = make_double2(0.0, 0.0), sp1 = sp0, sp2 = sp0;
  if (slot && lane == 0 && e0 < N) {
    sp0 = reinterpret_cast<const double2*>(slot)[0];
    sp1 = reinterpret_cast<const double2*>(slot)[1];
    sp2 = reinterpret_cast<const double2*>(slot)[2];
  }
#pragma unroll
  for (int j = 0; j < TL; ++j) reinterpret_cast<uint4*>(&t_wave[w])[min(tt0 + j * TB, TW - 1)] = tword[j];
  // this wave's copy of the tables staged (state loads retire in order as used): a wave barrier, no
  // block barrier in the kernel -- 6.38-6.40 against 6.45-6.46 us with one block copy under a block
  // barrier (profiles/r04_step2_wave_tables_ab.txt; round 2 had measured the two the same)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  DIAG(1);
  if (DBG(DBG_EXIT_BARRIER)) return;
  if (DBG(DBG_WAIT_LOADS)) {   // diagnostics: when has every load of this wave landed?
    __builtin_amdgcn_s_waitcnt(0);
    DIAG(15);
  }

  // ---- this lane's dynamic obstacles: draws and moves first (no action needed; ballenv_env.py:323-353)
  int counter = (int)((double)len0 * p.inv_g1);   // counter == ep_len mod (G+1)
  counter = len0 - counter * (p.goal_change + 1);
  if (counter < 0) counter += p.goal_change + 1;
  if (counter > p.goal_change) counter -= p.goal_change + 1;
  const bool change = counter >= p.goal_change;
  const u4 b0 = DBG(DBG_NO_PHILOX) ? u4{gid, episode, (uint32_t)len0, gid ^ episode}   // (ablation: wrong draws)
                                   : philox(gid, episode, (uint32_t)len0, tag(PURPOSE_STEP_OBS, 0u), p.seed);
  DIAG(7);
  uint32_t st_flags = 0u;
  int ngs[SD];
  int32_t dnew[SD];
#pragma unroll
  for (int j = 0; j < SD; ++j) {
    const int k = L * j + h;
    const bool real = k < NDC;
    int ox = px(dp[j]), oy = py(dp[j]);
    const uint32_t f = h ? pick_field(b0, min(L * j + 1, 4)) : pick_field(b0, L * j);
    uint32_t fl = 0u;
    ngs[j] = dyn_move_fixed(p, t, ox, oy, dgi[j], t.speed[min(k, NDC - 1)], change, f, fl);
    st_flags |= real ? fl : 0u;
    dnew[j] = pk(ox, oy);
  }
  DIAG(11);
  // ---- action -> agent move + clamp (ballenv_env.py:247-259); unit moves and speeds
  st_flags |= a >= p.num_actions ? (uint32_t)BE_STATUS_BAD_ACTION : 0u;
  const uint32_t sh = 2u * (uint32_t)(a < p.num_actions ? a : 0);
  int ax = min(max(px(agent0) + (int)((p.amx >> sh) & 3u) - 1, 0), p.screen_w);
  int ay = min(max(py(agent0) + (int)((p.amy >> sh) & 3u) - 1, 0), p.screen_h);
  int gx = px(goal0), gy = py(goal0);
  const Win g0(p, 0, 0);
  const uint32_t R2 = (uint32_t)g0.R2;
  const NearBox nb0(g0);
  typedef unsigned short v2u __attribute__((ext_vector_type(2)));
  const v2s boxo = {(short)(WT / 2 + g0.R), (short)(WT / 2 + g0.R)};
  const v2u boxw = {(unsigned short)nb0.bw, (unsigned short)nb0.bh};
  const v2s agv = __builtin_bit_cast(v2s, pk(ax, ay));
  const double dist = calc_dist(gx, gy, ax, ay);
  // the distance and the distance term of the reward (ballenv_env.py:268-275) right after the
  // move: the f64 sqrt / divide chain then overlaps the obstacle tests
  const double rbase = (0.0 - p.time_penalty) + (old_dist - dist) / total;
  DIAG(8);
  // ---- collision + window-box tests (be_kernel's packed int16x2 form), near list
  bool hs = false, hd = false;
  // the near list's next free slot as an LDS address, advanced by sat(1 - over) slots: no compare /
  // select / carry chain (and its VCC hazard nops) per obstacle
  uint32_t* nlp = nl.base;
  auto obstacle_pk = [&](int32_t opk, bool real, bool& hit) {
    const v2s d = __builtin_elementwise_sub_sat(__builtin_bit_cast(v2s, opk), agv);
    hit |= real & ((uint32_t)dot2_sq(d) <= R2);
    const v2u b = __builtin_bit_cast(v2u, __builtin_elementwise_add_sat(d, boxo));
    const v2u over = __builtin_elementwise_sub_sat(b, boxw);   // (0, 0) iff inside the box
    *nlp = __builtin_bit_cast(uint32_t, d);
    // 1 iff inside the box (and a real slot): a saturating 1 - over, one VALU without VCC
    const uint32_t in = __builtin_elementwise_sub_sat(1u, __builtin_bit_cast(uint32_t, over) | (real ? 0u : 1u));
    nlp += CT * in;
  };
#pragma unroll
  for (int j = 0; j < SD; ++j) obstacle_pk(dnew[j], L * j + h < NDC, hd);
#pragma unroll
  for (int j = 0; j < SS; ++j) obstacle_pk(so[j], L * j + h < NSC, hs);
  nl.cnt = (int)(lds_bytes(nl.base, nlp) / (CT * 4u));
  hs = pair_or((uint32_t)hs) != 0u;
  hd = pair_or((uint32_t)hd) != 0u;
  DIAG(10);

  // ---- distance, reward, done (ballenv_env.py:268-286, 200-229), on both lanes
  double reward = rbase;
  if (hs) reward -= p.static_penalty;          // statics come first in obstacle_list (Q3)
  else if (hd) reward -= p.dynamic_penalty;
  ret += reward;
  const int len = len0 + 1;
  const bool env_done = (dist < p.threshold_goal) || hs || hd;
  const bool trunc = p.time_limit > 0 && len >= p.time_limit;
  const bool done = env_done || trunc;
  const bool do_reset = valid && done && p.autoreset;
  // ---- a finished env's next episode from the autoreset pool: its tag and its 112-byte body (both
  //      lanes, the same addresses) are loaded here and land while the wave stores the physics
  // (POOL instances are launched only with KParams::pool set; testing the pointer as well measured
  // faster -- the compiler schedules the kernel around the branch differently: 5.65-5.71 against
  // 5.81-5.85 us at 65 536 envs, 4.58-4.59 against 4.78-4.79 at 32 768, profiles/r06_pool_ab.txt)
  const bool ptry = POOL && do_reset && p.pool != nullptr;
  uint2 q_tv = make_uint2(0u, 0u);
  uint4 qb[7];
#if BE_POOL_MODE == 1 || BE_POOL_MODE == 6
  if constexpr (POOL)
#if BE_POOL_MODE == 6   // (A/B) a uniform scalar branch around the divergent one
  if (__ballot(ptry))
#endif
  if (ptry) {
    const uint32_t x = ((episode + 1u) & 1u) * (uint32_t)N + (uint32_t)i;
    q_tv = pool_ld<uint2>(p.pool, x * 8u);
    const uint32_t bo = pool_body((uint32_t)N, x, 28);
#pragma unroll
    for (int j = 0; j < 7; ++j) qb[j] = pool_ld<uint4>(p.pool, bo, 16u * j);
    __builtin_amdgcn_s_waitcnt(0);   // here, in the branch: no pending pool load past its end
  }
#ifdef BE_DIAG_STAMPS
  if (__ballot(ptry)) DIAG(9);   // (stamps build: this wave's entries landed)
#endif
#endif
  if (valid) {   // both lanes of the pair store the env's scalars (the same value to the same address:
                 // one full-wave store per array, no per-lane pointer selects or exec masking)
    const uint32_t iu = (uint32_t)i;
    st_ws(p.reward, iu, reward);
    st_ws(p.ep_return, iu, ret);
    st_ws(p.agent, iu, pk(ax, ay));
    st_ws(p.ep_len, iu, len);
    if (p.done) st_ws(p.done, iu, (uint8_t)done);
    if (p.truncated) st_ws(p.truncated, iu, (uint8_t)(trunc && !env_done));
    st_ws(p.prev_dist, iu, dist);
    if (done) {
      if (p.final_return) st_ws(p.final_return, iu, ret);
      if (p.final_len) st_ws(p.final_len, iu, len);
    }
    // (stored after done is known: measured faster than storing inside the obstacle loop)
#pragma unroll
    for (int j = 0; j < SD; ++j) {
      const int k = L * j + h;
      if (k < NDC) {
        st_wt(&ld_s_ptr(p.dyn_obs, (uint32_t)k * (uint32_t)N + (uint32_t)i), dnew[j]);
        if (change) st_wt(&ld_s_ptr(p.dyn_goal, (uint32_t)k * (uint32_t)N + (uint32_t)i), (uint8_t)ngs[j]);
      }
    }
  }
  DIAG(2);
  if (__ballot(st_flags != 0u)) {   // rare: OR the wave's flags, one atomic
    uint32_t f = st_flags;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) f |= (uint32_t)__shfl_xor((int)f, o);
    if (lane == 0) atomicOr(p.status, (int)f);
  }
  if (DBG(DBG_EXIT_PHYSICS)) return;

  // ---- episode boundary: terminal obs, then the reset of the finished envs
  uint32_t xrows[KR];
#pragma unroll
  for (int k = 0; k < KR; ++k) xrows[k] = 0u;
  if (do_reset && p.terminal_obs) {   // both lanes of the pair take this branch together
    uint32_t rows[KR], flat[NW];
    raster_rows_span<WT, CT>(nl, p.R, rows, span);
#pragma unroll
    for (int k = 0; k < KR; ++k) rows[k] = pair_or(rows[k]);
    flatten<WT>(rows, flat);
    if (!h) write_row_global<WT>(p.terminal_obs + (int64_t)i * F, flat, quadrant(ax, ay, gx, gy));
  }
  // a pool entry for the new episode (e + 1) that was written and is still current: copy it.  Only
  // the waves with a finished env take this (uniform) branch, so no other wave waits for the loads
  // above -- every use of a loaded value is inside it
  bool hit = false;
#if BE_POOL_MODE == 5
  const unsigned long long m0 = DBG(DBG_NO_RESET) ? 0ull : __ballot(do_reset && h == 0);
  if (m0) {   // (uniform) the waves with a finished env
  if (POOL) {
    if (ptry) {
      const uint32_t x = ((episode + 1u) & 1u) * (uint32_t)N + (uint32_t)i;
      q_tv = pool_ld<uint2>(p.pool, x * 8u);
      const uint32_t bo = pool_body((uint32_t)N, x, 28);
#pragma unroll
      for (int j = 0; j < 7; ++j) qb[j] = pool_ld<uint4>(p.pool, bo, 16u * j);
    }
#else
  if (__ballot(ptry)) {
#endif
    hit = ptry && q_tv.x == episode + 1u && (q_tv.y & POOL_VALID) != 0u;
    if (hit) {   // both lanes store the env's scalars (as the physics did) and their own obstacle slots
      auto qw = [&](int k) -> uint32_t { return u4w(qb[k >> 2], k & 3); };   // body word k (compile-time k)
      const uint32_t iu = (uint32_t)i;
      const int32_t ag = (int32_t)qw(PB_AGENT), go = (int32_t)qw(PB_GOAL);
      st_ws(p.ep_return, iu, 0.0);
      st_ws(p.ep_len, iu, 0);
      st_ws(p.agent, iu, ag);
      st_ws(p.prev_dist, iu, u2d(qw(PB_PREV), qw(PB_PREV + 1)));
      st_ws(p.goal, iu, go);
      st_ws(p.total_dist, iu, u2d(qw(PB_TOTAL), qw(PB_TOTAL + 1)));
      st_ws(p.episode, iu, episode + 1u);
#pragma unroll
      for (int j = 0; j < SD; ++j) {
        const int k = L * j + h;
        const uint32_t o = h ? qw(PB_OBS + NSC + min(L * j + 1, NDC - 1)) : qw(PB_OBS + NSC + L * j);
        if (k < NDC) {
          st_ws(p.dyn_obs, (uint32_t)k * (uint32_t)N + iu, (int32_t)o);
          st_ws(p.dyn_goal, (uint32_t)k * (uint32_t)N + iu, (uint8_t)k);
        }
      }
#pragma unroll
      for (int j = 0; j < SS; ++j) {
        const int k = L * j + h;
        const uint32_t o = h ? qw(PB_OBS + min(L * j + 1, NSC - 1)) : qw(PB_OBS + L * j);
        if (k < NSC) st_ws(p.static_obs, (uint32_t)k * (uint32_t)N + iu, (int32_t)o);
      }
      ax = px(ag); ay = py(ag); gx = px(go); gy = py(go);
#pragma unroll
      for (int k = 0; k < KR; ++k) xrows[k] = (qw(PB_ROWS + k / 3) >> (10 * (k % 3))) & 0x3FFu;   // three rows per word
      nl.cnt = 0;
    }
    if (__ballot(hit && (q_tv.y & POOL_REJ)) && lane == 0) atomicOr(p.status, BE_STATUS_REJECTION_LIMIT);
  }
  const unsigned long long m = DBG(DBG_NO_RESET) ? 0ull : __ballot(do_reset && !hit && h == 0);
  if (m) {   // stale entries (or no pool): wave-cooperative, this wave runs its own resets
    auto osink = [&](int, int k, int il, int32_t o) {   // (32-bit element offsets: pick_kernel keeps NS*N < 2^30)
      if (k < NSC) {
        st_ws(p.static_obs, (uint32_t)k * (uint32_t)N + (uint32_t)il, o);
      } else {
        st_ws(p.dyn_obs, (uint32_t)(k - NSC) * (uint32_t)N + (uint32_t)il, o);
        st_ws(p.dyn_goal, (uint32_t)(k - NSC) * (uint32_t)N + (uint32_t)il, (uint8_t)(k - NSC));
      }
    };
    auto esink = [&](int, int32_t ag, int32_t go, int32_t a0) {
      // both lanes take the new agent / goal / rows and store the env's scalars, as in the physics
      // above.  Ordering against the physics stores is the wave's program order (wave_resets' note)
      double prev;
      const double td = reset_dists(ag, go, a0, prev);
      const uint32_t iu = (uint32_t)i;
      st_ws(p.ep_return, iu, 0.0);
      st_ws(p.ep_len, iu, 0);
      st_ws(p.agent, iu, ag);
      st_ws(p.prev_dist, iu, prev);
      st_ws(p.goal, iu, go);
      st_ws(p.total_dist, iu, td);
      st_ws(p.episode, iu, episode + 1u);
    };
    if (!(m & (m - 1)))
      wave_resets<WT, NSC, NDC, 1, decltype(osink)&, decltype(esink)&, L>(p, t, m, i, gid, episode, ax, ay, gx, gy,
                                                                        nl.cnt, xrows, &s_rows[w][0], osink, esink, span);
    else
      wave_resets<WT, NSC, NDC, 64, decltype(osink)&, decltype(esink)&, L>(p, t, m, i, gid, episode, ax, ay, gx, gy,
                                                                         nl.cnt, xrows, &s_rows[w][0], osink, esink, span);
  }
#if BE_POOL_MODE == 5
  }
#endif
  DIAG(3);
  if (DBG(DBG_NO_OBS)) return;
  if (DBG(DBG_NO_RASTER)) nl.cnt = 0;

  // ---- observation (prep_state4): own near list -> rows, OR-ed over the pair, half a row each
  {
    uint32_t rows[KR];
    raster_rows_span<WT, CT>(nl, p.R, rows, span, xrows);   // from a reset env's new rows (else 0)
    // three 10-bit rows per word, OR-ed over the pair (3 DPP ops); then this lane's cells from its
    // first nibble: lane 0 cells -4.. (its word 0 is the quadrant one-hot), lane 1 cells 52..  Window
    // row r is distinct row max(r-1, 0) (quirk Q1): V = sum_r R_r << (10 r + 4) over the lane's six
    // window rows (lane 0: 0-5; lane 1: 5-9), c = V >> 6h, from the packed words directly.
    const uint32_t P0 = pair_or(rows[0] | (rows[1] << 10) | (rows[2] << 20));
    const uint32_t P1 = pair_or(rows[3] | (rows[4] << 10) | (rows[5] << 20));
    const uint32_t P2 = pair_or(rows[6] | (rows[7] << 10) | (rows[8] << 20));
    const uint32_t vlo = h ? ((P1 >> 6) & 0xFFFFF0u) | (P2 << 24) : ((P0 << 4) & 0x3FF0u) | (P0 << 14);
    const uint32_t vhi = h ? P2 >> 8 : (P0 >> 18) | (P1 << 12);
    const unsigned long long c = (((unsigned long long)vhi << 32) | vlo) >> (6 * h);
    // nibble jj of c is byte jj/2 of the even- / odd-nibble masks: one byte-select multiply and an AND
    const uint32_t clo = (uint32_t)c, chi = (uint32_t)(c >> 32);
    const uint32_t ne0 = clo & 0x0F0F0F0Fu, no0 = (clo >> 4) & 0x0F0F0F0Fu;
    const uint32_t ne1 = chi & 0x0F0F0F0Fu, no1 = (chi >> 4) & 0x0F0F0F0Fu;
    const uint32_t kx = 0x00204081u;
    auto word = [&](int jj) -> uint32_t {   // jj: this lane's word 0 .. 2*HQ-1
      const int b = jj >> 1;
      const uint32_t src = (jj & 1) ? (b < 4 ? no0 : no1) : (b < 4 ? ne0 : ne1);
      return mul24_byte(src, kx, b & 3) & 0x01010101u;
    };
    // quadrant(ax, ay, gx, gy) one-hot: byte 2 sy + (1 ^ sx ^ sy), s = the sign of goal - agent
    const uint32_t sx = (uint32_t)(gx - ax) >> 31, sy = (uint32_t)(gy - ay) >> 31;
    const uint32_t onehot = 1u << ((sy << 4) | ((sx ^ sy ^ 1u) << 3));
    uint2* dst = reinterpret_cast<uint2*>(stage + (tid & 62) / 2 * F) + HQ * h;
#pragma unroll
    for (int q = 0; q < HQ; ++q) {
      const uint32_t w0 = q == 0 ? (h ? word(0) : onehot) : word(2 * q);
      if (q < NQ - HQ || !h) dst[q] = make_uint2(w0, word(2 * q + 1));
    }
  }
  DIAG(4);
  // the wave's contiguous rows out (no block barrier: a wave that reset delays nobody)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  DIAG(5);
  if (!DBG(DBG_NO_COPY)) {
    const int e0u = __builtin_amdgcn_readfirstlane(e0);
    if (e0u + EPW <= N && p.obs && !p.obs_f32)   // the common case: a full wave, u8 obs only
      copy_wave_full<EPW * F / 16>(stage, p.obs + (size_t)e0u * F, lane);
    else
      copy_out<64>(stage, F, max(0, min(EPW, N - e0u)), (int64_t)e0u, p.obs, p.obs_f32, lane);
  }
  // the episode statistics fold after the obs stores are issued: off the path to the last store
  // (6.55 -> 6.45 us; a reset leaves this lane's ret / len registers as the finished episode's)
  WaveStats ws{0.0, 0.0, 0.0, 0.0, INFINITY, -INFINITY};
  if (slot && !DBG(DBG_NO_STATS)) ws = wave_stats(done && valid && h == 0, ret, len);   // even lanes: env order
  if (slot && lane == 0 && ws.n > 0.0) {
    reinterpret_cast<double2*>(slot)[0] = make_double2(sp0.x + ws.n, sp0.y + ws.s1);
    reinterpret_cast<double2*>(slot)[1] = make_double2(sp1.x + ws.s2, sp1.y + ws.sl);
    reinterpret_cast<double2*>(slot)[2] = make_double2(fmin(sp2.x, ws.mn), fmax(sp2.y, ws.mx));
  }
  DIAG(6);
}

// ------------------------------------------------------------------ small batches at W = 5
// stepw_kernel<5, NS, ND, L>: the fixed-shape step of be_kernel<5, MODE_STEP, NS, ND>, bit for
// bit, with L (4 or 8) lanes per env, for BASELINE config 2 (4 096 envs, W=5).  With one lane
// per env 4 096 envs are 16 blocks: 64 waves on a 1 024-SIMD chip, each wave running the whole
// per-env chain for 64 envs.  Here a block is 32 envs (one be_stats_slots slot) on 32 L lanes:
//  * lane h of an env takes obstacles k = L j + h (at L = 8: one dynamic and two static slots,
//    the slot past the count re-reads a real obstacle and is masked out), moves, tests and
//    stores them, and rasterises the ones that can light a cell straight into a packed row
//    word (W = 5: the 4 distinct rows of quirk Q1 are 20 bits, row k at bits 5k..5k+4);
//  * the group ORs its rows and both collision flags as one word (log2 L DPP ops);
//  * the Philox block, the agent move, the f64 distance / reward and done run on every lane of
//    the group (the same instruction stream: no extra issue), the per-env scalar stores are
//    spread over the group's lanes;
//  * lane h writes bytes [4h, 4h+4) (L = 8) or [8h, 8h+8) (L = 4) of its env's obs row into the
//    wave's LDS stage, and the wave copies its 64/L rows (a contiguous 232 / 464 B) out;
//  * autoreset is wave_resets (the owner is the group's lane 0), as in step2_kernel;
//  * the block's 32 envs share one stats slot: every wave leaves its finished envs' return and
//    length in LDS after the physics, and after a block barrier at the very end (behind every
//    wave's obs stores: 4.01 against 4.03 us with the barrier right after the physics,
//    profiles/r04_stepw_late_fold_ab.txt) wave 0 folds them in env order -- the same sums, in
//    the same order, as the one-lane kernel.
template <int L>
__device__ __forceinline__ uint32_t lane_group_or(uint32_t x) {   // OR over the aligned group of L lanes
  static_assert(L == 4 || L == 8, "L must be 4 or 8");
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);     // quad_perm 1,0,3,2
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);     // quad_perm 2,3,0,1
  if constexpr (L == 8) x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
  return x;
}

template <int WT, int NSC, int NDC, int L, bool POOL = false>
__global__ __launch_bounds__(32 * L) void stepw_kernel(KParams p) {
  constexpr int CT = 32 * L, EPW = 64 / L, NWAVE = CT / 64;
  constexpr int SS = (NSC + L - 1) / L, SD = (NDC + L - 1) / L;   // obstacle slots per lane
  constexpr int KR = Geo<WT>::K, F = Geo<WT>::F;
  constexpr int BPL = (F + L - 1) / L;                             // obs bytes per lane
  constexpr int WB = EPW * F, SW = (WB + 15) & ~15;                // a wave's obs bytes, its stage stride
  static_assert(WT * KR <= 20, "packed rows: 20 bits + the two collision flags");
  static_assert(NDC <= 5, "one Philox block of 24-bit fields");
  static_assert(16 * KR >= (64 / (NSC + NDC)) * (KR + 4), "wave reset scratch");
  static_assert(WB % 8 == 0, "a wave's rows are whole 8-byte words");
  // one copy of the tables per wave, staged under a wave barrier: no block barrier at the start
  // (3.97 against 4.01 us with one block copy, profiles/r04_stepw_wave_tables_ab.txt)
  __shared__ Tables t_wave[NWAVE];
  __shared__ uint32_t s_rows[NWAVE][16 * KR];      // wave_resets scratch (row masks + stash)
  __shared__ __align__(16) uint8_t s_stage[NWAVE][SW];
  __shared__ double s_fret[32];
  __shared__ int32_t s_flen[32];
  __shared__ uint8_t s_fin[32];
  constexpr int TW = (int)(sizeof(Tables) / 4);

  if (DBG(DBG_EXIT_ENTRY)) return;
  PH_INIT;
  const int N = p.n, tid = (int)threadIdx.x, w = tid >> 6, lane = tid & 63, h = lane & (L - 1);
  const int el = tid / L, blk0 = (int)blockIdx.x * 32, i = blk0 + el, e0 = blk0 + w * EPW;
  const bool valid = i < N;
  const uint32_t ic = (uint32_t)min(i, N - 1), gid = (uint32_t)p.gid0 + (uint32_t)i;
  uint8_t* stage = &s_stage[w][0];
  Tables& t = t_wave[w];

  // ---- every load, straight-line, in use order (as step2_kernel)
  constexpr int TL = (TW + 63) / 64;   // table words per lane
  uint32_t tword[TL];
#pragma unroll
  for (int j = 0; j < TL; ++j)
    tword[j] = ld_s(reinterpret_cast<const uint32_t*>(p.tables), (uint32_t)min(lane + j * 64, TW - 1));
  const uint32_t episode = ld_s(p.episode, ic);
  const int len0 = ld_s(p.ep_len, ic);
  const int32_t agent0 = ld_s(p.agent, ic), goal0 = ld_s(p.goal, ic);
  int32_t dp[SD], so[SS];
  int dgi[SD];
  // (the slot offsets k * N are kept apart from + ic: fused into one v_mad_u64_u32, whose 64-bit
  // addend pair took a pending load's register as its high half, the compiler waited for the first
  // loads before issuing these -- a second memory latency in the prologue)
#pragma unroll
  for (int j = 0; j < SD; ++j) {
    uint32_t kn = (uint32_t)min(L * j + h, NDC - 1) * (uint32_t)N;
    asm volatile("" : "+v"(kn));
    const uint32_t e = kn + ic;
    dp[j] = ld_s(p.dyn_obs, e);
    dgi[j] = ld_s(p.dyn_goal, e);
  }
#pragma unroll
  for (int j = 0; j < SS; ++j) {
    uint32_t kn = (uint32_t)min(L * j + h, NSC - 1) * (uint32_t)N;
    asm volatile("" : "+v"(kn));
    so[j] = ld_s(p.static_obs, kn + ic);
  }
  const double old_read = ld_s(p.prev_dist, ic);   // (read even when unused: no branch among the loads)
  const double total = ld_s(p.total_dist, ic);
  double ret = ld_s(p.ep_return, ic);
  const int a = ld_s(p.actions, ic);
  __builtin_amdgcn_sched_barrier(0);   // every load above is issued before any of them is used
  const double old_dist = p.prev_read ? old_read : calc_dist(px(goal0), py(goal0), px(agent0), py(agent0));
  double* const slot = p.stats ? p.stats + (size_t)blockIdx.x * 8 : nullptr;
  double2 sp0 = make_double2(0.0, 0.0), sp1 = sp0, sp2 = sp0;
  if (slot && tid == 0) {   // the block's stats slot, read now (wave 0 folds into it)
    sp0 = reinterpret_cast<const double2*>(slot)[0];
    sp1 = reinterpret_cast<const double2*>(slot)[1];
    sp2 = reinterpret_cast<const double2*>(slot)[2];
  }
#pragma unroll
  for (int j = 0; j < TL; ++j) reinterpret_cast<uint32_t*>(&t)[min(lane + j * 64, TW - 1)] = tword[j];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // this wave's copy staged
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (DBG(DBG_EXIT_BARRIER)) {   // diagnostics: the loads issued, nothing else
    if (valid && (agent0 ^ goal0 ^ so[0] ^ dp[0] ^ len0 ^ a ^ (int)old_dist ^ (int)ret) == 0x7fffffff) p.obs[i] = 1;
    return;
  }
  if (DBG(DBG_WAIT_LOADS)) __builtin_amdgcn_s_waitcnt(0);
  PH(0);

  // ---- this lane's dynamic obstacles (ballenv_env.py:323-353): draws and moves need no action
  int counter = (int)((double)len0 * p.inv_g1);   // counter == ep_len mod (G+1)
  counter = len0 - counter * (p.goal_change + 1);
  if (counter < 0) counter += p.goal_change + 1;
  if (counter > p.goal_change) counter -= p.goal_change + 1;
  const bool change = counter >= p.goal_change;
  const u4 b0 = DBG(DBG_NO_PHILOX) ? u4{gid, episode, 7u, 9u} : philox(gid, episode, (uint32_t)len0, tag(PURPOSE_STEP_OBS, 0u), p.seed);
  uint32_t st_flags = 0u;
  int ngs[SD];
  int32_t dnew[SD];
#pragma unroll
  for (int j = 0; j < SD; ++j) {
    const int k = L * j + h;
    int ox = px(dp[j]), oy = py(dp[j]);
    uint32_t fl = 0u;
    ngs[j] = dyn_move_fixed(p, t, ox, oy, dgi[j], t.speed[min(k, NDC - 1)], change, pick_field(b0, min(k, 4)), fl);
    st_flags |= k < NDC ? fl : 0u;
    dnew[j] = pk(ox, oy);
  }
  PH(1);
  // ---- action -> agent move + clamp (ballenv_env.py:247-259); unit moves and speeds
  st_flags |= a >= p.num_actions ? (uint32_t)BE_STATUS_BAD_ACTION : 0u;
  const uint32_t sh = 2u * (uint32_t)(a < p.num_actions ? a : 0);
  int ax = min(max(px(agent0) + (int)((p.amx >> sh) & 3u) - 1, 0), p.screen_w);
  int ay = min(max(py(agent0) + (int)((p.amy >> sh) & 3u) - 1, 0), p.screen_h);
  int gx = px(goal0), gy = py(goal0);
  const int R = p.R;
  const uint32_t R2 = (uint32_t)(R * R);
  const v2s agv = __builtin_bit_cast(v2s, pk(ax, ay));
  const double dist = calc_dist(gx, gy, ax, ay);
  const double rbase = (0.0 - p.time_penalty) + (old_dist - dist) / total;
  PH(2);

  // ---- collision test, and the row masks of the obstacles that can light a cell
  //      (prep_state4 with quirk Q1, ball_cnn_ac3.py:384-412: row k is y offset k - W/2)
  uint32_t word = 0u;   // rows (20 bits) | static hit << 20 | dynamic hit << 21
  auto obstacle = [&](int32_t opk, bool real, uint32_t hit_bit) {
    const v2s d = __builtin_elementwise_sub_sat(__builtin_bit_cast(v2s, opk), agv);
    word |= (real & ((uint32_t)__builtin_amdgcn_sdot2(d, d, 0, false) <= R2)) ? hit_bit : 0u;
    const int f = d.x + WT / 2, e = d.y + WT / 2;   // window column / distinct-row coordinates
    if (real & ((uint32_t)(f + R) <= (uint32_t)(WT - 1 + 2 * R)) & ((uint32_t)(e + R) <= (uint32_t)(KR - 1 + 2 * R))) {
#pragma unroll
      for (int k = 0; k < KR; ++k) {
        const int ady = abs(e - k);
        const int hw = t.hw[min(ady, HW_MAX)];
        const int lo = max(f - hw, 0), hi = min(f + hw, WT - 1);
        word |= (ady <= R && lo <= hi) ? ((2u << hi) - (1u << lo)) << (WT * k) : 0u;
      }
    }
  };
#pragma unroll
  for (int j = 0; j < SD; ++j) obstacle(dnew[j], L * j + h < NDC, 1u << 21);
#pragma unroll
  for (int j = 0; j < SS; ++j) obstacle(so[j], L * j + h < NSC, 1u << 20);
  word = lane_group_or<L>(word);
  const bool hs = (word >> 20) & 1u, hd = (word >> 21) & 1u;
  uint32_t rows = word & 0xFFFFFu;
  PH(3);

  // ---- reward, done (ballenv_env.py:268-286, 200-229), on every lane of the group
  double reward = rbase;
  if (hs) reward -= p.static_penalty;          // statics come first in obstacle_list (Q3)
  else if (hd) reward -= p.dynamic_penalty;
  ret += reward;
  const int len = len0 + 1;
  const bool env_done = (dist < p.threshold_goal) || hs || hd;
  const bool trunc = p.time_limit > 0 && len >= p.time_limit;
  const bool done = env_done || trunc;
  const bool do_reset = valid && done && p.autoreset;
  // ---- a finished env's next episode from the autoreset pool, loads issued now (as step2_kernel):
  //      lane h loads the tag, the body's rows / agent / goal / distances and its own obstacle slots
  // (POOL instances are launched only with KParams::pool set; testing the pointer as well measured
  // faster -- the compiler schedules the kernel around the branch differently: 5.65-5.71 against
  // 5.81-5.85 us at 65 536 envs, 4.58-4.59 against 4.78-4.79 at 32 768, profiles/r06_pool_ab.txt)
  const bool ptry = POOL && do_reset && p.pool != nullptr;
  uint2 q_tv = make_uint2(0u, 0u);
  uint4 q0, q1;
  uint2 q2;
  uint32_t q_dp[SD], q_so[SS];
#if BE_POOL_MODE == 1
  if constexpr (POOL) if (ptry) {
    const uint32_t x = ((episode + 1u) & 1u) * (uint32_t)N + (uint32_t)i;
    q_tv = pool_ld<uint2>(p.pool, x * 8u);
    const uint32_t bo = pool_body((uint32_t)N, x, 28);
    q0 = pool_ld<uint4>(p.pool, bo, 0u);     // rows, -, -, agent
    q1 = pool_ld<uint4>(p.pool, bo, 16u);    // goal, -, prev
    q2 = pool_ld<uint2>(p.pool, bo, 32u);    // total
#pragma unroll
    for (int j = 0; j < SD; ++j) q_dp[j] = pool_ld<uint32_t>(p.pool, bo + 4u * (uint32_t)min(L * j + h, NDC - 1), 4u * (PB_OBS + NSC));
#pragma unroll
    for (int j = 0; j < SS; ++j) q_so[j] = pool_ld<uint32_t>(p.pool, bo + 4u * (uint32_t)min(L * j + h, NSC - 1), 4u * PB_OBS);
    __builtin_amdgcn_s_waitcnt(0);   // here, in the branch: no pending pool load past its end
  }
#endif
  if (valid) {   // the per-env scalars: one full-wave store per array
    const uint32_t iu = (uint32_t)i;   // every lane of the group: the same value to the same address
    st_ws(p.reward, iu, reward);
    st_ws(p.ep_return, iu, ret);
    st_ws(p.prev_dist, iu, dist);
    st_ws(p.agent, iu, pk(ax, ay));
    st_ws(p.ep_len, iu, len);
    if (p.done) st_ws(p.done, iu, (uint8_t)done);
    if (p.truncated) st_ws(p.truncated, iu, (uint8_t)(trunc && !env_done));
    if (done) {
      if (p.final_return) st_ws(p.final_return, iu, ret);
      if (p.final_len) st_ws(p.final_len, iu, len);
    }
#pragma unroll
    for (int j = 0; j < SD; ++j) {
      const int k = L * j + h;
      if (k < NDC) {
        st_wt(&ld_s_ptr(p.dyn_obs, (uint32_t)k * (uint32_t)N + (uint32_t)i), dnew[j]);
        if (change) st_wt(&ld_s_ptr(p.dyn_goal, (uint32_t)k * (uint32_t)N + (uint32_t)i), (uint8_t)ngs[j]);
      }
    }
  }
  if (__ballot(st_flags != 0u)) {   // rare: OR the wave's flags, one atomic
    uint32_t f = st_flags;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) f |= (uint32_t)__shfl_xor((int)f, o);
    if (lane == 0) atomicOr(p.status, (int)f);
  }
  // ---- the block's stats slot (32 envs): every wave leaves its finished envs' return / length in
  //      LDS right after the physics (before a reset overwrites ret / len); the fold is at the end
  if (slot && !DBG(DBG_NO_STATS)) {
    const bool fin = done && valid;   // (the same on every lane of the group: they all write it)
    s_fin[el] = fin ? 1 : 0;
    if (fin && h == 0) { s_fret[el] = ret; s_flen[el] = len; }
  }
  PH(4);
  if (DBG(DBG_EXIT_PHYSICS)) return;

  // ---- episode boundary: terminal obs, then the wave's resets
  if (do_reset && p.terminal_obs && h == 0) {
    const uint32_t fl[Geo<WT>::NW] = {(rows & ((1u << WT) - 1u)) | (rows << WT), 0u};
    write_row_global<WT>(p.terminal_obs + (int64_t)i * F, fl, quadrant(ax, ay, gx, gy));
  }
  // a pool entry for episode e + 1 that was written and is still current: copy it (a uniform branch:
  // no wave without a finished env waits for the pool loads; every use of a loaded value is inside)
  bool hit = false;
  if (__ballot(ptry)) {
#if BE_POOL_MODE == 5
    if (ptry) {
      const uint32_t x = ((episode + 1u) & 1u) * (uint32_t)N + (uint32_t)i;
      q_tv = pool_ld<uint2>(p.pool, x * 8u);
      const uint32_t bo = pool_body((uint32_t)N, x, 28);
      q0 = pool_ld<uint4>(p.pool, bo, 0u);
      q1 = pool_ld<uint4>(p.pool, bo, 16u);
      q2 = pool_ld<uint2>(p.pool, bo, 32u);
#pragma unroll
      for (int j = 0; j < SD; ++j) q_dp[j] = pool_ld<uint32_t>(p.pool, bo + 4u * (uint32_t)min(L * j + h, NDC - 1), 4u * (PB_OBS + NSC));
#pragma unroll
      for (int j = 0; j < SS; ++j) q_so[j] = pool_ld<uint32_t>(p.pool, bo + 4u * (uint32_t)min(L * j + h, NSC - 1), 4u * PB_OBS);
    }
#endif
    hit = ptry && q_tv.x == episode + 1u && (q_tv.y & POOL_VALID) != 0u;
    if (hit) {   // every lane of the group stores the scalars (as the physics did) and its own slots
      const uint32_t iu = (uint32_t)i;
      const int32_t q_ag = (int32_t)q0.w, q_go = (int32_t)q1.x;
      st_ws(p.agent, iu, q_ag);
      st_ws(p.goal, iu, q_go);
      st_ws(p.total_dist, iu, u2d(q2.x, q2.y));
      st_ws(p.episode, iu, episode + 1u);
      st_ws(p.ep_return, iu, 0.0);
      st_ws(p.ep_len, iu, 0);
      st_ws(p.prev_dist, iu, u2d(q1.z, q1.w));
#pragma unroll
      for (int j = 0; j < SD; ++j) {
        const int k = L * j + h;
        if (k < NDC) {
          st_ws(p.dyn_obs, (uint32_t)k * (uint32_t)N + iu, (int32_t)q_dp[j]);
          st_ws(p.dyn_goal, (uint32_t)k * (uint32_t)N + iu, (uint8_t)k);
        }
      }
#pragma unroll
      for (int j = 0; j < SS; ++j) {
        const int k = L * j + h;
        if (k < NSC) st_ws(p.static_obs, (uint32_t)k * (uint32_t)N + iu, (int32_t)q_so[j]);
      }
      ax = px(q_ag); ay = py(q_ag); gx = px(q_go); gy = py(q_go);
      rows = q0.x & 0xFFFFFu;
    }
    if (__ballot(hit && (q_tv.y & POOL_REJ)) && lane == 0) atomicOr(p.status, BE_STATUS_REJECTION_LIMIT);
  }
  const unsigned long long m = DBG(DBG_NO_RESET) ? 0ull : __ballot(do_reset && !hit && h == 0);
  if (m) {   // stale entries (or no pool): the wave's inline resets
    uint32_t xrows[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) xrows[k] = 0u;
    int kept = 1;   // wave_resets zeroes it for the lanes of a reset env
    auto osink = [&](int, int k, int il, int32_t o) {   // (32-bit element offsets: NS*N < 2^30 here)
      if (k < NSC) {
        st_ws(p.static_obs, (uint32_t)k * (uint32_t)N + (uint32_t)il, o);
      } else {
        st_ws(p.dyn_obs, (uint32_t)(k - NSC) * (uint32_t)N + (uint32_t)il, o);
        st_ws(p.dyn_goal, (uint32_t)(k - NSC) * (uint32_t)N + (uint32_t)il, (uint8_t)(k - NSC));
      }
    };
    auto esink = [&](int, int32_t ag, int32_t go, int32_t a0) {
      // every lane of the group takes the new agent / goal / rows and stores the env's scalars, as
      // in the physics above.  Ordering against the physics stores is the wave's program order
      // (wave_resets' note)
      double prev;
      const double td = reset_dists(ag, go, a0, prev);
      const uint32_t iu = (uint32_t)i;
      st_ws(p.agent, iu, ag);
      st_ws(p.goal, iu, go);
      st_ws(p.total_dist, iu, td);
      st_ws(p.episode, iu, episode + 1u);
      st_ws(p.ep_return, iu, 0.0);
      st_ws(p.ep_len, iu, 0);
      st_ws(p.prev_dist, iu, prev);
    };
    if (!(m & (m - 1)))
      wave_resets<WT, NSC, NDC, 1, decltype(osink)&, decltype(esink)&, L>(p, t, m, i, gid, episode, ax, ay, gx, gy,
                                                                        kept, xrows, &s_rows[w][0], osink, esink);
    else
      wave_resets<WT, NSC, NDC, 64, decltype(osink)&, decltype(esink)&, L>(p, t, m, i, gid, episode, ax, ay, gx, gy,
                                                                         kept, xrows, &s_rows[w][0], osink, esink);
    if (!kept) {
      rows = 0u;
#pragma unroll
      for (int k = 0; k < KR; ++k) rows |= xrows[k] << (WT * k);
    }
  }

  PH(5);
  // ---- observation (prep_state4): lane h writes bytes [BPL h, BPL (h+1)) of its env's row
  if (!DBG(DBG_NO_OBS)) {
    const int quad = quadrant(ax, ay, gx, gy);
    const uint32_t flat = (rows & ((1u << WT) - 1u)) | (rows << WT);   // row r uses distinct row max(r-1, 0)
    uint8_t* dst = stage + (el - w * EPW) * F;
#pragma unroll
    for (int j = 0; j < BPL; ++j) {
      const int b = BPL * h + j;
      if (BPL * L == F || b < F) dst[b] = (uint8_t)(b < 4 ? (b == quad) : (flat >> (b - 4)) & 1u);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (!DBG(DBG_NO_OBS)) {
    const int e0u = __builtin_amdgcn_readfirstlane(e0);
    if (e0u + EPW <= N && p.obs && !p.obs_f32) {   // the common case: the wave's rows, one store per lane
      typedef int v2i_ __attribute__((ext_vector_type(2)));
      typedef int v4i_ __attribute__((ext_vector_type(4)));
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(p.obs + (size_t)e0u * F, (short)0, WB, 0x00020000);
      if constexpr (WB % 16 == 0) {
        const v4i_ x = reinterpret_cast<const v4i_*>(stage)[min(lane, WB / 16 - 1)];
        __builtin_amdgcn_raw_buffer_store_b128(x, rsrc, lane * 16, 0, AUX_SC1);
      } else {
        const v2i_ x = reinterpret_cast<const v2i_*>(stage)[min(lane, WB / 8 - 1)];
        __builtin_amdgcn_raw_buffer_store_b64(x, rsrc, lane * 8, 0, AUX_SC1);
      }
    } else {   // a partial last wave, or f32 obs: byte by byte
      const int nb = max(0, min(EPW, N - e0u)) * F;
      for (int b = lane; b < nb; b += 64) {
        if (p.obs) p.obs[(size_t)e0u * F + b] = stage[b];
        if (p.obs_f32) p.obs_f32[(size_t)e0u * F + b] = (float)stage[b];
      }
    }
  }
  // ---- the block's stats slot (32 envs), folded after every wave's obs stores are issued: one
  //      block barrier, then wave 0 folds the 32 finished flags / returns / lengths in env order
  if (slot && !DBG(DBG_NO_STATS)) {
    __syncthreads();
    if (w == 0) {
      const bool d = lane < 32 && s_fin[lane & 31];
      if (__ballot(d)) {
        const WaveStats ws = wave_stats(d, d ? s_fret[lane & 31] : 0.0, d ? s_flen[lane & 31] : 0);
        if (lane == 0) {
          reinterpret_cast<double2*>(slot)[0] = make_double2(sp0.x + ws.n, sp0.y + ws.s1);
          reinterpret_cast<double2*>(slot)[1] = make_double2(sp1.x + ws.s2, sp1.y + ws.sl);
          reinterpret_cast<double2*>(slot)[2] = make_double2(fmin(sp2.x, ws.mn), fmax(sp2.y, ws.mx));
        }
      }
    }
  }

  PH(6);
  PH_STORE;
}

// ------------------------------------------------------------------ the pool's fill
// pool_fill_kernel<W, NS, ND>: one lane per env; an env at episode e needs the entries of episodes
// e+1 (slot (e+1) & 1) and e+2 (the other slot).  Each wave ballots its envs with a stale entry per
// slot and draws them with wave_resets -- the step kernels' own inline reset, so an entry is the
// reset those kernels would draw, bit for bit -- with sinks into the pool instead of the state.
// Stream-ordered with the step kernels (be_step queues it every pool_period calls, be_reset and
// be_load_state after their copies): no step kernel reads an entry while it is written.
template <int WT, int NSC, int NDC>
__global__ __launch_bounds__(256) void pool_fill_kernel(KParams p) {
  constexpr int KR = Geo<WT>::K, NWAVE = 4;
  static_assert(WT == 10 || WT == 5, "the pool's row packing is laid out for the W = 10 and W = 5 step kernels");
  __shared__ __align__(16) TablesX t_wave[NWAVE];
  __shared__ uint32_t s_rows[NWAVE][16 * KR];
  constexpr int TW = (int)(sizeof(TablesX) / 16);
  const int N = p.n, tid = (int)threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int i = (int)blockIdx.x * 256 + tid;
  const bool valid = i < N;
  const uint32_t ic = (uint32_t)min(i, N - 1), gid = (uint32_t)p.gid0 + (uint32_t)i;
  constexpr int NBW = pool_body_words(NSC, NDC);
  uint4 tword[(TW + 63) / 64];
#pragma unroll
  for (int j = 0; j < (TW + 63) / 64; ++j)
    tword[j] = ld_s(reinterpret_cast<const uint4*>(p.tables), (uint32_t)min(lane + j * 64, TW - 1));
  const uint32_t e = ld_s(p.episode, ic);
  const uint2 tv0 = pool_ld<uint2>(p.pool, ic * 8u), tv1 = pool_ld<uint2>(p.pool, ((uint32_t)N + ic) * 8u);
#pragma unroll
  for (int j = 0; j < (TW + 63) / 64; ++j) reinterpret_cast<uint4*>(&t_wave[w])[min(lane + j * 64, TW - 1)] = tword[j];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const Tables& t = t_wave[w].t;
  const uint64_t* span = span_fits(WT, p.R) ? t_wave[w].span : nullptr;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const uint32_t target = (((e + 1u) & 1u) == (uint32_t)s) ? e + 1u : e + 2u;   // the episode slot s holds
    const uint2 tv = s ? tv1 : tv0;
    const bool need = valid && !(tv.x == target && (tv.y & POOL_VALID));
    const unsigned long long m = __ballot(need);
    if (!m) continue;
    const uint32_t xs = (uint32_t)s * (uint32_t)N;   // this slot's first entry
    auto osink = [&](int, int k, int il, int32_t o) {   // obstacle k of env il, from the lane that drew it
      pool_st(p.pool, pool_body((uint32_t)N, xs + (uint32_t)il, NBW), (uint32_t)o, 4u * (uint32_t)(PB_OBS + k));
    };
    auto esink = [&](int, int32_t ag, int32_t go, int32_t a0) {   // on the env's own lane
      double prev;
      const double td = reset_dists(ag, go, a0, prev);
      const uint32_t bo = pool_body((uint32_t)N, xs + (uint32_t)i, NBW);
      pool_st(p.pool, bo, (uint32_t)ag, 4u * PB_AGENT);
      pool_st(p.pool, bo, (uint32_t)go, 4u * PB_GOAL);
      pool_st(p.pool, bo, prev, 4u * PB_PREV);
      pool_st(p.pool, bo, td, 4u * PB_TOTAL);
    };
    int ax = 0, ay = 0, gx = 0, gy = 0, ncnt = 0;
    uint32_t xrows[KR], rej = 0u;
#pragma unroll
    for (int k = 0; k < KR; ++k) xrows[k] = 0u;
    wave_resets<WT, NSC, NDC, 64, decltype(osink)&, decltype(esink)&, 1>(p, t, m, i, gid, target - 1u, ax, ay, gx, gy,
                                                                         ncnt, xrows, &s_rows[w][0], osink, esink,
                                                                         span, &rej);
    if (need) {   // the rows, packed as the consuming kernel ORs its rows, then the tag (written flag)
      uint32_t q0, q1 = 0u, q2 = 0u;
      if constexpr (WT == 10) {
        q0 = xrows[0] | (xrows[1] << 10) | (xrows[2] << 20);
        q1 = xrows[3] | (xrows[4] << 10) | (xrows[5] << 20);
        q2 = xrows[6] | (xrows[7] << 10) | (xrows[8] << 20);
      } else {
        q0 = xrows[0] | (xrows[1] << 5) | (xrows[2] << 10) | (xrows[3] << 15);
      }
      const uint32_t x = xs + (uint32_t)i, bo = pool_body((uint32_t)N, x, NBW);
      pool_st(p.pool, bo, q0, 4u * PB_ROWS);
      pool_st(p.pool, bo, q1, 4u * (PB_ROWS + 1));
      pool_st(p.pool, bo, q2, 4u * (PB_ROWS + 2));
      pool_st(p.pool, x * 8u, make_uint2(target, POOL_VALID | (rej ? POOL_REJ : 0u)));
    }
  }
}

template <int WT, int NSC, int NDC, int L>
__global__ __launch_bounds__(32 * L) void rolloutw_kernel(KParams p) {
  constexpr int CT = 32 * L, EPW = 64 / L, NWAVE = CT / 64, G = NSC + NDC;
  constexpr int SS = (NSC + L - 1) / L, SD = (NDC + L - 1) / L;
  constexpr int KR = Geo<WT>::K, F = Geo<WT>::F;
  constexpr int BPL = (F + L - 1) / L;
  constexpr int WB = EPW * F, SW = (WB + 15) & ~15;
  constexpr int SC = 32;                         // steps per stats fold
  static_assert(WT * KR <= 20, "packed rows: 20 bits + the two collision flags");
  static_assert(NDC <= 5, "one Philox block of 24-bit fields");
  static_assert(16 * KR >= (64 / G) * (KR + 4) && (64 / G) * G <= 64, "wave reset scratch");
  static_assert(WB % 8 == 0, "a wave's rows are whole 8-byte words");
  __shared__ Tables t;
  __shared__ uint32_t s_rows[NWAVE][16 * KR];    // wave_resets scratch (row masks + stash)
  __shared__ int32_t s_ost[NWAVE][64];           // a reset pass's new obstacle positions [slot][k]
  __shared__ __align__(16) uint8_t s_stage[NWAVE][SW];
  __shared__ double s_fret[SC][32];              // finished envs' return / length per step of the fold window
  __shared__ int32_t s_flen[SC][32];
  __shared__ uint32_t s_fdone[SC][NWAVE];        // per step and wave: its finished envs (bit g = env g of the wave)
  constexpr int TW = (int)(sizeof(Tables) / 4);

  const int N = p.n, tid = (int)threadIdx.x, w = tid >> 6, lane = tid & 63, h = lane & (L - 1);
  const int el = tid / L, blk0 = (int)blockIdx.x * 32, i = blk0 + el, e0 = blk0 + w * EPW;
  const bool valid = i < N;
  const uint32_t ic = (uint32_t)min(i, N - 1), gid = (uint32_t)p.gid0 + (uint32_t)i;
  uint8_t* stage = &s_stage[w][0];

  // ---- state into registers (straight-line, use order); each lane its own obstacle slots
  constexpr int TL = (TW + CT - 1) / CT;
  uint32_t tword[TL];
#pragma unroll
  for (int j = 0; j < TL; ++j)
    tword[j] = ld_s(reinterpret_cast<const uint32_t*>(p.tables), (uint32_t)min(tid + j * CT, TW - 1));
  uint32_t episode = ld_s(p.episode, ic);
  int len = ld_s(p.ep_len, ic);
  int a = ld_s(p.actions, ic);
  const int32_t agent0 = ld_s(p.agent, ic);
  int32_t goal = ld_s(p.goal, ic);
  int32_t dp[SD], so[SS];
  int dgi[SD];
#pragma unroll
  for (int j = 0; j < SD; ++j) {
    const uint32_t e = (uint32_t)min(L * j + h, NDC - 1) * (uint32_t)N + ic;
    dp[j] = ld_s(p.dyn_obs, e);
    dgi[j] = ld_s(p.dyn_goal, e);
  }
#pragma unroll
  for (int j = 0; j < SS; ++j) so[j] = ld_s(p.static_obs, (uint32_t)min(L * j + h, NSC - 1) * (uint32_t)N + ic);
  double old_dist = ld_s(p.prev_dist, ic), total = ld_s(p.total_dist, ic), ret = ld_s(p.ep_return, ic);
  double* const slot = p.stats ? p.stats + (size_t)blockIdx.x * 8 : nullptr;   // one per 32 envs
  WaveStats acc{0.0, 0.0, 0.0, 0.0, INFINITY, -INFINITY};
  if (slot && tid == 0) acc = WaveStats{slot[0], slot[1], slot[2], slot[3], slot[4], slot[5]};
#pragma unroll
  for (int j = 0; j < TL; ++j) reinterpret_cast<uint32_t*>(&t)[min(tid + j * CT, TW - 1)] = tword[j];
  __syncthreads();   // tables staged

  int ax = px(agent0), ay = py(agent0);
  uint32_t st_flags = 0u;
  bool was_reset = false;   // statics / goal / total / episode changed: store them at the end
  const int R = p.R;
  const uint32_t R2 = (uint32_t)(R * R);
  // fold the stats window's steps [0, n) in order (wave 0; after a block barrier)
  auto fold = [&](int n) {
    if (w != 0) return;
#pragma unroll 1
    for (int u = 0; u < n; ++u) {
      uint32_t m32 = 0u;
#pragma unroll
      for (int ww = 0; ww < NWAVE; ++ww) m32 |= s_fdone[u][ww] << (ww * EPW);
      if (m32 == 0u) continue;   // (uniform)
      const bool d = lane < 32 && ((m32 >> (lane & 31)) & 1u);
      const WaveStats ws = wave_stats(d, d ? s_fret[u][lane & 31] : 0.0, d ? s_flen[u][lane & 31] : 0);
      acc.n += ws.n; acc.s1 += ws.s1; acc.s2 += ws.s2; acc.sl += ws.sl;
      acc.mn = fmin(acc.mn, ws.mn); acc.mx = fmax(acc.mx, ws.mx);
    }
  };

  // the obstacles' goal-change counter (== ep_len mod (G+1)) kept incrementally, and each step's
  // Philox block computed one step ahead: the next step's (episode, ep_len + 1) block runs beside
  // this step's work, off its critical path (recomputed after a reset for the envs that reset)
  int counter = (int)((double)len * p.inv_g1);
  counter = len - counter * (p.goal_change + 1);
  if (counter < 0) counter += p.goal_change + 1;
  if (counter > p.goal_change) counter -= p.goal_change + 1;
  u4 bnext = philox(gid, episode, (uint32_t)len, tag(PURPOSE_STEP_OBS, 0u), p.seed);
  PH_INIT;
  for (int s = 0; s < p.steps; ++s) {
    const size_t so_n = (size_t)s * N;
    // next step's action: in flight while this step runs
    const int a_next = s + 1 < p.steps ? ld_s(p.actions + so_n + N, ic) : 0;
    const int gx = px(goal), gy = py(goal);
    // ---- this lane's dynamic obstacles (ballenv_env.py:323-353)
    const bool change = counter >= p.goal_change;
    counter = change ? 0 : counter + 1;
    const u4 b0 = bnext;
    bnext = philox(gid, episode, (uint32_t)(len + 1), tag(PURPOSE_STEP_OBS, 0u), p.seed);
#pragma unroll
    for (int j = 0; j < SD; ++j) {
      const int k = L * j + h;
      int ox = px(dp[j]), oy = py(dp[j]);
      uint32_t fl = 0u;
      dgi[j] = dyn_move_fixed(p, t, ox, oy, dgi[j], t.speed[min(k, NDC - 1)], change, pick_field(b0, min(k, 4)), fl);
      st_flags |= k < NDC ? fl : 0u;
      dp[j] = pk(ox, oy);
    }
    PH(0);
    // ---- action -> agent move + clamp (ballenv_env.py:247-259)
    st_flags |= a >= p.num_actions ? (uint32_t)BE_STATUS_BAD_ACTION : 0u;
    const uint32_t sh = 2u * (uint32_t)(a < p.num_actions ? a : 0);
    ax = min(max(ax + (int)((p.amx >> sh) & 3u) - 1, 0), p.screen_w);
    ay = min(max(ay + (int)((p.amy >> sh) & 3u) - 1, 0), p.screen_h);
    const v2s agv = __builtin_bit_cast(v2s, pk(ax, ay));
    const double dist = calc_dist_lib(gx, gy, ax, ay);
    const double rbase = (0.0 - p.time_penalty) + (old_dist - dist) / total;
    PH(1);
    // ---- collision test and row masks (stepw_kernel's)
    uint32_t word = 0u;
    auto obstacle = [&](int32_t opk, bool real, uint32_t hit_bit) {
      const v2s d = __builtin_elementwise_sub_sat(__builtin_bit_cast(v2s, opk), agv);
      word |= (real & ((uint32_t)__builtin_amdgcn_sdot2(d, d, 0, false) <= R2)) ? hit_bit : 0u;
      const int f = d.x + WT / 2, e = d.y + WT / 2;
      if (real & ((uint32_t)(f + R) <= (uint32_t)(WT - 1 + 2 * R)) & ((uint32_t)(e + R) <= (uint32_t)(KR - 1 + 2 * R))) {
#pragma unroll
        for (int k = 0; k < KR; ++k) {
          const int ady = abs(e - k);
          const int hw = t.hw[min(ady, HW_MAX)];
          const int lo = max(f - hw, 0), hi = min(f + hw, WT - 1);
          word |= (ady <= R && lo <= hi) ? ((2u << hi) - (1u << lo)) << (WT * k) : 0u;
        }
      }
    };
#pragma unroll
    for (int j = 0; j < SD; ++j) obstacle(dp[j], L * j + h < NDC, 1u << 21);
#pragma unroll
    for (int j = 0; j < SS; ++j) obstacle(so[j], L * j + h < NSC, 1u << 20);
    word = lane_group_or<L>(word);
    const bool hs = (word >> 20) & 1u, hd = (word >> 21) & 1u;
    uint32_t rows = word & 0xFFFFFu;
    PH(2);
    // ---- reward, done (ballenv_env.py:268-286, 200-229)
    double reward = rbase;
    if (hs) reward -= p.static_penalty;          // statics come first in obstacle_list (Q3)
    else if (hd) reward -= p.dynamic_penalty;
    ret += reward;
    ++len;
    const bool env_done = (dist < p.threshold_goal) || hs || hd;
    const bool trunc = p.time_limit > 0 && len >= p.time_limit;
    const bool done = env_done || trunc;
    old_dist = dist;
    if (valid) {   // per-step outputs over the group's lanes
      if (h == 0) p.reward[so_n + i] = reward;
      if (h == 1) p.done[so_n + i] = (uint8_t)done;
      if (h == 2 && p.truncated) p.truncated[so_n + i] = (uint8_t)(trunc && !env_done);
      if (done) {
        if (h == 3 && p.final_return) p.final_return[so_n + i] = ret;
        if (h == 1 && p.final_len) p.final_len[so_n + i] = len;
      }
    }
    // ---- this step's finished envs for the stats fold
    const int u = s % SC;
    if (slot) {
      const bool fin = done && valid;
      if (fin && h == 0) { s_fret[u][el] = ret; s_flen[u][el] = len; }
      const unsigned long long fm = __ballot(fin && h == 0);
      uint32_t wm = 0u;
#pragma unroll
      for (int g = 0; g < EPW; ++g) wm |= (uint32_t)((fm >> (g * L)) & 1ull) << g;
      if (lane == 0) s_fdone[u][w] = wm;
    }
    PH(3);
    // ---- autoreset: terminal obs, then the wave's resets (new obstacles through the LDS stash)
    const unsigned long long m = __ballot(valid && done && p.autoreset && h == 0);
    if (m) {
      if (p.terminal_obs && valid && done && h == 0) {
        const uint32_t fl[Geo<WT>::NW] = {(rows & ((1u << WT) - 1u)) | (rows << WT), 0u};
        write_row_global<WT>(p.terminal_obs + (so_n + i) * F, fl, quadrant(ax, ay, gx, gy));
      }
      uint32_t xrows[KR];
#pragma unroll
      for (int k = 0; k < KR; ++k) xrows[k] = 0u;
      int kept = 1;
      int gxr = gx, gyr = gy;
      int32_t* ost = &s_ost[w][0];
      auto osink = [&](int sl, int k, int, int32_t o) { ost[sl * G + k] = o; };
      bool reset_now = false;
      auto esink = [&](int own, int32_t ag, int32_t go, int32_t a0) {   // every lane of the env's group
        goal = go;
        total = reset_dists<true>(ag, go, a0, old_dist);
        ret = 0.0; len = 0; ++episode; was_reset = true; reset_now = true; counter = 0;
#pragma unroll
        for (int j = 0; j < SS; ++j) so[j] = ost[own * G + min(L * j + h, NSC - 1)];
#pragma unroll
        for (int j = 0; j < SD; ++j) { dp[j] = ost[own * G + NSC + min(L * j + h, NDC - 1)]; dgi[j] = min(L * j + h, NDC - 1); }
      };
      if (!(m & (m - 1)))
        wave_resets<WT, NSC, NDC, 1, decltype(osink)&, decltype(esink)&, L>(p, t, m, i, gid, episode, ax, ay, gxr, gyr,
                                                                          kept, xrows, &s_rows[w][0], osink, esink);
      else
        wave_resets<WT, NSC, NDC, 64, decltype(osink)&, decltype(esink)&, L>(p, t, m, i, gid, episode, ax, ay, gxr, gyr,
                                                                           kept, xrows, &s_rows[w][0], osink, esink);
      if (!kept) {
        rows = 0u;
#pragma unroll
        for (int k = 0; k < KR; ++k) rows |= xrows[k] << (WT * k);
      }
      if (reset_now) bnext = philox(gid, episode, 0u, tag(PURPOSE_STEP_OBS, 0u), p.seed);
    }
    PH(4);
    // ---- observation (prep_state4) into the wave's stage, its 64/L rows out
    if (p.obs) {
      const int quad = quadrant(ax, ay, px(goal), py(goal));
      const uint32_t flat = (rows & ((1u << WT) - 1u)) | (rows << WT);
      uint8_t* dst = stage + (el - w * EPW) * F;
#pragma unroll
      for (int j = 0; j < BPL; ++j) {
        const int b = BPL * h + j;
        if (BPL * L == F || b < F) dst[b] = (uint8_t)(b < 4 ? (b == quad) : (flat >> (b - 4)) & 1u);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int e0u = __builtin_amdgcn_readfirstlane(e0);
      uint8_t* orow = p.obs + (so_n + (size_t)e0u) * F;
      if (e0u + EPW <= N) {
        typedef int v2i_ __attribute__((ext_vector_type(2)));
        typedef int v4i_ __attribute__((ext_vector_type(4)));
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(orow, (short)0, WB, 0x00020000);
        if constexpr (WB % 16 == 0) {
          const v4i_ x = reinterpret_cast<const v4i_*>(stage)[min(lane, WB / 16 - 1)];
          __builtin_amdgcn_raw_buffer_store_b128(x, rsrc, lane * 16, 0, 0);
        } else {
          const v2i_ x = reinterpret_cast<const v2i_*>(stage)[min(lane, WB / 8 - 1)];
          __builtin_amdgcn_raw_buffer_store_b64(x, rsrc, lane * 8, 0, 0);
        }
      } else {
        const int nb = max(0, min(EPW, N - e0u)) * F;
        for (int b = lane; b < nb; b += 64) orow[b] = stage[b];
      }
      // the next step's stage writes follow this step's stage reads
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    PH(5);
    if (slot && (u == SC - 1 || s + 1 == p.steps)) {   // (uniform: every wave runs every step)
      __syncthreads();
      fold(u + 1);
      __syncthreads();   // the window's LDS is free again
    }
    a = a_next;
    PH(6);
  }
  PH_STORE;

  // ---- state back to HBM, once
  if (valid) {
    if (h == 0) {
      p.agent[i] = pk(ax, ay);
      p.prev_dist[i] = old_dist;
      p.ep_return[i] = ret;
      p.ep_len[i] = len;
      if (was_reset) {
        p.goal[i] = goal;
        p.total_dist[i] = total;
        p.episode[i] = episode;
      }
    }
#pragma unroll
    for (int j = 0; j < SD; ++j) {
      const int k = L * j + h;
      if (k < NDC) {
        (p.dyn_obs + (size_t)k * N)[i] = dp[j];
        (p.dyn_goal + (size_t)k * N)[i] = (uint8_t)dgi[j];
      }
    }
    if (was_reset) {
#pragma unroll
      for (int j = 0; j < SS; ++j) {
        const int k = L * j + h;
        if (k < NSC) (p.static_obs + (size_t)k * N)[i] = so[j];
      }
    }
  }
  if (slot && tid == 0) {
    slot[0] = acc.n; slot[1] = acc.s1; slot[2] = acc.s2; slot[3] = acc.sl; slot[4] = acc.mn; slot[5] = acc.mx;
  }
  if (__ballot(st_flags != 0u)) {
    uint32_t f = st_flags;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) f |= (uint32_t)__shfl_xor((int)f, o);
    if (lane == 0) atomicOr(p.status, (int)f);
  }
}

// ------------------------------------------------------------------ fused multi-step rollout
// rollout_kernel<W, NS, ND>: p.steps consecutive be_step calls of the fixed-shape kernel in one
// launch, for a caller-given (steps, N) action tape.  Each env's state stays in registers for
// the whole rollout; per step only the action is read and the reward / done (/ truncated,
// final return / length) and the obs row are written, into (steps, N, ...) buffers.  State
// goes back to HBM once, at the end.  Every draw is Philox keyed by (global env id, episode,
// ep_len), so the outputs are bit-identical to p.steps launches of be_kernel<W, STEP, NS, ND>
// (tests/test_gpu_rollout.py); the per-step physics below is that kernel's fixed-shape path
// (ballenv_env.py:232-289, 323-353, 200-229; ball_cnn_ac3.py:384-412).  Autoreset is
// wave-cooperative (wave_resets) with the new state stashed in LDS and picked up by the env's
// own lane.  SURVEY 8(d) prices this mode at 1 + 8 + 1 + (4+W^2) bytes per env-step plus the
// state round trip once per launch.
//
// HT > 0: the fused config-5 rollout (be_policy_rollout).  The action of every step comes from
// select_action on the obs in the block's LDS stage (policy_core.h, the packed Policy(W) image
// staged in LDS once per launch): envs with a lit window cell are compacted into a block list
// and go through tile_forward in 16-env MFMA tiles (one wave per tile), the others take the
// empty-window table; policy_finish draws the action.  Same functions, same inputs and the
// same Philox keys as be_policy_act, so the trajectory is bit-identical to the two-launch
// loop (tests/test_gpu_rollout.py::test_policy_rollout_matches_two_launch_loop).  The obs is
// written per step only when recorded (p.obs), and the last one to p.obs_last.
template <int WT, int NSC, int NDC, int HT = 0, int KS = 1, int NO = 10>
__global__ __launch_bounds__(BLOCK_THREADS) void rollout_kernel(KParams p) {
  constexpr int KR = Geo<WT>::K, F = Geo<WT>::F, G = NSC + NDC, NWAVE = BLOCK_THREADS / 64;
  constexpr bool POL = HT > 0;
  constexpr PolLayout PL = pol_layout(HT > 0 ? HT : 1, KS, NO);
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ Tables t;
  __shared__ uint32_t s_rows[NWAVE][16 * KR];    // wave_resets scratch (row masks + stash)
  __shared__ int32_t s_ost[NWAVE][64];           // a reset pass's new obstacle positions [slot][k]
  constexpr int TW = (int)(sizeof(Tables) / 4);
  const int N = p.n, tid = (int)threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int blk0 = (int)blockIdx.x * BLOCK_THREADS, i = blk0 + tid, e0 = blk0 + w * 64;
  const bool valid = i < N;
  const int nrows = max(0, min(64, N - e0));     // this wave's valid obs rows
  const uint32_t ic = (uint32_t)min(i, N - 1), gid = (uint32_t)p.gid0 + (uint32_t)i;
  NearList<BLOCK_THREADS> nl{reinterpret_cast<uint32_t*>(smem) + tid, 0};
  uint8_t* stage_blk = smem + (size_t)(G + 1) * BLOCK_THREADS * 4;   // [256 envs][F]: row = tid
  uint8_t* stage = stage_blk + (size_t)w * 64 * F;                    // this wave's 64 rows
  // POL: PolLayout image + scratch, 16-byte aligned (a constant offset from the LDS base keeps the
  // accesses ds_* -- an integer round trip of the pointer would turn them into flat accesses)
  constexpr int POL_OFF = ((G + 1) * BLOCK_THREADS * 4 + BLOCK_THREADS * F + 15) & ~15;
  uint8_t* pimg = smem + POL_OFF;
  // the row-span table (build_span_table): after the stage, or (POL) after the chunk partials
  uint16_t* mt = reinterpret_cast<uint16_t*>(POL ? pimg + PL.lds + POL_CHUNKS * NWAVE * 16 * NO * 4 : smem + POL_OFF);

  // ---- state into registers (straight-line, use order)
  const uint32_t tword = ld_s(reinterpret_cast<const uint32_t*>(p.tables), (uint32_t)min(tid, TW - 1));
  uint32_t episode = ld_s(p.episode, ic);
  int len = ld_s(p.ep_len, ic);
  int a = POL ? 0 : ld_s(p.actions, ic);
  const int32_t agent0 = ld_s(p.agent, ic);
  int32_t goal = ld_s(p.goal, ic);
  int32_t dp[NDC], so[NSC];
  int dgi[NDC];
#pragma unroll
  for (int j = 0; j < NDC; ++j) { dp[j] = ld_s(p.dyn_obs + (size_t)j * N, ic); dgi[j] = ld_s(p.dyn_goal + (size_t)j * N, ic); }
#pragma unroll
  for (int j = 0; j < NSC; ++j) so[j] = ld_s(p.static_obs + (size_t)j * N, ic);
  double old_dist = ld_s(p.prev_dist, ic), total = ld_s(p.total_dist, ic), ret = ld_s(p.ep_return, ic);
  // stats slot of this lane's half-wave (be_stats_slots: one per 32 envs; none past N)
  const int e32 = e0 + (lane & 32);
  double* slot = (p.stats && e32 < N) ? p.stats + (((size_t)blockIdx.x * NWAVE + w) * 2 + (lane >> 5)) * 8 : nullptr;
  WaveStats acc{0.0, 0.0, 0.0, 0.0, INFINITY, -INFINITY};
  if (slot) acc = WaveStats{slot[0], slot[1], slot[2], slot[3], slot[4], slot[5]};
  reinterpret_cast<uint32_t*>(&t)[min(tid, TW - 1)] = tword;
  build_span_table<WT>(mt, p.R, tid, BLOCK_THREADS);
  int pquad = 0;          // POL: quadrant of the current obs
  bool pnz = false;       // POL: the current obs needs the dense forward (a lit cell / not one-hot)
  if constexpr (POL) {
    // the packed policy image, once per launch; the current obs rows (obs of the state)
    const uint4* src = reinterpret_cast<const uint4*>(p.pol_img);
    stage_image<BLOCK_THREADS, 8>(reinterpret_cast<uint4*>(pimg), src, p.pol_bytes / 16, tid);
    const int bytes = nrows * F;
    const uint8_t* orow = p.obs_in + (size_t)e0 * F;
    stage_image<64, 8>(reinterpret_cast<uint4*>(stage), reinterpret_cast<const uint4*>(orow), bytes / 16, lane);
    for (int b = (bytes & ~15) + lane; b < bytes; b += 64) stage[b] = orow[b];
    if (tid < 3) reinterpret_cast<int*>(pimg + PL.count)[tid] = 0;
  }
  __syncthreads();   // tables (and the policy image, the obs rows, the list counters) staged
  float* pbuf_base = reinterpret_cast<float*>(pimg + PL.lds);   // POL: chunk partials of a round of tiles
  if constexpr (POL) {
    if (valid) {   // what be_policy_act's scan decides from the same bytes
      const uint8_t* row = stage + lane * F;
      const uint32_t q4 = (uint32_t)row[0] | ((uint32_t)row[1] << 8) | ((uint32_t)row[2] << 16) | ((uint32_t)row[3] << 24);
      uint32_t lit = 0;
      for (int b = 4; b < F; ++b) lit |= row[b];
      pquad = q4 == 1u ? 0 : (q4 == 0x100u ? 1 : (q4 == 0x10000u ? 2 : 3));
      const bool onehot = q4 == 1u || q4 == 0x100u || q4 == 0x10000u || q4 == 0x1000000u;
      pnz = lit != 0u || !onehot;
    }
  }

  int ax = px(agent0), ay = py(agent0);
  uint32_t st_flags = 0;
  bool was_reset = false;   // statics / goal / total / episode changed: store them at the end
  const Win g0(p, 0, 0);
  const uint32_t R2 = (uint32_t)g0.R2;
  const NearBox nb0(g0);
  const int bxo = WT / 2 + g0.R, byo = WT / 2 + g0.R;   // unit speeds
  typedef unsigned short v2u __attribute__((ext_vector_type(2)));
  const v2s boxo = {(short)bxo, (short)byo};
  const v2u boxw = {(unsigned short)nb0.bw, (unsigned short)nb0.bh};

  PH_INIT;
  for (int s = 0; s < p.steps; ++s) {
    const size_t so_n = (size_t)s * N;
    // next step's action (tape mode): in flight while this step runs
    const int a_next = (!POL && s + 1 < p.steps) ? ld_s(p.actions + so_n + N, ic) : 0;
    if constexpr (POL) {
      // ---- select_action (ball_cnn_ac3.py:210-220) on the obs in the stage
      // list counters, one per step mod 3: thread 0 clears step s+2's right after this step's
      // barrier, which every wave passes again (step s+1) before it counts into that one
      int* cnt3 = reinterpret_cast<int*>(pimg + PL.count);
      int16_t* list = reinterpret_cast<int16_t*>(pimg + PL.list);
      float* lg = reinterpret_cast<float*>(pimg + PL.logits);
      if (DBG(DBG_POL_TABLE)) pnz = false;
      const int c3 = s % 3;
      // the draw's uniform, a function of this env's state (in flight across the barrier)
      const float u = policy_uniform(gid, episode, (uint32_t)len, p.pol_seed);
      int my_k = 0;   // this env's place in the list
      if (valid && pnz) {
        my_k = atomicAdd(&cnt3[c3], 1);
        list[my_k] = (int16_t)tid;
      }
      PH(0);
      if (!DBG(DBG_POL_NO_SYNC)) __syncthreads();   // list complete (and every wave's stage rows written)
      PH(1);
      const int cnt = cnt3[c3];
      if (tid == 0) cnt3[c3 == 0 ? 2 : c3 - 1] = 0;   // (s + 2) % 3
      const int g4 = lane >> 4;
      // the listed envs in 16-env tiles, rounds of up to NWAVE tiles: every wave runs its chunk
      // of hidden rows (tile_chunk, wave w = chunk w) for each tile of the round into pbuf, then
      // the listed envs' lanes add the four chunks in order (tile_forward's sum, bit for bit)
      float* pbuf = pbuf_base;   // [NWAVE chunks][NWAVE tiles][16][NO]
      const int ntiles = (cnt + 15) >> 4;
      for (int r0 = 0; r0 < ntiles; r0 += NWAVE) {
        const int nt = min(NWAVE, ntiles - r0);
        // obs fragments of tile r0 + tt (load_obs16's bytes: row e, columns c .. c+15, zero past F)
        auto load_b = [&](int tt, v4i (&Bt)[KS]) {
          const int k = (r0 + tt) * 16 + (lane & 15);
          const int e = k < cnt ? list[k] : -1;
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            const int c = 64 * ks + 16 * g4;
            const uint8_t* row = stage_blk + (e >= 0 ? e : 0) * F;
            v4i v = {0, 0, 0, 0};
            if constexpr ((F & 7) == 0) {
              const int c0 = c < F - 8 ? c : F - 8, c1 = c + 8 < F - 8 ? c + 8 : F - 8;
              const uint2 lo = *reinterpret_cast<const uint2*>(row + c0), hi = *reinterpret_cast<const uint2*>(row + c1);
              const bool vlo = e >= 0 && c + 8 <= F, vhi = e >= 0 && c + 16 <= F;
              v[0] = vlo ? (int)lo.x : 0; v[1] = vlo ? (int)lo.y : 0;
              v[2] = vhi ? (int)hi.x : 0; v[3] = vhi ? (int)hi.y : 0;
            } else {
              uint32_t wd[4] = {0u, 0u, 0u, 0u};
#pragma unroll
              for (int j = 0; j < 16; ++j)
                if (e >= 0 && c + j < F) wd[j >> 2] |= (uint32_t)row[c + j] << (8 * (j & 3));
              v[0] = (int)wd[0]; v[1] = (int)wd[1]; v[2] = (int)wd[2]; v[3] = (int)wd[3];
            }
            Bt[ks] = v;
          }
        };
        auto put = [&](int tt, const float (&part)[PolQ<NO>::N]) {   // lane group g4: outputs g4, g4 + 4, ...
#pragma unroll
          for (int q = 0; q < PolQ<NO>::N; ++q)
            if (4 * q + g4 < NO) pbuf[((w * NWAVE + tt) * 16 + (lane & 15)) * NO + 4 * q + g4] = part[q];
        };
        constexpr int HTC = HT > 0 ? HT : 1;
        const int h0 = pol_chunk_begin(HTC, w), h1 = pol_chunk_begin(HTC, w + 1);
        for (int tt = 0; tt < nt; tt += 2) {   // two tiles at a time: shared weight reads, interleaved chains
          v4i Ba[KS], Bb[KS];
          float pa[PolQ<NO>::N], pb[PolQ<NO>::N];
          load_b(tt, Ba);
          if (tt + 1 < nt && !DBG(0xF0000u)) {
            load_b(tt + 1, Bb);
            // chunk lengths are HT/4 or HT/4 + 1: unrolled bodies for both
            constexpr int LS = HTC / POL_CHUNKS;
            if (h1 - h0 == LS) tile_chunk2<HTC, KS, NO, LS>(pimg, Ba, Bb, lane, h0, h1, pa, pb);
            else tile_chunk2<HTC, KS, NO, LS + 1>(pimg, Ba, Bb, lane, h0, h1, pa, pb);
            put(tt, pa);
            put(tt + 1, pb);
          } else {
            // (diagnostics builds: tile_chunk's own ablation bits 2 / 4 from dbg bits 17 / 18)
            constexpr int LS = HTC / POL_CHUNKS;
            if (DBG(0xF0000u)) tile_chunk<HTC, KS, NO>(pimg, Ba, lane, (int)(DBG(0xF0000u) >> 16), h0, h1, pa);
            else if (h1 - h0 == LS) tile_chunk<HTC, KS, NO, LS>(pimg, Ba, lane, 0, h0, h1, pa);
            else tile_chunk<HTC, KS, NO, LS + 1>(pimg, Ba, lane, 0, h0, h1, pa);
            put(tt, pa);
            if (tt + 1 < nt) {
              load_b(tt + 1, Bb);
              tile_chunk<HTC, KS, NO>(pimg, Bb, lane, (int)(DBG(0xF0000u) >> 16), h0, h1, pb);
              put(tt + 1, pb);
            }
          }
        }
        PH(2);
        __syncthreads();   // every chunk of the round's tiles
        PH(3);
        if (ntiles <= NWAVE) break;   // one round (the common case): each env reads its chunks below
        if (tid < nt * 16 && r0 * 16 + tid < cnt) {   // one thread per listed env: the chunks in order
          const int e = list[r0 * 16 + tid];
          const int tt = tid >> 4, col = tid & 15;
#pragma unroll
          for (int o = 0; o < NO; ++o) {
            float v = pbuf[((0 * NWAVE + tt) * 16 + col) * NO + o];
#pragma unroll
            for (int c = 1; c < NWAVE; ++c) v = v + pbuf[((c * NWAVE + tt) * 16 + col) * NO + o];
            lg[e * NO + o] = v;
          }
        }
        __syncthreads();   // round done: pbuf free, these logits visible
      }
      static_assert(NWAVE == POL_CHUNKS, "one hidden-row chunk per wave");
      // select_action's tail (policy_finish with the uniform drawn above) on the raw logits: the
      // chunk partials added in order (one round), the combined logits (several), or the table
      float raw[NO];
      if (pnz && ntiles <= NWAVE) {
        const int tt = my_k >> 4, col = my_k & 15;
#pragma unroll
        for (int o = 0; o < NO; ++o) {
          float v = pbuf_base[((0 * NWAVE + tt) * 16 + col) * NO + o];
#pragma unroll
          for (int c = 1; c < NWAVE; ++c) v = v + pbuf_base[((c * NWAVE + tt) * 16 + col) * NO + o];
          raw[o] = v;
        }
      } else {
        const float* src = pnz ? lg + tid * NO : reinterpret_cast<const float*>(pimg + PL.table) + pquad * NO;
#pragma unroll
        for (int o = 0; o < NO; ++o) raw[o] = src[o];
      }
      float lp = 0.f, val = 0.f;
      if (DBG(DBG_POL_NO_FINISH)) {
        a = (int)((gid + (uint32_t)len * 7u) % 9u);
      } else {
        const PolDist<NO> d = policy_dist<NO>(raw, reinterpret_cast<const float*>(pimg + PL.hbias), p.pol_actions,
                                              nullptr);
        a = policy_pick<NO>(d.cdf, d.lp, d.last_nz, p.pol_actions, u, lp);
        val = d.value;
      }
      if (valid) {
        p.act_out[so_n + i] = (uint8_t)a;
        if (p.logp_out) p.logp_out[so_n + i] = lp;
        if (p.value_out) p.value_out[so_n + i] = val;
      }
    }
    const int gx = px(goal), gy = py(goal);
    PH(4);
    // ---- action -> agent move + clamp (ballenv_env.py:247-259)
    st_flags |= a >= p.num_actions ? (uint32_t)BE_STATUS_BAD_ACTION : 0u;
    const uint32_t sh = 2u * (uint32_t)(a < p.num_actions ? a : 0);
    const int dx = (int)((p.amx >> sh) & 3u) - 1, dy = (int)((p.amy >> sh) & 3u) - 1;
    ax = min(max(ax + dx, 0), p.screen_w);   // unit speeds (pick_rollout's precondition)
    ay = min(max(ay + dy, 0), p.screen_h);
    bool hs = false, hd = false;
    nl.cnt = 0;
    // ---- dynamic obstacles (counter == ep_len mod (G+1): all start at 0 on reset)
    int counter = (int)((double)len * p.inv_g1);
    counter = len - counter * (p.goal_change + 1);
    if (counter < 0) counter += p.goal_change + 1;
    if (counter > p.goal_change) counter -= p.goal_change + 1;
    const bool change = counter >= p.goal_change;
    const u4 b0 = philox(gid, episode, (uint32_t)len, tag(PURPOSE_STEP_OBS, 0u), p.seed);
    u4 b1{0u, 0u, 0u, 0u};
    if (NDC > 5) b1 = philox(gid, episode, (uint32_t)len, tag(PURPOSE_STEP_OBS, 1u), p.seed);
    const v2s agv = __builtin_bit_cast(v2s, pk(ax, ay));
    uint32_t* nlp = nl.base;   // (step2_kernel's saturating slot advance; nl.cnt set after the tests)
    auto obstacle_pk = [&](int32_t opk, bool& hit) {   // be_kernel's packed int16x2 test
      const v2s d = __builtin_elementwise_sub_sat(__builtin_bit_cast(v2s, opk), agv);
      hit |= (uint32_t)__builtin_amdgcn_sdot2(d, d, 0, false) <= R2;
      const v2u b = __builtin_bit_cast(v2u, __builtin_elementwise_add_sat(d, boxo));
      const v2u over = __builtin_elementwise_sub_sat(b, boxw);
      *nlp = __builtin_bit_cast(uint32_t, d);
      nlp += BLOCK_THREADS * __builtin_elementwise_sub_sat(1u, __builtin_bit_cast(uint32_t, over));
    };
#pragma unroll
    for (int j = 0; j < NDC; ++j) {
      int ox = px(dp[j]), oy = py(dp[j]);
      const uint32_t wf = j < 5 ? pick_field(b0, j) : pick_field(b1, j - 5);
      dgi[j] = dyn_move_fixed(p, t, ox, oy, dgi[j], t.speed[j], change, wf, st_flags);
      dp[j] = pk(ox, oy);
      obstacle_pk(dp[j], hd);
    }
#pragma unroll
    for (int j = 0; j < NSC; ++j) obstacle_pk(so[j], hs);
    nl.cnt = (int)(lds_bytes(nl.base, nlp) / (BLOCK_THREADS * 4u));

    // ---- distance, reward, done (ballenv_env.py:268-286, 200-229)
    // (computing this right after the move, as step2_kernel does, measured slower here)
    const double dist = calc_dist_lib(gx, gy, ax, ay);
    double reward = 0.0 - p.time_penalty;
    reward += (old_dist - dist) / total;
    if (hs) reward -= p.static_penalty;          // statics come first in obstacle_list (Q3)
    else if (hd) reward -= p.dynamic_penalty;
    ret += reward;
    ++len;
    const bool env_done = (dist < p.threshold_goal) || hs || hd;
    const bool trunc = p.time_limit > 0 && len >= p.time_limit;
    const bool done = env_done || trunc;
    old_dist = dist;
    if (valid) {
      p.reward[so_n + i] = reward;
      p.done[so_n + i] = (uint8_t)done;
      if (p.truncated) p.truncated[so_n + i] = (uint8_t)(trunc && !env_done);
      if (done) {
        if (p.final_return) p.final_return[so_n + i] = ret;
        if (p.final_len) p.final_len[so_n + i] = len;
      }
    }
    if (p.stats) {   // the step kernel's per-half-wave fold, step by step (same order: bit-identical sums)
      WaveStats lo, hi;
      wave_stats2(done && valid, ret, len, lo, hi);
      const bool lh = lane < 32;   // this lane's half (per-field selects: no runtime-selected struct)
      const double wn = lh ? lo.n : hi.n;
      if (slot && wn > 0.0) {
        acc.n += wn; acc.s1 += lh ? lo.s1 : hi.s1; acc.s2 += lh ? lo.s2 : hi.s2; acc.sl += lh ? lo.sl : hi.sl;
        acc.mn = fmin(acc.mn, lh ? lo.mn : hi.mn); acc.mx = fmax(acc.mx, lh ? lo.mx : hi.mx);
      }
    }

    PH(5);
    // ---- autoreset: new state stashed in LDS, picked up into this lane's registers
    uint32_t xrows[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) xrows[k] = 0u;
    int gxr = gx, gyr = gy;
    const unsigned long long m = __ballot(valid && done && p.autoreset);
    if (m) {
      if (p.terminal_obs && valid && done) {   // obs of the terminal state, rows of reset envs (as be_step)
        uint32_t rows[KR], flat[Geo<WT>::NW];
        raster_rows_mt<WT, BLOCK_THREADS>(nl, p.R, rows, mt);
        flatten<WT>(rows, flat);
        write_row_global<WT>(p.terminal_obs + (so_n + i) * F, flat, quadrant(ax, ay, gx, gy));
      }
      int32_t* ost = &s_ost[w][0];
      auto osink = [&](int sl, int k, int, int32_t o) { ost[sl * G + k] = o; };
      auto esink = [&](int own, int32_t ag, int32_t go, int32_t a0) {
        goal = go;
        total = reset_dists<true>(ag, go, a0, old_dist);
        ret = 0.0; len = 0; ++episode; was_reset = true;
#pragma unroll
        for (int k = 0; k < NSC; ++k) so[k] = ost[own * G + k];
#pragma unroll
        for (int j = 0; j < NDC; ++j) { dp[j] = ost[own * G + NSC + j]; dgi[j] = j; }
      };
      if (!(m & (m - 1)))
        wave_resets<WT, NSC, NDC, 1>(p, t, m, i, gid, episode, ax, ay, gxr, gyr, nl.cnt, xrows, &s_rows[w][0], osink, esink);
      else
        wave_resets<WT, NSC, NDC, 64>(p, t, m, i, gid, episode, ax, ay, gxr, gyr, nl.cnt, xrows, &s_rows[w][0], osink, esink);
    }

    PH(6);
    // ---- observation (prep_state4) into this wave's stage, then 64 rows out
    {
      uint32_t rows[KR], flat[Geo<WT>::NW];
      raster_rows_mt<WT, BLOCK_THREADS>(nl, p.R, rows, mt);
#pragma unroll
      for (int k = 0; k < KR; ++k) rows[k] |= xrows[k];
      flatten<WT>(rows, flat);
      const int quad = quadrant(ax, ay, gxr, gyr);
      if constexpr (POL) {
        uint32_t any = 0u;
#pragma unroll
        for (int k = 0; k < Geo<WT>::NW; ++k) any |= flat[k];
        pquad = quad;
        pnz = valid && any != 0u;   // (lanes past N are never listed)
      }
      if constexpr ((F & 7) == 0) {   // 8-byte LDS stores
        auto word = [&](int wd) -> uint32_t {
          const int jc = 4 * (wd - 1);
          return wd == 0 ? 1u << (8 * quad) : (((flat[jc >> 5] >> (jc & 31)) & 0xFu) * 0x00204081u) & 0x01010101u;
        };
        uint2* dst = reinterpret_cast<uint2*>(stage + lane * F);
#pragma unroll
        for (int wd = 0; wd < F / 8; ++wd) dst[wd] = make_uint2(word(2 * wd), word(2 * wd + 1));
      } else {
        stage_row<WT>(stage, lane, flat, quad);
      }
    }
    if (p.obs) {   // recorded obs (always in tape mode)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (nrows == 64)   // a full wave (wave-uniform): one unrolled pass, reads ahead of stores
        copy_wave_full<64 * F / 16, ST_PLAIN>(stage, p.obs + (so_n + (size_t)__builtin_amdgcn_readfirstlane(e0)) * F, lane);
      else
        copy_out<64, ST_PLAIN>(stage, F, nrows, (int64_t)e0, p.obs + so_n * F, nullptr, lane);
      // the next step's stage writes must follow this step's stage reads (LDS ops issue in order)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    a = a_next;
    PH(7);
  }

  PH_STORE;
  // ---- state back to HBM, once
  if (valid) {
    p.agent[i] = pk(ax, ay);
    p.prev_dist[i] = old_dist;
    p.ep_return[i] = ret;
    p.ep_len[i] = len;
#pragma unroll
    for (int j = 0; j < NDC; ++j) {
      (p.dyn_obs + (size_t)j * N)[i] = dp[j];
      (p.dyn_goal + (size_t)j * N)[i] = (uint8_t)dgi[j];
    }
    if (was_reset) {
      p.goal[i] = goal;
      p.total_dist[i] = total;
      p.episode[i] = episode;
#pragma unroll
      for (int k = 0; k < NSC; ++k) (p.static_obs + (size_t)k * N)[i] = so[k];
    }
  }
  if (p.obs_last) {   // the obs of the final state (the env's obs buffer)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (nrows == 64)
      copy_wave_full<64 * F / 16, ST_PLAIN>(stage, p.obs_last + (size_t)__builtin_amdgcn_readfirstlane(e0) * F, lane);
    else
      copy_out<64, ST_PLAIN>(stage, F, nrows, (int64_t)e0, p.obs_last, nullptr, lane);
  }
  if (slot && (lane & 31) == 0) {
    slot[0] = acc.n; slot[1] = acc.s1; slot[2] = acc.s2; slot[3] = acc.sl; slot[4] = acc.mn; slot[5] = acc.mx;
  }
  if (__ballot(st_flags != 0u)) {
    uint32_t f = st_flags;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) f |= (uint32_t)__shfl_xor((int)f, o);
    if (lane == 0) atomicOr(p.status, (int)f);
  }
}

__global__ void sample_actions_kernel(uint8_t* out, int32_t n, int32_t steps, int64_t env_offset,
                                      int32_t num_actions, unsigned long long seed) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)n * steps;
  for (; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
    const int32_t t = (int32_t)(idx / n), i = (int32_t)(idx - (int64_t)t * n);
    const u4 b = philox((uint32_t)(env_offset + i), (uint32_t)t, 0u, tag(PURPOSE_SAMPLE, 0), seed);
    out[idx] = (uint8_t)map_range(b.x, 0, num_actions);
  }
}

// ------------------------------------------------------------------ dispatch
using KFn = void (*)(KParams);
template <int WT>
KFn kernel_for(int mode) {
  return mode == MODE_STEP ? be_kernel<WT, MODE_STEP>
                           : (mode == MODE_RESET ? be_kernel<WT, MODE_RESET> : be_kernel<WT, MODE_OBSERVE>);
}

struct Launch { KFn fn; int epb; int lds; char name[48]; int threads = BLOCK_THREADS; };

// Fixed-shape step kernels for the reference's default obstacle counts (ball_cnn_ac3.py:40-41).
constexpr int FIX_NS = 13, FIX_ND = 5;   // the reference's obstacle counts (ball_cnn_ac3.py:40-41)
// The fixed-shape kernels address per-env arrays as a uniform base + a 32-bit byte offset (ld_s /
// st_ws): element i of an 8-byte array needs i < 2^29.  Larger batches (~150 GB of state and outputs)
// take the generic kernels, which index in 64 bits.
constexpr int64_t FIX_MAX_ENVS = 1ll << 29;

// pool: the variant that copies finished envs' resets from the autoreset pool (step2_kernel /
// stepw_kernel<..., true>; the context passes it only with a pool allocated)
Launch pick_kernel(const be_config& c, int mode, bool fixed_ok = false, int lanes10 = 1, int lpe5 = 0, bool pool = false) {
  int W = c.window;
  const int F = 4 + W * W, nobs = c.num_static + c.num_dynamic;
  Launch L{nullptr, 0, 0, {0}};
  bool staged = true;
  const bool fixed = fixed_ok && mode == MODE_STEP && c.num_static == FIX_NS && c.num_dynamic == FIX_ND &&
                     c.speed_x == 1 && c.speed_y == 1 && c.radius_obstacle + c.radius_agent <= HW_MAX &&
                     (int64_t)c.num_envs < FIX_MAX_ENVS;
  if (fixed && lanes10 == 2 && W == 10 && span_fits(W, c.radius_obstacle + c.radius_agent) &&
      (int64_t)c.num_envs * FIX_NS < (1ll << 30)) {
    // two lanes per env (step2_kernel): 32 envs per wave, 128 per block
    L.fn = pool ? step2_kernel<10, FIX_NS, FIX_ND, true> : step2_kernel<10, FIX_NS, FIX_ND, false>;
    L.epb = S2_CT / 2;
    L.threads = S2_CT;
    constexpr int SLOTS = (FIX_NS + 1) / 2 + (FIX_ND + 1) / 2 + 1;
    L.lds = SLOTS * S2_CT * 4 + L.epb * F;
    snprintf(L.name, sizeof L.name, "step2_kernel<10, %d, %d, %s>", FIX_NS, FIX_ND, pool ? "true" : "false");
    return L;
  }
  if (fixed && W == 5 && (lpe5 == 4 || lpe5 == 8) && (int64_t)c.num_envs * FIX_NS < (1ll << 30)) {
    // L lanes per env (stepw_kernel): 32 envs per block (its reset sink stores obstacles at 32-bit
    // byte offsets, as step2_kernel's does: NS*N < 2^30)
    L.fn = lpe5 == 8 ? (pool ? stepw_kernel<5, FIX_NS, FIX_ND, 8, true> : stepw_kernel<5, FIX_NS, FIX_ND, 8, false>)
                     : (pool ? stepw_kernel<5, FIX_NS, FIX_ND, 4, true> : stepw_kernel<5, FIX_NS, FIX_ND, 4, false>);
    L.epb = 32;
    L.threads = 32 * lpe5;
    L.lds = 0;
    snprintf(L.name, sizeof L.name, "stepw_kernel<5, %d, %d, %d, %s>", FIX_NS, FIX_ND, lpe5, pool ? "true" : "false");
    return L;
  }
  if (fixed && W == 10) {
    L.fn = pool ? be_kernel<10, MODE_STEP, FIX_NS, FIX_ND, true> : be_kernel<10, MODE_STEP, FIX_NS, FIX_ND, false>;
    L.epb = BLOCK_THREADS; W = -1;
  } else if (fixed && W == 5) {
    L.fn = pool ? be_kernel<5, MODE_STEP, FIX_NS, FIX_ND, true> : be_kernel<5, MODE_STEP, FIX_NS, FIX_ND, false>;
    L.epb = BLOCK_THREADS; W = -1;
  }
  switch (W) {
    case -1: break;
#define BE_CASE(n) case n: L.fn = kernel_for<n>(mode); L.epb = envs_per_block(n); break;
    BE_CASE(1) BE_CASE(2) BE_CASE(3) BE_CASE(4) BE_CASE(5) BE_CASE(6) BE_CASE(7) BE_CASE(8)
    BE_CASE(9) BE_CASE(10) BE_CASE(11) BE_CASE(12) BE_CASE(13) BE_CASE(14) BE_CASE(15) BE_CASE(16)
    BE_CASE(21)
#undef BE_CASE
    default: L.fn = kernel_for<0>(mode); L.epb = envs_per_block(0); staged = false; break;
  }
  if (L.fn) {
    if (W == -1) snprintf(L.name, sizeof L.name, "be_kernel<%d, %d, %d, %d, %s>", c.window, mode, FIX_NS, FIX_ND, pool ? "true" : "false");
    else snprintf(L.name, sizeof L.name, "be_kernel<%d, %d, 0, 0, false>", staged ? W : 0, mode);
  }
  const int near_bytes = (nobs + 1) * BLOCK_THREADS * 4;   // +1: predicated pushes write one slot ahead
  const int stage_bytes = staged ? L.epb * F : 0;
  L.lds = (near_bytes + stage_bytes + 15) & ~15;
  if (L.lds == 0) L.lds = 16;
  return L;
}

// The fused rollout kernel for the same fixed shapes (nullptr: not applicable).
Launch pick_rollout(const be_config& c, bool fixed_ok, int lpe5 = 0) {
  Launch L{nullptr, BLOCK_THREADS, 0, {0}};
  const bool fixed = fixed_ok && c.num_static == FIX_NS && c.num_dynamic == FIX_ND && c.speed_x == 1 &&
                     c.speed_y == 1 && c.radius_obstacle + c.radius_agent <= HW_MAX && (int64_t)c.num_envs < FIX_MAX_ENVS;
  if (fixed && c.window == 5 && (lpe5 == 4 || lpe5 == 8)) {   // small batches: L lanes per env, 32-env blocks
    L.fn = lpe5 == 8 ? rolloutw_kernel<5, FIX_NS, FIX_ND, 8> : rolloutw_kernel<5, FIX_NS, FIX_ND, 4>;
    L.epb = 32;
    L.threads = 32 * lpe5;
    L.lds = 0;
    snprintf(L.name, sizeof L.name, "rolloutw_kernel<5, %d, %d, %d>", FIX_NS, FIX_ND, lpe5);
    return L;
  }
  if (fixed && c.window == 10) L.fn = rollout_kernel<10, FIX_NS, FIX_ND>;
  else if (fixed && c.window == 5) L.fn = rollout_kernel<5, FIX_NS, FIX_ND>;
  L.lds = ((FIX_NS + FIX_ND + 1) * BLOCK_THREADS * 4 + BLOCK_THREADS * (4 + c.window * c.window) + 15) & ~15;
  const int R = c.radius_obstacle + c.radius_agent;
  L.lds += (c.window + 2 * R) * (R + 2) * 2;   // the row-span table
  if (L.fn) snprintf(L.name, sizeof L.name, "rollout_kernel<%d, %d, %d, 0, 1, 10>", c.window, FIX_NS, FIX_ND);
  return L;
}

// The fused policy rollout kernel: fixed env shape and the select_action kernel's Policy(W)
// shapes (H 208 / W 10 and H 128 / W 5, 9 actions).
Launch pick_policy_rollout(const be_config& c, bool fixed_ok, int HT, int KS, int NO) {
  Launch L{nullptr, BLOCK_THREADS, 0, {0}};
  const bool fixed = fixed_ok && c.num_static == FIX_NS && c.num_dynamic == FIX_ND && c.speed_x == 1 &&
                     c.speed_y == 1 && c.radius_obstacle + c.radius_agent <= HW_MAX && (int64_t)c.num_envs < FIX_MAX_ENVS;
  if (fixed && c.window == 10 && HT == 13 && KS == 2 && NO == 10)
    L.fn = rollout_kernel<10, FIX_NS, FIX_ND, 13, 2, 10>;
  else if (fixed && c.window == 5 && HT == 8 && KS == 1 && NO == 10)
    L.fn = rollout_kernel<5, FIX_NS, FIX_ND, 8, 1, 10>;
  const PolLayout PL = pol_layout(HT, KS, NO);
  L.lds = (FIX_NS + FIX_ND + 1) * BLOCK_THREADS * 4 + BLOCK_THREADS * (4 + c.window * c.window);
  L.lds = ((L.lds + 15) & ~15) + PL.lds;
  L.lds = ((L.lds + 15) & ~15) + POL_CHUNKS * (BLOCK_THREADS / 64) * 16 * NO * 4;   // chunk partials
  const int R = c.radius_obstacle + c.radius_agent;
  L.lds += (c.window + 2 * R) * (R + 2) * 2;   // the row-span table (3.2 KB at W = 10, R = 25: fits the CU's 160 KB)
  return L;
}

}  // namespace

// ====================================================================== C ABI
struct be_ctx {
  be_config cfg;
  TablesX tables;
  KParams base;      // config-derived part of every launch's KParams
  int device;
  int* status;
  TablesX* d_tables;
  bool generic_only;   // BALLENV_GENERIC_KERNELS=1: never use the fixed-shape step kernels (A/B diagnostics)
  bool unit_moves;     // every action move in {-1,0,1}^2 (fixed-shape kernels' packed table)
  bool distinct_goals; // >= 2 pairwise-distinct goals (fixed-shape kernels' arithmetic newGoalList)
  int step_lanes;      // W = 10: lanes per env of the fixed step kernel (1: be_kernel; 2: step2_kernel)
  int step5_lpe;       // W = 5: lanes per env of the fixed step kernel (1: be_kernel; 4 / 8: stepw_kernel)
  int roll5_lpe;       // W = 5: lanes per env of the fused rollout (1: rollout_kernel; 4 / 8: rolloutw_kernel)
  int max_lds;         // the device's LDS bytes per workgroup
  Launch step_launch[2];   // be_step's kernel without / with the fixed-shape preconditions (fixed per context)
  Launch step_launch_pool; // the fixed-shape kernel's pool variant (when the context has a pool)
  int64_t blob_hdr[8]; // be_save_state's header (host memory that outlives the async copy)
  // the autoreset pool (layout at pool_body): allocated when be_step's fixed-shape kernel consumes it
  uint32_t* pool;      // nullptr: no pool (every reset inline)
  int64_t pool_bytes;
  KFn pool_fill;       // pool_fill_kernel<W, 13, 5>
  int pool_period;     // be_step queues a fill every pool_period step launches (0: only be_reset / be_load_state / be_pool_fill)
  int pool_calls;      // step launches since the last fill
  const void* pool_owner;   // the state (its episode array) the pool serves: other states step without it
  mutable struct { KFn fn; int lds; bool ok; } lds_cache[4];   // fits_lds() answers per (kernel, dynamic LDS)
  mutable std::mutex lds_mu;                                    // guards lds_cache (const entries may race)
  char err[512];
};

// Does a fused kernel's LDS (static + this launch's dynamic bytes) fit one workgroup?  The fused
// rollouts' dynamic LDS grows with R = radius_obstacle + radius_agent (near lists, row-span
// table) and the config-5 kernel is within 72 B of the CU's 160 KB at the default R = 25, so a
// larger R must take the per-step fallback instead of failing the launch.
static bool fits_lds(const be_ctx* ctx, const Launch& L) {
  if (!L.fn) return false;
  std::lock_guard<std::mutex> lock(ctx->lds_mu);
  for (auto& c : ctx->lds_cache)
    if (c.fn == L.fn && c.lds == L.lds) return c.ok;
  hipFuncAttributes fa;
  bool ok = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(L.fn)) == hipSuccess &&
            (int64_t)fa.sharedSizeBytes + L.lds <= (int64_t)ctx->max_lds;
  for (auto& c : ctx->lds_cache)
    if (!c.fn) { c.fn = L.fn; c.lds = L.lds; c.ok = ok; break; }
  return ok;
}

static thread_local char g_err[512];

static int fail(be_ctx* ctx, int code, const char* fmt, const char* detail) {
  char* dst = ctx ? ctx->err : g_err;
  snprintf(dst, 512, fmt, detail ? detail : "");
  return code;
}

#define HIP_TRY(ctx, expr)                                                                     \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) return fail(ctx, BE_E_HIP, "HIP error: %s", hipGetErrorString(e_)); \
  } while (0)

// library-internal accessors for the other translation units (csrc/internal.h)
be_ctx_view be_ctx_get(const be_ctx* ctx) {
  be_ctx_view v;
  v.num_envs = ctx->cfg.num_envs; v.window = ctx->cfg.window; v.device = ctx->device;
  v.num_static = ctx->cfg.num_static; v.num_dynamic = ctx->cfg.num_dynamic;
  v.env_offset = ctx->cfg.env_offset;
  return v;
}
int be_ctx_fail(be_ctx* ctx, int code, const char* msg) { return fail(ctx, code, "%s", msg); }
static int check_state(be_ctx* ctx, const be_state* st);
int be_ctx_check_state(be_ctx* ctx, const be_state* st) { return check_state(ctx, st); }

extern "C" {

int be_abi_version(void) { return BE_ABI_VERSION; }

BE_DIAG_STEP_ENTRIES   // diagnostics builds only (diag.h)

int be_config_default(be_config* c, int32_t num_envs, int32_t window) {
  if (!c) return fail(nullptr, BE_E_INVALID, "%s", "cfg is NULL");
  memset(c, 0, sizeof(*c));
  c->num_envs = num_envs; c->window = window; c->env_offset = 0; c->seed = 0xBA11ull;
  c->screen_width = 500; c->screen_height = 500;                                     // ballenv_env.py:11-18
  c->strip_obs_x = 0; c->strip_obs_y = 20; c->strip_goal_x = 500; c->strip_goal_y = 20;
  c->strip_agent_x = 500; c->strip_agent_y = 10;
  c->radius_obstacle = 20; c->radius_agent = 5; c->speed_x = 1; c->speed_y = 1;     // :49-54
  c->threshold_goal = 10.0; c->time_penalty = 0.0; c->min_spawn_dist = 50.0;        // :64-65, :122
  c->num_static = 13; c->num_dynamic = 5; c->static_penalty = 1.0; c->dynamic_penalty = 8000.0;  // ball_cnn_ac3.py:40-51
  c->goal_change_step = 50; c->obs_certainty = 60;
  static const int goals[5][2] = {{12, 122}, {123, 93}, {87, 150}, {430, 440}, {230, 11}};
  c->num_goals = 5;
  for (int g = 0; g < 5; ++g) { c->goals[g][0] = goals[g][0]; c->goals[g][1] = goals[g][1]; }
  for (int k = 0; k < 5; ++k) c->obstacle_speed[k] = 1;
  static const int moves[9][2] = {{1, 1}, {1, -1}, {1, 0}, {0, 1}, {0, -1}, {0, 0}, {-1, 1}, {-1, 0}, {-1, -1}};
  c->num_actions = 9;                                                                // ball_cnn_ac3.py:530
  for (int a = 0; a < 9; ++a) { c->actions[a][0] = moves[a][0]; c->actions[a][1] = moves[a][1]; }
  c->time_limit = 1000; c->autoreset = 1;                                            // gym_ballenv/__init__.py:7
  return BE_OK;
}

int be_config_check(const be_config* c, char* msg, int32_t msg_len) {
  char buf[256] = {0};
#define BE_REQ(cond, text) do { if (!(cond)) { snprintf(buf, sizeof buf, "%s", text); goto bad; } } while (0)
  BE_REQ(c != nullptr, "cfg is NULL");
  BE_REQ(c->num_envs >= 1, "num_envs must be >= 1");
  BE_REQ(c->window >= 1 && c->window <= BE_MAX_WINDOW, "window must be in [1, 64]");
  BE_REQ(c->num_static >= 0 && c->num_static <= BE_MAX_STATIC, "num_static must be in [0, 64]");
  BE_REQ(c->num_dynamic >= 0 && c->num_dynamic <= BE_MAX_DYNAMIC, "num_dynamic must be in [0, 32]");
  BE_REQ(c->env_offset >= 0 && c->env_offset + (int64_t)c->num_envs <= (1ll << 32), "global env ids must fit in 32 bits");
  BE_REQ(c->screen_width >= 1 && c->screen_width <= 16384 && c->screen_height >= 1 && c->screen_height <= 16384,
         "screen size must be in [1, 16384]");
  BE_REQ(c->strip_goal_x >= 1 && c->strip_goal_x <= c->screen_width + 16384 && c->strip_goal_y >= 1 &&
         c->strip_goal_y <= c->screen_height + 16384, "goal strips must give non-empty randint ranges");
  BE_REQ(c->strip_agent_x >= 1 && c->strip_agent_x <= 16384 && c->strip_agent_y >= 1 && c->strip_agent_y <= 16384,
         "agent strips must give non-empty randint ranges");
  BE_REQ(c->screen_width - 2 * c->strip_obs_x >= 1 && c->screen_height - 2 * c->strip_obs_y >= 1,
         "obstacle strips must give non-empty randint ranges");
  BE_REQ(c->radius_obstacle >= 0 && c->radius_agent >= 0 && c->radius_obstacle + c->radius_agent <= 2047,
         "radii must be >= 0 with r_obstacle + r_agent <= 2047");
  BE_REQ(c->speed_x >= 1 && c->speed_y >= 1 && c->speed_x <= 1024 && c->speed_y <= 1024,
         "agent speeds (window cell steps) must be in [1, 1024]");
  BE_REQ(c->speed_x * (c->window / 2) <= 16384 && c->speed_y * (c->window / 2) <= 16384, "window too wide");
  BE_REQ(c->goal_change_step >= 0 && c->goal_change_step < (1 << 30), "goal_change_step out of range");
  BE_REQ(c->num_goals >= 0 && c->num_goals <= BE_MAX_GOALS, "num_goals must be in [0, 16]");
  BE_REQ(c->num_goals >= c->num_dynamic, "need a goal per dynamic obstacle (obs_goal_position)");
  BE_REQ(c->num_actions >= 1 && c->num_actions <= BE_MAX_ACTIONS, "num_actions must be in [1, 16]");
  for (int k = 0; k < c->num_dynamic; ++k)
    BE_REQ(c->obstacle_speed[k] >= -1024 && c->obstacle_speed[k] <= 1024, "obstacle speed out of range");
  for (int g = 0; g < c->num_goals; ++g)
    BE_REQ(c->goals[g][0] >= -16384 && c->goals[g][0] <= 16384 && c->goals[g][1] >= -16384 && c->goals[g][1] <= 16384,
           "goal coordinates out of range");
  for (int a = 0; a < c->num_actions; ++a)
    BE_REQ(c->actions[a][0] >= -1024 && c->actions[a][0] <= 1024 && c->actions[a][1] >= -1024 && c->actions[a][1] <= 1024,
           "action deltas out of range");
  BE_REQ(c->time_limit >= 0, "time_limit must be >= 0");
  BE_REQ(!(c->threshold_goal != c->threshold_goal), "threshold_goal is NaN");
  {  // int16 coordinates.  The reference's dynamic obstacles are unbounded Python ints (no clamp,
     // ballenv_env.py:334-347); here they are int16.  An obstacle spawns inside the obstacle strips
     // and moves at most |speed| per axis per step, and with autoreset and a time limit an episode
     // has at most time_limit moves, so the bound below holds for every episode and such a config
     // can never leave int16.  Without that bound (time_limit 0, or autoreset 0: a caller may step
     // past done) the kernels flag BE_STATUS_COORD_RANGE, the stored coordinate wraps (two's
     // complement int16) and the caller must poll be_status.
    int64_t ms = 0;
    for (int k = 0; k < c->num_dynamic; ++k) ms = std::max<int64_t>(ms, std::abs((int64_t)c->obstacle_speed[k]));
    const int64_t ex = std::max<int64_t>(std::abs((int64_t)c->strip_obs_x),
                                         std::abs((int64_t)c->screen_width - c->strip_obs_x));
    const int64_t ey = std::max<int64_t>(std::abs((int64_t)c->strip_obs_y),
                                         std::abs((int64_t)c->screen_height - c->strip_obs_y));
    BE_REQ(!(c->autoreset && c->time_limit > 0 && c->num_dynamic > 0) ||
               std::max(ex, ey) + ms * (int64_t)c->time_limit <= 32767,
           "dynamic obstacles can leave the int16 coordinate range within one episode: need "
           "max spawn extent + max|obstacle_speed| * time_limit <= 32767 (or time_limit 0 / autoreset 0 "
           "and poll status())");
  }
#undef BE_REQ
  if (msg && msg_len > 0) msg[0] = 0;
  return BE_OK;
bad:
  if (msg && msg_len > 0) snprintf(msg, (size_t)msg_len, "%s", buf);
  return fail(nullptr, BE_E_INVALID, "invalid config: %s", buf);
}

// Can a reset re-sample the agent (ballenv_env.py:121-126, quirk Q9)?  Only if some agent spawn
// point lies closer than min_spawn_dist to some goal spawn point: with the reference's strips
// (agent y < 10, goal y >= 480) never.  When it cannot, prev_dist (state[2]) always equals
// calc_dist(goal, agent) -- after a step it is that distance, after a reset total_distance -- so
// the fixed-shape step kernels may recompute it instead of reading it (an A/B option, KParams).
static bool q9_possible(const be_config* c) {
  const int64_t dx = std::max<int64_t>(0, (int64_t)(c->screen_width - c->strip_goal_x) - (c->strip_agent_x - 1));
  const int64_t dy = std::max<int64_t>(0, (int64_t)(c->screen_height - c->strip_goal_y) - (c->strip_agent_y - 1));
  const double D = c->min_spawn_dist;
  return D > 0.0 && sqrt((double)(dx * dx + dy * dy)) < D;
}

int64_t be_step_bytes(const be_config* c) {
  if (!c) return 0;
  // agent R+W 8 | goal R 4 | prev_dist R+W 16 | total_dist R 8 | ep_return R+W 16 | ep_len R+W 8
  // | episode R 4 | action R 1 | reward W 8 | done W 1                                     = 74
  // | statics R 4*Ns | dyn xy R+W 8*Nd | dyn goal R 1*Nd | obs W 4+W^2
  return 74 + 4ll * c->num_static + 9ll * c->num_dynamic + 4 + (int64_t)c->window * c->window;
}

const char* be_last_error(const be_ctx* ctx) { return ctx ? ctx->err : g_err; }

const char* be_kernel_name(const be_ctx* ctx, int32_t entry) {
  static thread_local char name[48];
  if (!ctx) return nullptr;
  const bool fixed_ok = !ctx->generic_only && ctx->unit_moves && ctx->distinct_goals;
  Launch L{nullptr, 0, 0, {0}};
  switch (entry) {
    case BE_ENTRY_STEP_ACTIONS:   // (the pool variant when the context has a pool: its state's steps run it)
      L = pick_kernel(ctx->cfg, MODE_STEP, fixed_ok, ctx->step_lanes, ctx->step5_lpe, ctx->pool != nullptr);
      break;
    case BE_ENTRY_STEP_SAMPLED: L = pick_kernel(ctx->cfg, MODE_STEP, false); break;
    case BE_ENTRY_ROLLOUT: {
      L = pick_rollout(ctx->cfg, fixed_ok, ctx->roll5_lpe);
      const DeviceGuard dg(ctx->device);   // fits_lds queries the context's device
      if (dg.err != hipSuccess || !fits_lds(ctx, L)) L.fn = nullptr;
      break;
    }
    case BE_ENTRY_RESET: L = pick_kernel(ctx->cfg, MODE_RESET, false); break;
    case BE_ENTRY_OBSERVE: L = pick_kernel(ctx->cfg, MODE_OBSERVE, false); break;
    default: return nullptr;
  }
  if (!L.fn) return nullptr;
  memcpy(name, L.name, sizeof name);
  return name;
}

int64_t be_stats_slots(const be_config* c) {
  if (!c || c->num_envs < 1 || c->window < 1) return 0;
  // one slot per 32 envs: the fixed-shape kernels settle stats per half-wave (LPE 1) or per
  // wave (LPE 2), the generic ones per block (fewer slots, a prefix of these)
  return ((int64_t)c->num_envs + 31) / 32;
}

int be_create(const be_config* cfg, int32_t device, be_ctx** out) {
  if (!out) return fail(nullptr, BE_E_INVALID, "%s", "out is NULL");
  *out = nullptr;
  char msg[256];
  if (be_config_check(cfg, msg, sizeof msg) != BE_OK) return fail(nullptr, BE_E_INVALID, "invalid config: %s", msg);
  be_ctx* ctx = new (std::nothrow) be_ctx();
  if (!ctx) return fail(nullptr, BE_E_NOMEM, "%s", "out of host memory");
  ctx->cfg = *cfg;
  ctx->device = device;
  KParams& b = ctx->base;
  memset(&b, 0, sizeof b);
  b.n = cfg->num_envs; b.window = cfg->window; b.ns = cfg->num_static; b.nd = cfg->num_dynamic;
  b.R = cfg->radius_obstacle + cfg->radius_agent; b.speed_x = cfg->speed_x; b.speed_y = cfg->speed_y;
  b.screen_w = cfg->screen_width; b.screen_h = cfg->screen_height; b.goal_change = cfg->goal_change_step;
  b.certainty = cfg->obs_certainty; b.time_limit = cfg->time_limit; b.num_actions = cfg->num_actions;
  b.autoreset = cfg->autoreset; b.gid0 = (int32_t)(uint32_t)cfg->env_offset;
  b.threshold_goal = cfg->threshold_goal; b.time_penalty = cfg->time_penalty;
  b.static_penalty = cfg->static_penalty; b.dynamic_penalty = cfg->dynamic_penalty;
  b.min_spawn_dist = cfg->min_spawn_dist; b.seed = cfg->seed;
  b.num_goals = cfg->num_goals;
  // prev_dist is read: recomputing it (possible when q9_possible() is false) measured slower, the
  // f64 sqrt lands on the reward's chain (step2 6.52 vs 6.38 us, stepw 4.36 vs 4.20 us, A/B in one
  // process, profiles/r03_prev_dist_ab.txt); BALLENV_PREV_READ=0 selects it where it is exact (A/B)
  b.prev_read = 1;
  if (const char* r = getenv("BALLENV_PREV_READ")) { if (!strcmp(r, "0") && !q9_possible(cfg)) b.prev_read = 0; }
  ctx->unit_moves = cfg->num_actions <= 16;
  for (int a = 0; a < cfg->num_actions && a < 16; ++a) {
    const int mx = cfg->actions[a][0], my = cfg->actions[a][1];
    if (mx < -1 || mx > 1 || my < -1 || my > 1) ctx->unit_moves = false;
    else { b.amx |= (uint32_t)(mx + 1) << (2 * a); b.amy |= (uint32_t)(my + 1) << (2 * a); }
  }
  ctx->distinct_goals = cfg->num_goals >= 2;
  for (int g = 0; g < cfg->num_goals; ++g)
    for (int h = 0; h < g; ++h)
      if (cfg->goals[g][0] == cfg->goals[h][0] && cfg->goals[g][1] == cfg->goals[h][1]) ctx->distinct_goals = false;
  {  // smallest integer n with sqrt(n) >= min_spawn_dist (f64, correctly rounded: monotone in n)
    const double D = cfg->min_spawn_dist;
    long long n = D <= 0.0 ? 0 : (long long)ceil(D * D);
    if (n > (1ll << 30)) n = 1ll << 30;
    while (n > 0 && sqrt((double)(n - 1)) >= D) --n;
    while (n < (1ll << 30) && sqrt((double)n) < D) ++n;
    b.min_spawn_d2 = (int32_t)n;
  }
  b.inv_g1 = 1.0 / ((double)cfg->goal_change_step + 1.0);
  if (const char* d = getenv("BALLENV_DEBUG_SKIP")) b.dbg = (int32_t)strtoul(d, nullptr, 0);
  if (const char* g = getenv("BALLENV_GENERIC_KERNELS")) ctx->generic_only = atoi(g) != 0;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
  {  // Two lanes per env (step2_kernel) shorten each wave's dependent chain where one lane per env
     // leaves at most ~1.5 waves per SIMD; past that the one-lane kernel has the waves to hide its
     // latency and the pair's duplicated per-env work costs more than it saves (measured on MI355X,
     // 256 CUs: step2 6.42 / 7.51 us at 65 536 / 98 304 envs against 6.97 / 7.92; one lane 8.13 /
     // 14.5 / 48.9 us at 131 072 / 262 144 / 2^20 against 8.54 / 16.2 / 52.6).
     // BALLENV_STEP_LPE=1 / 2 forces one or two lanes (A/B).
    ctx->step_lanes = (int64_t)cfg->num_envs > (int64_t)96 * 4 * cus ? 1 : 2;
  }
  // W = 5 (BASELINE config 2): stepw_kernel's 8 lanes per env while one lane per env would leave
  // most of the chip idle (<= 64 envs per CU), the one-lane kernel above that.
  ctx->step5_lpe = (int64_t)cfg->num_envs <= (int64_t)64 * cus ? 8 : 1;
  ctx->roll5_lpe = ctx->step5_lpe;
  if (const char* l = getenv("BALLENV_ROLLOUT5_LPE")) {   // A/B override: "1", "4" or "8", else ignored
    if (!strcmp(l, "1")) ctx->roll5_lpe = 1;
    else if (!strcmp(l, "4")) ctx->roll5_lpe = 4;
    else if (!strcmp(l, "8")) ctx->roll5_lpe = 8;
  }
  if (const char* l = getenv("BALLENV_STEP5_LPE")) {   // A/B override: "1", "4" or "8", else ignored
    if (!strcmp(l, "1")) ctx->step5_lpe = 1;
    else if (!strcmp(l, "4")) ctx->step5_lpe = 4;
    else if (!strcmp(l, "8")) ctx->step5_lpe = 8;
  }
  // (four lanes per env, step2_kernel<10, 13, 5, 4, 128> of commit b0bc389, was bit-exact but slower
  // at every size: 6.08 vs 5.28 us at 32 768 envs, profiles/r04_w10_lanes_2_4.jsonl)
  if (const char* l = getenv("BALLENV_STEP_LPE")) {   // A/B override: exactly "1" or "2", else ignored
    if (!strcmp(l, "1")) ctx->step_lanes = 1;
    else if (!strcmp(l, "2")) ctx->step_lanes = 2;
  }
  if (hipDeviceGetAttribute(&ctx->max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess ||
      ctx->max_lds <= 0)
    ctx->max_lds = 65536;
  memset(&ctx->tables, 0, sizeof ctx->tables);
  Tables& t = ctx->tables.t;
  for (int k = 0; k < cfg->num_dynamic; ++k) t.speed[k] = cfg->obstacle_speed[k];
  t.strip_obs_x = cfg->strip_obs_x; t.strip_obs_y = cfg->strip_obs_y;
  t.strip_goal_x = cfg->strip_goal_x; t.strip_goal_y = cfg->strip_goal_y;
  t.strip_agent_x = cfg->strip_agent_x; t.strip_agent_y = cfg->strip_agent_y;
  t.radius_obstacle = cfg->radius_obstacle; t.radius_agent = cfg->radius_agent;
  for (int g = 0; g < cfg->num_goals; ++g)
    t.goal[g] = (int32_t)(((uint32_t)cfg->goals[g][0] & 0xFFFFu) | ((uint32_t)cfg->goals[g][1] << 16));
  for (int a = 0; a < cfg->num_actions; ++a)
    t.action[a] = (int32_t)(((uint32_t)cfg->actions[a][0] & 0xFFFFu) | ((uint32_t)cfg->actions[a][1] << 16));
  for (int g = 0; g < cfg->num_goals; ++g) {  // newGoalList, ballenv_env.py:351
    int n = 0;
    for (int q = 0; q < cfg->num_goals; ++q)
      if (cfg->goals[q][0] != cfg->goals[g][0] || cfg->goals[q][1] != cfg->goals[g][1]) t.other[g][n++] = (uint8_t)q;
    t.n_other[g] = (uint8_t)n;
  }
  const int R = cfg->radius_obstacle + cfg->radius_agent;
  for (int d = 0; d <= R && d <= HW_MAX; ++d) {   // exact integer sqrt
    int h = 0;
    while ((h + 1) * (h + 1) <= R * R - d * d) ++h;
    t.hw[d] = (uint8_t)h;
  }
  if (span_fits(cfg->window, R)) {   // step2_kernel's row-span table (TablesX)
    const int W = cfg->window, C = W - 1 + R, J0 = R + W - 2;   // K = W-1 rows
    for (int j = 0; j < SPAN_N; ++j) {
      const int a = abs(j - J0), hw = a <= R ? t.hw[a] : 0;
      ctx->tables.span[j] = a <= R && j <= 2 * J0 ? ((2ull << (2 * hw)) - 1ull) << (C - hw) : 0ull;
    }
  }
  const DeviceGuard dg(device);   // the caller's current device is restored on return
  hipError_t e = dg.err;
  if (e == hipSuccess) e = hipMalloc(&ctx->status, sizeof(int));
  if (e == hipSuccess) e = hipMemset(ctx->status, 0, sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&ctx->d_tables, sizeof(TablesX));
  if (e == hipSuccess) e = hipMemcpy(ctx->d_tables, &ctx->tables, sizeof(TablesX), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  // be_step's two possible kernels, picked once (pick_kernel formats a name: not per launch)
  ctx->step_launch[0] = pick_kernel(ctx->cfg, MODE_STEP, false, ctx->step_lanes, ctx->step5_lpe);
  ctx->step_launch[1] = pick_kernel(ctx->cfg, MODE_STEP, true, ctx->step_lanes, ctx->step5_lpe);
  {  // the autoreset pool, for the fixed-shape kernels that consume it (step2_kernel, stepw_kernel, the one-lane kernel)
    const KFn f = ctx->step_launch[1].fn;
    int64_t onelane_max = (int64_t)2 * 64 * 4 * cus;   // BALLENV_POOL_ONELANE_MAX: the bound below, for A/B runs
    if (const char* v = getenv("BALLENV_POOL_ONELANE_MAX")) onelane_max = atoll(v);
    const bool consumes = ctx->unit_moves && ctx->distinct_goals && !ctx->generic_only && cfg->autoreset &&
                          (f == step2_kernel<10, FIX_NS, FIX_ND, false> || f == stepw_kernel<5, FIX_NS, FIX_ND, 8, false> ||
                           f == stepw_kernel<5, FIX_NS, FIX_ND, 4, false> ||
                           // the one-lane kernel up to two waves per SIMD: 7.51-7.59 against 7.76-7.85 us at
                           // 131 072 envs; at 262 144 (four waves per SIMD hide the reset draws, and the
                           // fill costs more) 14.11-14.24 against 13.71-13.72 (profiles/r06_onelane_pool_ab.txt)
                           ((f == be_kernel<10, MODE_STEP, FIX_NS, FIX_ND> || f == be_kernel<5, MODE_STEP, FIX_NS, FIX_ND>) &&
                            (int64_t)cfg->num_envs <= onelane_max));
    bool want = consumes && (int64_t)cfg->num_envs <= POOL_MAX_ENVS;
    if (const char* v = getenv("BALLENV_POOL")) want = want && strcmp(v, "0") != 0;   // A/B: "0" = no pool
    ctx->pool_period = 128;
    if (const char* v = getenv("BALLENV_POOL_PERIOD")) ctx->pool_period = std::max(0, atoi(v));
    if (want && e == hipSuccess) {
      ctx->pool_bytes = pool_bytes_per_env(FIX_NS, FIX_ND) * cfg->num_envs;
      ctx->pool_fill = cfg->window == 10 ? pool_fill_kernel<10, FIX_NS, FIX_ND> : pool_fill_kernel<5, FIX_NS, FIX_ND>;
      e = hipMalloc(&ctx->pool, (size_t)ctx->pool_bytes);
      if (e == hipSuccess) e = hipMemset(ctx->pool, 0, (size_t)ctx->pool_bytes);   // every entry unwritten
      if (e == hipSuccess) e = hipDeviceSynchronize();
      ctx->step_launch_pool = pick_kernel(ctx->cfg, MODE_STEP, true, ctx->step_lanes, ctx->step5_lpe, true);
    }
  }
  if (e != hipSuccess) {
    int rc = fail(nullptr, BE_E_HIP, "HIP error in be_create: %s", hipGetErrorString(e));
    if (ctx->status) (void)hipFree(ctx->status);
    if (ctx->d_tables) (void)hipFree(ctx->d_tables);
    if (ctx->pool) (void)hipFree(ctx->pool);
    delete ctx;
    return rc;
  }
  *out = ctx;
  return BE_OK;
}

int be_destroy(be_ctx* ctx) {
  if (!ctx) return BE_OK;
  const DeviceGuard dg(ctx->device);   // the caller's current device is restored on return
  if (ctx->status) (void)hipFree(ctx->status);
  if (ctx->d_tables) (void)hipFree(ctx->d_tables);
  if (ctx->pool) (void)hipFree(ctx->pool);
  delete ctx;
  return BE_OK;
}

static int check_state(be_ctx* ctx, const be_state* st) {
  if (!st || !st->agent || !st->goal || !st->prev_dist || !st->total_dist || !st->ep_return || !st->ep_len ||
      !st->episode)
    return fail(ctx, BE_E_INVALID, "%s", "be_state has a NULL pointer");
  if (ctx->cfg.num_static > 0 && !st->static_obs) return fail(ctx, BE_E_INVALID, "%s", "static_obs is NULL");
  if (ctx->cfg.num_dynamic > 0 && (!st->dyn_obs || !st->dyn_goal))
    return fail(ctx, BE_E_INVALID, "%s", "dyn_obs/dyn_goal is NULL");
  return BE_OK;
}

// Per-call KParams: the context's config part + this call's pointers.
static KParams make_params(be_ctx* ctx, const be_state* st, const be_out* out) {
  KParams a = ctx->base;
  a.agent = st->agent; a.goal = st->goal; a.prev_dist = st->prev_dist; a.total_dist = st->total_dist;
  a.ep_return = st->ep_return; a.ep_len = st->ep_len; a.episode = st->episode; a.static_obs = st->static_obs;
  a.dyn_obs = st->dyn_obs; a.dyn_goal = st->dyn_goal;
  if (out) {
    a.obs = out->obs; a.obs_f32 = out->obs_f32; a.reward = out->reward; a.done = out->done;
    a.truncated = out->truncated; a.terminal_obs = out->terminal_obs; a.final_return = out->final_return;
    a.final_len = out->final_len; a.stats = out->stats;
  }
  a.tables = &ctx->d_tables->t;
  a.status = ctx->status;
  return a;
}

// pool_fill_kernel over every env of the state (the caller holds the DeviceGuard)
static void launch_pool_fill(be_ctx* ctx, const KParams& a, void* stream) {
  KParams f = a;
  f.pool = ctx->pool;
  const int N = ctx->cfg.num_envs;
  hipLaunchKernelGGL(ctx->pool_fill, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, f);
  ctx->pool_calls = 0;
}

// steps > 1 (be_step_n): `steps` launches of the same kernel, actions advancing by N per step.
static int launch(be_ctx* ctx, int mode, KParams& a, void* stream, int32_t steps = 1) {
  const bool fixed_ok = mode == MODE_STEP && a.tape == nullptr && a.actions != nullptr && !ctx->generic_only &&
                        ctx->unit_moves && ctx->distinct_goals;
  if (((uintptr_t)a.obs & 15) || ((uintptr_t)a.obs_f32 & 15))
    return fail(ctx, BE_E_INVALID, "%s", "obs / obs_f32 must be 16-byte aligned");
  const DeviceGuard dg(ctx->device);   // the caller's current device is restored on return
  HIP_TRY(ctx, dg.err);
  // the pool serves one state (its owner: the state last reset / loaded, else the first one stepped);
  // a step of any other state draws its resets inline, so a context's entries are only ever written
  // and read by the launches of one state, which the caller orders on its stream anyway
  if (ctx->pool && mode == MODE_STEP && fixed_ok && !ctx->pool_owner) ctx->pool_owner = a.episode;
  const bool use_pool = ctx->pool && mode == MODE_STEP && fixed_ok && a.episode == ctx->pool_owner;
  a.pool = use_pool ? ctx->pool : nullptr;
  const Launch L = mode == MODE_STEP ? (use_pool ? ctx->step_launch_pool : ctx->step_launch[fixed_ok ? 1 : 0])
                                     : pick_kernel(ctx->cfg, mode, fixed_ok, ctx->step_lanes, ctx->step5_lpe);
  const int N = ctx->cfg.num_envs;
  const dim3 grid((unsigned)((N + L.epb - 1) / L.epb)), block((unsigned)L.threads);
  for (int32_t s = 0; s < steps; ++s) {
    hipLaunchKernelGGL(L.fn, grid, block, (size_t)L.lds, (hipStream_t)stream, a);
    a.actions += N;
    if (use_pool && ctx->pool_period > 0 && ++ctx->pool_calls >= ctx->pool_period) launch_pool_fill(ctx, a, stream);
  }
  HIP_TRY(ctx, hipGetLastError());
  return BE_OK;
}

int be_reset(be_ctx* ctx, const be_state* st, const uint8_t* mask, const int16_t* reset_tape, int32_t tape_len,
             const be_out* out, void* stream) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (int rc = check_state(ctx, st)) return rc;
  if (reset_tape && tape_len < 0) return fail(ctx, BE_E_INVALID, "%s", "tape_len < 0");
  if (!out || (!out->obs && !out->obs_f32)) return fail(ctx, BE_E_INVALID, "%s", "be_reset needs out->obs or out->obs_f32");
  KParams a = make_params(ctx, st, out);
  a.reward = nullptr; a.done = nullptr; a.truncated = nullptr; a.terminal_obs = nullptr;
  a.final_return = nullptr; a.final_len = nullptr; a.stats = nullptr;
  a.mask = mask; a.reset_tape = reset_tape; a.reset_tape_len = reset_tape ? tape_len : 0;
  if (int rc = launch(ctx, MODE_RESET, a, stream)) return rc;
  if (ctx->pool) {   // this state's next two episodes per env, ahead of its first step
    ctx->pool_owner = st->episode;
    const DeviceGuard dg(ctx->device);
    HIP_TRY(ctx, dg.err);
    launch_pool_fill(ctx, a, stream);
    HIP_TRY(ctx, hipGetLastError());
  }
  return BE_OK;
}

int be_step(be_ctx* ctx, const be_state* st, const uint8_t* actions, const int16_t* action_deltas,
            const int16_t* draw_tape, const be_out* out, void* stream) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (int rc = check_state(ctx, st)) return rc;
  if (!out || !out->reward || !out->done) return fail(ctx, BE_E_INVALID, "%s", "be_step needs out->reward and out->done");
  if (draw_tape && ctx->cfg.autoreset) return fail(ctx, BE_E_INVALID, "%s", "draw tapes (parity mode) need autoreset = 0");
  KParams a = make_params(ctx, st, out);
  a.actions = actions; a.deltas = action_deltas; a.tape = draw_tape;
  return launch(ctx, MODE_STEP, a, stream);
}

int be_step_n(be_ctx* ctx, const be_state* st, const uint8_t* actions, int32_t steps, const be_out* out,
              void* stream) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (int rc = check_state(ctx, st)) return rc;
  if (!actions || steps < 0) return fail(ctx, BE_E_INVALID, "%s", "be_step_n needs actions and steps >= 0");
  if (!out || !out->reward || !out->done) return fail(ctx, BE_E_INVALID, "%s", "be_step_n needs out->reward and out->done");
  if (steps == 0) return BE_OK;
  KParams a = make_params(ctx, st, out);
  a.actions = actions;
  return launch(ctx, MODE_STEP, a, stream, steps);
}

int be_rollout(be_ctx* ctx, const be_state* st, const uint8_t* actions, int32_t steps, const be_out* out,
               void* stream) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (int rc = check_state(ctx, st)) return rc;
  if (!actions || steps < 0) return fail(ctx, BE_E_INVALID, "%s", "be_rollout needs actions and steps >= 0");
  if (!out || !out->obs || !out->reward || !out->done)
    return fail(ctx, BE_E_INVALID, "%s", "be_rollout needs out->obs, out->reward and out->done");
  if (out->obs_f32) return fail(ctx, BE_E_INVALID, "%s", "be_rollout writes u8 obs only (obs_f32 must be NULL)");
  const int64_t N = ctx->cfg.num_envs, F = 4 + (int64_t)ctx->cfg.window * ctx->cfg.window;
  if (((uintptr_t)out->obs & 15) || (N * F) % 16)
    return fail(ctx, BE_E_INVALID, "%s", "be_rollout needs a 16-byte aligned obs and num_envs * (4+W*W) % 16 == 0");
  if (steps == 0) return BE_OK;
  const Launch L = pick_rollout(ctx->cfg, !ctx->generic_only && ctx->unit_moves && ctx->distinct_goals, ctx->roll5_lpe);
  bool fused = false;
  {   // every HIP query (fits_lds' function attributes) on the context's device
    const DeviceGuard dg(ctx->device);   // the caller's current device is restored on return
    HIP_TRY(ctx, dg.err);
    fused = fits_lds(ctx, L);
  }
  if (fused) {
    KParams a = make_params(ctx, st, out);
    a.actions = actions; a.steps = steps;
    const DeviceGuard dg(ctx->device);   // the caller's current device is restored on return
    HIP_TRY(ctx, dg.err);
    const dim3 grid((unsigned)((N + L.epb - 1) / L.epb)), block((unsigned)L.threads);
    hipLaunchKernelGGL(L.fn, grid, block, (size_t)L.lds, (hipStream_t)stream, a);
    HIP_TRY(ctx, hipGetLastError());
    return BE_OK;
  }
  // any other config: one be_step per step into the (steps, N, ...) slices (same results)
  for (int32_t s = 0; s < steps; ++s) {
    be_out o = *out;
    o.obs = out->obs + s * N * F;
    o.reward = out->reward + s * N;
    o.done = out->done + s * N;
    if (o.truncated) o.truncated = out->truncated + s * N;
    if (o.terminal_obs) o.terminal_obs = out->terminal_obs + s * N * F;
    if (o.final_return) o.final_return = out->final_return + s * N;
    if (o.final_len) o.final_len = out->final_len + s * N;
    if (int rc = be_step(ctx, st, actions + s * N, nullptr, nullptr, &o, stream)) return rc;
  }
  return BE_OK;
}

}  // extern "C"

int be_internal_policy_rollout(be_ctx* ctx, const be_state* st, const be_pol_rollout_args* r, void* stream) {
  const Launch L = pick_policy_rollout(ctx->cfg, !ctx->generic_only && ctx->unit_moves && ctx->distinct_goals, r->HT,
                                       r->KS, r->NO);
  const DeviceGuard dg(ctx->device);   // the caller's current device is restored on return; every
  HIP_TRY(ctx, dg.err);                // HIP query below (fits_lds) runs on the context's device
  if (!fits_lds(ctx, L)) return 0;   // the caller loops select_action + be_step instead
  KParams a = make_params(ctx, st, r->out);
  a.steps = r->steps;
  a.pol_bytes = r->img_bytes; a.pol_actions = r->num_actions; a.pol_img = r->img; a.pol_seed = r->seed;
  a.obs_in = r->obs_in; a.obs_last = r->obs_last;
  a.act_out = r->act->action; a.logp_out = r->act->log_prob; a.value_out = r->act->value;
  const int N = ctx->cfg.num_envs;
  const dim3 grid((unsigned)((N + L.epb - 1) / L.epb)), block((unsigned)BLOCK_THREADS);
  hipLaunchKernelGGL(L.fn, grid, block, (size_t)L.lds, (hipStream_t)stream, a);
  HIP_TRY(ctx, hipGetLastError());
  return 1;
}

extern "C" {

int be_observe(be_ctx* ctx, const be_state* st, const be_out* out, void* stream) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (int rc = check_state(ctx, st)) return rc;
  if (!out || (!out->obs && !out->obs_f32)) return fail(ctx, BE_E_INVALID, "%s", "be_observe needs out->obs or out->obs_f32");
  KParams a = make_params(ctx, st, out);
  a.reward = nullptr; a.done = nullptr; a.truncated = nullptr; a.terminal_obs = nullptr;
  a.final_return = nullptr; a.final_len = nullptr; a.stats = nullptr;
  return launch(ctx, MODE_OBSERVE, a, stream);
}

int be_sample_actions(be_ctx* ctx, uint8_t* actions_out, int32_t steps, uint64_t seed, void* stream) {
  if (!ctx || !actions_out || steps < 0) return fail(ctx, BE_E_INVALID, "%s", "bad arguments to be_sample_actions");
  if (steps == 0) return BE_OK;
  const DeviceGuard dg(ctx->device);   // the caller's current device is restored on return
  HIP_TRY(ctx, dg.err);
  const int64_t total = (int64_t)ctx->cfg.num_envs * steps;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(sample_actions_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, actions_out,
                     ctx->cfg.num_envs, steps, ctx->cfg.env_offset, ctx->cfg.num_actions, (unsigned long long)seed);
  HIP_TRY(ctx, hipGetLastError());
  return BE_OK;
}

// ---- env-state checkpoint: header + the be_state arrays at 16-byte aligned offsets
struct BlobLayout { int64_t off[10], bytes[10], total; };
static BlobLayout blob_layout(const be_config* c) {
  BlobLayout b;
  const int64_t N = c->num_envs, ns = c->num_static, nd = c->num_dynamic;
  const int64_t sz[10] = {4 * N, 4 * N, 8 * N, 8 * N, 8 * N, 4 * N, 4 * N, 4 * ns * N, 4 * nd * N, nd * N};
  int64_t o = 64;
  for (int k = 0; k < 10; ++k) { b.off[k] = o; b.bytes[k] = sz[k]; o += (sz[k] + 15) & ~15ll; }
  b.total = o;
  return b;
}
static void blob_header(const be_config* c, int64_t total, int64_t (&hdr)[8]) {
  memset(hdr, 0, sizeof hdr);
  memcpy(&hdr[0], "BALLENV1", 8);
  hdr[1] = BE_ABI_VERSION; hdr[2] = c->num_envs; hdr[3] = c->num_static; hdr[4] = c->num_dynamic; hdr[5] = total;
}
static void state_ptrs(const be_state* st, void* (&p)[10]) {
  p[0] = st->agent; p[1] = st->goal; p[2] = st->prev_dist; p[3] = st->total_dist; p[4] = st->ep_return;
  p[5] = st->ep_len; p[6] = st->episode; p[7] = st->static_obs; p[8] = st->dyn_obs; p[9] = st->dyn_goal;
}

int64_t be_state_blob_bytes(const be_config* cfg) {
  if (!cfg || cfg->num_envs < 1) return 0;
  return blob_layout(cfg).total;
}

int be_save_state(be_ctx* ctx, const be_state* st, void* blob, void* stream) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (int rc = check_state(ctx, st)) return rc;
  if (!blob) return fail(ctx, BE_E_INVALID, "%s", "blob is NULL");
  const DeviceGuard dg(ctx->device);   // the caller's current device is restored on return
  HIP_TRY(ctx, dg.err);
  const BlobLayout L = blob_layout(&ctx->cfg);
  blob_header(&ctx->cfg, L.total, ctx->blob_hdr);   // lives in the context: safe for an async copy
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(ctx, hipMemcpyAsync(blob, ctx->blob_hdr, sizeof ctx->blob_hdr, hipMemcpyDefault, s));
  void* src[10];
  state_ptrs(st, src);
  for (int k = 0; k < 10; ++k)
    if (L.bytes[k] > 0)
      HIP_TRY(ctx, hipMemcpyAsync(static_cast<char*>(blob) + L.off[k], src[k], (size_t)L.bytes[k], hipMemcpyDefault, s));
  return BE_OK;
}

int be_load_state(be_ctx* ctx, const be_state* st, const void* blob, void* stream) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (int rc = check_state(ctx, st)) return rc;
  if (!blob) return fail(ctx, BE_E_INVALID, "%s", "blob is NULL");
  const DeviceGuard dg(ctx->device);   // the caller's current device is restored on return
  HIP_TRY(ctx, dg.err);
  const BlobLayout L = blob_layout(&ctx->cfg);
  hipStream_t s = (hipStream_t)stream;
  int64_t got[8], want[8];
  HIP_TRY(ctx, hipMemcpyAsync(got, blob, sizeof got, hipMemcpyDefault, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  blob_header(&ctx->cfg, L.total, want);
  if (memcmp(got, want, sizeof got) != 0)
    return fail(ctx, BE_E_INVALID, "%s", "state blob header does not match this context (magic, ABI, N, Ns, Nd)");
  void* dst[10];
  state_ptrs(st, dst);
  for (int k = 0; k < 10; ++k)
    if (L.bytes[k] > 0)
      HIP_TRY(ctx, hipMemcpyAsync(dst[k], static_cast<const char*>(blob) + L.off[k], (size_t)L.bytes[k], hipMemcpyDefault, s));
  if (ctx->pool) {   // the loaded episodes' next entries (the pool's entries need no invalidation:
                     // each is a pure function of (seed, global id, episode) and is checked by its tag)
    ctx->pool_owner = st->episode;
    launch_pool_fill(ctx, make_params(ctx, st, nullptr), stream);
    HIP_TRY(ctx, hipGetLastError());
  }
  return BE_OK;
}

int be_pool_fill(be_ctx* ctx, const be_state* st, void* stream) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (int rc = check_state(ctx, st)) return rc;
  if (!ctx->pool) return BE_OK;
  const DeviceGuard dg(ctx->device);
  HIP_TRY(ctx, dg.err);
  ctx->pool_owner = st->episode;
  launch_pool_fill(ctx, make_params(ctx, st, nullptr), stream);
  HIP_TRY(ctx, hipGetLastError());
  return BE_OK;
}

int be_pool_invalidate(be_ctx* ctx, void* stream) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (!ctx->pool) return BE_OK;
  const DeviceGuard dg(ctx->device);
  HIP_TRY(ctx, dg.err);
  HIP_TRY(ctx, hipMemsetAsync(ctx->pool, 0, (size_t)ctx->pool_bytes, (hipStream_t)stream));
  return BE_OK;
}

int be_pool_set_period(be_ctx* ctx, int32_t period) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (period < 0) return fail(ctx, BE_E_INVALID, "%s", "pool period must be >= 0");
  ctx->pool_period = period;
  ctx->pool_calls = 0;
  return BE_OK;
}

int64_t be_pool_bytes(const be_ctx* ctx) { return ctx && ctx->pool ? ctx->pool_bytes : 0; }

int32_t be_pool_period(const be_ctx* ctx) { return ctx ? ctx->pool_period : 0; }

int be_pool_entry(be_ctx* ctx, int32_t env, int32_t slot, uint32_t* words, double* f64, int32_t write) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (!ctx->pool) return fail(ctx, BE_E_INVALID, "%s", "this context has no autoreset pool");
  if (env < 0 || env >= ctx->cfg.num_envs || slot < 0 || slot > 1 || !words || !f64)
    return fail(ctx, BE_E_INVALID, "%s", "bad arguments to be_pool_entry");
  const DeviceGuard dg(ctx->device);
  HIP_TRY(ctx, dg.err);
  HIP_TRY(ctx, hipDeviceSynchronize());
  // the header's word order (TAG, AGENT, GOAL, ROWS0 | flags << 30, ROWS1, ROWS2, obstacles) from / to
  // the tags array and the entry body
  const int64_t n = ctx->cfg.num_envs, x = (int64_t)slot * n + env;
  constexpr int NBW = pool_body_words(FIX_NS, FIX_ND), NO = FIX_NS + FIX_ND;
  char* tv = reinterpret_cast<char*>(ctx->pool) + x * 8;
  char* body = reinterpret_cast<char*>(ctx->pool) + 16 * n + x * 4 * NBW;
  uint32_t t[2], b[NBW];
  HIP_TRY(ctx, hipMemcpy(t, tv, sizeof t, hipMemcpyDeviceToHost));
  HIP_TRY(ctx, hipMemcpy(b, body, sizeof b, hipMemcpyDeviceToHost));
  if (!write) {
    words[0] = t[0]; words[1] = b[PB_AGENT]; words[2] = b[PB_GOAL];
    words[3] = (b[PB_ROWS] & 0x3FFFFFFFu) | ((t[1] & 3u) << 30);
    words[4] = b[PB_ROWS + 1]; words[5] = b[PB_ROWS + 2];
    for (int k = 0; k < NO; ++k) words[6 + k] = b[PB_OBS + k];
    memcpy(&f64[0], &b[PB_PREV], 8);
    memcpy(&f64[1], &b[PB_TOTAL], 8);
    return BE_OK;
  }
  t[0] = words[0]; t[1] = (words[3] >> 30) & 3u;
  b[PB_AGENT] = words[1]; b[PB_GOAL] = words[2];
  b[PB_ROWS] = words[3] & 0x3FFFFFFFu; b[PB_ROWS + 1] = words[4]; b[PB_ROWS + 2] = words[5];
  for (int k = 0; k < NO; ++k) b[PB_OBS + k] = words[6 + k];
  memcpy(&b[PB_PREV], &f64[0], 8);
  memcpy(&b[PB_TOTAL], &f64[1], 8);
  HIP_TRY(ctx, hipMemcpy(tv, t, sizeof t, hipMemcpyHostToDevice));
  HIP_TRY(ctx, hipMemcpy(body, b, sizeof b, hipMemcpyHostToDevice));
  return BE_OK;
}

int be_status(be_ctx* ctx, int32_t* status_out, void* stream) {
  if (!ctx || !status_out) return fail(ctx, BE_E_INVALID, "%s", "bad arguments to be_status");
  const DeviceGuard dg(ctx->device);   // the caller's current device is restored on return
  HIP_TRY(ctx, dg.err);
  HIP_TRY(ctx, hipStreamSynchronize((hipStream_t)stream));
  int v = 0;
  HIP_TRY(ctx, hipMemcpy(&v, ctx->status, sizeof v, hipMemcpyDeviceToHost));
  const int zero = 0;
  HIP_TRY(ctx, hipMemcpy(ctx->status, &zero, sizeof zero, hipMemcpyHostToDevice));
  *status_out = v;
  return BE_OK;
}

}  // extern "C"
