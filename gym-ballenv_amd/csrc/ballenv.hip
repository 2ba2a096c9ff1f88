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
// Memory: every per-env word the step needs is loaded up front (obstacles in
// register chunks of 16 static / 8 dynamic), so a wave has ~30 independent
// loads in flight instead of a chain of dependent HBM round trips.  There is
// no cross-block communication at all: randomness is Philox keyed by per-env
// state (global env id, episode, ep_len), so no global counter or atomics.
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
#include <hip/hip_runtime.h>

#include <math.h>
#include <new>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "ballenv.h"

namespace {

// Philox purposes (counter word 3, high byte); oracle/ballenv_oracle.c uses the same.
constexpr uint32_t PURPOSE_STEP_OBS = 1, PURPOSE_ACTION = 2, PURPOSE_RESET = 3, PURPOSE_SAMPLE = 4;
constexpr int REJECT_LIMIT = 4096;
constexpr int CS = 16;  // static obstacles per register chunk
constexpr int CD = 8;   // dynamic obstacles per register chunk

enum Mode { MODE_STEP = 0, MODE_RESET = 1, MODE_OBSERVE = 2 };

// Host-precomputed lookup tables (read from the kernarg segment).
struct Tables {
  int32_t goal[BE_MAX_GOALS];                 // packed goal xy
  int32_t action[BE_MAX_ACTIONS];             // packed (dx, dy)
  uint8_t n_other[BE_MAX_GOALS];              // goals with a different value than goal g
  uint8_t other[BE_MAX_GOALS][BE_MAX_GOALS];  // pick -> goal index, per current goal g (newGoalList)
};

struct KArgs {
  be_config c;
  Tables t;
  be_state st;
  be_out out;
  const uint8_t* actions;
  const int16_t* deltas;
  const int16_t* tape;        // (Nd, 2, N) step draw tape or NULL
  const uint8_t* mask;        // reset mask or NULL
  const int16_t* reset_tape;  // (L, N) or NULL
  int32_t reset_tape_len;
  int* status;
};

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
__device__ __forceinline__ int isqrt_small(int n) {  // floor(sqrt(n)), 0 <= n < 2^22
  int s = (int)__builtin_amdgcn_sqrtf((float)n);
  if (s * s > n) --s;
  if ((s + 1) * (s + 1) <= n) ++s;
  return s;
}
__device__ __forceinline__ int floordiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

struct u4 { uint32_t x, y, z, w; };

// Philox4x32-10 (Salmon et al., SC'11); same as oracle/ballenv_oracle.c
__device__ __forceinline__ u4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, unsigned long long seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return u4{c0, c1, c2, c3};
}
__device__ __forceinline__ uint32_t tag(uint32_t purpose, uint32_t sub) { return (purpose << 24) | (sub & 0xFFFFFFu); }
__device__ __forceinline__ uint32_t pick_word(const u4& b, int w) {
  return w == 0 ? b.x : (w == 1 ? b.y : (w == 2 ? b.z : b.w));
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

__device__ __forceinline__ double calc_dist(int x1, int y1, int x2, int y2) {
  // math.sqrt(math.pow(dx,2)+math.pow(dy,2)): the squares are exact integers in f64
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
  __device__ Win(const be_config& c, int ax, int ay) {
    w = c.window; int h = w / 2;
    sx = c.speed_x; sy = c.speed_y;
    x0 = ax - sx * h; y0 = ay - sy * h;
    kr = w > 1 ? w - 1 : 1;
    R = c.radius_obstacle + c.radius_agent; R2 = R * R;
  }
  // Can obstacle (ox,oy) light any cell?  (f, e) = its window-relative position.
  __device__ __forceinline__ bool near(int ox, int oy, int& f, int& e) const {
    f = ox - x0; e = oy - y0;
    int cx = min(max(f, 0), sx * (w - 1));
    int cy = min(max(e, 0), sy * (kr - 1));
    return d2u(f - cx, e - cy) <= (uint32_t)R2;
  }
};

__device__ __forceinline__ int quadrant(int ax, int ay, int gx, int gy) {
  // prep_state2, examples/ball_cnn_ac3.py:343-351
  int dx = gx - ax, dy = gy - ay;
  if (dx >= 0 && dy >= 0) return 1;
  if (dx < 0 && dy >= 0) return 0;
  if (dx < 0 && dy < 0) return 3;
  return 2;
}

// Per-thread list of window-relevant obstacles in LDS, laid out [slot][BLOCK].
template <int BLOCK>
struct NearList {
  uint32_t* base; int cnt;
  __device__ __forceinline__ void push(int f, int e) {
    base[cnt * BLOCK] = (uint32_t)(f & 0xFFFF) | ((uint32_t)e << 16);
    ++cnt;
  }
  __device__ __forceinline__ void get(int n, int& f, int& e) const {
    uint32_t v = base[n * BLOCK];
    f = (int)(int16_t)(v & 0xFFFF); e = (int)v >> 16;
  }
};

template <int WT> struct Geo {
  static constexpr int K = WT > 1 ? WT - 1 : 1;       // distinct rows
  static constexpr int NW = (WT * WT + 31) / 32 + 1;  // flat cell words (+1 spill word)
  static constexpr int F = 4 + WT * WT;
};

// Rasterise the near list into K row bitmasks (compile-time W).
template <int WT, int BLOCK>
__device__ __forceinline__ void raster_rows(const NearList<BLOCK>& nl, const Win& g, uint32_t (&rows)[Geo<WT>::K]) {
  constexpr int K = Geo<WT>::K;
#pragma unroll
  for (int k = 0; k < K; ++k) rows[k] = 0u;
  for (int n = 0; n < nl.cnt; ++n) {
    int f, e;
    nl.get(n, f, e);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      int ady = abs(e - g.sy * k);
      if (ady <= g.R) {
        int hw = isqrt_small(g.R2 - ady * ady);
        int lo, hi;
        if (g.sx == 1) { lo = f - hw; hi = f + hw; }
        else { lo = -floordiv(hw - f, g.sx); hi = floordiv(f + hw, g.sx); }
        lo = max(lo, 0); hi = min(hi, WT - 1);
        if (lo <= hi) rows[k] |= (2u << hi) - (1u << lo);
      }
    }
  }
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
      uint32_t nib = (flat[j >> 5] >> (j & 31)) & 0xFu;
      dst[w] = (nib * 0x00204081u) & 0x01010101u;
    }
  } else {
    uint8_t* dst = stage + tid * F;
#pragma unroll
    for (int b = 0; b < F; ++b) dst[b] = (uint8_t)obs_byte<WT>(flat, quad, b);
  }
}

// Copy the block's staged rows to obs (u8) and/or obs_f32 with 16-byte stores.
template <int BLOCK>
__device__ __forceinline__ void copy_out(const uint8_t* stage, int F, int nvalid, int64_t row0,
                                         uint8_t* obs, float* obs_f32) {
  const int tid = threadIdx.x;
  const int bytes = nvalid * F;
  if (obs) {
    uint8_t* dst = obs + row0 * F;
    const int nv = bytes >> 4;
    for (int v = tid; v < nv; v += BLOCK)
      reinterpret_cast<uint4*>(dst)[v] = reinterpret_cast<const uint4*>(stage)[v];
    for (int b = (nv << 4) + tid; b < bytes; b += BLOCK) dst[b] = stage[b];
  }
  if (obs_f32) {
    float* dst = obs_f32 + row0 * F;
    const int nv = bytes >> 2;
    for (int v = tid; v < nv; v += BLOCK) {
      uint32_t q = reinterpret_cast<const uint32_t*>(stage)[v];
      reinterpret_cast<float4*>(dst)[v] =
          make_float4((float)(q & 0xFF), (float)((q >> 8) & 0xFF), (float)((q >> 16) & 0xFF), (float)(q >> 24));
    }
    for (int b = (nv << 2) + tid; b < bytes; b += BLOCK) dst[b] = (float)stage[b];
  }
}

// Generic-W (runtime W, no staging) obs writer: per cell over the near list.
template <int BLOCK>
__device__ void write_row_generic(const NearList<BLOCK>& nl, const Win& g, int quad, uint8_t* row, float* rowf) {
  for (int b = 0; b < 4; ++b) {
    if (row) row[b] = (uint8_t)(b == quad);
    if (rowf) rowf[b] = (float)(b == quad);
  }
  for (int r = 0; r < g.w; ++r) {
    int k = r > 0 ? r - 1 : 0;
    for (int cc = 0; cc < g.w; ++cc) {
      int hit = 0;
      for (int n = 0; n < nl.cnt && !hit; ++n) {
        int f, e;
        nl.get(n, f, e);
        hit = d2u(f - g.sx * cc, e - g.sy * k) <= (uint32_t)g.R2;
      }
      int b = 4 + r * g.w + cc;
      if (row) row[b] = (uint8_t)hit;
      if (rowf) rowf[b] = (float)hit;
    }
  }
}

// ------------------------------------------------------------------ reset
// BallEnv.reset for one env (ballenv_env.py:113-167); also rebuilds the near list.
template <int BLOCK>
__device__ void reset_env(const KArgs& p, int i, ResetDraws& ds, int& ax, int& ay, int& gx, int& gy,
                          NearList<BLOCK>& nl) {
  const be_config& c = p.c;
  const int N = c.num_envs, W = c.screen_width, H = c.screen_height;
  gx = ds.draw(W - c.strip_goal_x, W);                                  // :115
  gy = ds.draw(H - c.strip_goal_y, H);                                  // :116
  ax = ds.draw(0, c.strip_agent_x);                                     // :117
  ay = ds.draw(0, c.strip_agent_y);                                     // :118
  const double dist = calc_dist(gx, gy, ax, ay);                        // :119
  for (int guard = 0; calc_dist(gx, gy, ax, ay) < c.min_spawn_dist;) {  // :121-126
    if (++guard > REJECT_LIMIT) { atomicOr(p.status, BE_STATUS_REJECTION_LIMIT); break; }
    ax = ds.draw(0, c.strip_agent_x);
    ay = ds.draw(0, c.strip_agent_y);
  }
  p.st.agent[i] = pk(ax, ay);
  p.st.goal[i] = pk(gx, gy);
  p.st.prev_dist[i] = dist;  // state[2] keeps the pre-resample distance (Q9)
  p.st.total_dist[i] = calc_dist(ax, ay, gx, gy);                       // :166
  p.st.ep_return[i] = 0.0;
  p.st.ep_len[i] = 0;
  p.st.episode[i] = ds.episode;
  Win g(c, ax, ay);
  nl.cnt = 0;
  // check_overlap_rect (:193-197): |dx| < rad + r_a and |dy| < rad/2 + r_a  <=>  2|dy| < rad + 2 r_a
  const int rx = c.radius_obstacle + c.radius_agent, ry2 = c.radius_obstacle + 2 * c.radius_agent;
  for (int k = 0; k < c.num_static; ++k) {                              // :131-149
    int ox = 0, oy = 0;
    for (int guard = 0;;) {
      ox = ds.draw(c.strip_obs_x, W - c.strip_obs_x);                   // obstacles.__init__ :24-25
      oy = ds.draw(c.strip_obs_y, H - c.strip_obs_y);
      const bool ra = abs(ox - ax) < rx && 2 * abs(oy - ay) < ry2;
      const bool rg = abs(ox - gx) < rx && 2 * abs(oy - gy) < ry2;
      if (!ra && !rg) break;
      if (++guard > REJECT_LIMIT) { atomicOr(p.status, BE_STATUS_REJECTION_LIMIT); break; }
    }
    p.st.static_obs[(int64_t)k * N + i] = pk(ox, oy);
    int f, e;
    if (g.near(ox, oy, f, e)) nl.push(f, e);
  }
  for (int k = 0; k < c.num_dynamic; ++k) {                             // :153-164
    const int ox = ds.draw(c.strip_obs_x, W - c.strip_obs_x);
    const int oy = ds.draw(c.strip_obs_y, H - c.strip_obs_y);
    p.st.dyn_obs[(int64_t)k * N + i] = pk(ox, oy);
    p.st.dyn_goal[(int64_t)k * N + i] = (uint8_t)k;                    // curr_goal = goal list[k]
    int f, e;
    if (g.near(ox, oy, f, e)) nl.push(f, e);
  }
}

// ------------------------------------------------------------------ statistics
__device__ __forceinline__ void atomic_min_f64(double* a, double v) {
  unsigned long long* u = reinterpret_cast<unsigned long long*>(a);
  unsigned long long old = *u;
  while (v < __longlong_as_double((long long)old)) {
    unsigned long long prev = atomicCAS(u, old, (unsigned long long)__double_as_longlong(v));
    if (prev == old) break;
    old = prev;
  }
}
__device__ __forceinline__ void atomic_max_f64(double* a, double v) {
  unsigned long long* u = reinterpret_cast<unsigned long long*>(a);
  unsigned long long old = *u;
  while (v > __longlong_as_double((long long)old)) {
    unsigned long long prev = atomicCAS(u, old, (unsigned long long)__double_as_longlong(v));
    if (prev == old) break;
    old = prev;
  }
}

// Wave-level reduction of finished-episode statistics (called by all 64 lanes).
__device__ void wave_stats(double* stats, bool done, double ret, int len) {
  const unsigned long long m = __ballot(done);
  if (m == 0ull) return;  // wave-uniform: nobody finished (the common case)
  double s1 = done ? ret : 0.0, s2 = done ? ret * ret : 0.0, sl = done ? (double)len : 0.0;
  double mn = done ? ret : INFINITY, mx = done ? ret : -INFINITY;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o); s2 += __shfl_xor(s2, o); sl += __shfl_xor(sl, o);
    mn = fmin(mn, __shfl_xor(mn, o)); mx = fmax(mx, __shfl_xor(mx, o));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&stats[0], (double)__popcll(m));
    atomicAdd(&stats[1], s1); atomicAdd(&stats[2], s2); atomicAdd(&stats[3], sl);
    atomic_min_f64(&stats[4], mn); atomic_max_f64(&stats[5], mx);
  }
}

constexpr int block_for(int WT) {
  return WT == 0 ? 64 : ((4 + WT * WT) <= 256 ? 256 : ((4 + WT * WT) <= 512 ? 128 : 64));
}

// One dynamic obstacle's move_obstacles (ballenv_env.py:323-353).  d0/d1 are
// the values of its first/second randint call (tape or Philox mapped below).
struct DynMove {
  __device__ static void apply(const KArgs& p, int64_t a, int& ox, int& oy, int gi, int speed, bool change,
                               bool tape, int t0, int t1, uint32_t w0, uint32_t w1) {
    const be_config& c = p.c;
    if (!change) {
      const int32_t gp = p.t.goal[gi];
      const int tx = px(gp) - ox, ty = py(gp) - oy;
      int mv;  // -1 = directed move toward the current goal
      if (tx != 0 && ty != 0) {
        const int u = tape ? t0 : map_range(w0, 0, 100);
        mv = u < c.obs_certainty ? -1 : (tape ? t1 : map_range(w1, 0, 9));
      } else {
        mv = tape ? t0 : map_range(w0, 0, 9);
      }
      int mx, my;
      if (mv < 0) { mx = tx > 0 ? 1 : -1; my = ty > 0 ? 1 : -1; }
      else {  // move_list of ballenv_env.py:324: (-1,-1) twice, no (-1,0) (Q4)
        mx = mv < 3 ? 1 : (mv < 6 ? 0 : -1);
        const int r3 = mv - 3 * (mv / 3);
        my = mv == 8 ? -1 : (r3 == 0 ? 1 : (r3 == 1 ? -1 : 0));
      }
      ox += mx * speed; oy += my * speed;
      if (ox < -32768 || ox > 32767 || oy < -32768 || oy > 32767) atomicOr(p.status, BE_STATUS_COORD_RANGE);
      p.st.dyn_obs[a] = pk(ox, oy);
    } else {  // new goal from the other goals; no move this step (Q5)
      const int n_other = p.t.n_other[gi];
      if (n_other == 0) atomicOr(p.status, BE_STATUS_NO_GOAL);
      else p.st.dyn_goal[a] = p.t.other[gi][tape ? t0 : map_range(w0, 0, n_other)];
    }
  }
};

// ------------------------------------------------------------------ the kernel
// MODE_STEP: physics + (autoreset) + obs.  MODE_RESET: reset masked envs + obs.
// MODE_OBSERVE: obs only.  WT = compile-time W (0 = runtime W, no LDS staging).
template <int WT, int MODE>
__global__ __launch_bounds__(block_for(WT)) void be_kernel(KArgs p) {
  constexpr int BLOCK = block_for(WT);
  extern __shared__ __align__(16) uint8_t smem[];

  const be_config& c = p.c;
  const int N = c.num_envs, Ns = c.num_static, Nd = c.num_dynamic;
  const int tid = threadIdx.x;
  const int i = blockIdx.x * BLOCK + tid;
  const bool valid = i < N;

  NearList<BLOCK> nl{reinterpret_cast<uint32_t*>(smem) + tid, 0};
  int ax = 0, ay = 0, gx = 0, gy = 0;
  bool done = false;
  double fin_ret = 0.0;
  int fin_len = 0;
  uint32_t episode = 0;
  const uint32_t gid = (uint32_t)(c.env_offset + i);

  if (valid) {
    if (MODE == MODE_STEP) {
      // ---- issue every load of this env first (independent, coalesced across the wave)
      int a = 0, dx = 0, dy = 0;
      if (p.actions) a = p.actions[i];
      else if (p.deltas) { dx = p.deltas[2 * (int64_t)i]; dy = p.deltas[2 * (int64_t)i + 1]; }
      const int32_t agent0 = p.st.agent[i];
      const int32_t goal0 = p.st.goal[i];
      const double old_dist = p.st.prev_dist[i];
      const double total = p.st.total_dist[i];
      double ret = p.st.ep_return[i];
      const int len0 = p.st.ep_len[i];
      episode = p.st.episode[i];
      const int ns0 = min(Ns, CS), nd0 = min(Nd, CD);
      int32_t so[CS], dp[CD];
      int dgi[CD], t0[CD], t1[CD];
#pragma unroll
      for (int k = 0; k < CS; ++k) so[k] = k < ns0 ? p.st.static_obs[(int64_t)k * N + i] : 0;
#pragma unroll
      for (int k = 0; k < CD; ++k) {
        dp[k] = k < nd0 ? p.st.dyn_obs[(int64_t)k * N + i] : 0;
        dgi[k] = k < nd0 ? p.st.dyn_goal[(int64_t)k * N + i] : 0;
        t0[k] = (p.tape && k < nd0) ? p.tape[(int64_t)(2 * k) * N + i] : 0;
        t1[k] = (p.tape && k < nd0) ? p.tape[(int64_t)(2 * k + 1) * N + i] : 0;
      }

      // ---- action -> agent move + clamp (ballenv_env.py:247-259)
      if (p.actions) {
        if (a >= c.num_actions) { atomicOr(p.status, BE_STATUS_BAD_ACTION); a = 0; }
        const int32_t m = p.t.action[a]; dx = px(m); dy = py(m);
      } else if (!p.deltas) {  // sampled actions
        const u4 b = philox(gid, episode, (uint32_t)len0, tag(PURPOSE_ACTION, 0), c.seed);
        const int32_t m = p.t.action[map_range(b.x, 0, c.num_actions)]; dx = px(m); dy = py(m);
      }
      gx = px(goal0); gy = py(goal0);
      ax = min(max(px(agent0) + c.speed_x * dx, 0), c.screen_width);
      ay = min(max(py(agent0) + c.speed_y * dy, 0), c.screen_height);
      const Win g(c, ax, ay);
      const uint32_t R2 = (uint32_t)g.R2;
      bool hs = false, hd = false;

      // ---- dynamic obstacles: move (counter == ep_len mod (G+1): all start at 0 on reset)
      const int counter = len0 % (c.goal_change_step + 1);
      const bool change = counter >= c.goal_change_step;
      const bool tape = p.tape != nullptr;
      u4 blk{0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < CD; ++k) {
        if (k < nd0) {
          // Philox block k>>1 holds both draws of obstacles 2j and 2j+1
          if (!tape && (k & 1) == 0) blk = philox(gid, episode, (uint32_t)len0, tag(PURPOSE_STEP_OBS, k >> 1), c.seed);
          int ox = px(dp[k]), oy = py(dp[k]);
          DynMove::apply(p, (int64_t)k * N + i, ox, oy, dgi[k], c.obstacle_speed[k], change, tape, t0[k], t1[k],
                         (k & 1) ? blk.z : blk.x, (k & 1) ? blk.w : blk.y);
          hd |= d2u(ox - ax, oy - ay) <= R2;
          int f, e;
          if (g.near(ox, oy, f, e)) nl.push(f, e);
        }
      }
      for (int kb = CD; kb < Nd; ++kb) {  // configs with more than CD dynamic obstacles
        const int64_t aa = (int64_t)kb * N + i;
        int ox = px(p.st.dyn_obs[aa]), oy = py(p.st.dyn_obs[aa]);
        if (!tape && (kb & 1) == 0) blk = philox(gid, episode, (uint32_t)len0, tag(PURPOSE_STEP_OBS, kb >> 1), c.seed);
        const int tt0 = tape ? p.tape[(int64_t)(2 * kb) * N + i] : 0, tt1 = tape ? p.tape[(int64_t)(2 * kb + 1) * N + i] : 0;
        DynMove::apply(p, aa, ox, oy, p.st.dyn_goal[aa], c.obstacle_speed[kb], change, tape, tt0, tt1,
                       (kb & 1) ? blk.z : blk.x, (kb & 1) ? blk.w : blk.y);
        hd |= d2u(ox - ax, oy - ay) <= R2;
        int f, e;
        if (g.near(ox, oy, f, e)) nl.push(f, e);
      }
      // ---- static obstacles: collision + near test
#pragma unroll
      for (int k = 0; k < CS; ++k) {
        if (k < ns0) {
          const int ox = px(so[k]), oy = py(so[k]);
          hs |= d2u(ox - ax, oy - ay) <= R2;
          int f, e;
          if (g.near(ox, oy, f, e)) nl.push(f, e);
        }
      }
      for (int kb = CS; kb < Ns; ++kb) {
        const int32_t o = p.st.static_obs[(int64_t)kb * N + i];
        const int ox = px(o), oy = py(o);
        hs |= d2u(ox - ax, oy - ay) <= R2;
        int f, e;
        if (g.near(ox, oy, f, e)) nl.push(f, e);
      }

      // ---- distance, reward, done (ballenv_env.py:268-286, 200-229)
      const double dist = calc_dist(gx, gy, ax, ay);
      double reward = 0.0 - c.time_penalty;
      reward += (old_dist - dist) / total;
      if (hs) reward -= c.static_penalty;          // statics come first in obstacle_list (Q3)
      else if (hd) reward -= c.dynamic_penalty;
      ret += reward;
      const int len = len0 + 1;
      const bool env_done = (dist < c.threshold_goal) || hs || hd;
      const bool trunc = c.time_limit > 0 && len >= c.time_limit;
      done = env_done || trunc;
      p.out.reward[i] = reward;
      p.out.done[i] = (uint8_t)done;
      if (p.out.truncated) p.out.truncated[i] = (uint8_t)(trunc && !env_done);
      p.st.agent[i] = pk(ax, ay);
      p.st.prev_dist[i] = dist;
      p.st.ep_return[i] = ret;
      p.st.ep_len[i] = len;
      if (done) {
        if (p.out.final_return) p.out.final_return[i] = ret;
        if (p.out.final_len) p.out.final_len[i] = len;
      }
      fin_ret = ret; fin_len = len;
    } else {
      const int32_t agent0 = p.st.agent[i];
      const int32_t goal0 = p.st.goal[i];
      ax = px(agent0); ay = py(agent0); gx = px(goal0); gy = py(goal0);
      if (MODE == MODE_RESET) episode = p.st.episode[i];
    }
  }
  if (MODE == MODE_STEP && p.out.stats) wave_stats(p.out.stats, done, fin_ret, fin_len);  // all lanes converged

  // ---- episode boundary: terminal obs + reset (rare, divergent)
  bool do_reset = false;
  if (valid) {
    if (MODE == MODE_STEP) do_reset = done && c.autoreset;
    if (MODE == MODE_RESET) do_reset = p.mask ? (p.mask[i] != 0) : true;
  }
  if (valid && do_reset) {
    if (MODE == MODE_STEP && p.out.terminal_obs) {
      const int F = 4 + c.window * c.window;
      const Win g(c, ax, ay);
      const int quad = quadrant(ax, ay, gx, gy);
      if constexpr (WT > 0) {
        uint32_t rows[Geo<WT>::K], flat[Geo<WT>::NW];
        raster_rows<WT, BLOCK>(nl, g, rows);
        flatten<WT>(rows, flat);
        write_row_global<WT>(p.out.terminal_obs + (int64_t)i * F, flat, quad);
      } else {
        write_row_generic<BLOCK>(nl, g, quad, p.out.terminal_obs + (int64_t)i * F, nullptr);
      }
    }
    ResetDraws ds{MODE == MODE_RESET ? p.reset_tape : nullptr, p.reset_tape_len, N, i, 0, gid, episode + 1u,
                  c.seed, p.status};
    reset_env<BLOCK>(p, i, ds, ax, ay, gx, gy, nl);
  } else if (valid && MODE != MODE_STEP) {
    // observe / reset of an unmasked env: near list of the current state
    const Win g(c, ax, ay);
    for (int k = 0; k < Ns; ++k) {
      const int32_t o = p.st.static_obs[(int64_t)k * N + i];
      int f, e;
      if (g.near(px(o), py(o), f, e)) nl.push(f, e);
    }
    for (int k = 0; k < Nd; ++k) {
      const int32_t o = p.st.dyn_obs[(int64_t)k * N + i];
      int f, e;
      if (g.near(px(o), py(o), f, e)) nl.push(f, e);
    }
  }

  // ---- observation (prep_state4)
  if constexpr (WT > 0) {
    uint32_t flat[Geo<WT>::NW];
    int quad = 0;
    if (valid) {
      const Win g(c, ax, ay);
      uint32_t rows[Geo<WT>::K];
      raster_rows<WT, BLOCK>(nl, g, rows);
      flatten<WT>(rows, flat);
      quad = quadrant(ax, ay, gx, gy);
    }
    __syncthreads();  // near lists consumed: the stage reuses the same LDS
    if (valid) stage_row<WT>(smem, tid, flat, quad);
    __syncthreads();
    const int nvalid = min(BLOCK, N - (int)blockIdx.x * BLOCK);
    copy_out<BLOCK>(smem, Geo<WT>::F, nvalid, (int64_t)blockIdx.x * BLOCK, p.out.obs, p.out.obs_f32);
  } else {
    if (valid) {
      const int F = 4 + c.window * c.window;
      const Win g(c, ax, ay);
      write_row_generic<BLOCK>(nl, g, quadrant(ax, ay, gx, gy), p.out.obs ? p.out.obs + (int64_t)i * F : nullptr,
                               p.out.obs_f32 ? p.out.obs_f32 + (int64_t)i * F : nullptr);
    }
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
using KFn = void (*)(KArgs);
template <int WT>
KFn kernel_for(int mode) {
  return mode == MODE_STEP ? be_kernel<WT, MODE_STEP>
                           : (mode == MODE_RESET ? be_kernel<WT, MODE_RESET> : be_kernel<WT, MODE_OBSERVE>);
}

struct Launch { KFn fn; int block; int lds; };

Launch pick_kernel(const be_config& c, int mode) {
  const int W = c.window, F = 4 + W * W, nobs = c.num_static + c.num_dynamic;
  Launch L{nullptr, 0, 0};
  bool staged = true;
  switch (W) {
#define BE_CASE(n) case n: L.fn = kernel_for<n>(mode); L.block = block_for(n); break;
    BE_CASE(1) BE_CASE(2) BE_CASE(3) BE_CASE(4) BE_CASE(5) BE_CASE(6) BE_CASE(7) BE_CASE(8)
    BE_CASE(9) BE_CASE(10) BE_CASE(11) BE_CASE(12) BE_CASE(13) BE_CASE(14) BE_CASE(15) BE_CASE(16)
    BE_CASE(21)
#undef BE_CASE
    default: L.fn = kernel_for<0>(mode); L.block = block_for(0); staged = false; break;
  }
  const int near_bytes = nobs * L.block * 4;
  const int stage_bytes = staged ? L.block * F : 0;
  L.lds = ((near_bytes > stage_bytes ? near_bytes : stage_bytes) + 15) & ~15;
  if (L.lds == 0) L.lds = 16;
  return L;
}

}  // namespace

// ====================================================================== C ABI
struct be_ctx {
  be_config cfg;
  Tables tables;
  int device;
  int* status;
  char err[512];
};

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

extern "C" {

int be_abi_version(void) { return BE_ABI_VERSION; }

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
#undef BE_REQ
  if (msg && msg_len > 0) msg[0] = 0;
  return BE_OK;
bad:
  if (msg && msg_len > 0) snprintf(msg, (size_t)msg_len, "%s", buf);
  return fail(nullptr, BE_E_INVALID, "invalid config: %s", buf);
}

int64_t be_step_bytes(const be_config* c) {
  if (!c) return 0;
  // agent R+W 8 | goal R 4 | prev_dist R+W 16 | total_dist R 8 | ep_return R+W 16 | ep_len R+W 8
  // | episode R 4 | action R 1 | reward W 8 | done W 1                                     = 74
  // | statics R 4*Ns | dyn xy R+W 8*Nd | dyn goal R 1*Nd | obs W 4+W^2
  return 74 + 4ll * c->num_static + 9ll * c->num_dynamic + 4 + (int64_t)c->window * c->window;
}

const char* be_last_error(const be_ctx* ctx) { return ctx ? ctx->err : g_err; }

int be_create(const be_config* cfg, int32_t device, be_ctx** out) {
  if (!out) return fail(nullptr, BE_E_INVALID, "%s", "out is NULL");
  *out = nullptr;
  char msg[256];
  if (be_config_check(cfg, msg, sizeof msg) != BE_OK) return fail(nullptr, BE_E_INVALID, "invalid config: %s", msg);
  be_ctx* ctx = new (std::nothrow) be_ctx();
  if (!ctx) return fail(nullptr, BE_E_NOMEM, "%s", "out of host memory");
  ctx->cfg = *cfg;
  ctx->device = device;
  Tables& t = ctx->tables;
  memset(&t, 0, sizeof t);
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
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc(&ctx->status, sizeof(int));
  if (e == hipSuccess) e = hipMemset(ctx->status, 0, sizeof(int));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    int rc = fail(nullptr, BE_E_HIP, "HIP error in be_create: %s", hipGetErrorString(e));
    if (ctx->status) (void)hipFree(ctx->status);
    delete ctx;
    return rc;
  }
  *out = ctx;
  return BE_OK;
}

int be_destroy(be_ctx* ctx) {
  if (!ctx) return BE_OK;
  if (ctx->status) (void)hipFree(ctx->status);
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

static int launch(be_ctx* ctx, int mode, KArgs& a, void* stream) {
  if (((uintptr_t)a.out.obs & 15) || ((uintptr_t)a.out.obs_f32 & 15))
    return fail(ctx, BE_E_INVALID, "%s", "obs / obs_f32 must be 16-byte aligned");
  int cur = -1;
  HIP_TRY(ctx, hipGetDevice(&cur));
  if (cur != ctx->device) HIP_TRY(ctx, hipSetDevice(ctx->device));
  a.c = ctx->cfg;
  a.t = ctx->tables;
  a.status = ctx->status;
  const Launch L = pick_kernel(ctx->cfg, mode);
  const int N = ctx->cfg.num_envs;
  const dim3 grid((unsigned)((N + L.block - 1) / L.block)), block((unsigned)L.block);
  hipLaunchKernelGGL(L.fn, grid, block, (size_t)L.lds, (hipStream_t)stream, a);
  HIP_TRY(ctx, hipGetLastError());
  return BE_OK;
}

int be_reset(be_ctx* ctx, const be_state* st, const uint8_t* mask, const int16_t* reset_tape, int32_t tape_len,
             const be_out* out, void* stream) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (int rc = check_state(ctx, st)) return rc;
  if (reset_tape && tape_len < 0) return fail(ctx, BE_E_INVALID, "%s", "tape_len < 0");
  KArgs a;
  memset(&a, 0, sizeof a);
  a.st = *st;
  if (out) a.out = *out;
  if (!a.out.obs && !a.out.obs_f32) return fail(ctx, BE_E_INVALID, "%s", "be_reset needs out->obs or out->obs_f32");
  a.mask = mask; a.reset_tape = reset_tape; a.reset_tape_len = reset_tape ? tape_len : 0;
  return launch(ctx, MODE_RESET, a, stream);
}

int be_step(be_ctx* ctx, const be_state* st, const uint8_t* actions, const int16_t* action_deltas,
            const int16_t* draw_tape, const be_out* out, void* stream) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (int rc = check_state(ctx, st)) return rc;
  if (!out || !out->reward || !out->done) return fail(ctx, BE_E_INVALID, "%s", "be_step needs out->reward and out->done");
  if (draw_tape && ctx->cfg.autoreset) return fail(ctx, BE_E_INVALID, "%s", "draw tapes (parity mode) need autoreset = 0");
  KArgs a;
  memset(&a, 0, sizeof a);
  a.st = *st; a.out = *out;
  a.actions = actions; a.deltas = action_deltas; a.tape = draw_tape;
  return launch(ctx, MODE_STEP, a, stream);
}

int be_observe(be_ctx* ctx, const be_state* st, const be_out* out, void* stream) {
  if (!ctx) return fail(nullptr, BE_E_INVALID, "%s", "ctx is NULL");
  if (int rc = check_state(ctx, st)) return rc;
  if (!out || (!out->obs && !out->obs_f32)) return fail(ctx, BE_E_INVALID, "%s", "be_observe needs out->obs or out->obs_f32");
  KArgs a;
  memset(&a, 0, sizeof a);
  a.st = *st; a.out = *out;
  return launch(ctx, MODE_OBSERVE, a, stream);
}

int be_sample_actions(be_ctx* ctx, uint8_t* actions_out, int32_t steps, uint64_t seed, void* stream) {
  if (!ctx || !actions_out || steps < 0) return fail(ctx, BE_E_INVALID, "%s", "bad arguments to be_sample_actions");
  if (steps == 0) return BE_OK;
  int cur = -1;
  HIP_TRY(ctx, hipGetDevice(&cur));
  if (cur != ctx->device) HIP_TRY(ctx, hipSetDevice(ctx->device));
  const int64_t total = (int64_t)ctx->cfg.num_envs * steps;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(sample_actions_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, actions_out,
                     ctx->cfg.num_envs, steps, ctx->cfg.env_offset, ctx->cfg.num_actions, (unsigned long long)seed);
  HIP_TRY(ctx, hipGetLastError());
  return BE_OK;
}

int be_status(be_ctx* ctx, int32_t* status_out, void* stream) {
  if (!ctx || !status_out) return fail(ctx, BE_E_INVALID, "%s", "bad arguments to be_status");
  HIP_TRY(ctx, hipStreamSynchronize((hipStream_t)stream));
  int v = 0;
  HIP_TRY(ctx, hipMemcpy(&v, ctx->status, sizeof v, hipMemcpyDeviceToHost));
  const int zero = 0;
  HIP_TRY(ctx, hipMemcpy(ctx->status, &zero, sizeof zero, hipMemcpyHostToDevice));
  *status_out = v;
  return BE_OK;
}

}  // extern "C"
