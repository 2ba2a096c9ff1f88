// board.hip -- the createBoard physics profile, batched: N
// independent ``ballenv_pygame.createBoard`` worlds stepped by one launch, each step
// followed by ``featureExtractor.featureExtractor`` (the 20 IRL features step() computes).
//
// Reference (ballenv_pygame.py / featureExtractor.py):
//   Obstacle.__init__            :21-50   x = randint(0, W), y = randint(0, H), rad 20, vel 0
//   createBoard.reset            :460-513 goal / agent = generate_randomval (ranf), agent
//                                          re-sampled while dist < 50 (state[2] keeps the first
//                                          distance), statics rejected while within 15+20 of the
//                                          agent or 5+20 of the goal (check_overlap :381-387)
//   createBoard.step             :650-675 old = |agent-goal|; agent += action, clamp [0, W];
//                                          state[2] = |agent-goal|; calc_reward; features
//   createBoard.calc_reward      :680-706 any obstacle within 20 (<=) -> -1, done; else
//                                          |agent-goal| < 15 -> +1, done; else (old-cur)/total
//   featureExtractor             featureExtractor.py:247-265 (+ :36-193): [distance bin,
//                                          relative goal direction x4, density x3, speed x
//                                          orientation 3x3, social forces x3]
//
// Every coordinate is f64 as in the reference (ranf spawns; the actions are the integer
// actionArray moves or arbitrary float deltas).  Distances are sqrt(fl(x*x) + fl(y*y)) --
// math.sqrt(math.pow(x, 2) + math.pow(y, 2)) with correctly rounded pow(x, 2) and sqrt, no
// FMA contraction -- so positions, rewards, returns and done are bit-exact.  The features
// use hypot / acos / exp (1-ulp libraries on both sides): their bins and counts are exact
// away from measure-zero boundaries and the social-force sum agrees to ~1e-16 relative.
//
// createBoard's velocities are identically zero (the agent's agent_x_vel is never changed,
// :338; Obstacle vel defaults to 0, :40-47), so for every obstacle relvel = 0 -> speed bin 0
// and angle_between(v1, 0) = arccos(0) = pi/2 -> orientation bin 1, and the social-force
// factor lam + 0.5 (1 - lam)(1 + cos(pi/2)) is exactly 1.5 in f64 (featureExtractor.py:61-86,
// 115-130, 170-193).  The kernel computes those terms from that identity.
//
// One lane per env; the env index is the unit-stride HBM axis of every array.  Resets
// (reset(), or autoreset inside step) draw from a tape on the env's own lane (parity mode:
// the reference's ranf/randint values in call order), or from Philox(seed; gid, episode, 0,
// BOARD<<24 | sub), wave-cooperatively (wave_board_resets_fast: one Philox chain per lane covers
// the goal and the first attempts of every rejection loop; wave_board_resets, for the rare env
// that needs more: every rejection loop becomes one ballot over 64 candidate attempts).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <math.h>
#include <new>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ballenv.h"
#include "internal.h"
#include "philox.h"

namespace {

constexpr uint32_t PURPOSE_BOARD_RESET = 6;

// diagnostics hooks (BPH phase stamps, BCOUNT): no-ops in the release build (diag.h)
#define BE_DIAG_UNIT_BOARD 1
#include "diag.h"
constexpr int BOARD_REJECT_LIMIT = 4096;
constexpr double PI = 3.141592653589793;   // math.pi

struct BoardTables {
  double actions[BE_BOARD_MAX_ACTIONS][2];
};

struct BParams {
  double* agent; double* goal; double* dist; double* total; double* ep_return;
  int32_t* ep_len; uint32_t* episode; int32_t* statics;
  float* features; double* reward; uint8_t* done; uint8_t* truncated;
  const uint8_t* actions; const double* deltas; const uint8_t* mask;
  const double* tape; int32_t tape_len;
  const BoardTables* tables;
  int* status;
  unsigned long long seed;
  int32_t n, ns, num_actions, time_limit, autoreset, gid0, mode;   // mode: 0 step, 1 reset, 2 observe, 3 rollout
  int32_t steps;                                                   // mode 3
  int32_t W, H, sox, soy, sgx, sgy, sax, say;
  double r_collide, r_feature_obs, r_agent, goal_thr, min_spawn, thr_agent, thr_goal;
  uint32_t* pool;   // the autoreset pool (below; nullptr: every reset drawn inline)
};

// ------------------------------------------------------------------ the autoreset pool (createBoard)
// ballenv.hip's pool for this profile: a Philox reset of env i into episode x is a pure
// function of (seed, global id, x) and the config, so board_pool_fill draws every env's resets into
// episodes e+1 and e+2 ahead of time and the per-step kernel copies the entry of a finishing env
// (its reset pass -- goal, agent and static rejection chains -- was the step's tail), drawing it
// inline when the entry is stale.  Two entries per env, slot = episode & 1, entry x = slot * N + env:
//   tags    uint2 [2N] at byte 0       (episode, flags: BPOOL_VALID written, BPOOL_REJ a rejection
//                                       loop hit its bound)
//   bodies  [2N] at byte 16 N, 4 * bpool_words(ns) bytes each: agent x, y, goal x, y, state[2] (the
//           first attempt's distance), total_distance (f64), then the ns statics' packed xy
constexpr uint32_t BPOOL_VALID = 1u, BPOOL_REJ = 2u;
__host__ __device__ constexpr int bpool_words(int ns) { return 12 + ((ns + 3) & ~3); }
constexpr int64_t BPOOL_MAX_ENVS = 1ll << 22;   // every byte offset below 2^32 (48 statics' words at most)
__device__ __forceinline__ uint32_t bpool_body(uint32_t n, uint32_t x, int ns) { return 16u * n + x * (4u * (uint32_t)bpool_words(ns)); }
template <class T>
__device__ __forceinline__ T bp_ld(const uint32_t* pool, uint32_t off, uint32_t imm = 0) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(pool) + (size_t)off + imm);
}
template <class T>
__device__ __forceinline__ void bp_st(uint32_t* pool, uint32_t off, T v, uint32_t imm = 0) {
  *reinterpret_cast<T*>(reinterpret_cast<char*>(pool) + (size_t)off + imm) = v;
}

__device__ __forceinline__ double dist2(double x1, double y1, double x2, double y2) {
  const double dx = x1 - x2, dy = y1 - y2;
  return sqrt(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)));   // math.sqrt(math.pow(dx,2)+math.pow(dy,2))
}
// Per-step outputs and state of be_board_step: write-through stores (sc1, a relaxed agent-scope
// atomic store; the features as sc1 buffer stores), so they drain while the wave runs instead of in
// the kernel-end L2 write-back -- as the step kernels of ballenv.hip do: 8.75 -> 8.22 us per step at
// 65 536 envs; the fused rollout too (3.68 -> 3.62 us per step; profiles/r03_board_wt_ab.txt).
template <bool WT, class T>
__device__ __forceinline__ void bst(T* p, T v) {
  if constexpr (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
__device__ __forceinline__ int sx(int32_t p) { return (int)(int16_t)(p & 0xFFFF); }
__device__ __forceinline__ int sy(int32_t p) { return p >> 16; }

// Sequential draw source of one reset: tape column (f64 values in call order) or Philox words.
struct Draws {
  const double* tape; int32_t len, n, env, cur;
  uint32_t gid, episode; unsigned long long seed;
  u4 blk; int32_t have;
  int* status;
  __device__ uint32_t word() {
    if ((cur & 3) == 0) blk = philox(gid, episode, 0u, tag(PURPOSE_BOARD_RESET, (uint32_t)(cur >> 2)), seed);
    const uint32_t w = (cur & 3) == 0 ? blk.x : ((cur & 3) == 1 ? blk.y : ((cur & 3) == 2 ? blk.z : blk.w));
    ++cur;
    return w;
  }
  __device__ double tape_next() {
    if (cur >= len) { atomicOr(status, BE_STATUS_RESET_TAPE_EXHAUSTED); return 0.0; }
    return tape[(int64_t)(cur++) * n + env];
  }
  __device__ double ranf() {   // np.random.ranf: 53-bit uniform in [0, 1)
    if (tape) return tape_next();
    const uint32_t a = word() >> 5, b = word() >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
  }
  __device__ int randint(int lo, int hi) {
    if (tape) return (int)tape_next();
    return lo + (int)__umulhi(word(), (uint32_t)(hi - lo));
  }
};

// Lane-pair helpers (L = 2 lanes per env: lanes 2e and 2e+1 hold env e)
template <int L>
__device__ __forceinline__ double pair_other_f64(double v) {   // the other lane's value (L = 2)
  static_assert(L == 2, "pairs only");
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), 0xB1, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <int L>
__device__ __forceinline__ double pair_lead_f64(double v) {    // the pair's lane-0 value
  static_assert(L == 2, "pairs only");
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, 0xA0, 0xF, 0xF, false);   // quad_perm 0,0,2,2
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), 0xA0, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// featureExtractor(state, obstacle_list, (0, 0), agent_rad) -> 20 f32 (featureExtractor.py:247-265).
// L lanes per env: lane h takes obstacles k = L j + h; dk[j] = |obstacle k - agent| (the
// collision test's distances: the same value, sqrt(fl(dx*dx) + fl(dy*dy)) is symmetric in sign).
// The pair's counts are exact small integers; the social-force sum adds the per-obstacle terms in
// the reference's obstacle order on both lanes.  Lane h writes the row's float4 words h, h+L, ...
template <int MAXS, int L>
__device__ void features(const BParams& p, float4* out, double ax, double ay, double gx, double gy,
                         const double (&dk)[(MAXS + L - 1) / L], int h) {
  constexpr int SPL = (MAXS + L - 1) / L;
  float f[20];
#pragma unroll
  for (int k = 0; k < 20; ++k) f[k] = 0.f;
  const double vx = gx - ax, vy = gy - ay;
  const double nv = sqrt(__dadd_rn(__dmul_rn(vx, vx), __dmul_rn(vy, vy)));   // |goal - agent|
  // calcDistanceFromGoal (:132-144): floor(hypot(ax - gx, ay - gy) / 5), capped at 5.  nv is the
  // same length (correctly rounded sqrt of the rounded sum; within a few ulps of hypot's 1-ulp
  // result), so floor(nv / 5) is floor(hypot / 5) unless nv / 5 lies within 1e-9 of an integer:
  // only a wave with such a lane (never seen in practice) evaluates hypot.
  const double tq = nv / 5.0, tf = floor(tq);
  double dg = tf;
  if (tq - tf < 1e-9 || tf + 1.0 - tq < 1e-9)
    dg = floor(hypot(ax - gx, ay - gy) / 5.0);
  f[0] = (float)(dg > 5.0 ? 5.0 : dg);
  // relativeGoalPos (:146-166): angle between (0, 1) and (gx - ax, gy - ay), acos(c) of the
  // clipped cosine c.  acos decreases, so ang < pi/4 is c > cos(pi/4) and ang > 3 pi/4 is
  // c < -cos(pi/4); acos (1 ulp) only decides a lane within 1e-9 of those cuts.
  double c = nv > 0.0 ? vy / nv : 0.0;
  c = c < -1.0 ? -1.0 : (c > 1.0 ? 1.0 : c);
  constexpr double COS_PI4 = 0.70710678118654752;
  int bin;   // 0: ang < pi/4, 1: pi/4 < ang < 3 pi/4, 2: otherwise
  bin = c > COS_PI4 ? 0 : (c > -COS_PI4 ? 1 : 2);
  if (fabs(fabs(c) - COS_PI4) < 1e-9)
  {
    const double ang = acos(c);
    bin = ang < PI / 4 ? 0 : ((ang > PI / 4 && ang < PI * 3 / 4) ? 1 : 2);
  }
  if (bin == 0) f[1] = 1.f;
  else if (bin == 1) { if (vx > 0) f[2] = 1.f; else f[4] = 1.f; }
  else f[3] = 1.f;
  // density (:91-112), speed/orientation (:115-130), social forces (:170-193)
  // branch-free over this lane's slots (slots past ns are masked out), so the obstacles' f64
  // chains (exp) interleave
  double tk[SPL];
  float c5 = 0.f, c6 = 0.f, c7 = 0.f, c11 = 0.f;
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    const bool real = L * j + h < p.ns;
    const double N = dk[j] - p.r_agent - p.r_feature_obs;   // calcDistance
    c7 += (real && N < 1000.0) ? 1.f : 0.f;
    c6 += (real && N < 230.0) ? 1.f : 0.f;
    c5 += (real && N < 101.0) ? 1.f : 0.f;
    c11 += real ? 1.f : 0.f;                               // orientation bin 1, speed bin 0
    // a*exp(-N/b)*N*thrPart, a = 1, b = 10; -N*0.1 is within an ulp of -N/10 (exp's own
    // accuracy class; only sf's f32 value and its > 1 cut, a measure-zero boundary, see it)
    const double fsoc = exp(N * -0.1) * N * 1.5;
    tk[j] = (real && fsoc > 1.0) ? fsoc : 0.0;             // -> phi_SF[orientation bin 1]
  }
  double sf = 0.0;
  if constexpr (L == 1) {
#pragma unroll
    for (int j = 0; j < SPL; ++j) sf += tk[j];
  } else {
    c5 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, c5), 0xB1, 0xF, 0xF, false));
    c6 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, c6), 0xB1, 0xF, 0xF, false));
    c7 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, c7), 0xB1, 0xF, 0xF, false));
    c11 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, c11), 0xB1, 0xF, 0xF, false));
#pragma unroll
    for (int j = 0; j < SPL; ++j) {   // obstacle order: k = 2j (lane 0's), then 2j + 1 (lane 1's)
      const double o = pair_other_f64<L>(tk[j]);
      sf += h ? o : tk[j];
      sf += h ? tk[j] : o;
    }
  }
  f[5] = c5; f[6] = c6; f[7] = c7; f[8 + 3 * 1 + 0] = c11;
  f[17 + 1] = (float)sf;
  // out: this env's 80-B row (5 x 16 B) in the wave's LDS stage (board_kernel copies the rows out)
#pragma unroll
  for (int k = 0; k < 5; ++k)
    if (k % L == h) out[k] = make_float4(f[4 * k], f[4 * k + 1], f[4 * k + 2], f[4 * k + 3]);
}

// createBoard.reset for env i (ballenv_pygame.py:460-513)
template <int MAXS>
__device__ void reset_env(const BParams& p, int i, uint32_t episode, double& ax, double& ay, double& gx, double& gy,
                          double& d0, double& total, int32_t (&so)[MAXS]) {
  Draws dr{p.tape, p.tape_len, p.n, i, 0, (uint32_t)p.gid0 + (uint32_t)i, episode, p.seed, u4{0, 0, 0, 0}, 0,
           p.status};
  // generate_randomval(lower, upper) = lower + ranf * (upper - lower)
  auto rv = [&](int lo, int hi) { return (double)lo + dr.ranf() * (double)(hi - lo); };
  gx = rv(p.W - p.sgx, p.W);
  gy = rv(p.H - p.sgy, p.H);
  ax = rv(0, p.sax);
  ay = rv(0, p.say);
  d0 = dist2(gx, gy, ax, ay);                                    // state[2]: the first distance
  int guard = 0;
  while (dist2(gx, gy, ax, ay) < p.min_spawn) {
    if (++guard > BOARD_REJECT_LIMIT) { atomicOr(p.status, BE_STATUS_REJECTION_LIMIT); break; }
    ax = rv(0, p.sax);
    ay = rv(0, p.say);
  }
#pragma unroll
  for (int k = 0; k < MAXS; ++k) {
    if (k >= p.ns) break;
    int ox = 0, oy = 0;
    for (int a = 0;; ++a) {
      if (a > BOARD_REJECT_LIMIT) { atomicOr(p.status, BE_STATUS_REJECTION_LIMIT); break; }
      ox = dr.randint(p.sox, p.W - p.sox);
      oy = dr.randint(p.soy, p.H - p.soy);
      // not check_overlap(obs, agent, thresh=15) and not check_overlap(obs, goal, thresh=5)
      const bool ok_a = dist2((double)ox, (double)oy, ax, ay) - p.thr_agent > p.r_collide;
      const bool ok_g = dist2((double)ox, (double)oy, gx, gy) - p.thr_goal > p.r_collide;
      if (ok_a && ok_g) break;
    }
    so[k] = (int32_t)(((uint32_t)ox & 0xFFFFu) | ((uint32_t)oy << 16));
  }
  total = dist2(ax, ay, gx, gy);                                 // total_distance
}

// Philox-mode resets, wave-cooperative: the wave's finished envs (mask m) are reset one after
// the other by all 64 lanes.  Lane r draws agent attempt r, and lane a*ns + k draws attempt a
// of static k, so the reference's rejection loops (the first accepted attempt, in attempt
// order) become a ballot instead of a serial chain on one lane.  Counter layout (purpose 6,
// c1 = the new episode): sub 0 = the goal, 1<<20 | r = agent attempt r, 2<<20 | k<<12 | a =
// static k attempt a; ranf = 53 bits from two words, randint = multiply-shift of one.
__device__ __forceinline__ double ranf2(uint32_t w0, uint32_t w1) {
  return ((double)(w0 >> 5) * 67108864.0 + (double)(w1 >> 6)) * (1.0 / 9007199254740992.0);
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// P envs per pass (P = 1, 2, 4): the wave's lanes split into P slots of LS = 64 / P lanes, slot s
// resetting the pass's s-th finished env.  A slot checks its attempts in order, LS agent attempts
// or LS / ns attempts per static at a time, so every env gets the first accepted attempt of its
// rejection loop whatever P is; the give-up points (BOARD_REJECT_LIMIT) are those of the 64-lane
// passes (64 agent attempts, 64 / ns per static), which oracle/board_oracle.c restates.  Needs
// ns <= LS.  The slot's lanes end up holding its env's new state; the env's own lane (the owner)
// picks it up with uniform readlanes.
// OWN (board_pool_fill): the owner lanes get their env's rejection-limit flag in *rej_own and the
// status word is left alone (the step kernel that consumes the entry raises it).  A template flag,
// not a null test: the step kernels' instance is the code without the pool, instruction for instruction.
template <int MAXS, int P, bool OWN = false>
__device__ void wave_board_resets(const BParams& p, unsigned long long m, uint32_t gid, uint32_t episode_new,
                                  double& ax, double& ay, double& gx, double& gy, double& d0, double& total,
                                  int32_t (&so)[MAXS], uint32_t* rej_own = nullptr) {
  constexpr int LS = 64 / P;
  constexpr unsigned long long SMASK = LS == 64 ? ~0ull : (1ull << LS) - 1;
  constexpr int AG_END = (BOARD_REJECT_LIMIT / 64 + 1) * 64;   // the 64-lane agent passes give up after this
  const int lane = (int)(threadIdx.x & 63), slot = lane / LS, sl = lane - slot * LS;
  const int ns = p.ns;
  const int per64 = ns > 0 ? 64 / ns : 64;                      // 64-lane static pass length
  const int st_g0 = BOARD_REJECT_LIMIT / per64 * per64;         // first 64-lane pass a0 with a0 + per64 > LIMIT
  const int st_end = st_g0 + per64;                             // attempts past this are never taken
  const int per = ns > 0 ? LS / ns : LS;                        // this slot's attempts per static per pass
  const int k_l = ns > 0 ? sl % ns : 0, a_l = ns > 0 ? sl / ns : 0;
  unsigned long long kbase = 0;                                 // lanes (a, k = 0) of a slot
  for (int a = 0; a < per; ++a) kbase |= 1ull << (a * ns);
  while (m) {
    int ls[P], n = 0;
#pragma unroll
    for (int s2 = 0; s2 < P; ++s2) {   // the next (up to) P finished lanes, in lane order
      ls[s2] = m ? __ffsll((long long)m) - 1 : 0;
      n += m ? 1 : 0;
      m &= m - 1;
    }
    uint32_t u = 0, ep = 0;
#pragma unroll
    for (int s2 = 0; s2 < P; ++s2) {
      const uint32_t u2 = (uint32_t)__builtin_amdgcn_readlane((int)gid, ls[s2]);
      const uint32_t e2 = (uint32_t)__builtin_amdgcn_readlane((int)episode_new, ls[s2]);
      u = slot == s2 ? u2 : u; ep = slot == s2 ? e2 : ep;
    }
    const bool act = slot < n;
    [[maybe_unused]] uint32_t rejs = 0u;   // (OWN, uniform) slots whose loops hit the bound in this pass
    // goal (ballenv_pygame.py:462-463), on every lane of the slot
    const u4 bg = philox(u, ep, 0u, tag(PURPOSE_BOARD_RESET, 0u), p.seed);
    const double rgx = (double)(p.W - p.sgx) + ranf2(bg.x, bg.y) * (double)p.sgx;
    const double rgy = (double)(p.H - p.sgy) + ranf2(bg.z, bg.w) * (double)p.sgy;
    // agent attempts r0 + sl (:464-481)
    double rax = 0.0, ray = 0.0, rd0 = 0.0;
    unsigned open = (1u << n) - 1u;
    for (int r0 = 0; open; r0 += LS) {
      const u4 ba = philox(u, ep, 0u, tag(PURPOSE_BOARD_RESET, (1u << 20) | (uint32_t)(r0 + sl)), p.seed);
      const double cx = ranf2(ba.x, ba.y) * (double)p.sax, cy = ranf2(ba.z, ba.w) * (double)p.say;
      const double dc = dist2(rgx, rgy, cx, cy);
      if (r0 == 0) {
#pragma unroll
        for (int s2 = 0; s2 < P; ++s2) {   // state[2]: the first attempt's distance
          const double d = readlane_f64(dc, s2 * LS);
          rd0 = slot == s2 ? d : rd0;
        }
      }
      const unsigned long long ok = __ballot(act && !(dc < p.min_spawn));
      const bool last = r0 + LS >= AG_END;
#pragma unroll
      for (int s2 = 0; s2 < P; ++s2) {
        if (!((open >> s2) & 1u)) continue;
        const unsigned long long hit = (ok >> (s2 * LS)) & SMASK;
        if (hit || last) {
          if constexpr (OWN) { if (!hit) rejs |= 1u << s2; }
          else if (!hit && lane == 0) atomicOr(p.status, BE_STATUS_REJECTION_LIMIT);
          const int q = s2 * LS + (hit ? __ffsll((long long)hit) - 1 : LS - 1);
          const double x = readlane_f64(cx, q), y = readlane_f64(cy, q);
          rax = slot == s2 ? x : rax; ray = slot == s2 ? y : ray;
          open &= ~(1u << s2);
        }
      }
    }
    // statics (:489-498): slot lane a * ns + k draws attempt a0 + a of static k
    unsigned long long need[P];
#pragma unroll
    for (int s2 = 0; s2 < P; ++s2) need[s2] = s2 < n && ns > 0 ? (ns >= 64 ? ~0ull : (1ull << ns) - 1) : 0ull;
    int32_t got[MAXS];
#pragma unroll
    for (int k = 0; k < MAXS; ++k) got[k] = 0;
    for (int a0 = 0;; a0 += per) {
      unsigned long long any = 0;
#pragma unroll
      for (int s2 = 0; s2 < P; ++s2) any |= need[s2];
      if (!any) break;
      unsigned long long mine = 0;
#pragma unroll
      for (int s2 = 0; s2 < P; ++s2) mine = slot == s2 ? need[s2] : mine;
      const int a = a0 + a_l;
      bool ok = false;
      int32_t cand = 0;
      if (act && ns > 0 && a_l < per && a < st_end && ((mine >> k_l) & 1ull)) {
        const u4 bo = philox(u, ep, 0u, tag(PURPOSE_BOARD_RESET, (2u << 20) | ((uint32_t)k_l << 12) | (uint32_t)a), p.seed);
        const int ox = p.sox + (int)__umulhi(bo.x, (uint32_t)(p.W - 2 * p.sox));
        const int oy = p.soy + (int)__umulhi(bo.y, (uint32_t)(p.H - 2 * p.soy));
        ok = dist2((double)ox, (double)oy, rax, ray) - p.thr_agent > p.r_collide &&
             dist2((double)ox, (double)oy, rgx, rgy) - p.thr_goal > p.r_collide;
        cand = (int32_t)(((uint32_t)ox & 0xFFFFu) | ((uint32_t)oy << 16));
      }
      const unsigned long long okm = __ballot(ok);
      const bool last = a0 + per >= st_end;
#pragma unroll
      for (int s2 = 0; s2 < P; ++s2) {
#pragma unroll
        for (int k = 0; k < MAXS; ++k) {
          if (k >= ns || !((need[s2] >> k) & 1ull)) continue;
          const unsigned long long hit = okm & ((kbase << k) << (s2 * LS));
          if (hit || last) {
            int32_t v;
            if (hit) {
              v = __builtin_amdgcn_readlane(cand, __ffsll((long long)hit) - 1);
            } else {   // rejection limit: the static's first attempt of the last 64-lane pass
              if constexpr (OWN) rejs |= 1u << s2;
              else if (lane == 0) atomicOr(p.status, BE_STATUS_REJECTION_LIMIT);
              const u4 bo = philox(u, ep, 0u, tag(PURPOSE_BOARD_RESET, (2u << 20) | ((uint32_t)k << 12) | (uint32_t)st_g0),
                                   p.seed);
              const int ox = p.sox + (int)__umulhi(bo.x, (uint32_t)(p.W - 2 * p.sox));
              const int oy = p.soy + (int)__umulhi(bo.y, (uint32_t)(p.H - 2 * p.soy));
              v = __builtin_amdgcn_readlane((int)(((uint32_t)ox & 0xFFFFu) | ((uint32_t)oy << 16)), s2 * LS);
            }
            got[k] = slot == s2 ? v : got[k];
            need[s2] &= ~(1ull << k);
          }
        }
      }
    }
    // the owners pick up their slot's state
#pragma unroll
    for (int s2 = 0; s2 < P; ++s2) {
      if (s2 >= n) break;
      const int src = s2 * LS;
      const double sgx = readlane_f64(rgx, src), sgy = readlane_f64(rgy, src);
      const double sax = readlane_f64(rax, src), say = readlane_f64(ray, src), sd0 = readlane_f64(rd0, src);
      const bool own = lane == ls[s2];
      if (own) { gx = sgx; gy = sgy; ax = sax; ay = say; d0 = sd0; total = dist2(sax, say, sgx, sgy); }   // total_distance
      if constexpr (OWN) { if (own) *rej_own = (rejs >> s2) & 1u; }
#pragma unroll
      for (int k = 0; k < MAXS; ++k) {
        const int32_t v = __builtin_amdgcn_readlane(got[k], src);
        if (own) so[k] = v;
      }
    }
  }
}

// Single-chain reset pass (1 <= ns <= 12), one finished env at a time on all 64 lanes: lane 0
// draws the goal, lanes 1..FA agent attempts 0..FA-1 and lane FS + a*ns + k attempt a of static
// k (a < (64 - FS) / ns), each lane with its own counter of the layout above -- one Philox chain
// per lane where the general passes run three (goal, agent attempts, static attempts) one after
// the other.  The agent is checked against the goal (lane 0's draw, read back), then the statics
// against both; each rejection loop takes its first accepted attempt in attempt order, as the
// general passes do, so an env whose loops all accept within these attempts gets the same state
// bit for bit.  The others (the agent rejected FA times, or a static rejected every time) are
// returned in the mask and take the general passes.
constexpr int FAST_AG = 12, FAST_S0 = FAST_AG + 1;
template <int MAXS>
__device__ unsigned long long wave_board_resets_fast(const BParams& p, unsigned long long m, uint32_t gid,
                                                     uint32_t episode_new, double& ax, double& ay, double& gx,
                                                     double& gy, double& d0, double& total, int32_t (&so)[MAXS]) {
  const int lane = (int)(threadIdx.x & 63), ns = p.ns;
  const int per = (64 - FAST_S0) / ns;
  const int sl = lane - FAST_S0, k_l = sl >= 0 ? sl % ns : 0, a_l = sl >= 0 ? sl / ns : 0;
  const bool is_ag = lane >= 1 && lane <= FAST_AG, is_st = sl >= 0 && a_l < per;
  const uint32_t sub = is_ag ? (1u << 20) | (uint32_t)(lane - 1)
                             : (is_st ? (2u << 20) | ((uint32_t)k_l << 12) | (uint32_t)a_l : 0u);
  unsigned long long kbase = 0;                                 // lanes (a, k = 0)
  for (int a = 0; a < per; ++a) kbase |= 1ull << (FAST_S0 + a * ns);
  unsigned long long rest = 0;
  while (m) {
    const int l = __ffsll((long long)m) - 1;
    m &= m - 1;
    const uint32_t u = (uint32_t)__builtin_amdgcn_readlane((int)gid, l);
    const uint32_t ep = (uint32_t)__builtin_amdgcn_readlane((int)episode_new, l);
    const u4 b = philox(u, ep, 0u, tag(PURPOSE_BOARD_RESET, sub), p.seed);
    const double r0 = ranf2(b.x, b.y), r1 = ranf2(b.z, b.w);
    // goal (ballenv_pygame.py:462-463): lane 0's block
    const double rgx = readlane_f64((double)(p.W - p.sgx) + r0 * (double)p.sgx, 0);
    const double rgy = readlane_f64((double)(p.H - p.sgy) + r1 * (double)p.sgy, 0);
    // candidates: agent attempts (ranf) or static attempts (randint)
    const int ox = p.sox + (int)__umulhi(b.x, (uint32_t)(p.W - 2 * p.sox));
    const int oy = p.soy + (int)__umulhi(b.y, (uint32_t)(p.H - 2 * p.soy));
    const double fx = is_ag ? r0 * (double)p.sax : (double)ox, fy = is_ag ? r1 * (double)p.say : (double)oy;
    const double dg = dist2(fx, fy, rgx, rgy);                  // |candidate - goal| (symmetric in sign)
    // agent (:464-481): the first attempt with dist >= min_spawn; state[2] = attempt 0's distance
    const unsigned long long oka = __ballot(is_ag && !(dg < p.min_spawn));
    if (!oka) { rest |= 1ull << l; continue; }
    const double d0v = readlane_f64(dg, 1);
    const int qa = __ffsll((long long)oka) - 1;
    const double rax = readlane_f64(fx, qa), ray = readlane_f64(fy, qa);
    // statics (:489-498): not within thresh of the agent or the goal
    const bool oks = is_st && dist2(fx, fy, rax, ray) - p.thr_agent > p.r_collide && dg - p.thr_goal > p.r_collide;
    const unsigned long long okm = __ballot(oks);
    const int32_t cand = (int32_t)(((uint32_t)ox & 0xFFFFu) | ((uint32_t)oy << 16));
    int32_t got[MAXS];
    bool all = true;
#pragma unroll
    for (int k = 0; k < MAXS; ++k) {
      got[k] = 0;
      if (k >= ns) continue;
      const unsigned long long hit = okm & (kbase << k);
      if (!hit) { all = false; continue; }
      got[k] = __builtin_amdgcn_readlane(cand, __ffsll((long long)hit) - 1);
    }
    if (!all) { rest |= 1ull << l; continue; }
    if (lane == l) {
      gx = rgx; gy = rgy; ax = rax; ay = ray; d0 = d0v; total = dist2(rax, ray, rgx, rgy);   // total_distance
#pragma unroll
      for (int k = 0; k < MAXS; ++k) so[k] = got[k];
    }
  }
  return rest;
}

// MAXS: compile-time bound on the static-obstacle count (4 .. 32), so the obstacle loops unroll
// with a runtime guard and the positions stay in registers (no scratch).  L lanes per env (1 or
// 2): every lane holds the env's whole state; lane h runs the collision test and the feature
// terms of obstacles k = L j + h (the pair combines them, above), the per-env chains (distance,
// reward, the goal features) run on both lanes, and the pair splits the stores.  Two lanes give
// two waves per SIMD at 65 536 envs where one lane per env leaves one.
// A wave's feature rows (EPW x 80 B, contiguous in the output) from its LDS stage to HBM with
// 16-byte stores in lane order: whole cache lines per store instruction, where a lane's own row
// would scatter 5 stores over 64 rows at an 80-B stride.
template <int EPW, bool WT>
__device__ __forceinline__ void copy_feat(const float4* stage, float* dst, int nrows, int lane) {
  const int nv = nrows * 5;
  if constexpr (WT) {   // nrows / dst are wave-uniform: a scalar descriptor whose size drops the tail
    typedef int v4i_ __attribute__((ext_vector_type(4)));
    const int nvu = __builtin_amdgcn_readfirstlane(nv);
    const uint64_t du = (uint64_t)dst;
    float* dstu = reinterpret_cast<float*>(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(du >> 32)) << 32) |
                                           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)du));
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(dstu, (short)0, nvu * 16, 0x00020000);
#pragma unroll
    for (int j = 0; j < (EPW * 5 + 63) / 64; ++j) {
      const int v = lane + 64 * j;
      const float4 x = stage[min(v, EPW * 5 - 1)];
      const v4i_ y = {__builtin_bit_cast(int, x.x), __builtin_bit_cast(int, x.y), __builtin_bit_cast(int, x.z),
                      __builtin_bit_cast(int, x.w)};
      __builtin_amdgcn_raw_buffer_store_b128(y, rsrc, v * 16, 0, 16);   // aux 16 = sc1
    }
  } else {
    float4* d4 = reinterpret_cast<float4*>(dst);
#pragma unroll
    for (int j = 0; j < (EPW * 5 + 63) / 64; ++j) {
      const int v = lane + 64 * j;
      if (v < nv) d4[v] = stage[v];
    }
  }
}

template <int MAXS, bool ROLL, int L, bool POOL = false>
__global__ __launch_bounds__(256) void board_kernel(BParams p) {
  constexpr int SPL = (MAXS + L - 1) / L, EPW = 64 / L;
  constexpr bool WT = true;   // write-through in both kernels (profiles/r03_board_wt_ab.txt)
  __shared__ float4 s_feat[4][EPW * 5];   // per wave: its envs' feature rows
  const int lane = (int)(threadIdx.x & 63), w = (int)(threadIdx.x >> 6);
  float4* fstage = &s_feat[w][0];
  float4* frow = fstage + (lane / L) * 5;
  const int e0 = (int)blockIdx.x * (256 / L) + w * EPW;          // the wave's first env
  const int nrows = max(0, min(EPW, p.n - e0));
  auto feat_out = [&](int64_t row0) {   // the wave's staged rows to features[row0 ..]
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    copy_feat<EPW, WT>(fstage, p.features + row0 * 20, nrows, lane);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // the next step's stage writes follow
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // every lane of a wave stays to the end (the Philox resets are wave-cooperative); lanes past
  // N work on a clamped index and store nothing
  const int h = (int)(threadIdx.x & (L - 1));
  const int i0 = blockIdx.x * (256 / L) + (int)threadIdx.x / L;
  const bool valid = i0 < p.n;
  const int i = valid ? i0 : p.n - 1;
  int32_t so[MAXS];
#pragma unroll
  for (int k = 0; k < MAXS; ++k) so[k] = k < p.ns ? p.statics[(int64_t)k * p.n + i] : 0;
  const double2 ag = reinterpret_cast<const double2*>(p.agent)[i];
  const double2 gl = reinterpret_cast<const double2*>(p.goal)[i];
  double ax = ag.x, ay = ag.y, gx = gl.x, gy = gl.y;
  double dk[SPL];   // this lane's obstacle distances |obstacle - agent|
  auto obstacle_dists = [&]() {
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
      const int32_t o = so[min(L * j + h, MAXS - 1)];
      dk[j] = dist2(ax, ay, (double)sx(o), (double)sy(o));
    }
  };
  if (p.mode == 2) {
    obstacle_dists();
    if (valid) features<MAXS, L>(p, frow, ax, ay, gx, gy, dk, h);
    feat_out(e0);
    return;
  }
  BPH_INIT;
  uint32_t episode = p.episode[i];
  double total = p.total[i], ret = p.ep_return[i], dist = p.dist[i];
  int32_t len = p.ep_len[i];
  bool was_reset = false;   // goal / total / episode / statics changed: store them at the end
  bool fresh = true;        // dist may differ from |agent - goal| (a reset's state[2], or loaded state)
  // mode 3 (be_board_rollout): p.steps steps with the state in registers, per-step outputs in
  // (steps, N, ...) rows; modes 0 / 1 are one pass of the same body
  const int steps = ROLL ? p.steps : 1;   // ROLL: the mode-3 instantiation
  // the action table in LDS (a table read from memory is a second load on the move's chain), and
  // the next step's action read one step ahead in the fused rollout, so its latency overlaps a step.
  // One copy per wave under a wave barrier, no block barrier (step 8.08-8.12 against 8.10-8.16 us,
  // fused 2.96-3.05 against 3.05-3.08: profiles/r04_board_wave_actions_ab.txt)
  __shared__ double s_act_w[4][2 * BE_BOARD_MAX_ACTIONS];
  double* s_act = &s_act_w[w][0];
  int a_pf = 0;
  double dx_pf = 0.0, dy_pf = 0.0;
  auto fetch = [&](int s) {
    const int64_t r = (int64_t)s * p.n + i;
    if (p.actions) a_pf = p.actions[r];
    else { dx_pf = p.deltas[2 * r]; dy_pf = p.deltas[2 * r + 1]; }
  };
  const bool stage_act = p.mode != 1 && p.actions;   // (uniform)
  auto act_barrier = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  if constexpr (!ROLL) {
    // the per-step kernel: the table word (a clamped index: no branch around the load), then step
    // 0's action, then the LDS write, which waits for the table word only -- the other way round the
    // action load was issued after that wait, a second memory latency in the prologue (step
    // 8.06-8.10 -> 7.89-7.91 us, profiles/r05_board_prologue_ab.txt)
    double tword = 0.0;
    if (stage_act) tword = (&p.tables->actions[0][0])[min(lane, 2 * BE_BOARD_MAX_ACTIONS - 1)];
    if (p.mode != 1) fetch(0);
    if (stage_act) {
      if (lane < 2 * p.num_actions) s_act[lane] = tword;
      act_barrier();
    }
  } else {
    // the fused kernel keeps the table first: its prologue is once per launch, and the per-step
    // kernel's order cost its loop 0.25 us per step (the same A/B)
    if (stage_act) {
      if (lane < 2 * p.num_actions) s_act[lane] = (&p.tables->actions[0][0])[lane];
      act_barrier();
    }
    if (p.mode != 1) {
      fetch(0);
      // step 0's action lands before the loop: inside it the only pending read of a_pf is the one
      // issued a step earlier, so its wait need not cover that step's stores (vmcnt(#stores), where a
      // loop entered with a_pf in flight merges to vmcnt(0))
      asm volatile("" ::"v"(a_pf), "v"(dx_pf), "v"(dy_pf));
    }
  }
  for (int s = 0; s < steps; ++s) {
    const int64_t row = (int64_t)s * p.n + i;   // this step's output row (i for modes 0 / 1)
    bool do_reset = valid && p.mode == 1 && (!p.mask || p.mask[i]);
    bool moved = false;
    if (p.mode != 1) {
      double dx = dx_pf, dy = dy_pf;
      int a = a_pf;
      if (ROLL && s + 1 < steps) fetch(s + 1);
      if (p.actions) {
        if (a >= p.num_actions) { atomicOr(p.status, BE_STATUS_BAD_ACTION); a = 0; }
        dx = s_act[2 * a]; dy = s_act[2 * a + 1];
      }
      BPH(0);
      // self.old_dist (:652) = |agent - goal|, which the previous step of this launch left in dist
      const double old = fresh ? dist2(ax, ay, gx, gy) : dist;
      double nx = ax + dx, ny = ay + dy;
      if (nx < 0) nx = 0;
      if (nx > p.W) nx = p.W;
      if (ny < 0) ny = 0;
      if (ny > p.H) ny = p.H;
      ax = nx; ay = ny;
      dist = dist2(ax, ay, gx, gy);                                // state[2] (:668)
      fresh = false;
      moved = true;
      // calc_reward (:680-706)
      obstacle_dists();
      double r;
      bool done = false;
#pragma unroll
      for (int j = 0; j < SPL; ++j)   // any hit (the reference stops at the first; the result is the same)
        done |= (L * j + h < p.ns) & !(dk[j] > p.r_collide);
      if constexpr (L == 2) done = (__builtin_amdgcn_update_dpp(0, (int)done, 0xB1, 0xF, 0xF, false) | (int)done) != 0;
      if (done) { r = -1.0; ret += -1.0; }
      else if (dist < p.goal_thr) { done = true; r = 1.0; ret += 1.0; }
      else { r = (old - dist) / total; ret += r; }
      ++len;
      const bool trunc = !done && p.time_limit > 0 && len >= p.time_limit;
      done = done || trunc;
      if (valid) {   // the pair splits the per-step stores
        if (h == 0) bst<WT>(p.reward + row, r);
        if (h == L - 1) bst<WT>(p.done + row, (uint8_t)(done ? 1 : 0));
        if (h == L - 1 && p.truncated) bst<WT>(p.truncated + row, (uint8_t)(trunc ? 1 : 0));
      }
      do_reset = valid && done && p.autoreset;
      BPH(1);
    }
    if (p.tape) {   // parity mode: the reference's draw order, on the env's own lane(s)
      if (do_reset) reset_env(p, i, episode + 1u, ax, ay, gx, gy, dist, total, so);
    } else {
      const unsigned long long m0 = __ballot(do_reset && h == 0);
      if (m0) {
        const uint32_t g = (uint32_t)p.gid0 + (uint32_t)i;
        unsigned long long m = m0;
        if constexpr (POOL) {   // (L == 1) the pool's entry for episode + 1 when it is current
          static_assert(L == 1 && !ROLL, "the pool instance is the one-lane per-step kernel");
          const bool ptry = do_reset && p.pool != nullptr;
          uint2 q_tv = make_uint2(0u, 0u);
          double2 qa = make_double2(0.0, 0.0), qg = qa, qd = qa;
          if (ptry) {   // (the statics load straight into so: a finishing lane's are dead, and a stale
                        // entry's lane gets them again from the inline passes below)
            const uint32_t x = ((episode + 1u) & 1u) * (uint32_t)p.n + (uint32_t)i;
            q_tv = bp_ld<uint2>(p.pool, x * 8u);
            const uint32_t bo = bpool_body((uint32_t)p.n, x, p.ns);
            qa = bp_ld<double2>(p.pool, bo, 0u);
            qg = bp_ld<double2>(p.pool, bo, 16u);
            qd = bp_ld<double2>(p.pool, bo, 32u);
#pragma unroll
            for (int k = 0; k < MAXS; ++k)
              if (k < p.ns) so[k] = bp_ld<int32_t>(p.pool, bo, 48u + 4u * (uint32_t)k);
            __builtin_amdgcn_s_waitcnt(0);   // here, in the branch: no pending pool load past its end
          }
          const bool hit = ptry && q_tv.x == episode + 1u && (q_tv.y & BPOOL_VALID) != 0u;
          if (hit) { ax = qa.x; ay = qa.y; gx = qg.x; gy = qg.y; dist = qd.x; total = qd.y; }
          if (__ballot(hit && (q_tv.y & BPOOL_REJ)) && lane == 0) atomicOr(p.status, BE_STATUS_REJECTION_LIMIT);
          m = __ballot(do_reset && !hit);
        }
        if constexpr (MAXS <= 12) {   // one Philox chain per reset; the rare rest take the general passes
          if (p.ns >= 1) m = wave_board_resets_fast<MAXS>(p, m, g, episode + 1u, ax, ay, gx, gy, dist, total, so);
        }
        BCOUNT(5, __popcll(m0));
        BCOUNT(6, __popcll(m));
        if (m) {   // several finished envs: 2 or 4 per pass (ns must fit a slot: ns <= 64 / P)
          const int nf = __popcll(m);
          if constexpr (MAXS > 16) {   // (ns > 16 never fits two slots)
            wave_board_resets<MAXS, 1>(p, m, g, episode + 1u, ax, ay, gx, gy, dist, total, so);
          } else {
            if (nf == 1) wave_board_resets<MAXS, 1>(p, m, g, episode + 1u, ax, ay, gx, gy, dist, total, so);
            else if (nf == 2 || p.ns > 8) wave_board_resets<MAXS, 2>(p, m, g, episode + 1u, ax, ay, gx, gy, dist, total, so);
            else wave_board_resets<MAXS, 4>(p, m, g, episode + 1u, ax, ay, gx, gy, dist, total, so);
          }
        }
        if constexpr (L == 2) {   // the owner (lane 0) took the new state: its partner copies it
          if (__ballot(do_reset)) {
            ax = pair_lead_f64<L>(ax); ay = pair_lead_f64<L>(ay); gx = pair_lead_f64<L>(gx); gy = pair_lead_f64<L>(gy);
            dist = pair_lead_f64<L>(dist); total = pair_lead_f64<L>(total);
#pragma unroll
            for (int k = 0; k < MAXS; ++k) so[k] = __builtin_amdgcn_update_dpp(0, so[k], 0xA0, 0xF, 0xF, false);
          }
        }
      }
    }
    if (do_reset) {
      ++episode;
      ret = 0.0; len = 0;
      was_reset = true;
      fresh = true;
      obstacle_dists();
    }
    BPH(2);
    if (p.features) {   // (uniform)
      if (valid) {
        if (!moved) obstacle_dists();
        features<MAXS, L>(p, frow, ax, ay, gx, gy, dk, h);
      }
      BPH(3);
      feat_out((int64_t)s * p.n + e0);
      BPH(4);
    }
  }
  BPH_STORE;
  if (!valid) return;
  if (was_reset && h == L - 1) {
#pragma unroll
    for (int k = 0; k < MAXS; ++k)
      if (k < p.ns) bst<WT>(p.statics + (int64_t)k * p.n + i, so[k]);
    bst<WT>(p.goal + 2 * (int64_t)i, gx);
    bst<WT>(p.goal + 2 * (int64_t)i + 1, gy);
    bst<WT>(p.total + i, total);
    bst<WT>(p.episode + i, episode);
  }
  if (h == 0) {
    bst<WT>(p.agent + 2 * (int64_t)i, ax);
    bst<WT>(p.agent + 2 * (int64_t)i + 1, ay);
    bst<WT>(p.dist + i, dist);
  }
  if (h == L - 1) {
    bst<WT>(p.ep_return + i, ret);
    bst<WT>(p.ep_len + i, len);
  }
}

// The pool's fill (one lane per env): an env at episode e needs the entries of e+1 (slot (e+1) & 1)
// and e+2; a wave draws its stale ones with the step kernel's own passes (the single-chain pass,
// then the general passes for its rest), so an entry is the reset the step would draw, bit for bit.
// Stream-ordered with the steps (be_board_step queues it every pool period, be_board_reset after its
// kernel).
template <int MAXS>
__global__ __launch_bounds__(256) void board_pool_fill(BParams p) {
  const int i0 = (int)blockIdx.x * 256 + (int)threadIdx.x;
  const bool valid = i0 < p.n;
  const int i = valid ? i0 : p.n - 1;
  const uint32_t g = (uint32_t)p.gid0 + (uint32_t)i, e = p.episode[i];
  const uint2 tv0 = bp_ld<uint2>(p.pool, (uint32_t)i * 8u), tv1 = bp_ld<uint2>(p.pool, ((uint32_t)p.n + (uint32_t)i) * 8u);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const uint32_t target = (((e + 1u) & 1u) == (uint32_t)s) ? e + 1u : e + 2u;   // the episode slot s holds
    const uint2 tv = s ? tv1 : tv0;
    const bool need = valid && !(tv.x == target && (tv.y & BPOOL_VALID));
    unsigned long long m = __ballot(need);
    if (!m) continue;
    double ax = 0.0, ay = 0.0, gx = 0.0, gy = 0.0, d0 = 0.0, total = 0.0;
    int32_t so[MAXS];
#pragma unroll
    for (int k = 0; k < MAXS; ++k) so[k] = 0;
    uint32_t rej = 0u;
    if constexpr (MAXS <= 12) {
      if (p.ns >= 1) m = wave_board_resets_fast<MAXS>(p, m, g, target, ax, ay, gx, gy, d0, total, so);
    }
    if (m) {
      const int nf = __popcll(m);
      if constexpr (MAXS > 16) {
        wave_board_resets<MAXS, 1, true>(p, m, g, target, ax, ay, gx, gy, d0, total, so, &rej);
      } else {
        if (nf == 1) wave_board_resets<MAXS, 1, true>(p, m, g, target, ax, ay, gx, gy, d0, total, so, &rej);
        else if (nf == 2 || p.ns > 8) wave_board_resets<MAXS, 2, true>(p, m, g, target, ax, ay, gx, gy, d0, total, so, &rej);
        else wave_board_resets<MAXS, 4, true>(p, m, g, target, ax, ay, gx, gy, d0, total, so, &rej);
      }
    }
    if (need) {   // the body, then the tag (its written flag)
      const uint32_t x = (uint32_t)s * (uint32_t)p.n + (uint32_t)i, bo = bpool_body((uint32_t)p.n, x, p.ns);
      bp_st(p.pool, bo, make_double2(ax, ay), 0u);
      bp_st(p.pool, bo, make_double2(gx, gy), 16u);
      bp_st(p.pool, bo, make_double2(d0, total), 32u);
#pragma unroll
      for (int k = 0; k < MAXS; ++k)
        if (k < p.ns) bp_st(p.pool, bo, so[k], 48u + 4u * (uint32_t)k);
      bp_st(p.pool, x * 8u, make_uint2(target, BPOOL_VALID | (rej ? BPOOL_REJ : 0u)));
    }
  }
}

}  // namespace

struct be_board {
  be_board_config cfg;
  int device;
  bool lpe2;           // BALLENV_BOARD_LPE=2: two lanes per env (A/B)
  int* status;
  BoardTables* d_tables;
  uint32_t* pool;      // the autoreset pool (Philox autoreset, one lane per env), or nullptr
  int64_t pool_bytes;
  int pool_period, pool_calls;
  const void* pool_owner;   // the state (its episode array) the pool serves
  char err[512];
};

static thread_local char g_board_err[512];

static int bfail(be_board* b, int code, const char* msg) {
  snprintf(b ? b->err : g_board_err, 512, "%s", msg);
  return code;
}

static int bhip(be_board* b, hipError_t e) {
  char buf[256];
  snprintf(buf, sizeof buf, "HIP error: %s", hipGetErrorString(e));
  return bfail(b, BE_E_HIP, buf);
}

extern "C" {

int be_board_config_default(be_board_config* c, int32_t num_envs, int32_t num_static) {
  if (!c) return bfail(nullptr, BE_E_INVALID, "cfg is NULL");
  memset(c, 0, sizeof *c);
  c->num_envs = num_envs; c->num_static = num_static; c->seed = 0xB0A2Dull;
  c->screen_width = 100; c->screen_height = 100;                       // ballenv_pygame.py:8-15
  c->strip_obs_x = 0; c->strip_obs_y = 0; c->strip_goal_x = 100; c->strip_goal_y = 100;
  c->strip_agent_x = 100; c->strip_agent_y = 100;
  c->agent_radius = 10.0; c->static_radius = 10.0; c->obstacle_feature_radius = 20.0;   // :316, Obstacle rad :35-38
  c->goal_threshold = 15.0; c->min_spawn_dist = 50.0; c->spawn_thresh_agent = 15.0; c->spawn_thresh_goal = 5.0;
  static const double acts[4][2] = {{0, -1}, {1, 0}, {0, 1}, {-1, 0}};   // actionArray :352-353
  c->num_actions = 4;
  for (int a = 0; a < 4; ++a) { c->actions[a][0] = acts[a][0]; c->actions[a][1] = acts[a][1]; }
  c->time_limit = 0; c->autoreset = 0;
  return BE_OK;
}

int be_board_create(const be_board_config* cfg, int32_t device, be_board** out) {
  if (!cfg || !out) return bfail(nullptr, BE_E_INVALID, "bad arguments to be_board_create");
  *out = nullptr;
  if (cfg->num_envs < 1) return bfail(nullptr, BE_E_INVALID, "num_envs must be >= 1");
  if (cfg->num_static < 0 || cfg->num_static > BE_BOARD_MAX_STATIC)
    return bfail(nullptr, BE_E_INVALID, "num_static must be in [0, 32]");
  if (cfg->num_actions < 1 || cfg->num_actions > BE_BOARD_MAX_ACTIONS)
    return bfail(nullptr, BE_E_INVALID, "num_actions must be in [1, 16]");
  if (cfg->screen_width < 1 || cfg->screen_height < 1 || cfg->screen_width > 16384 || cfg->screen_height > 16384 ||
      cfg->screen_width - 2 * cfg->strip_obs_x < 1 || cfg->screen_height - 2 * cfg->strip_obs_y < 1)
    return bfail(nullptr, BE_E_INVALID, "screen / obstacle strips give an empty randint range");
  if (cfg->env_offset < 0 || cfg->env_offset + (int64_t)cfg->num_envs > (1ll << 32))
    return bfail(nullptr, BE_E_INVALID, "global env ids must fit in 32 bits");
  be_board* b = new (std::nothrow) be_board();
  if (!b) return bfail(nullptr, BE_E_NOMEM, "out of host memory");
  b->cfg = *cfg;
  b->device = device;
  if (const char* l = getenv("BALLENV_BOARD_LPE")) b->lpe2 = !strcmp(l, "2");
  BoardTables t;
  memset(&t, 0, sizeof t);
  for (int a = 0; a < cfg->num_actions; ++a) { t.actions[a][0] = cfg->actions[a][0]; t.actions[a][1] = cfg->actions[a][1]; }
  const DeviceGuard dg(device);   // the caller's current device is restored on return
  hipError_t e = dg.err;
  if (e == hipSuccess) e = hipMalloc(&b->status, sizeof(int));
  if (e == hipSuccess) e = hipMemset(b->status, 0, sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&b->d_tables, sizeof t);
  if (e == hipSuccess) e = hipMemcpy(b->d_tables, &t, sizeof t, hipMemcpyHostToDevice);
  {  // the autoreset pool: Philox autoreset, one lane per env (BALLENV_POOL=0 disables it, A/B)
    bool want = cfg->autoreset && !b->lpe2 && (int64_t)cfg->num_envs <= BPOOL_MAX_ENVS;
    if (const char* v = getenv("BALLENV_POOL")) want = want && strcmp(v, "0") != 0;
    b->pool_period = 128;
    if (const char* v = getenv("BALLENV_POOL_PERIOD")) b->pool_period = std::max(0, atoi(v));
    if (want && e == hipSuccess) {
      b->pool_bytes = 2ll * cfg->num_envs * (8 + 4ll * bpool_words(cfg->num_static));
      e = hipMalloc(&b->pool, (size_t)b->pool_bytes);
      if (e == hipSuccess) e = hipMemset(b->pool, 0, (size_t)b->pool_bytes);   // every entry unwritten
      if (e == hipSuccess) e = hipDeviceSynchronize();
    }
  }
  if (e != hipSuccess) {
    const int rc = bhip(nullptr, e);
    if (b->status) (void)hipFree(b->status);
    if (b->d_tables) (void)hipFree(b->d_tables);
    if (b->pool) (void)hipFree(b->pool);
    delete b;
    return rc;
  }
  *out = b;
  return BE_OK;
}

int be_board_destroy(be_board* b) {
  if (!b) return BE_OK;
  const DeviceGuard dg(b->device);   // the caller's current device is restored on return
  if (b->status) (void)hipFree(b->status);
  if (b->d_tables) (void)hipFree(b->d_tables);
  if (b->pool) (void)hipFree(b->pool);
  delete b;
  return BE_OK;
}

int64_t be_board_pool_bytes(const be_board* b) { return b && b->pool ? b->pool_bytes : 0; }

const char* be_board_last_error(const be_board* b) { return b ? b->err : g_board_err; }

static int board_launch(be_board* b, const be_board_state* st, const be_board_out* out, int mode,
                        const uint8_t* actions, const double* deltas, const uint8_t* mask, const double* tape,
                        int32_t tape_len, void* stream, int32_t steps = 1) {
  if (!b) return bfail(nullptr, BE_E_INVALID, "board is NULL");
  if (!st || !st->agent || !st->goal || !st->dist || !st->total_dist || !st->ep_return || !st->ep_len ||
      !st->episode || (b->cfg.num_static > 0 && !st->static_obs))
    return bfail(b, BE_E_INVALID, "be_board_state has a NULL pointer");
  if (!out) return bfail(b, BE_E_INVALID, "out is NULL");
  if ((mode == 0 || mode == 3) && (!out->reward || !out->done))
    return bfail(b, BE_E_INVALID, "be_board_step / be_board_rollout need out->reward and out->done");
  if ((mode == 0 || mode == 3) && !actions && !deltas)
    return bfail(b, BE_E_INVALID, "be_board_step / be_board_rollout need actions or deltas");
  if (mode == 3 && steps < 0) return bfail(b, BE_E_INVALID, "steps < 0");
  if (mode == 3 && steps == 0) return BE_OK;
  if (mode == 2 && !out->features) return bfail(b, BE_E_INVALID, "be_board_observe needs out->features");
  if (tape && tape_len < 0) return bfail(b, BE_E_INVALID, "tape_len < 0");
  const DeviceGuard dg(b->device);   // the caller's current device is restored on return
  hipError_t e = dg.err;
  if (e != hipSuccess) return bhip(b, e);
  const be_board_config& c = b->cfg;
  BParams p;
  memset(&p, 0, sizeof p);
  p.agent = st->agent; p.goal = st->goal; p.dist = st->dist; p.total = st->total_dist; p.ep_return = st->ep_return;
  p.ep_len = st->ep_len; p.episode = st->episode; p.statics = st->static_obs;
  p.features = out->features; p.reward = out->reward; p.done = out->done; p.truncated = out->truncated;
  p.actions = actions; p.deltas = deltas; p.mask = mask; p.tape = tape; p.tape_len = tape ? tape_len : 0;
  p.tables = b->d_tables; p.status = b->status; p.seed = c.seed;
  p.n = c.num_envs; p.ns = c.num_static; p.num_actions = c.num_actions; p.time_limit = c.time_limit;
  p.autoreset = c.autoreset; p.gid0 = (int32_t)(uint32_t)c.env_offset; p.mode = mode; p.steps = steps;
  p.W = c.screen_width; p.H = c.screen_height; p.sox = c.strip_obs_x; p.soy = c.strip_obs_y;
  p.sgx = c.strip_goal_x; p.sgy = c.strip_goal_y; p.sax = c.strip_agent_x; p.say = c.strip_agent_y;
  p.r_collide = c.static_radius + c.agent_radius; p.r_feature_obs = c.obstacle_feature_radius;
  p.r_agent = c.agent_radius; p.goal_thr = c.goal_threshold; p.min_spawn = c.min_spawn_dist;
  p.thr_agent = c.spawn_thresh_agent; p.thr_goal = c.spawn_thresh_goal;
  // the obstacle loops run MAXS slots branch-free: the smallest bound that covers num_static;
  // one lane per env: two (BALLENV_BOARD_LPE=2, A/B) measured slower, 9.66 vs 9.45 us per step
  // and 4.96 vs 3.97 us fused at 65 536 envs -- the per-env f64 chains (acos, hypot, the reward
  // divide) run on both lanes and outweigh the halved obstacle terms (profiles/r03_board_lanes_ab.txt)
  const int lpe = (tape || !b->lpe2) ? 1 : 2;
  // the pool serves one state (the one last reset, else the first one stepped): its steps run the
  // pool instance, any other state's steps draw every reset inline
  if (b->pool && mode == 0 && !b->pool_owner) b->pool_owner = st->episode;
  const bool use_pool = b->pool && mode == 0 && lpe == 1 && st->episode == b->pool_owner;
  p.pool = use_pool ? b->pool : nullptr;
  void (*fn)(BParams) = nullptr;
#define BE_BOARD_PICK(R, LL, ...)                                                                                       \
  fn = c.num_static <= 4 ? board_kernel<4, R, LL, ##__VA_ARGS__> : c.num_static <= 6 ? board_kernel<6, R, LL, ##__VA_ARGS__>   \
     : c.num_static <= 8 ? board_kernel<8, R, LL, ##__VA_ARGS__> : c.num_static <= 12 ? board_kernel<12, R, LL, ##__VA_ARGS__> \
     : c.num_static <= 16 ? board_kernel<16, R, LL, ##__VA_ARGS__> : board_kernel<32, R, LL, ##__VA_ARGS__>
  if (mode == 3) { if (lpe == 2) BE_BOARD_PICK(true, 2); else BE_BOARD_PICK(true, 1); }
  else if (use_pool) BE_BOARD_PICK(false, 1, true);
  else { if (lpe == 2) BE_BOARD_PICK(false, 2); else BE_BOARD_PICK(false, 1); }
#undef BE_BOARD_PICK
  const int epb = 256 / lpe;
  hipLaunchKernelGGL(fn, dim3((unsigned)((c.num_envs + epb - 1) / epb)), dim3(256), 0, (hipStream_t)stream, p);
  // the pool's fill: after a reset (its state's next two episodes), and every pool period of steps
  const bool fill = b->pool && (mode == 1 || (use_pool && b->pool_period > 0 && ++b->pool_calls >= b->pool_period));
  if (fill) {
    if (mode == 1) b->pool_owner = st->episode;
    if (st->episode == b->pool_owner) {
      b->pool_calls = 0;
      BParams f = p;
      f.pool = b->pool; f.tape = nullptr; f.tape_len = 0;
      void (*ff)(BParams) = c.num_static <= 4 ? board_pool_fill<4> : c.num_static <= 6 ? board_pool_fill<6>
                          : c.num_static <= 8 ? board_pool_fill<8> : c.num_static <= 12 ? board_pool_fill<12>
                          : c.num_static <= 16 ? board_pool_fill<16> : board_pool_fill<32>;
      hipLaunchKernelGGL(ff, dim3((unsigned)((c.num_envs + 255) / 256)), dim3(256), 0, (hipStream_t)stream, f);
    }
  }
  e = hipGetLastError();
  if (e != hipSuccess) return bhip(b, e);
  return BE_OK;
}

int be_board_reset(be_board* b, const be_board_state* st, const uint8_t* mask, const double* reset_tape,
                   int32_t tape_len, const be_board_out* out, void* stream) {
  return board_launch(b, st, out, 1, nullptr, nullptr, mask, reset_tape, tape_len, stream);
}

int be_board_step(be_board* b, const be_board_state* st, const uint8_t* actions, const double* deltas,
                  const be_board_out* out, void* stream) {
  return board_launch(b, st, out, 0, actions, deltas, nullptr, nullptr, 0, stream);
}

int be_board_rollout(be_board* b, const be_board_state* st, const uint8_t* actions, const double* deltas,
                     int32_t steps, const be_board_out* out, void* stream) {
  return board_launch(b, st, out, 3, actions, deltas, nullptr, nullptr, 0, stream, steps);
}

int be_board_observe(be_board* b, const be_board_state* st, const be_board_out* out, void* stream) {
  return board_launch(b, st, out, 2, nullptr, nullptr, nullptr, nullptr, 0, stream);
}

BE_DIAG_BOARD_ENTRIES   // diagnostics builds only (diag.h)

int be_board_status(be_board* b, int32_t* status_out, void* stream) {
  if (!b || !status_out) return bfail(b, BE_E_INVALID, "bad arguments to be_board_status");
  const DeviceGuard dg(b->device);   // the caller's current device is restored on return
  hipError_t e = dg.err;
  if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
  int v = 0;
  if (e == hipSuccess) e = hipMemcpy(&v, b->status, sizeof v, hipMemcpyDeviceToHost);
  const int zero = 0;
  if (e == hipSuccess) e = hipMemcpy(b->status, &zero, sizeof zero, hipMemcpyHostToDevice);
  if (e != hipSuccess) return bhip(b, e);
  *status_out = v;
  return BE_OK;
}

}  // extern "C"
