// policy_core.h -- the Policy(W) forward pieces shared by the select_action kernel
// (policy.hip) and the fused policy rollout kernel (ballenv.hip): the packed-weight
// layout, one 16-env column tile of fc1 on the int8 matrix cores + heads, and the
// softmax / Categorical draw.  The design notes are at the top of policy.hip.
// Reference: examples/ball_cnn_ac3.py:109-146 (Policy), :210-220 (select_action).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "philox.h"

namespace {

constexpr uint32_t PURPOSE_POLICY = 5;
constexpr int POL_MAXH = 256, POL_MAXF = 128, POL_MAXA = 15;
constexpr int POL_ENVS = 256;                    // envs per workgroup
constexpr int POL_THREADS = 64 * POL_ENVS / 16;  // one wave per 16-env tile
constexpr int POL_FIN_WAVES = POL_ENVS / 64;     // waves that run the epilogue

typedef int v4i __attribute__((ext_vector_type(4)));

// Packed-weight image (bytes), identical in HBM and in each workgroup's LDS.
struct PolLayout {
  int HT, KS, NO;            // 16-row hidden tiles, 64-wide K steps, outputs (actions + value)
  int frag, bias, head, hbias, table, total, logits, info, list, count, lds;
};
__host__ __device__ constexpr PolLayout pol_layout(int HT, int KS, int NO) {
  PolLayout L{};
  L.HT = HT; L.KS = KS; L.NO = NO;
  L.frag = 0;                                   // [HT][3 digits, high first][KS][64 lanes][16 B] int8
  L.bias = L.frag + HT * 3 * KS * 1024;         // [HT*16] i32   bq_k = rint(b1_k / s_k)
  L.head = L.bias + HT * 16 * 4;                // [HT][4 groups][NO][4] f32  W_o,k * s_k, k = 16ht+4g+r
  L.hbias = L.head + HT * 4 * NO * 4 * 4;       // [NO] f32 (pad actions: -inf; value last)
  L.table = L.hbias + NO * 4;                   // [4][NO] f32 raw logits of the obs e_0..e_3 (empty window)
  L.total = (L.table + 4 * NO * 4 + 15) & ~15;
  L.logits = L.total;                           // LDS only: [POL_ENVS][NO] f32 for the epilogue
  L.info = L.logits + POL_ENVS * NO * 4;        // LDS only: [POL_ENVS] u8
  L.list = L.info + POL_ENVS;                   // LDS only: [POL_ENVS] i16 envs with a lit window cell
  L.count = L.list + POL_ENVS * 2;              // LDS only: i32
  L.lds = L.count + 16;
  return L;
}


// Sum over the 4 lane groups (lanes l, l^16, l^32, l^48) of four values at once: lane group
// (row) r gets the full sum of value r, added as ((g0 + g1) + (g2 + g3)) -- two permlane16
// swaps pair the values' rows, one permlane32 swap finishes all four (6 VALU instructions
// where one value at a time takes 16).
__device__ __forceinline__ float sum_groups4(float x0, float x1, float x2, float x3) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x0), __float_as_uint(x1), false, false);
  const float c = __uint_as_float(a[0]) + __uint_as_float(a[1]);   // rows: x0 01, x1 01, x0 23, x1 23
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(x2), __float_as_uint(x3), false, false);
  const float e = __uint_as_float(b[0]) + __uint_as_float(b[1]);   // rows: x2 01, x3 01, x2 23, x3 23
  const auto d = __builtin_amdgcn_permlane32_swap(__float_as_uint(c), __float_as_uint(e), false, false);
  return __uint_as_float(d[0]) + __uint_as_float(d[1]);
}

// A tile's NO outputs in NQ = ceil(NO/4) registers: register q of lane group g holds output 4q + g.
template <int NO> struct PolQ { static constexpr int N = (NO + 3) / 4; };
template <int NO>
__device__ __forceinline__ void sum_outputs(const float (&part)[NO], float (&out)[PolQ<NO>::N]) {
#pragma unroll
  for (int q = 0; q < PolQ<NO>::N; ++q) {
    auto at = [&](int o) { return o < NO ? part[o] : 0.f; };
    out[q] = sum_groups4(at(4 * q), at(4 * q + 1), at(4 * q + 2), at(4 * q + 3));
  }
}


// OR of x over lanes l, l^16, l^32, l^48
// The packed image (global, 16-B words) into LDS by NT threads, U loads in flight per thread: a
// plain `for (k = tid; k < n16; k += NT) dst[k] = src[k]` waits for each load before the next
// one is issued (the LDS write needs it), one memory latency per pass -- 22 passes for the 89-KB
// W=10 image in a 256-thread block.  Slots past the end re-read and re-write the last word (the same
// value): no branch, which would let the compiler sink each load next to its write again.
template <int NT, int U>
__device__ __forceinline__ void stage_image(uint4* dst, const uint4* src, int n16, int tid) {
  for (int k0 = tid; k0 < n16; k0 += U * NT) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[min(k0 + u * NT, n16 - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) dst[min(k0 + u * NT, n16 - 1)] = v[u];
  }
}

__device__ __forceinline__ uint32_t or_groups(uint32_t x) {
  const auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  x = a[0] | a[1];
  const auto b = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return b[0] | b[1];
}

// fc1 pre-activation from its three digit-plane accumulators: hi * 2^16 + mid * 2^8 + lo (mod 2^32),
// as (((hi << 8) + mid) << 8) + lo: two v_lshl_add_u32.  The empty asm keeps the inner sum from
// being re-associated into the compiler's form (two shifts and an add3, one VALU instruction more
// per element); the instructions themselves stay the compiler's, so it still inserts the wait
// states a VALU read of an MFMA result needs.
__device__ __forceinline__ int digits(int hi, int mid, int lo) {
  uint32_t t = ((uint32_t)hi << 8) + (uint32_t)mid;
  asm("" : "+v"(t));
  return (int)((t << 8) + (uint32_t)lo);
}

// Hidden rows are summed in 4 fixed chunks of 16-row tiles, chunk c = [c*HT/4, (c+1)*HT/4):
// logit = ((s_0 + s_1) + s_2) + s_3 with s_c the chunk's FMA chain summed over the lane groups.
// One wave can run all four (tile_forward) or four waves one each (the fused rollout kernel),
// with the same result bit for bit.
constexpr int POL_CHUNKS = 4;
__host__ __device__ constexpr int pol_chunk_begin(int HT, int c) { return (c * HT) / POL_CHUNKS; }

// One chunk [ht0, ht1) of the dense forward of a 16-env column tile (env of lane = lane & 15,
// obs fragments B): fc1 on the int8 MFMA, relu, heads.  Returns the chunk's raw logit partials
// (no head bias), summed over the lane groups, in PolQ layout: register q of lane group g holds
// output 4q + g of the env of column lane & 15.
template <int HT, int KS, int NO, int LEN = 0>
__device__ __forceinline__ void tile_chunk(const uint8_t* lds, const v4i (&B)[KS], int lane, int dbg, int ht0,
                                           int ht1, float (&out)[PolQ<NO>::N]) {
  constexpr PolLayout L = pol_layout(HT, KS, NO);
  const int g = lane >> 4;
  float part[NO];
#pragma unroll
  for (int o = 0; o < NO; ++o) part[o] = 0.f;
  const int n = LEN > 0 ? LEN : ht1 - ht0;
#pragma unroll
  for (int j = 0; j < (LEN > 0 ? LEN : HT); ++j) {
    if (LEN == 0 && j >= n) break;
    const int ht = ht0 + j;
    v4i acc[3];   // one accumulator per digit plane: no VALU between a tile row's MFMAs
    acc[0] = v4i{0, 0, 0, 0};
    acc[1] = v4i{0, 0, 0, 0};
    acc[2] = *(const v4i*)(lds + L.bias + (ht * 16 + 4 * g) * 4);
    if (!(dbg & 2)) {
#pragma unroll
      for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const v4i a = *(const v4i*)(lds + L.frag + ((((ht * 3 + d) * KS + ks) * 64 + lane) << 4));
          acc[d] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, B[ks], acc[d], 0, 0, 0);
        }
    } else {
      acc[2] += B[0];
    }
    float h[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = digits(acc[0][r], acc[1][r], acc[2][r]);
      h[r] = (float)(q > 0 ? q : 0);
    }
    if (!(dbg & 4)) {
#pragma unroll
      for (int o = 0; o < NO; ++o) {
        const float4 w = *(const float4*)(lds + L.head + (((ht * 4 + g) * NO + o) * 4) * 4);
        part[o] = fmaf(w.w, h[3], fmaf(w.z, h[2], fmaf(w.y, h[1], fmaf(w.x, h[0], part[o]))));
      }
    } else {
      part[0] += h[0] + h[1] + h[2] + h[3];
    }
  }
  sum_outputs<NO>(part, out);
}

// tile_chunk for two tiles at once (B0, B1): the fc1 digit fragments and head weights are
// read once for both, and the two tiles' chains interleave.  Each tile's arithmetic is
// tile_chunk's, in the same order (bit-identical partials).
// LEN > 0: the chunk has exactly LEN rows (fully unrolled: the loads of row j+1 can be issued
// under row j's MFMAs); LEN == 0: a runtime trip count.
template <int HT, int KS, int NO, int LEN = 0>
__device__ __forceinline__ void tile_chunk2(const uint8_t* lds, const v4i (&B0)[KS], const v4i (&B1)[KS], int lane,
                                            int ht0, int ht1, float (&out0)[PolQ<NO>::N],
                                            float (&out1)[PolQ<NO>::N]) {
  constexpr PolLayout L = pol_layout(HT, KS, NO);
  const int g = lane >> 4;
  float p0[NO], p1[NO];
#pragma unroll
  for (int o = 0; o < NO; ++o) { p0[o] = 0.f; p1[o] = 0.f; }
  const int n = LEN > 0 ? LEN : ht1 - ht0;
#pragma unroll
  for (int j = 0; j < (LEN > 0 ? LEN : HT); ++j) {
    if (LEN == 0 && j >= n) break;
    const int ht = ht0 + j;
    v4i a0[3], a1[3];
    a0[0] = v4i{0, 0, 0, 0};
    a0[1] = v4i{0, 0, 0, 0};
    a0[2] = *(const v4i*)(lds + L.bias + (ht * 16 + 4 * g) * 4);
    a1[0] = a0[0]; a1[1] = a0[1]; a1[2] = a0[2];
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const v4i a = *(const v4i*)(lds + L.frag + ((((ht * 3 + d) * KS + ks) * 64 + lane) << 4));
        a0[d] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, B0[ks], a0[d], 0, 0, 0);
        a1[d] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, B1[ks], a1[d], 0, 0, 0);
      }
    float h0[4], h1[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q0 = digits(a0[0][r], a0[1][r], a0[2][r]);
      const int q1 = digits(a1[0][r], a1[1][r], a1[2][r]);
      h0[r] = (float)(q0 > 0 ? q0 : 0);
      h1[r] = (float)(q1 > 0 ? q1 : 0);
    }
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const float4 w = *(const float4*)(lds + L.head + (((ht * 4 + g) * NO + o) * 4) * 4);
      p0[o] = fmaf(w.w, h0[3], fmaf(w.z, h0[2], fmaf(w.y, h0[1], fmaf(w.x, h0[0], p0[o]))));
      p1[o] = fmaf(w.w, h1[3], fmaf(w.z, h1[2], fmaf(w.y, h1[1], fmaf(w.x, h1[0], p1[o]))));
    }
  }
  sum_outputs<NO>(p0, out0);
  sum_outputs<NO>(p1, out1);
}

// The whole dense forward of one tile on one wave: the four chunks in order.
template <int HT, int KS, int NO>
__device__ __forceinline__ void tile_forward(const uint8_t* lds, const v4i (&B)[KS], int lane, int dbg,
                                             float (&out)[PolQ<NO>::N]) {
#pragma unroll
  for (int c = 0; c < POL_CHUNKS; ++c) {
    float part[PolQ<NO>::N];
    tile_chunk<HT, KS, NO>(lds, B, lane, dbg, pol_chunk_begin(HT, c), pol_chunk_begin(HT, c + 1), part);   // (inlined: constant bounds)
#pragma unroll
    for (int q = 0; q < PolQ<NO>::N; ++q) out[q] = c == 0 ? part[q] : out[q] + part[q];
  }
}

// select_action's tail for one env (ball_cnn_ac3.py:139-146, 210-220), in two parts:
// policy_dist turns raw logits src (no head bias) + hb into the Categorical's CDF over the A
// actions (softmax, pads are -inf), the log-probability of each action and the value head;
// policy_pick draws by inverse CDF of u.  policy_finish is both, with u from
// Philox(seed; gid, episode, ep_len, POLICY).  An env on the empty-window table has one of 4
// distributions, which the fused rollout computes once per launch -- same ops, same result.
// pick_policy builds the NO = 10 layouts only for A = 9 actions (NO = A + 1: no pad outputs); the
// generic NO = 16 layout pads with -inf logits.  With no pads every `o < A` test below is true at
// compile time (a runtime A kept nine loop-invariant lane masks live in spilled SGPRs).
__host__ __device__ constexpr bool pol_unpadded(int NO) { return NO == 10; }

template <int NO>
struct PolDist {
  float cdf[NO - 1];   // running sum of the probabilities (the draw's comparison values)
  float lp[NO - 1];    // log_prob of each action
  float value;
  int last_nz;         // last action with a nonzero probability
};

template <int NO>
__device__ __forceinline__ PolDist<NO> policy_dist(const float* src, const float* hb, int A, float* probs_row) {
  if constexpr (pol_unpadded(NO)) A = NO - 1;
  PolDist<NO> d;
  float logit[NO];
#pragma unroll
  for (int o = 0; o < NO; ++o) logit[o] = src[o] + hb[o];
  float mx = logit[0];
#pragma unroll
  for (int o = 1; o < NO - 1; ++o) mx = fmaxf(mx, logit[o]);
  float e[NO - 1], sum = 0.f;
#pragma unroll
  for (int o = 0; o < NO - 1; ++o) { e[o] = __expf(logit[o] - mx); sum += e[o]; }
  const float inv = __builtin_amdgcn_rcpf(sum);
  const float lsum = __logf(sum);
  float c = 0.f;
  d.last_nz = 0;
#pragma unroll
  for (int o = 0; o < NO - 1; ++o) {
    const float pr = e[o] * inv;
    c += pr;
    d.cdf[o] = c;
    d.lp[o] = (logit[o] - mx) - lsum;
    d.last_nz = (o < A && pr > 0.f) ? o : d.last_nz;
    if (probs_row && o < A) probs_row[o] = pr;
  }
  d.value = logit[NO - 1];
  return d;
}

__device__ __forceinline__ float policy_uniform(uint32_t gid, uint32_t episode, uint32_t len, unsigned long long seed) {
  const u4 r = philox(gid, episode, len, tag(PURPOSE_POLICY, 0), seed);
  return (float)(r.x >> 8) * (1.0f / 16777216.0f);
}

// cdf / lp / last_nz may point into LDS (the fused rollout's per-quadrant table)
template <int NO>
__device__ __forceinline__ int policy_pick(const float* cdf, const float* lp, int last_nz, int A, float u,
                                           float& log_prob) {
  if constexpr (pol_unpadded(NO)) A = NO - 1;
  int act = 0;
#pragma unroll
  for (int o = 0; o < NO - 1; ++o) act += (o < A && cdf[o] <= u) ? 1 : 0;
  act = act > last_nz ? last_nz : act;
  float la = lp[0];
#pragma unroll
  for (int o = 1; o < NO - 1; ++o) {
    la = o == act ? lp[o] : la;
    // a select chain the compiler would otherwise turn into lp[act] on a scratch copy of lp
    asm volatile("" : "+v"(la));
  }
  log_prob = la;
  return act;
}

template <int NO>
__device__ __forceinline__ int policy_finish(const float* src, const float* hb, int A, uint32_t gid, uint32_t episode,
                                             uint32_t len, unsigned long long seed, float* probs_row, float& log_prob,
                                             float& value) {
  const PolDist<NO> d = policy_dist<NO>(src, hb, A, probs_row);
  value = d.value;
  return policy_pick<NO>(d.cdf, d.lp, d.last_nz, A, policy_uniform(gid, episode, len, seed), log_prob);
}

}  // namespace
