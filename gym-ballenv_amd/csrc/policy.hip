// policy.hip -- on-GPU select_action for the batched rollout (BASELINE config 5,
// SURVEY.md §8 a8): the reference's A2C Policy(W) forward plus Categorical
// sampling, one launch for every env, reading the u8 window obs the step
// kernel wrote.  Its own translation unit, built with -fno-slp-vectorize
// (packed f32 FMAs beside MFMAs cost more than scalar ones on gfx950) and linked
// into libballenv.so; it shares philox.h with the step kernels and reaches the
// context through internal.h.
//
// Reference (examples/ball_cnn_ac3.py):
//   Policy.__init__ / forward   :109-146   h = relu(fc1(x)); probs = softmax(action_head(h)); v = value_head(h)
//   select_action               :210-220   a ~ Categorical(probs); saved (log_prob(a), v)
//   hidden = 128 (W=5) / 208 (W=10), 9 actions (move_list :530)
//
// fc1 on the int8 matrix cores, exactly.  The obs is 0/1, so fc1(x) = b1 + the
// sum of the weight columns of the set inputs.  Each fc1 row k is quantised
// once (pack kernel) to fixed point with step s_k = max(max|W1[k,:]|, |b1_k|/64)
// / (127 * 2^16): weights to 24 bits, q = rint(w / s_k), split into three
// signed int8 digits (q = d2*2^16 + d1*2^8 + d0), and the bias to bq_k =
// rint(b1_k / s_k).  The obs bytes ARE the int8 B operand of
// v_mfma_i32_16x16x64_i8, the three digit planes accumulate in three i32
// accumulators (the d0 one starts at bq_k), and Q = acc2<<16 + acc1<<8 + acc0
// is the exact integer sum.  relu is max(Q, 0) on the integer, and s_k is
// folded into the head weights (pack: (W_head * s)[o][k] in f32), so
//   logit_o = b_o + sum_k (W_o,k s_k) * float(max(Q_k, 0)).
// Error per set input <= s_k/2 (2^-24 of the row's largest weight, one fp32
// half-ulp), plus fp32 roundings in the head sums -- the accuracy of an fp32
// GEMM (tests/test_gpu_policy.py bounds it against an fp64 evaluation).
//
// Work split (256 envs per workgroup, one workgroup per CU at 65536 envs):
//  * compute: 16 waves (4 per SIMD), one 16-env column tile each.  D = W1q
//    (hidden x K) . obs^T (K x env), so the env is the MFMA column (lane & 15)
//    and each lane holds 4 hidden units of its env per 16-row tile; the heads
//    are per-lane fp32 FMAs over those units, summed over the 4 lane groups
//    with v_permlane16/32_swap;
//  * epilogue: the logits go through LDS and 4 waves finish 64 envs each with
//    every lane busy -- softmax, log_prob, value, and an inverse-CDF draw from
//    Philox(seed; gid, episode, ep_len, POLICY), a pure function of per-env
//    state like every other draw in this library.
#include <hip/hip_runtime.h>

#include <math.h>
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

struct PolPack {             // pack kernel arguments (device f32 weights in torch state_dict layout)
  const float* w1; const float* b1; const float* wa; const float* ba; const float* wv; const float* bv;
  int H, F, A;
};

// One block, one thread per padded hidden row (HT*16 <= 256).
__global__ void policy_pack_kernel(PolPack a, uint8_t* img, PolLayout L) {
  const int m = threadIdx.x;
  if (m >= L.HT * 16) return;
  int32_t* bias = (int32_t*)(img + L.bias);
  float* head = (float*)(img + L.head);
  float* hb = (float*)(img + L.hbias);
  const bool real = m < a.H;
  float mx = 0.f;
  if (real) {
    for (int k = 0; k < a.F; ++k) mx = fmaxf(mx, fabsf(a.w1[(int64_t)m * a.F + k]));
    mx = fmaxf(mx, fabsf(a.b1[m]) * (1.0f / 64.0f));
  }
  const double s = mx > 0.f ? (double)(float)((double)mx / 8323072.0) : 1.0;   // 127 * 2^16
  bias[m] = real ? (int32_t)llrint((double)a.b1[m] / s) : 0;
  const int ht = m >> 4, row = m & 15;
  for (int k = 0; k < L.KS * 64; ++k) {
    long long q = 0;
    if (real && k < a.F) {
      q = llrint((double)a.w1[(int64_t)m * a.F + k] / s);
      q = q > 8323072 ? 8323072 : (q < -8323072 ? -8323072 : q);
    }
    const int d0 = (int)(((q + 128) & 255) - 128);
    const long long q1 = (q - d0) >> 8;
    const int d1 = (int)(((q1 + 128) & 255) - 128);
    const int d2 = (int)((q1 - d1) >> 8);
    const int ks = k >> 6, g = (k >> 4) & 3, j = k & 15, lane = row + 16 * g;
    const int dig[3] = {d2, d1, d0};
    for (int d = 0; d < 3; ++d)
      img[L.frag + ((((ht * 3 + d) * L.KS + ks) * 64 + lane) * 16 + j)] = (uint8_t)(int8_t)dig[d];
  }
  // head weights, scaled by s_k: output o < A -> action_head[o], o == NO-1 -> value_head, else 0
  const int g = (m >> 2) & 3, r = m & 3;
  for (int o = 0; o < L.NO; ++o) {
    double w = 0.0;
    if (real) {
      if (o < a.A) w = a.wa[(int64_t)o * a.H + m];
      else if (o == L.NO - 1) w = a.wv[m];
    }
    head[((ht * 4 + g) * L.NO + o) * 4 + r] = (float)(w * s);
  }
  if (m < L.NO) hb[m] = m < a.A ? a.ba[m] : (m == L.NO - 1 ? a.bv[0] : -INFINITY);
}

struct PParams {
  const uint8_t* img;        // packed weights (PolLayout)
  const uint8_t* obs;        // (N, F) u8
  const uint32_t* episode;   // (N) Philox key words (be_state.episode / ep_len)
  const int32_t* ep_len;
  uint8_t* action;           // (N) u8
  float* log_prob;           // (N) or NULL
  float* value;              // (N) or NULL
  float* probs;              // (N, A) or NULL
  float* table_out;          // table mode: (N, NO) raw logits, every env dense, no draw
  unsigned long long seed;
  int32_t n, F, A, gid0;
  int32_t img_bytes;
  int32_t dbg;               // BALLENV_POLICY_DEBUG ablation bits (timing only): 1 no staging, 2 no MFMA,
                             // 4 no head FMAs, 8 no epilogue, 16 exit at entry, 32 every env dense
};

// 16 obs bytes of env `env` starting at column c (zero beyond F / beyond N).
// ALIGNED8 (F % 8 == 0): two 8-byte loads at clamped, always in-bounds addresses and
// selects -- no branches around the loads.
template <bool ALIGNED8>
__device__ __forceinline__ v4i load_obs16(const PParams& p, int env, int c) {
  v4i v = {0, 0, 0, 0};
  if (ALIGNED8) {
    const bool ok = env < p.n;
    const uint8_t* row = p.obs + (int64_t)(ok ? env : p.n - 1) * p.F;
    const int c0 = c < p.F - 8 ? c : p.F - 8, c1 = c + 8 < p.F - 8 ? c + 8 : p.F - 8;
    const uint2 lo = *(const uint2*)(row + c0), hi = *(const uint2*)(row + c1);
    const bool vlo = ok && c + 8 <= p.F, vhi = ok && c + 16 <= p.F;
    v[0] = vlo ? (int)lo.x : 0; v[1] = vlo ? (int)lo.y : 0;
    v[2] = vhi ? (int)hi.x : 0; v[3] = vhi ? (int)hi.y : 0;
    return v;
  }
  if (env >= p.n || c >= p.F) return v;
  const uint8_t* row = p.obs + (int64_t)env * p.F;
  uint32_t w[4] = {0, 0, 0, 0};
  for (int j = 0; j < 16 && c + j < p.F; ++j) w[j >> 2] |= (uint32_t)row[c + j] << (8 * (j & 3));
  v[0] = (int)w[0]; v[1] = (int)w[1]; v[2] = (int)w[2]; v[3] = (int)w[3];
  return v;
}

// Sparse structure of the input: an env whose window has no lit cell has the obs e_q (its
// quadrant one-hot) -- over 90 % of envs in rollouts (0.7 % of obs have a lit cell under
// random actions, 7.6 % under the reference's trained Policy(10)).  Their logits are the
// 4-entry table the pack step computes by running tile_forward on the obs e_0..e_3, so they
// are bit-identical to the dense result.  Each workgroup compacts its envs with a lit cell
// into a list in LDS and only those go through the matrix cores, in 16-env tiles.
// p.table_out != NULL: "table mode" -- every env dense, raw logits to table_out (no draw).
template <int HT, int KS, int NO, bool ALIGNED8>
__global__ __launch_bounds__(POL_THREADS) void policy_kernel(PParams p) {
  extern __shared__ uint4 pol_lds[];
  constexpr PolLayout L = pol_layout(HT, KS, NO);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int blk0 = blockIdx.x * POL_ENVS;
  const int tile0 = blk0 + wave * 16;                 // this wave's 16 envs for the scan
  if (p.dbg & 16) return;                             // ablation: launch cost alone
  uint8_t* lds = (uint8_t*)pol_lds;
  uint8_t* info = lds + L.info;                       // per env: bit 7 = a lit cell, bits 0-1 = quadrant
  int16_t* list = (int16_t*)(lds + L.list);
  int* count = (int*)(lds + L.count);
  const bool dense = p.table_out != nullptr || (p.dbg & 32);
  if (tid == 0) *count = 0;

  // the epilogue's Philox key words, prefetched (lane l of wave w < 4 finishes env blk0 + 64w + l)
  const int e_loc = wave * 64 + lane, my_env = blk0 + e_loc;
  const bool fin = wave < POL_FIN_WAVES && my_env < p.n;
  const uint32_t episode = fin ? p.episode[my_env] : 0u;
  const int32_t len = fin ? p.ep_len[my_env] : 0;

  // scan: this wave's 16 envs, 16 obs bytes per lane and K step (the B-operand layout)
  v4i B[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) B[ks] = load_obs16<ALIGNED8>(p, tile0 + (lane & 15), 64 * ks + 16 * g);
  uint32_t lit = 0;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    lit |= ((ks == 0 && g == 0) ? 0u : (uint32_t)B[ks][0]) | (uint32_t)B[ks][1] | (uint32_t)B[ks][2] | (uint32_t)B[ks][3];
  lit = or_groups(lit);
  __syncthreads();   // *count = 0 is visible

  if (!(p.dbg & 1)) {  // stage the packed weights (overlaps the scan's loads)
    const uint4* src = (const uint4*)p.img;
    const int n16 = p.img_bytes >> 4;
    stage_image<POL_THREADS, 6>(pol_lds, src, n16, tid);
  }
  if (g == 0 && tile0 + lane < p.n) {
    // obs bytes 0..3 must be exactly a quadrant one-hot for the table (any other input is dense)
    const uint32_t q4 = (uint32_t)B[0][0];
    const int quad = q4 == 1u ? 0 : (q4 == 0x100u ? 1 : (q4 == 0x10000u ? 2 : 3));
    const bool onehot = q4 == 1u || q4 == 0x100u || q4 == 0x10000u || q4 == 0x1000000u;
    const bool nz = dense || lit != 0u || !onehot;
    info[wave * 16 + lane] = (uint8_t)(quad | (nz ? 0x80 : 0));
    if (nz) list[atomicAdd(count, 1)] = (int16_t)(wave * 16 + lane);
  }
  __syncthreads();   // weights staged, list complete

  float* lg = (float*)(lds + L.logits);
  const int cnt = *count;
  if (wave * 16 < cnt) {
    const int k = wave * 16 + (lane & 15);
    const int e = k < cnt ? list[k] : -1;
    v4i Bt[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) Bt[ks] = load_obs16<ALIGNED8>(p, e >= 0 ? blk0 + e : p.n, 64 * ks + 16 * g);
    float out[PolQ<NO>::N];
    tile_forward<HT, KS, NO>(lds, Bt, lane, p.dbg, out);
    if (e >= 0) {   // lane group g holds outputs g, g + 4, ...
#pragma unroll
      for (int q = 0; q < PolQ<NO>::N; ++q)
        if (4 * q + g < NO) lg[e * NO + 4 * q + g] = out[q];
    }
  }
  __syncthreads();
  if (wave >= POL_FIN_WAVES || (p.dbg & 8) || !fin) return;

  // epilogue: lane l of wave w finishes env blk0 + 64w + l
  const uint8_t inf = info[e_loc];
  const float* src = (inf & 0x80) ? lg + e_loc * NO : (const float*)(lds + L.table) + (inf & 3) * NO;
  if (p.table_out) {
#pragma unroll
    for (int o = 0; o < NO; ++o) p.table_out[(int64_t)my_env * NO + o] = src[o];
    return;
  }
  float lp, val;
  const int act = policy_finish<NO>(src, (const float*)(lds + L.hbias), p.A, (uint32_t)(p.gid0 + my_env), episode,
                                    (uint32_t)len, p.seed, p.probs ? p.probs + (int64_t)my_env * p.A : nullptr, lp, val);
  p.action[my_env] = (uint8_t)act;
  if (p.log_prob) p.log_prob[my_env] = lp;
  if (p.value) p.value[my_env] = val;
}

using PolFn = void (*)(PParams);
struct PolKernel { PolFn fn; int HT, KS, NO; };

PolKernel pick_policy(int H, int F, int A) {
  const bool a8 = (F % 8) == 0;
  if (A == 9 && H == 208 && F > 64 && F <= 128)
    return {a8 ? policy_kernel<13, 2, 10, true> : policy_kernel<13, 2, 10, false>, 13, 2, 10};
  if (A == 9 && H == 128 && F <= 64)
    return {a8 ? policy_kernel<8, 1, 10, true> : policy_kernel<8, 1, 10, false>, 8, 1, 10};
  return {a8 ? policy_kernel<16, 2, 16, true> : policy_kernel<16, 2, 16, false>, 16, 2, 16};
}

}  // namespace

#define POL_TRY(ctx, expr)                                  \
  do {                                                      \
    hipError_t e_ = (expr);                                 \
    if (e_ != hipSuccess) return pol_hip_fail(ctx, e_);     \
  } while (0)

static int pol_hip_fail(be_ctx* ctx, hipError_t e) {
  char buf[256];
  snprintf(buf, sizeof buf, "HIP error: %s", hipGetErrorString(e));
  return be_ctx_fail(ctx, BE_E_HIP, buf);
}


struct be_policy {
  be_ctx* ctx;
  be_ctx_view cv;
  int H, F, A;
  PolKernel k;
  PolLayout L;
  uint8_t* img;
  uint8_t* obs4;     // (4, F) u8: the empty-window obs e_0..e_3 (table pass input)
  uint32_t* zero4;   // (4) zero episode / ep_len words for the table pass
  bool loaded;
  int dbg;
};

extern "C" {

int be_policy_create(be_ctx* ctx, int32_t hidden, int32_t num_actions, be_policy** out) {
  if (!ctx || !out) return be_ctx_fail(ctx, BE_E_INVALID, "bad arguments to be_policy_create");
  *out = nullptr;
  const be_ctx_view cv = be_ctx_get(ctx);
  const int F = 4 + cv.window * cv.window;
  if (hidden < 1 || hidden > POL_MAXH) return be_ctx_fail(ctx, BE_E_INVALID, "policy hidden size must be in [1, 256]");
  if (F > POL_MAXF) return be_ctx_fail(ctx, BE_E_INVALID, "policy input 4+W*W must be <= 128 (W <= 11)");
  if (num_actions < 1 || num_actions > POL_MAXA)
    return be_ctx_fail(ctx, BE_E_INVALID, "policy actions must be in [1, 15]");
  be_policy* pol = new (std::nothrow) be_policy();
  if (!pol) return be_ctx_fail(ctx, BE_E_NOMEM, "out of host memory");
  pol->ctx = ctx; pol->cv = cv; pol->H = hidden; pol->F = F; pol->A = num_actions;
  pol->k = pick_policy(hidden, F, num_actions);
  if (pol_unpadded(pol->k.NO) && pol->k.NO != num_actions + 1) {   // the kernels' compile-time A
    delete pol;
    return be_ctx_fail(ctx, BE_E_INVALID, "policy layout / action count mismatch");
  }
  if (const char* d = getenv("BALLENV_POLICY_DEBUG")) pol->dbg = (int)strtoul(d, nullptr, 0);
  pol->L = pol_layout(pol->k.HT, pol->k.KS, pol->k.NO);
  if (pol->L.lds > 160 * 1024) {
    delete pol;
    return be_ctx_fail(ctx, BE_E_INVALID, "packed policy exceeds the LDS budget");
  }
  const DeviceGuard dg(cv.device);   // the caller's current device is restored on return
  int rc = dg.err == hipSuccess ? BE_OK : pol_hip_fail(ctx, dg.err);
  hipError_t e = hipSuccess;
  if (rc == BE_OK) e = hipMalloc(&pol->img, (size_t)pol->L.total);
  if (rc == BE_OK && e == hipSuccess) e = hipMemset(pol->img, 0, (size_t)pol->L.total);
  if (rc == BE_OK && e == hipSuccess) e = hipMalloc(&pol->obs4, (size_t)4 * F);
  if (rc == BE_OK && e == hipSuccess) e = hipMalloc(&pol->zero4, 4 * sizeof(uint32_t));
  if (rc == BE_OK && e == hipSuccess) e = hipMemset(pol->zero4, 0, 4 * sizeof(uint32_t));
  if (rc == BE_OK && e == hipSuccess) {
    uint8_t h[4 * POL_MAXF];
    memset(h, 0, sizeof h);
    for (int q = 0; q < 4; ++q) h[q * F + q] = 1;
    e = hipMemcpy(pol->obs4, h, (size_t)4 * F, hipMemcpyHostToDevice);
  }
  if (rc == BE_OK && e != hipSuccess) rc = pol_hip_fail(ctx, e);
  if (rc != BE_OK) {
    if (pol->img) (void)hipFree(pol->img);
    if (pol->obs4) (void)hipFree(pol->obs4);
    if (pol->zero4) (void)hipFree(pol->zero4);
    delete pol;
    return rc;
  }
  *out = pol;
  return BE_OK;
}

int be_policy_destroy(be_policy* pol) {
  if (!pol) return BE_OK;
  const DeviceGuard dg(pol->cv.device);   // the caller's current device is restored on return
  if (pol->img) (void)hipFree(pol->img);
  if (pol->obs4) (void)hipFree(pol->obs4);
  if (pol->zero4) (void)hipFree(pol->zero4);
  delete pol;
  return BE_OK;
}

int be_policy_load(be_policy* pol, const float* fc1_w, const float* fc1_b, const float* act_w, const float* act_b,
                   const float* val_w, const float* val_b, void* stream) {
  if (!pol) return be_ctx_fail(nullptr, BE_E_INVALID, "policy is NULL");
  be_ctx* ctx = pol->ctx;
  if (!fc1_w || !fc1_b || !act_w || !act_b || !val_w || !val_b)
    return be_ctx_fail(ctx, BE_E_INVALID, "be_policy_load: a weight pointer is NULL");
  const DeviceGuard dg(pol->cv.device);   // the caller's current device is restored on return
  POL_TRY(ctx, dg.err);
  const PolPack a{fc1_w, fc1_b, act_w, act_b, val_w, val_b, pol->H, pol->F, pol->A};
  hipLaunchKernelGGL(policy_pack_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, a, pol->img, pol->L);
  POL_TRY(ctx, hipGetLastError());
  // table pass: the dense forward of the 4 empty-window obs, into the image's table
  PParams p;
  memset(&p, 0, sizeof p);
  p.img = pol->img; p.obs = pol->obs4; p.episode = pol->zero4; p.ep_len = (const int32_t*)pol->zero4;
  p.table_out = (float*)(pol->img + pol->L.table);
  p.n = 4; p.F = pol->F; p.A = pol->A; p.img_bytes = pol->L.total;
  hipLaunchKernelGGL(pol->k.fn, dim3(1), dim3(POL_THREADS), (size_t)pol->L.lds, (hipStream_t)stream, p);
  POL_TRY(ctx, hipGetLastError());
  pol->loaded = true;
  return BE_OK;
}

int be_policy_act(be_policy* pol, const be_state* st, const uint8_t* obs, const be_act_out* out, uint64_t seed,
                  void* stream) {
  if (!pol) return be_ctx_fail(nullptr, BE_E_INVALID, "policy is NULL");
  be_ctx* ctx = pol->ctx;
  if (!pol->loaded) return be_ctx_fail(ctx, BE_E_INVALID, "be_policy_act before be_policy_load");
  if (!st || !st->episode || !st->ep_len || !obs || !out || !out->action)
    return be_ctx_fail(ctx, BE_E_INVALID, "be_policy_act needs state episode/ep_len, obs and out->action");
  const DeviceGuard dg(pol->cv.device);   // the caller's current device is restored on return
  POL_TRY(ctx, dg.err);
  PParams p;
  memset(&p, 0, sizeof p);
  p.img = pol->img; p.obs = obs; p.episode = st->episode; p.ep_len = st->ep_len;
  p.action = out->action; p.log_prob = out->log_prob; p.value = out->value; p.probs = out->probs;
  p.seed = (unsigned long long)seed; p.n = pol->cv.num_envs; p.F = pol->F; p.A = pol->A;
  p.gid0 = (int32_t)(uint32_t)pol->cv.env_offset; p.img_bytes = pol->L.total; p.dbg = pol->dbg;
  const dim3 grid((unsigned)((p.n + POL_ENVS - 1) / POL_ENVS));
  hipLaunchKernelGGL(pol->k.fn, grid, dim3(POL_THREADS), (size_t)pol->L.lds, (hipStream_t)stream, p);
  POL_TRY(ctx, hipGetLastError());
  return BE_OK;
}

int be_policy_rollout(be_policy* pol, const be_state* st, const uint8_t* obs_in, uint8_t* obs_last, int32_t steps,
                      const be_out* out, const be_act_out* act, uint64_t seed, void* stream) {
  if (!pol) return be_ctx_fail(nullptr, BE_E_INVALID, "policy is NULL");
  be_ctx* ctx = pol->ctx;
  if (!pol->loaded) return be_ctx_fail(ctx, BE_E_INVALID, "be_policy_rollout before be_policy_load");
  if (int rc = be_ctx_check_state(ctx, st)) return rc;
  if (!obs_in || steps < 0 || !out || !out->reward || !out->done || !act || !act->action)
    return be_ctx_fail(ctx, BE_E_INVALID, "be_policy_rollout needs obs_in, steps >= 0, out->reward/done, act->action");
  if (!out->obs && !obs_last) return be_ctx_fail(ctx, BE_E_INVALID, "be_policy_rollout needs out->obs or obs_last");
  if (out->obs_f32 || out->terminal_obs || act->probs)
    return be_ctx_fail(ctx, BE_E_INVALID, "be_policy_rollout: obs_f32, terminal_obs and probs must be NULL");
  const int64_t N = pol->cv.num_envs, F = pol->F;
  if (((uintptr_t)obs_in & 15) || ((uintptr_t)obs_last & 15) || ((uintptr_t)out->obs & 15) || (N * F) % 16)
    return be_ctx_fail(ctx, BE_E_INVALID,
                       "be_policy_rollout needs 16-byte aligned obs buffers and num_envs * (4+W*W) % 16 == 0");
  if (steps == 0) return BE_OK;
  const DeviceGuard dg(pol->cv.device);   // the caller's current device is restored on return
  POL_TRY(ctx, dg.err);
  const be_pol_rollout_args r{pol->img, pol->L.total, pol->k.HT, pol->k.KS, pol->k.NO, pol->A,
                              (unsigned long long)seed, obs_in, obs_last, steps, out, act};
  const int rc = be_internal_policy_rollout(ctx, st, &r, stream);
  if (rc != 0) return rc < 0 ? rc : BE_OK;
  // no fused kernel for this shape: be_policy_act + be_step per step (the same trajectory)
  for (int32_t s = 0; s < steps; ++s) {
    const uint8_t* o_in = s == 0 ? obs_in : (out->obs ? out->obs + (s - 1) * N * F : obs_last);
    const be_act_out ao{act->action + s * N, act->log_prob ? act->log_prob + s * N : nullptr,
                        act->value ? act->value + s * N : nullptr, nullptr};
    if (int e = be_policy_act(pol, st, o_in, &ao, seed, stream)) return e;
    be_out o = *out;
    o.obs = out->obs ? out->obs + s * N * F : obs_last;
    o.reward = out->reward + s * N;
    o.done = out->done + s * N;
    if (o.truncated) o.truncated = out->truncated + s * N;
    if (o.final_return) o.final_return = out->final_return + s * N;
    if (o.final_len) o.final_len = out->final_len + s * N;
    if (int e = be_step(ctx, st, ao.action, nullptr, nullptr, &o, stream)) return e;
  }
  if (out->obs && obs_last)
    POL_TRY(ctx, hipMemcpyAsync(obs_last, out->obs + (steps - 1) * N * F, (size_t)(N * F), hipMemcpyDeviceToDevice,
                                (hipStream_t)stream));
  return BE_OK;
}

int64_t be_policy_bytes(const be_policy* pol) { return pol ? (int64_t)pol->L.total : 0; }

}  // extern "C"
