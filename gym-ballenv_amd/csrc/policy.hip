// policy.hip -- on-GPU select_action for the batched rollout (BASELINE config 5,
// SURVEY.md §8 a8): the reference's A2C Policy(W) forward plus Categorical
// sampling, one launch for every env, reading the u8 window obs the step
// kernel wrote.  #included at the end of ballenv.hip (one translation unit:
// it shares philox(), be_ctx and the error helpers).
//
// Reference (examples/ball_cnn_ac3.py):
//   Policy.__init__ / forward   :109-146   h = relu(fc1(x)); probs = softmax(action_head(h)); v = value_head(h)
//   select_action               :210-220   a ~ Categorical(probs); saved (log_prob(a), v)
//   hidden = 128 (W=5) / 208 (W=10), 9 actions (move_list :530)
//
// fc1 on the matrix cores, exactly.  The obs is 0/1, so fc1(x) = b1 + sum of
// the weight columns of the set inputs.  Each fc1 row k is quantised once to
// 24-bit fixed point, q = rint(w / s_k) with s_k = max|W1[k,:]| / (127 * 2^16),
// and split into three signed int8 digits (q = d2*2^16 + d1*2^8 + d0).  The
// obs bytes ARE the int8 B operand of v_mfma_i32_16x16x64_i8 (no conversion),
// and the digits are Horner-combined in the i32 accumulator
// (acc = ((d2.x) << 8 + d1.x) << 8 + d0.x): the integer dot product is exact,
// so h_k = b1_k + s_k * Q_k carries one quantisation error of <= s_k/2 per set
// input (<= 2^-24 max|W1[k,:]|, the size of one fp32 half-ulp of the largest
// weight) and a final fp32 rounding -- the same order as torch's fp32 GEMM.
//
// Tile orientation: D = W1q (hidden x K) . obs^T (K x env), so the env is the
// MFMA column = the lane (lane & 15) and each lane holds 4 hidden units of its
// env per 16-row tile; the heads (action logits + value) are then per-lane
// fp32 FMAs over those hidden units, reduced over the 4 lane groups with two
// xor-shuffles.  A wave owns 64 contiguous envs (4 column tiles of 16) and
// reuses every weight fragment (one ds_read_b128 from LDS) for its 4 tiles.
// After the reduction lane l finalises env (wave base + l): softmax, log_prob,
// value and an inverse-CDF draw from Philox(seed; gid, episode, ep_len,
// POLICY) -- a pure function of per-env state, like every other draw here.

namespace {

constexpr uint32_t PURPOSE_POLICY = 5;
constexpr int POL_MAXH = 256, POL_MAXF = 128, POL_MAXA = 15;

typedef int v4i __attribute__((ext_vector_type(4)));

// Packed-weight image (bytes), identical in HBM and in each block's LDS.
struct PolLayout {
  int HT, KS, NO;            // 16-row hidden tiles, 64-wide K steps, outputs (actions + value)
  int frag, scale, bias, head, hbias, total;
};
__host__ __device__ constexpr PolLayout pol_layout(int HT, int KS, int NO) {
  PolLayout L{};
  L.HT = HT; L.KS = KS; L.NO = NO;
  L.frag = 0;                                   // [HT][3 digits, high first][KS][64 lanes][16 B] int8
  L.scale = L.frag + HT * 3 * KS * 1024;        // [HT*16] f32  s_k
  L.bias = L.scale + HT * 16 * 4;               // [HT*16] f32  b1_k
  L.head = L.bias + HT * 16 * 4;                // [HT][4 groups][NO][4] f32  head weight of hidden 16ht+4g+r
  L.hbias = L.head + HT * 4 * NO * 4 * 4;       // [NO] f32 (pad actions: -inf; value last)
  L.total = (L.hbias + NO * 4 + 15) & ~15;
  return L;
}

struct PolPack {             // pack kernel arguments (device f32 weights in torch state_dict layout)
  const float* w1; const float* b1; const float* wa; const float* ba; const float* wv; const float* bv;
  int H, F, A;
};

// One block, one thread per padded hidden row (HT*16 <= 256).
__global__ void policy_pack_kernel(PolPack a, uint8_t* img, PolLayout L) {
  const int m = threadIdx.x;
  if (m >= L.HT * 16) return;
  float* scale = (float*)(img + L.scale);
  float* bias = (float*)(img + L.bias);
  float* head = (float*)(img + L.head);
  float* hb = (float*)(img + L.hbias);
  const bool real = m < a.H;
  float mx = 0.f;
  if (real)
    for (int k = 0; k < a.F; ++k) mx = fmaxf(mx, fabsf(a.w1[(int64_t)m * a.F + k]));
  const float s = mx > 0.f ? (float)((double)mx / 8323072.0) : 1.0f;   // 127 * 2^16
  scale[m] = real ? s : 0.f;
  bias[m] = real ? a.b1[m] : 0.f;
  const int ht = m >> 4, row = m & 15;
  for (int k = 0; k < L.KS * 64; ++k) {
    long long q = 0;
    if (real && k < a.F) {
      q = llrint((double)a.w1[(int64_t)m * a.F + k] / (double)s);
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
  // head weights: output o < A -> action_head[o], o == NO-1 -> value_head, else 0
  const int g = (m >> 2) & 3, r = m & 3;
  for (int o = 0; o < L.NO; ++o) {
    float w = 0.f;
    if (real) {
      if (o < a.A) w = a.wa[(int64_t)o * a.H + m];
      else if (o == L.NO - 1) w = a.wv[m];
    }
    head[((ht * 4 + g) * L.NO + o) * 4 + r] = w;
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
  unsigned long long seed;
  int32_t n, F, A, gid0;
  int32_t img_bytes;
  int32_t dbg;               // BALLENV_POLICY_DEBUG ablation bits (timing only): 1 no staging, 2 no MFMA,
                             // 4 no head FMAs, 8 no epilogue
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

constexpr int POL_ENVS_PER_BLOCK = 256;   // one 90-KB weight image per CU at 65536 envs

// T = 16-env column tiles per wave; a block has 256/(16T) waves (T=2: 8 waves, two per SIMD).
template <int HT, int KS, int NO, bool ALIGNED8, int T>
__global__ __launch_bounds__(64 * POL_ENVS_PER_BLOCK / (16 * T)) void policy_kernel(PParams p) {
  extern __shared__ uint4 pol_lds[];
  constexpr PolLayout L = pol_layout(HT, KS, NO);
  constexpr int NT = 64 * POL_ENVS_PER_BLOCK / (16 * T);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int env0 = blockIdx.x * POL_ENVS_PER_BLOCK + wave * 16 * T;

  // obs fragments (B operand) and the sampling key words, issued before the staging barrier
  v4i B[T][KS];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) B[t][ks] = load_obs16<ALIGNED8>(p, env0 + 16 * t + (lane & 15), 64 * ks + 16 * g);
  const int my_env = env0 + lane;
  const bool mine = g < T && my_env < p.n;          // lane l finalises env env0 + l (tile l >> 4)
  const uint32_t episode = mine ? p.episode[my_env] : 0u;
  const int32_t len = mine ? p.ep_len[my_env] : 0;

  if (!(p.dbg & 1)) {  // stage the packed weights
    const uint4* src = (const uint4*)p.img;
    const int n16 = p.img_bytes >> 4;
    for (int i = tid; i < n16; i += NT) pol_lds[i] = src[i];
  }
  __syncthreads();
  if (env0 >= p.n) return;

  const uint8_t* lds = (const uint8_t*)pol_lds;
  float part[T][NO];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int o = 0; o < NO; ++o) part[t][o] = 0.f;

#ifndef BE_POL_UNROLL
#define BE_POL_UNROLL 1
#endif
#pragma unroll BE_POL_UNROLL
  for (int ht = 0; ht < HT; ++ht) {
    v4i acc[3][T];   // one accumulator per digit: no VALU between the MFMAs of a tile row
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
      for (int t = 0; t < T; ++t) acc[d][t] = v4i{0, 0, 0, 0};
    if (!(p.dbg & 2)) {
#pragma unroll
      for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const v4i a = *(const v4i*)(lds + L.frag + ((((ht * 3 + d) * KS + ks) * 64 + lane) << 4));
#pragma unroll
          for (int t = 0; t < T; ++t)
            acc[d][t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, B[t][ks], acc[d][t], 0, 0, 0);
        }
    } else {
#pragma unroll
      for (int t = 0; t < T; ++t) acc[0][t] = B[t][0];
    }
    const float4 s = *(const float4*)(lds + L.scale + (ht * 16 + 4 * g) * 4);
    const float4 b = *(const float4*)(lds + L.bias + (ht * 16 + 4 * g) * 4);
    float4 wh[NO];
#pragma unroll
    for (int o = 0; o < NO; ++o) wh[o] = *(const float4*)(lds + L.head + (((ht * 4 + g) * NO + o) * 4) * 4);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      float h[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = (int)(((uint32_t)acc[0][t][r] << 16) + ((uint32_t)acc[1][t][r] << 8)) + acc[2][t][r];
        const float sr = r == 0 ? s.x : (r == 1 ? s.y : (r == 2 ? s.z : s.w));
        const float br = r == 0 ? b.x : (r == 1 ? b.y : (r == 2 ? b.z : b.w));
        h[r] = fmaxf(fmaf(sr, (float)q, br), 0.f);
      }
      if (!(p.dbg & 4)) {
#pragma unroll
        for (int o = 0; o < NO; ++o)
          part[t][o] = fmaf(wh[o].w, h[3], fmaf(wh[o].z, h[2], fmaf(wh[o].y, h[1], fmaf(wh[o].x, h[0], part[t][o]))));
      } else {
        part[t][0] += h[0] + h[1] + h[2] + h[3];
      }
    }
  }

  // sum over the 4 lane groups (hidden-unit quarters); lane l keeps tile l >> 4
  float logit[NO];
#pragma unroll
  for (int o = 0; o < NO; ++o) {
    float v[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      float x = part[t][o];
      x += __shfl_xor(x, 16);
      x += __shfl_xor(x, 32);
      v[t] = x;
    }
    float sel = v[0];
#pragma unroll
    for (int t = 1; t < T; ++t) sel = g == t ? v[t] : sel;
    logit[o] = sel + *(const float*)(lds + L.hbias + 4 * o);
  }
  if (!mine || (p.dbg & 8)) return;

  // softmax over the action logits (pads are -inf), Categorical draw by inverse CDF
  float mx = logit[0];
#pragma unroll
  for (int o = 1; o < NO - 1; ++o) mx = fmaxf(mx, logit[o]);
  float e[NO - 1], sum = 0.f;
#pragma unroll
  for (int o = 0; o < NO - 1; ++o) { e[o] = __expf(logit[o] - mx); sum += e[o]; }
  const float inv = __frcp_rn(sum);
  const u4 r = philox((uint32_t)(p.gid0 + my_env), episode, (uint32_t)len, tag(PURPOSE_POLICY, 0), p.seed);
  const float u = (float)(r.x >> 8) * (1.0f / 16777216.0f);
  float c = 0.f;
  int act = 0, last_nz = 0;
#pragma unroll
  for (int o = 0; o < NO - 1; ++o) {
    const float pr = e[o] * inv;
    c += pr;
    act += (o < p.A && c <= u) ? 1 : 0;
    last_nz = (o < p.A && pr > 0.f) ? o : last_nz;
    if (p.probs && o < p.A) p.probs[(int64_t)my_env * p.A + o] = pr;
  }
  act = act > last_nz ? last_nz : act;
  float lg = logit[0];
#pragma unroll
  for (int o = 1; o < NO - 1; ++o) lg = o == act ? logit[o] : lg;
  p.action[my_env] = (uint8_t)act;
  if (p.log_prob) p.log_prob[my_env] = (lg - mx) - __logf(sum);
  if (p.value) p.value[my_env] = logit[NO - 1];
}

using PolFn = void (*)(PParams);
struct PolKernel { PolFn fn; int HT, KS, NO, threads; };

#ifndef BE_POL_TILES
#define BE_POL_TILES 2
#endif
constexpr int POL_T = BE_POL_TILES;
constexpr int POL_THREADS = 64 * POL_ENVS_PER_BLOCK / (16 * POL_T);

PolKernel pick_policy(int H, int F, int A) {
  const bool a8 = (F % 8) == 0;
  if (A == 9 && H == 208 && F > 64 && F <= 128)
    return {a8 ? policy_kernel<13, 2, 10, true, POL_T> : policy_kernel<13, 2, 10, false, POL_T>, 13, 2, 10,
            POL_THREADS};
  if (A == 9 && H == 128 && F <= 64)
    return {a8 ? policy_kernel<8, 1, 10, true, POL_T> : policy_kernel<8, 1, 10, false, POL_T>, 8, 1, 10,
            POL_THREADS};
  return {a8 ? policy_kernel<16, 2, 16, true, POL_T> : policy_kernel<16, 2, 16, false, POL_T>, 16, 2, 16,
          POL_THREADS};
}

}  // namespace

struct be_policy {
  be_ctx* ctx;
  int H, F, A;
  PolKernel k;
  PolLayout L;
  uint8_t* img;
  bool loaded;
  int dbg;
};

extern "C" {

int be_policy_create(be_ctx* ctx, int32_t hidden, int32_t num_actions, be_policy** out) {
  if (!ctx || !out) return fail(ctx, BE_E_INVALID, "%s", "bad arguments to be_policy_create");
  *out = nullptr;
  const int F = 4 + ctx->cfg.window * ctx->cfg.window;
  if (hidden < 1 || hidden > POL_MAXH) return fail(ctx, BE_E_INVALID, "%s", "policy hidden size must be in [1, 256]");
  if (F > POL_MAXF) return fail(ctx, BE_E_INVALID, "%s", "policy input 4+W*W must be <= 128 (W <= 11)");
  if (num_actions < 1 || num_actions > POL_MAXA) return fail(ctx, BE_E_INVALID, "%s", "policy actions must be in [1, 15]");
  be_policy* pol = new (std::nothrow) be_policy();
  if (!pol) return fail(ctx, BE_E_NOMEM, "%s", "out of host memory");
  pol->ctx = ctx; pol->H = hidden; pol->F = F; pol->A = num_actions;
  pol->k = pick_policy(hidden, F, num_actions);
  if (const char* d = getenv("BALLENV_POLICY_DEBUG")) pol->dbg = (int)strtoul(d, nullptr, 0);
  pol->L = pol_layout(pol->k.HT, pol->k.KS, pol->k.NO);
  int cur = -1;
  hipError_t e = hipGetDevice(&cur);
  if (e == hipSuccess && cur != ctx->device) e = hipSetDevice(ctx->device);
  if (e == hipSuccess) e = hipMalloc(&pol->img, (size_t)pol->L.total);
  if (e == hipSuccess) e = hipMemset(pol->img, 0, (size_t)pol->L.total);
  if (e != hipSuccess) {
    delete pol;
    return fail(ctx, BE_E_HIP, "HIP error in be_policy_create: %s", hipGetErrorString(e));
  }
  if (pol->L.total > 160 * 1024) {
    (void)hipFree(pol->img);
    delete pol;
    return fail(ctx, BE_E_INVALID, "%s", "packed policy exceeds the LDS budget");
  }
  *out = pol;
  return BE_OK;
}

int be_policy_destroy(be_policy* pol) {
  if (!pol) return BE_OK;
  if (pol->img) (void)hipFree(pol->img);
  delete pol;
  return BE_OK;
}

int be_policy_load(be_policy* pol, const float* fc1_w, const float* fc1_b, const float* act_w, const float* act_b,
                   const float* val_w, const float* val_b, void* stream) {
  if (!pol) return fail(nullptr, BE_E_INVALID, "%s", "policy is NULL");
  be_ctx* ctx = pol->ctx;
  if (!fc1_w || !fc1_b || !act_w || !act_b || !val_w || !val_b)
    return fail(ctx, BE_E_INVALID, "%s", "be_policy_load: a weight pointer is NULL");
  int cur = -1;
  HIP_TRY(ctx, hipGetDevice(&cur));
  if (cur != ctx->device) HIP_TRY(ctx, hipSetDevice(ctx->device));
  const PolPack a{fc1_w, fc1_b, act_w, act_b, val_w, val_b, pol->H, pol->F, pol->A};
  hipLaunchKernelGGL(policy_pack_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, a, pol->img, pol->L);
  HIP_TRY(ctx, hipGetLastError());
  pol->loaded = true;
  return BE_OK;
}

int be_policy_act(be_policy* pol, const be_state* st, const uint8_t* obs, const be_act_out* out, uint64_t seed,
                  void* stream) {
  if (!pol) return fail(nullptr, BE_E_INVALID, "%s", "policy is NULL");
  be_ctx* ctx = pol->ctx;
  if (!pol->loaded) return fail(ctx, BE_E_INVALID, "%s", "be_policy_act before be_policy_load");
  if (!st || !st->episode || !st->ep_len || !obs || !out || !out->action)
    return fail(ctx, BE_E_INVALID, "%s", "be_policy_act needs state episode/ep_len, obs and out->action");
  int cur = -1;
  HIP_TRY(ctx, hipGetDevice(&cur));
  if (cur != ctx->device) HIP_TRY(ctx, hipSetDevice(ctx->device));
  PParams p;
  p.img = pol->img; p.obs = obs; p.episode = st->episode; p.ep_len = st->ep_len;
  p.action = out->action; p.log_prob = out->log_prob; p.value = out->value; p.probs = out->probs;
  p.seed = (unsigned long long)seed; p.n = ctx->cfg.num_envs; p.F = pol->F; p.A = pol->A;
  p.gid0 = (int32_t)(uint32_t)ctx->cfg.env_offset; p.img_bytes = pol->L.total; p.dbg = pol->dbg;
  const dim3 grid((unsigned)((p.n + POL_ENVS_PER_BLOCK - 1) / POL_ENVS_PER_BLOCK));
  hipLaunchKernelGGL(pol->k.fn, grid, dim3(pol->k.threads), (size_t)pol->L.total, (hipStream_t)stream, p);
  HIP_TRY(ctx, hipGetLastError());
  return BE_OK;
}

int64_t be_policy_bytes(const be_policy* pol) { return pol ? (int64_t)pol->L.total : 0; }

}  // extern "C"
