// features.hip -- sibling observation formats of the reference's callers (SURVEY §8(f)
// rank 3), computed on the GPU from the same SoA state as the step kernels:
//
//   be_observe_blocks   prep_state2 of examples/ball_env_reinforce.py:130-172 (and
//                       block_to_arrpos :169-172): the 29-input block-count encoding the
//                       REINFORCE / supervised policies read -- quadrant one-hot, the
//                       agent's own cell set, +1 per obstacle in its 20-px block of a 5x5
//                       grid around the agent.
//
// One lane per env (the env index is the coalesced axis of every state array); the 29
// counters live in 8 packed 32-bit registers and each obstacle adds 1 << 8*(cell & 3) to
// the word of its cell with selects (no scratch memory).  All integer: the reference's
// sign(x)*(x-10)//20 on integer coordinates is exact.
//
// HBM-bound (80 B of state read, 29 B / 116 B of rows written per env): each wave's 64 rows
// are one contiguous run of the output (64 x 29 B = 116 16-B chunks; f32: 464), so the rows go
// through a per-wave LDS stage and out in 16-B stores, instead of 29 byte (dword) stores per
// lane at a 29-B (116-B) stride.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>

#include "ballenv.h"
#include "internal.h"

namespace {

__device__ __forceinline__ int floordiv20(int a) { return a >= 0 ? a / 20 : -((-a + 19) / 20); }
__device__ __forceinline__ int px(int32_t p) { return (int)(int16_t)(p & 0xFFFF); }
__device__ __forceinline__ int py(int32_t p) { return p >> 16; }

struct BParams {
  const int32_t* agent; const int32_t* goal; const int32_t* static_obs; const int32_t* dyn_obs;
  uint8_t* out; float* out_f32;
  int32_t n, ns, nd;
};

// a wave's N contiguous 16-B chunks from its LDS stage to dst (16-B aligned, wave-uniform) in one
// unrolled pass: every LDS read issued before the first store, write-through (sc1) buffer stores --
// they drain while the wave runs instead of in the kernel-end L2 write-back -- and a descriptor of
// N * 16 bytes that drops the last pass's extra lanes (no branch)
constexpr int BLOCKS_AUX = 16;   // cache-policy bits of the copy-out (gfx950: sc1 16)
template <int N>
__device__ __forceinline__ void copy_chunks(const uint8_t* stage, uint8_t* dst, int lane) {
  constexpr int IT = (N + 63) / 64;
  typedef int v4i_ __attribute__((ext_vector_type(4)));
  v4i_ x[IT];
#pragma unroll
  for (int j = 0; j < IT; ++j) x[j] = reinterpret_cast<const v4i_*>(stage)[min(lane + 64 * j, N - 1)];
  const uint64_t du = (uint64_t)dst;
  uint8_t* dstu = reinterpret_cast<uint8_t*>(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(du >> 32)) << 32) |
                                             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)du));
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(dstu, (short)0, N * 16, 0x00020000);
#pragma unroll
  for (int j = 0; j < IT; ++j) __builtin_amdgcn_raw_buffer_store_b128(x[j], rsrc, (lane + 64 * j) * 16, 0, BLOCKS_AUX);
}

constexpr int BLK_ROW = 29, BLK_WAVE_U8 = 64 * BLK_ROW, BLK_WAVE_F32 = 64 * BLK_ROW * 4;

// dynamic LDS: 4 wave stages of BLK_WAVE_U8 bytes, or BLK_WAVE_F32 when f32 rows are asked for (a
// u8-only launch keeps 7.4 KB per block, so LDS does not cap the waves per CU)
__global__ __launch_bounds__(256) void blocks_kernel(BParams p) {
  extern __shared__ __align__(16) uint8_t smem[];
  const int tid = (int)threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int i = blockIdx.x * 256 + tid, e0 = blockIdx.x * 256 + w * 64;
  const int nrows = max(0, min(64, p.n - e0));            // this wave's rows (uniform)
  if (nrows == 0) return;
  const bool valid = i < p.n;
  const int ic = valid ? i : p.n - 1;
  const int32_t a = p.agent[ic], gl = p.goal[ic];
  const int ax = px(a), ay = py(a), dx = px(gl) - ax, dy = py(gl) - ay;
  uint32_t w8[8] = {0, 0, 0, 0, 1u, 0, 0, 0};     // byte 16 (the agent's cell) = 1
  const int quad = dx >= 0 ? (dy >= 0 ? 1 : 2) : (dy >= 0 ? 0 : 3);
  w8[0] = 1u << (8 * quad);
  // obstacles in chunks of CH: every load of a chunk is issued before the first is used (clamped to
  // a real obstacle, the extra slots masked), so a wave waits for memory once per chunk instead of
  // once per pair of obstacles
  constexpr int CH = 6;   // obstacles per load chunk (18: slower at 65 536 envs, profiles/r03_blocks_ab.txt)
  const int nobs = p.ns + p.nd;
  for (int k0 = 0; k0 < nobs; k0 += CH) {
    int32_t o[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int k = min(k0 + j, nobs - 1);
      const int32_t* src = k < p.ns ? p.static_obs + (int64_t)k * p.n : p.dyn_obs + (int64_t)(k - p.ns) * p.n;
      o[j] = src[ic];
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int xd = ax - px(o[j]), yd = ay - py(o[j]);
      const bool off = xd == 0 || yd == 0;   // the reference's sign(0) = 0: block 0 on both axes
      const int xb = off ? 0 : floordiv20(xd > 0 ? xd - 10 : 10 - xd);
      const int yb = off ? 0 : floordiv20(yd > 0 ? yd - 10 : 10 - yd);
      const bool in = k0 + j < nobs && xb > -3 && xb < 3 && yb > -3 && yb < 3;
      const int cell = 16 + 5 * yb + xb;         // byte index 4 + (12 + 5 yb + xb)
      const uint32_t inc = in ? 1u << (8 * (cell & 3)) : 0u;
#pragma unroll
      for (int q = 1; q < 8; ++q) w8[q] += (cell >> 2) == q ? inc : 0u;
    }
  }
  uint8_t* stage = smem + w * (p.out_f32 ? BLK_WAVE_F32 : BLK_WAVE_U8);
  const bool full = nrows == 64;
  // wave barrier between a stage's writes and its copy-out (and the next format's writes)
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  if (p.out) {
    uint8_t* row = stage + lane * BLK_ROW;
#pragma unroll
    for (int b = 0; b < BLK_ROW; ++b) row[b] = (uint8_t)(w8[b >> 2] >> (8 * (b & 3)));
    wave_sync();
    uint8_t* dst = p.out + (int64_t)e0 * BLK_ROW;
    if (full && (reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
      copy_chunks<BLK_WAVE_U8 / 16>(stage, dst, lane);
    } else {
      for (int b = lane; b < nrows * BLK_ROW; b += 64) dst[b] = stage[b];
    }
    wave_sync();
  }
  if (p.out_f32) {
    float* rowf = reinterpret_cast<float*>(stage) + lane * BLK_ROW;
#pragma unroll
    for (int b = 0; b < BLK_ROW; ++b) rowf[b] = (float)(uint8_t)(w8[b >> 2] >> (8 * (b & 3)));
    wave_sync();
    float* dst = p.out_f32 + (int64_t)e0 * BLK_ROW;
    if (full && (reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
      copy_chunks<BLK_WAVE_F32 / 16>(stage, reinterpret_cast<uint8_t*>(dst), lane);
    } else {
      const float* sf = reinterpret_cast<const float*>(stage);
      for (int b = lane; b < nrows * BLK_ROW; b += 64) dst[b] = sf[b];
    }
  }
}

}  // namespace

extern "C" {

int be_observe_blocks(be_ctx* ctx, const be_state* st, uint8_t* out, float* out_f32, void* stream) {
  if (!ctx) return be_ctx_fail(nullptr, BE_E_INVALID, "ctx is NULL");
  if (int rc = be_ctx_check_state(ctx, st)) return rc;
  if (!out && !out_f32) return be_ctx_fail(ctx, BE_E_INVALID, "be_observe_blocks needs out or out_f32");
  const be_ctx_view cv = be_ctx_get(ctx);
  const DeviceGuard dg(cv.device);   // the caller's current device is restored on return
  hipError_t e = dg.err;
  if (e != hipSuccess) return be_ctx_fail(ctx, BE_E_HIP, hipGetErrorString(e));
  BParams p{st->agent, st->goal, st->static_obs, st->dyn_obs, out, out_f32, cv.num_envs, cv.num_static, cv.num_dynamic};
  const size_t lds = 4 * (size_t)(out_f32 ? BLK_WAVE_F32 : BLK_WAVE_U8);
  hipLaunchKernelGGL(blocks_kernel, dim3((unsigned)((cv.num_envs + 255) / 256)), dim3(256), lds, (hipStream_t)stream, p);
  e = hipGetLastError();
  if (e != hipSuccess) return be_ctx_fail(ctx, BE_E_HIP, hipGetErrorString(e));
  return BE_OK;
}

}  // extern "C"
