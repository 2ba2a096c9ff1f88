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
// the word of its cell with selects (no scratch memory); rows are written as bytes.
// All integer: the reference's sign(x)*(x-10)//20 on integer coordinates is exact.
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

__global__ __launch_bounds__(256) void blocks_kernel(BParams p) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= p.n) return;
  const int32_t a = p.agent[i], gl = p.goal[i];
  const int ax = px(a), ay = py(a), dx = px(gl) - ax, dy = py(gl) - ay;
  uint32_t w[8] = {0, 0, 0, 0, 1u, 0, 0, 0};     // byte 16 (the agent's cell) = 1
  const int quad = dx >= 0 ? (dy >= 0 ? 1 : 2) : (dy >= 0 ? 0 : 3);
  w[0] = 1u << (8 * quad);
  const int nobs = p.ns + p.nd;
  for (int k = 0; k < nobs; ++k) {
    const int32_t o = k < p.ns ? p.static_obs[(int64_t)k * p.n + i] : p.dyn_obs[(int64_t)(k - p.ns) * p.n + i];
    const int xd = ax - px(o), yd = ay - py(o);
    int xb = 0, yb = 0;
    if (xd != 0 && yd != 0) {
      xb = floordiv20(xd > 0 ? xd - 10 : 10 - xd);
      yb = floordiv20(yd > 0 ? yd - 10 : 10 - yd);
    }
    const bool in = xb > -3 && xb < 3 && yb > -3 && yb < 3;
    const int cell = 16 + 5 * yb + xb;           // byte index 4 + (12 + 5 yb + xb)
    const uint32_t inc = in ? 1u << (8 * (cell & 3)) : 0u;
#pragma unroll
    for (int q = 1; q < 8; ++q) w[q] += (cell >> 2) == q ? inc : 0u;
  }
  uint8_t* row = p.out ? p.out + (int64_t)i * 29 : nullptr;
  float* rowf = p.out_f32 ? p.out_f32 + (int64_t)i * 29 : nullptr;
#pragma unroll
  for (int b = 0; b < 29; ++b) {
    const uint8_t v = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
    if (row) row[b] = v;
    if (rowf) rowf[b] = (float)v;
  }
}

}  // namespace

extern "C" {

int be_observe_blocks(be_ctx* ctx, const be_state* st, uint8_t* out, float* out_f32, void* stream) {
  if (!ctx) return be_ctx_fail(nullptr, BE_E_INVALID, "ctx is NULL");
  if (int rc = be_ctx_check_state(ctx, st)) return rc;
  if (!out && !out_f32) return be_ctx_fail(ctx, BE_E_INVALID, "be_observe_blocks needs out or out_f32");
  const be_ctx_view cv = be_ctx_get(ctx);
  int cur = -1;
  hipError_t e = hipGetDevice(&cur);
  if (e == hipSuccess && cur != cv.device) e = hipSetDevice(cv.device);
  if (e != hipSuccess) return be_ctx_fail(ctx, BE_E_HIP, hipGetErrorString(e));
  BParams p{st->agent, st->goal, st->static_obs, st->dyn_obs, out, out_f32, cv.num_envs, cv.num_static, cv.num_dynamic};
  hipLaunchKernelGGL(blocks_kernel, dim3((unsigned)((cv.num_envs + 255) / 256)), dim3(256), 0, (hipStream_t)stream, p);
  e = hipGetLastError();
  if (e != hipSuccess) return be_ctx_fail(ctx, BE_E_HIP, hipGetErrorString(e));
  return BE_OK;
}

}  // extern "C"
