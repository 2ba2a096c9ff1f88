// Diagnostics: what bounds a be_step launch at small batch sizes?
// Times (hipEvents, median of 200 launches) for N in {65536, 262144, 1M}:
//   empty      : empty kernel, same grid
//   soa_copy   : reads/writes exactly the bytes be_step moves (275 B/env at W=10)
//   be_step    : the library's step kernel (Philox mode, random actions)
// build: hipcc --offload-arch=gfx950 -O3 -I include tools/microbench.hip -L gym-ballenv_amd -lballenv -o /tmp/mb
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

#include "ballenv.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void empty_kernel() {}

// Same traffic as be_step: R+W agent/prev/ret/len, R goal/total/episode/action, W reward/done,
// R 13 statics, R+W 5 dyn xy, R 5 dyn goal, W 104 B obs (u8, as 26 dwords per env, coalesced via row-major)
__global__ void soa_copy(int n, int32_t* agent, const int32_t* goal, double* prev, const double* total, double* ret,
                         int32_t* len, const uint32_t* episode, const uint8_t* act, double* reward, uint8_t* done,
                         const int32_t* so, int32_t* dy, const uint8_t* dg, uint32_t* obs) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t a = agent[i] + goal[i] + (int)episode[i] + act[i];
  double p = prev[i] + total[i];
  int32_t s = 0;
#pragma unroll
  for (int k = 0; k < 13; ++k) s += so[k * n + i];
#pragma unroll
  for (int k = 0; k < 5; ++k) { int32_t v = dy[k * n + i] + dg[k * n + i]; dy[k * n + i] = v + 1; s ^= v; }
  agent[i] = a + s; prev[i] = p; ret[i] += p; len[i] += 1; reward[i] = p; done[i] = (uint8_t)(s & 1);
  // obs: 26 dwords per env; write them as a block-contiguous stripe so stores coalesce
  uint32_t* o = obs + (size_t)blockIdx.x * blockDim.x * 26;
  for (int w = threadIdx.x; w < 26 * (int)blockDim.x; w += blockDim.x) o[w] = (uint32_t)(s + w);
}

// the step's read set alone / its write set alone (same SoA arrays, same per-env bytes)
__global__ void soa_read(int n, const int32_t* agent, const int32_t* goal, const double* prev, const double* total,
                         const double* ret, const int32_t* len, const uint32_t* episode, const uint8_t* act,
                         const int32_t* so, const int32_t* dy, const uint8_t* dg, int32_t* sink) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t s = agent[i] + goal[i] + (int)episode[i] + act[i] + len[i];
  double p = prev[i] + total[i] + ret[i];
#pragma unroll
  for (int k = 0; k < 13; ++k) s += so[k * n + i];
#pragma unroll
  for (int k = 0; k < 5; ++k) s ^= dy[k * n + i] + dg[k * n + i];
  if (s == 0x7FFFFFFF && p == 1.2345) sink[0] = s;   // keeps the loads
}
__global__ void soa_write(int n, int32_t* agent, double* prev, double* ret, int32_t* len, double* reward,
                          uint8_t* done, int32_t* dy, uint32_t* obs) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  agent[i] = i; prev[i] = 1.0; ret[i] = 2.0; len[i] = i; reward[i] = 3.0; done[i] = (uint8_t)i;
#pragma unroll
  for (int k = 0; k < 5; ++k) dy[k * n + i] = i + k;
  uint32_t* o = obs + (size_t)blockIdx.x * blockDim.x * 26;
  for (int w = threadIdx.x; w < 26 * (int)blockDim.x; w += blockDim.x) o[w] = (uint32_t)(i + w);
}

template <class F>
float time_b2b(F f, int iters = 500) {   // back-to-back launches, no events in between
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int t = 0; t < iters; ++t) f();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
  return ms * 1000.f / iters;
}

template <class F>
float time_median(F f, int iters = 200) {
  std::vector<hipEvent_t> ev(2 * iters);
  for (int k = 0; k < 2 * iters; ++k) CK(hipEventCreate(ev.data() + k));
  for (int t = 0; t < iters; ++t) { CK(hipEventRecord(ev[2 * t])); f(); CK(hipEventRecord(ev[2 * t + 1])); }
  CK(hipDeviceSynchronize());
  std::vector<float> d(iters);
  for (int t = 0; t < iters; ++t) CK(hipEventElapsedTime(&d[t], ev[2 * t], ev[2 * t + 1]));
  std::sort(d.begin(), d.end());
  for (int k = 0; k < 2 * iters; ++k) CK(hipEventDestroy(ev[k]));
  return d[iters / 2] * 1000.f;
}

int main(int argc, char** argv) {
  // argv[1] (optional): BALLENV_DEBUG_SKIP mask for the be_step context (diagnostics)
  const char* dbg = argc > 1 ? argv[1] : "0";
  for (int N : {65536, 262144, 1048576}) {
    be_config cfg;
    be_config_default(&cfg, N, 10);
    be_ctx* ctx = nullptr;
    setenv("BALLENV_DEBUG_SKIP", dbg, 1);
    if (be_create(&cfg, 0, &ctx)) { printf("create: %s\n", be_last_error(nullptr)); return 1; }
    unsetenv("BALLENV_DEBUG_SKIP");
    be_state st;
    be_out out;
    memset(&st, 0, sizeof st); memset(&out, 0, sizeof out);
    CK(hipMalloc(&st.agent, 4 * N)); CK(hipMalloc(&st.goal, 4 * N)); CK(hipMalloc(&st.prev_dist, 8 * N));
    CK(hipMalloc(&st.total_dist, 8 * N)); CK(hipMalloc(&st.ep_return, 8 * N)); CK(hipMalloc(&st.ep_len, 4 * N));
    CK(hipMalloc(&st.episode, 4 * N)); CK(hipMalloc(&st.static_obs, 4 * 13 * N)); CK(hipMalloc(&st.dyn_obs, 4 * 5 * N));
    CK(hipMalloc(&st.dyn_goal, 5 * N));
    CK(hipMalloc(&out.obs, 104 * N)); CK(hipMalloc(&out.reward, 8 * N)); CK(hipMalloc(&out.done, N));
    CK(hipMemset(st.episode, 0, 4 * N)); CK(hipMemset(st.ep_len, 0, 4 * N));
    uint8_t* acts; CK(hipMalloc(&acts, (size_t)N * 64));
    if (be_sample_actions(ctx, acts, 64, 7, nullptr)) return 1;
    if (be_reset(ctx, &st, nullptr, nullptr, 0, &out, nullptr)) { printf("reset: %s\n", be_last_error(ctx)); return 1; }
    CK(hipDeviceSynchronize());
    int blocks = (N + 255) / 256;
    float t_empty = time_median([&] { hipLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(256), 0, 0); });
    float t_copy = time_median([&] {
      hipLaunchKernelGGL(soa_copy, dim3(blocks), dim3(256), 0, 0, N, st.agent, st.goal, st.prev_dist, st.total_dist,
                         st.ep_return, st.ep_len, st.episode, acts, out.reward, out.done, st.static_obs, st.dyn_obs,
                         st.dyn_goal, (uint32_t*)out.obs);
    });
    int t = 0;
    float t_step = time_median([&] {
      be_step(ctx, &st, acts + (size_t)(t++ % 64) * N, nullptr, nullptr, &out, nullptr);
    });
    // back-to-back throughput (no events in between)
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int k = 0; k < 500; ++k) be_step(ctx, &st, acts + (size_t)(k % 64) * N, nullptr, nullptr, &out, nullptr);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    double bytes = (double)be_step_bytes(&cfg) * N;
    int32_t* sink; CK(hipMalloc(&sink, 4));
    const float b_empty = time_b2b([&] { hipLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(256), 0, 0); });
    const float b_copy = time_b2b([&] {
      hipLaunchKernelGGL(soa_copy, dim3(blocks), dim3(256), 0, 0, N, st.agent, st.goal, st.prev_dist, st.total_dist,
                         st.ep_return, st.ep_len, st.episode, acts, out.reward, out.done, st.static_obs, st.dyn_obs,
                         st.dyn_goal, (uint32_t*)out.obs);
    });
    const float b_read = time_b2b([&] {
      hipLaunchKernelGGL(soa_read, dim3(blocks), dim3(256), 0, 0, N, st.agent, st.goal, st.prev_dist, st.total_dist,
                         st.ep_return, st.ep_len, st.episode, acts, st.static_obs, st.dyn_obs, st.dyn_goal, sink);
    });
    const float b_write = time_b2b([&] {
      hipLaunchKernelGGL(soa_write, dim3(blocks), dim3(256), 0, 0, N, st.agent, st.prev_dist, st.ep_return, st.ep_len,
                         out.reward, out.done, st.dyn_obs, (uint32_t*)out.obs);
    });
    printf("{\"dbg\": \"%s\", \"envs\": %d, \"empty_us\": %.2f, \"soa_copy_us\": %.2f, \"soa_copy_GBs\": %.0f, \"be_step_us\": %.2f, "
           "\"be_step_GBs\": %.0f, \"b2b_us_per_step\": %.2f, \"b2b_empty_us\": %.2f, \"b2b_soa_copy_us\": %.2f, "
           "\"b2b_soa_read_us\": %.2f, \"b2b_soa_write_us\": %.2f}\n",
           dbg, N, t_empty, t_copy, bytes / (t_copy * 1e3), t_step, bytes / (t_step * 1e3), ms * 1000.f / 500,
           b_empty, b_copy, b_read, b_write);
    CK(hipFree(sink));
    be_destroy(ctx);
  }
  return 0;
}
