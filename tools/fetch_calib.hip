// Diagnostics: calibrate FETCH_SIZE / WRITE_SIZE on the access pattern of the config-2 step kernel
// (stepw_kernel<5, 13, 5, 8>: 4 096 envs, 32-env blocks of 256 threads, 8 lanes per env).
//
// MI355X_MICROARCH.md (HBM): FETCH_SIZE = TCC_EA0_RDREQ x 64 B, and it reads exactly half of the
// bytes of a wide (16 B/lane) coalesced streaming read -- hence the 2 x FETCH_SIZE correction the
// PMC reports use.  Other access widths are uncalibrated.  stepw_kernel reads 4-, 8- and 1-byte
// SoA words per env from 32-env blocks (128-B, 256-B and 32-B spans per block), so this program
// replays exactly that read set (and, separately, the write set) with known byte counts, under the
// same grid, so `rocprofv3 --pmc FETCH_SIZE` / `WRITE_SIZE` of each kernel says what the counters
// report for this pattern when nothing is wasted.
//
// Kernels (one template instantiation each, so the kernel trace names them):
//   rd<0, 0>  the whole read set (118 B/env), 8-lane groups, blocks in launch order
//   rd<0, 1>  the same with an XCD-aware block order (blocks b, b+8, ... take consecutive envs)
//   rd<1, 0>  only the 1-byte arrays (action, 5 x dyn_goal: 6 B/env)
//   rd<2, 0>  only the 4-byte arrays (agent, goal, ep_len, episode, 13 statics, 5 dyn: 88 B/env)
//   rd<3, 0>  only the 8-byte arrays (prev_dist, total_dist, ep_return: 24 B/env)
//   rd<4, 0>  the whole read set, one lane per env, 256-env blocks (64 envs per wave)
//   wr<0>     the write set (82 B/env: reward, ep_return, prev_dist 8 each; ep_len, agent 4 each;
//             done, truncated 1 each; 5 dyn 4 each; the 29-B obs row), write-through (sc1) stores in
//             stepw's pattern: per-env scalars spread over the group's lanes, the wave's 8 obs rows
//             (232 contiguous bytes) as 29 eight-byte stores
//   wr<1>     the same with the obs rows only
//
// build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
// run:   tools/fetch_calib [envs=4096] [launches=200] [mode 0..7: the kernels above, in order]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct Arrays {
  int32_t *agent, *goal, *len, *so, *dy;
  uint32_t* episode;
  uint8_t *act, *dg, *done, *trunc, *obs;
  double *prev, *total, *ret, *reward;
  int32_t* sink;
};

__device__ __forceinline__ int xcd_block(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

template <int SET, int XCD>
__global__ __launch_bounds__(256) void rd(Arrays a, int n) {
  constexpr int L = SET == 4 ? 1 : 8, EPB = 256 / L;
  const int tid = (int)threadIdx.x, h = tid & (L - 1);
  const int b = XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  const int i = min(b * EPB + tid / L, n - 1);
  int32_t s = 0;
  double f = 0.0;
  if (SET == 0 || SET == 1 || SET == 4) {
    s += a.act[i];
    for (int j = 0; j < (L == 8 ? 1 : 5); ++j) s += a.dg[(L == 8 ? min(h, 4) : j) * n + i];
  }
  if (SET == 0 || SET == 2 || SET == 4) {
    s ^= a.agent[i] + a.goal[i] + a.len[i] + (int)a.episode[i];
    for (int j = 0; j < (L == 8 ? 1 : 5); ++j) s += a.dy[(L == 8 ? min(h, 4) : j) * n + i];
    for (int j = 0; j < (L == 8 ? 2 : 13); ++j) s ^= a.so[(L == 8 ? min(8 * j + h, 12) : j) * n + i];
  }
  if (SET == 0 || SET == 3 || SET == 4) f = a.prev[i] + a.total[i] + a.ret[i];
  if (s == 0x7FFFFFFF && f == 1.2345) a.sink[0] = s;   // keeps the loads
}

template <class T>
__device__ __forceinline__ void st_wt(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

template <int SET>
__global__ __launch_bounds__(256) void wr(Arrays a, int n) {
  const int tid = (int)threadIdx.x, h = tid & 7, lane = tid & 63;
  const int i0 = (int)blockIdx.x * 32 + tid / 8;
  const bool valid = i0 < n;
  const int i = min(i0, n - 1);
  if (SET == 0 && valid) {
    if (h < 3) st_wt((h == 0 ? a.reward : h == 1 ? a.ret : a.prev) + i, (double)(i + h));
    if (h < 2) st_wt((h ? a.len : a.agent) + i, i + h);
    uint8_t* pb = h == 0 ? a.done : h == 1 ? a.trunc : nullptr;
    if (pb) st_wt(pb + i, (uint8_t)(i & 1));
    if (h < 5) st_wt(a.dy + h * n + i, i + h);
  }
  // the wave's 8 obs rows: 232 contiguous bytes, lanes 0..28 store 8 B each (stepw's copy-out)
  const int e0 = (int)blockIdx.x * 32 + (tid >> 6) * 8;
  const int nb = max(0, min(8, n - e0)) * 29;
  if (8 * lane < nb) st_wt(reinterpret_cast<uint64_t*>(a.obs + (size_t)e0 * 29) + lane, (uint64_t)(lane + e0));
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096, launches = argc > 2 ? atoi(argv[2]) : 200;
  Arrays a;
  auto alloc = [&](auto** p, size_t bytes) {
    CK(hipMalloc((void**)p, bytes));
    CK(hipMemset(*p, 1, bytes));
  };
  alloc(&a.agent, 4 * (size_t)n); alloc(&a.goal, 4 * (size_t)n); alloc(&a.len, 4 * (size_t)n);
  alloc(&a.so, 4 * 13 * (size_t)n); alloc(&a.dy, 4 * 5 * (size_t)n); alloc(&a.episode, 4 * (size_t)n);
  alloc(&a.act, n); alloc(&a.dg, 5 * (size_t)n); alloc(&a.done, n); alloc(&a.trunc, n); alloc(&a.obs, 29 * (size_t)n + 64);
  alloc(&a.prev, 8 * (size_t)n); alloc(&a.total, 8 * (size_t)n); alloc(&a.ret, 8 * (size_t)n); alloc(&a.reward, 8 * (size_t)n);
  alloc(&a.sink, 64);
  const dim3 g32((n + 31) / 32), g256((n + 255) / 256), blk(256);
  // one kernel per process, back to back (as the step kernel runs): the L2 state each launch
  // starts from is the one its own previous launch left
  const int mode = argc > 3 ? atoi(argv[3]) : 0;
  for (int t = 0; t < launches; ++t) {
    switch (mode) {
      case 0: rd<0, 0><<<g32, blk>>>(a, n); break;
      case 1: rd<0, 1><<<g32, blk>>>(a, n); break;
      case 2: rd<1, 0><<<g32, blk>>>(a, n); break;
      case 3: rd<2, 0><<<g32, blk>>>(a, n); break;
      case 4: rd<3, 0><<<g32, blk>>>(a, n); break;
      case 5: rd<4, 0><<<g256, blk>>>(a, n); break;
      case 6: wr<0><<<g32, blk>>>(a, n); break;
      default: wr<1><<<g32, blk>>>(a, n); break;
    }
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  printf("fetch_calib: %d envs, %d launches of each kernel\n", n, launches);
  return 0;
}
