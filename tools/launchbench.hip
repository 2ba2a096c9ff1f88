// Diagnostics: launch/dispatch cost of an (almost) empty kernel vs grid shape and LDS size.
// Each kernel records per-wave s_memrealtime start stamps; prints the start spread.
// build: hipcc --offload-arch=gfx950 -O3 tools/launchbench.hip -o tools/launchbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void stamp_kernel(unsigned long long* st, int lds_touch) {
  extern __shared__ int smem[];
  if (lds_touch) smem[threadIdx.x] = threadIdx.x;
  if ((threadIdx.x & 63) == 0) st[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = __builtin_amdgcn_s_memrealtime();
}

int main() {
  unsigned long long* d;
  CK(hipMalloc(&d, sizeof(unsigned long long) * 65536));
  struct Cfg { int blocks, threads, lds; };
  const Cfg cfgs[] = {{256, 256, 0}, {256, 256, 48 * 1024}, {256, 64, 0}, {1024, 64, 0}, {128, 512, 0},
                      {64, 1024, 0}, {512, 256, 0}, {1024, 256, 0}, {4096, 256, 48 * 1024}};
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (const Cfg& c : cfgs) {
    const int waves = c.blocks * c.threads / 64;
    std::vector<float> dur;
    std::vector<double> spread;
    std::vector<unsigned long long> h(waves);
    for (int r = 0; r < 50; ++r) {
      CK(hipMemset(d, 0, sizeof(unsigned long long) * waves));
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(stamp_kernel, dim3(c.blocks), dim3(c.threads), c.lds, 0, d, c.lds > 0);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b)); dur.push_back(ms * 1000.f);
      CK(hipMemcpy(h.data(), d, sizeof(unsigned long long) * waves, hipMemcpyDeviceToHost));
      auto mm = std::minmax_element(h.begin(), h.end());
      spread.push_back((*mm.second - *mm.first) * 0.01);
    }
    std::sort(dur.begin(), dur.end()); std::sort(spread.begin(), spread.end());
    printf("{\"blocks\": %d, \"threads\": %d, \"lds\": %d, \"waves\": %d, \"event_us_p50\": %.2f, \"start_spread_us_p50\": %.2f}\n",
           c.blocks, c.threads, c.lds, waves, dur[25], spread[25]);
  }
  return 0;
}
