// Diagnostics: host time per launch of a kernel with be_step's kernarg size (~400 B), by launch API.
// The eager step() is host-bound; this separates HIP's launch call from the rest.
// Bursts of 128 launches (timed on the host), a stream sync between bursts, the APIs interleaved.
// build: hipcc --offload-arch=gfx950 -O3 tools/launch_host.hip -o tools/launch_host
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <algorithm>
#include <chrono>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct KP {   // the size of ballenv.hip's KParams
  void* ptr[40];
  int flag;
  int pad[15];
};

__global__ void k(KP p) {
  if (p.flag && threadIdx.x == 0 && blockIdx.x == 0) *(int*)p.ptr[0] = 1;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  KP p{};
  p.flag = 0;
  const dim3 grid(512), block(256);
  const int B = 128, R = 40;
  const char* names[] = {"hipLaunchKernelGGL", "hipLaunchKernel", "hipExtLaunchKernel"};
  std::vector<double> t[3];
  for (int r = 0; r < R; ++r) {
    for (int v = 0; v < 3; ++v) {
      CK(hipStreamSynchronize(s));
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < B; ++i) {
        if (v == 0) {
          hipLaunchKernelGGL(k, grid, block, 0, s, p);
        } else if (v == 1) {
          void* args[] = {&p};
          (void)hipLaunchKernel((const void*)k, grid, block, args, 0, s);
        } else {
          void* args[] = {&p};
          (void)hipExtLaunchKernel((const void*)k, grid, block, args, 0, s, nullptr, nullptr, 0);
        }
      }
      const auto t1 = std::chrono::steady_clock::now();
      CK(hipGetLastError());
      if (r >= 5) t[v].push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / B);
    }
  }
  CK(hipStreamSynchronize(s));
  for (int v = 0; v < 3; ++v) {
    std::sort(t[v].begin(), t[v].end());
    printf("%-20s host us per launch: p10 %.3f p50 %.3f p90 %.3f\n", names[v], t[v][t[v].size() / 10],
           t[v][t[v].size() / 2], t[v][t[v].size() * 9 / 10]);
  }
  return 0;
}
