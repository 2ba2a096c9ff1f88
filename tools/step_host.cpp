// Diagnostics: host time per be_step call from C (no Python, no ctypes), 65 536 envs at W=10, the
// in-tree library; beside tools/launch_host (HIP's own launch call) it splits the eager step()'s
// host cost into Python/ctypes, the library and the HIP launch.
// build: hipcc -O2 -I include tools/step_host.cpp -L gym-ballenv_amd -l:libballenv.so
//        -Wl,-rpath,'$ORIGIN/../gym-ballenv_amd' -o tools/step_host
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <chrono>
#include <vector>
#include "ballenv.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define BK(x) do { int rc = (x); if (rc) { printf("be error %d at %d: %s\n", rc, __LINE__, be_last_error(ctx)); return 1; } } while (0)

template <class T>
static T* dalloc(size_t n) {
  void* p = nullptr;
  if (hipMalloc(&p, n * sizeof(T) + 16) != hipSuccess) return nullptr;
  (void)hipMemset(p, 0, n * sizeof(T) + 16);
  return (T*)p;
}

int main() {
  const int N = 65536, W = 10, F = 4 + W * W;
  be_config cfg;
  be_ctx* ctx = nullptr;
  BK(be_config_default(&cfg, N, W));
  BK(be_create(&cfg, 0, &ctx));
  const int ns = cfg.num_static, nd = cfg.num_dynamic;
  be_state st{dalloc<int32_t>(N), dalloc<int32_t>(N), dalloc<double>(N), dalloc<double>(N), dalloc<double>(N),
              dalloc<int32_t>(N), dalloc<uint32_t>(N), dalloc<int32_t>((size_t)ns * N), dalloc<int32_t>((size_t)nd * N),
              dalloc<uint8_t>((size_t)nd * N)};
  be_out out{dalloc<uint8_t>((size_t)N * F), nullptr, dalloc<double>(N), dalloc<uint8_t>(N), dalloc<uint8_t>(N), nullptr,
             dalloc<double>(N), dalloc<int32_t>(N), dalloc<double>((size_t)be_stats_slots(&cfg) * 8)};
  uint8_t* acts = dalloc<uint8_t>(N);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  BK(be_reset(ctx, &st, nullptr, nullptr, 0, &out, s));
  const int B = 128, R = 40;
  std::vector<double> t;
  for (int r = 0; r < R; ++r) {
    CK(hipStreamSynchronize(s));
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < B; ++i) BK(be_step(ctx, &st, acts, nullptr, nullptr, &out, s));
    const auto t1 = std::chrono::steady_clock::now();
    if (r >= 5) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / B);
  }
  CK(hipStreamSynchronize(s));
  std::sort(t.begin(), t.end());
  printf("be_step (C caller)    host us per call:   p10 %.3f p50 %.3f p90 %.3f  (%s)\n", t[t.size() / 10],
         t[t.size() / 2], t[t.size() * 9 / 10], be_kernel_name(ctx, 0));
  int32_t status = 0;
  BK(be_status(ctx, &status, s));
  CK(hipStreamSynchronize(s));
  printf("status %d\n", status);
  be_destroy(ctx);
  return 0;
}
