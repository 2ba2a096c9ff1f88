// Kernarg-preload probe (tools/probe/preload_probe.sh): the same tiny kernel compiled with and
// without -mllvm -amdgpu-kernarg-preload-count, timed per launch (graph-replayed).  If the
// firmware preloads kernel arguments into SGPRs, the preload build skips the kernarg s_load latency.
#include <hip/hip_runtime.h>
#ifndef KNAME
#define KNAME probe_plain
#endif
extern "C" __global__ __launch_bounds__(256) void KNAME(const int* __restrict__ a, const int* __restrict__ b,
                                                        int* __restrict__ c, int n) {
  const int i = (int)(blockIdx.x * 256 + threadIdx.x);
  if (i < n) c[i] = a[i] + b[i];
}
