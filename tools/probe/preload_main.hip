#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
extern "C" __global__ void probe_plain(const int*, const int*, int*, int);
extern "C" __global__ void probe_pre(const int*, const int*, int*, int);
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
static float run(void (*k)(const int*, const int*, int*, int), int n, int* a, int* b, int* c, hipStream_t s) {
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int t = 0; t < 500; ++t) hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, s, a, b, c, n);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < 4; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
  return ms * 1e3f / 2000.f;
}
int main() {
  const int nmax = 1 << 20;
  int *a, *b, *c;
  CK(hipMalloc(&a, 4 * nmax)); CK(hipMalloc(&b, 4 * nmax)); CK(hipMalloc(&c, 4 * nmax));
  CK(hipMemset(a, 0, 4 * nmax)); CK(hipMemset(b, 0, 4 * nmax));
  hipStream_t s; CK(hipStreamCreate(&s));
  for (int n : {1, 16384, 65536, 131072}) {
    for (int rep = 0; rep < 3; ++rep) {
      const float p0 = run(probe_plain, n, a, b, c, s), p1 = run(probe_pre, n, a, b, c, s);
      printf("n %7d rep %d: plain %.3f us  preload-build %.3f us per launch\n", n, rep, p0, p1);
    }
  }
  return 0;
}
