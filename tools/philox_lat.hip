// Philox4x32-10 dependent-chain latency on one wave (diagnostics): cycles per block for the
// library's philox() and for a variant that xors the key into the pass-through word first
// (hi ^ (c ^ k): one xor after each multiply on the chain instead of two), and for one whose round
// keys are scalar adds issued just before their round (v_xor takes the SGPR: no VALU key schedule).
//   hipcc --offload-arch=gfx950 -O3 -I gym-ballenv_amd/csrc tools/philox_lat.hip -o tools/diag/philox_lat
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "philox.h"

__device__ __forceinline__ u4 philox_kx(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, unsigned long long seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  asm volatile("" : "+v"(k0), "+v"(k1));
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t t0 = c1 ^ k0, t2 = c3 ^ k1;
    asm volatile("" : "+v"(t0), "+v"(t2));
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ t0, n2 = (uint32_t)(p0 >> 32) ^ t2;
    c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return u4{c0, c1, c2, c3};
}

__device__ __forceinline__ u4 philox_sk(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, unsigned long long seed) {
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);   // uniform: SGPRs
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t rk0, rk1;   // round keys on the scalar unit, per round (volatile: not hoisted, no SGPR pressure)
    asm volatile("s_add_u32 %0, %1, %2" : "=s"(rk0) : "s"(k0), "s"(0x9E3779B9u * (uint32_t)r));
    asm volatile("s_add_u32 %0, %1, %2" : "=s"(rk1) : "s"(k1), "s"(0xBB67AE85u * (uint32_t)r));
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ rk0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ rk1;
    c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
  }
  return u4{c0, c1, c2, c3};
}

template <int V>
__global__ void chain(uint32_t* out, long long* cyc, int iters, unsigned long long seed) {
  uint32_t a = threadIdx.x, b = 7, c = 9, d = 11;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    const u4 r = V == 0 ? philox(a, b, c, d, seed) : V == 1 ? philox_kx(a, b, c, d, seed) : philox_sk(a, b, c, d, seed);
    a = r.x; b = r.y; c = r.z; d = r.w;
  }
  const long long t1 = clock64();
  out[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  uint32_t* out; long long* cyc;
  hipMalloc(&out, 64 * 4 * 3); hipMalloc(&cyc, 8);
  const int iters = 4096;
  uint32_t h[3][64];
  for (int v = 0; v < 3; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      if (v == 0) chain<0><<<1, 64>>>(out + 64 * v, cyc, iters, 0x1234567890ull);
      else if (v == 1) chain<1><<<1, 64>>>(out + 64 * v, cyc, iters, 0x1234567890ull);
      else chain<2><<<1, 64>>>(out + 64 * v, cyc, iters, 0x1234567890ull);
      long long c = 0;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      printf("variant %d rep %d: %.1f clock64 ticks per Philox block (dependent chain, 1 wave)\n", v, rep, (double)c / iters);
    }
    hipMemcpy(h[v], out + 64 * v, 256, hipMemcpyDeviceToHost);
  }
  int same = 1;
  for (int l = 0; l < 64; ++l) same &= h[0][l] == h[1][l] && h[0][l] == h[2][l];
  printf("variants agree: %s\n", same ? "yes" : "NO");
  return same ? 0 : 1;
}
