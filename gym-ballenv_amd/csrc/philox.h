// philox.h -- Philox4x32-10 counter-based generator (Salmon et al., SC'11), shared by
// the step kernels (ballenv.hip) and the policy kernel (policy.hip); the same
// function as oracle/ballenv_oracle.c.  Counter layout: (global env id, c1, c2,
// purpose << 24 | sub) -- every draw is a pure function of per-env state.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

struct u4 { uint32_t x, y, z, w; };

// Philox4x32-10 (Salmon et al., SC'11); same as oracle/ballenv_oracle.c
__device__ __forceinline__ u4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, unsigned long long seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  // keep the key schedule in VGPRs: hoisted into SGPRs it pins 20 scalar registers and spills
  asm volatile("" : "+v"(k0), "+v"(k1));
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one v_mad_u64_u32 per product instead of a mul_hi + mul_lo pair
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return u4{c0, c1, c2, c3};
}
__device__ __forceinline__ uint32_t tag(uint32_t purpose, uint32_t sub) { return (purpose << 24) | (sub & 0xFFFFFFu); }

}  // namespace
