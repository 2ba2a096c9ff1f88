// internal.h -- library-internal interface between the translation units of
// libballenv.so (not part of the C ABI in include/ballenv.h).
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "ballenv.h"

// Makes `device` the calling thread's current HIP device for the scope of one entry point and
// restores the caller's device on exit, so no be_* call changes which GPU later torch / HIP calls
// of the same thread use (a one-process multi-device caller).  err != hipSuccess: the switch failed
// (nothing to restore).
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int device) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != device) err = hipSetDevice(device);
    else prev = -1;                        // already current (or the query failed): nothing to restore
    if (err != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

struct be_ctx_view {
  int32_t num_envs, window, device, num_static, num_dynamic;
  int64_t env_offset;
};
__attribute__((visibility("hidden"))) be_ctx_view be_ctx_get(const be_ctx* ctx);
// record msg as ctx's last error (or the process-wide one for a NULL ctx); returns code
__attribute__((visibility("hidden"))) int be_ctx_fail(be_ctx* ctx, int code, const char* msg);
// be_state pointer checks shared by the entry points (BE_OK or a be_ctx_fail code)
__attribute__((visibility("hidden"))) int be_ctx_check_state(be_ctx* ctx, const be_state* st);

// fused config-5 rollout (be_policy_rollout -> rollout_kernel with the policy in the loop)
struct be_pol_rollout_args {
  const uint8_t* img;          // packed Policy(W) image (device)
  int32_t img_bytes, HT, KS, NO, num_actions;
  unsigned long long seed;
  const uint8_t* obs_in;       // (N, F) obs of the current state
  uint8_t* obs_last;           // (N, F) or NULL
  int32_t steps;
  const be_out* out;           // per-step (steps, N, ...) outputs
  const be_act_out* act;       // (steps, N) action / log_prob / value
};
// 1: launched; 0: no fused kernel for this env / policy shape (the caller loops); < 0: error
__attribute__((visibility("hidden"))) int be_internal_policy_rollout(be_ctx* ctx, const be_state* st,
                                                                     const be_pol_rollout_args* a, void* stream);
