// internal.h -- library-internal interface between the translation units of
// libballenv.so (not part of the C ABI in include/ballenv.h).
#pragma once
#include <stdint.h>

#include "ballenv.h"

struct be_ctx_view {
  int32_t num_envs, window, device, num_static, num_dynamic;
  int64_t env_offset;
};
__attribute__((visibility("hidden"))) be_ctx_view be_ctx_get(const be_ctx* ctx);
// record msg as ctx's last error (or the process-wide one for a NULL ctx); returns code
__attribute__((visibility("hidden"))) int be_ctx_fail(be_ctx* ctx, int code, const char* msg);
// be_state pointer checks shared by the entry points (BE_OK or a be_ctx_fail code)
__attribute__((visibility("hidden"))) int be_ctx_check_state(be_ctx* ctx, const be_state* st);
