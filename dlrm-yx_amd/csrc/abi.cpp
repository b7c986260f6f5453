// Library-level entry points: version and thread-local error message.
#include <cstdarg>
#include <cstdio>

#include "common.hpp"

namespace dlrm {
namespace {
thread_local char g_last_error[1024] = {0};
constexpr int kTuneKeys = 8;
thread_local int64_t g_tuning[kTuneKeys] = {0};
}

int64_t tuning(int key) { return key > 0 && key < kTuneKeys ? g_tuning[key] : 0; }

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}
}  // namespace dlrm

extern "C" int dlrm_abi_version(void) { return DLRM_ABI_VERSION; }

extern "C" const char* dlrm_last_error(void) { return dlrm::g_last_error; }

extern "C" int dlrm_set_tuning(int32_t key, int64_t value) {
  DLRM_ARG(key >= DLRM_TUNE_GEMM_TILE && key <= DLRM_TUNE_INTERACT_FWD,
           "dlrm_set_tuning: unknown key %d", (int)key);
  DLRM_ARG(value >= 0, "dlrm_set_tuning: negative value");
  dlrm::g_tuning[key] = value;
  return DLRM_OK;
}

extern "C" int64_t dlrm_get_tuning(int32_t key) { return dlrm::tuning(key); }
