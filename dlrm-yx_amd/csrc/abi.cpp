// Library-level entry points: version and thread-local error message.
#include <cstdarg>
#include <cstdio>

#include "common.hpp"

namespace dlrm {
namespace {
thread_local char g_last_error[1024] = {0};
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}
}  // namespace dlrm

extern "C" int dlrm_abi_version(void) { return 4; }

extern "C" const char* dlrm_last_error(void) { return dlrm::g_last_error; }
