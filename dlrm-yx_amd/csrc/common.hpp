// Shared helpers for the gfx950 DLRM kernels (error plumbing, wave helpers).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "dlrm_hip.h"

namespace dlrm {

// Thread-local last-error message (dlrm_last_error()).
void set_error(const char* fmt, ...);

// Thread-local plan overrides of dlrm_set_tuning (autotuning sweeps and coverage tests of
// the alternative tiles / block lengths / sort paths); 0 = the planner's choice.  The
// library reads no environment variables.
int64_t tuning(int key);

inline hipStream_t as_stream(dlrm_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace dlrm

#define DLRM_REQUIRE(cond, code, ...)   \
  do {                                  \
    if (!(cond)) {                      \
      dlrm::set_error(__VA_ARGS__);     \
      return (code);                    \
    }                                   \
  } while (0)

#define DLRM_ARG(cond, ...) DLRM_REQUIRE(cond, DLRM_ERR_INVALID_ARG, __VA_ARGS__)

#define DLRM_LAUNCH_CHECK(name)                                                        \
  do {                                                                                 \
    hipError_t e_ = hipGetLastError();                                                 \
    if (e_ != hipSuccess) {                                                            \
      dlrm::set_error("%s: HIP launch failed: %s", (name), hipGetErrorString(e_));     \
      return DLRM_ERR_HIP;                                                             \
    }                                                                                  \
  } while (0)

#define DLRM_HIP_CALL(expr, name)                                                      \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) {                                                            \
      dlrm::set_error("%s: %s failed: %s", (name), #expr, hipGetErrorString(e_));      \
      return DLRM_ERR_HIP;                                                             \
    }                                                                                  \
  } while (0)

// Workspace carving: 256-B aligned sub-buffers of one caller-provided block.
struct WsCarver {
  char* base;
  size_t used = 0;
  explicit WsCarver(void* p) : base(static_cast<char*>(p)) {}
  template <typename T>
  T* take(size_t count) {
    used = (used + 255) & ~size_t(255);
    T* p = base ? reinterpret_cast<T*>(base + used) : nullptr;
    used += count * sizeof(T);
    return p;
  }
};
