// Status plumbing shared by the C-ABI translation units (capi_*.hip, precompute.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "../../include/gpmdm_hip.h"

namespace gpmdm {

extern thread_local std::string g_err;   // gpmdm_last_error()
int fail(int code, const std::string& msg);

#define HIPCHK(expr)                                                                       \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return ::gpmdm::fail(GPMDM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define CHECK(cond, msg)                                                                   \
  do {                                                                                     \
    if (!(cond)) return ::gpmdm::fail(GPMDM_E_INVALID, msg);                               \
  } while (0)

#define TRY(expr)                                                                          \
  do {                                                                                     \
    int rc_ = (expr);                                                                      \
    if (rc_ != GPMDM_OK) return rc_;                                                       \
  } while (0)

template <typename T>
int dalloc(T** p, size_t n) {
  *p = nullptr;
  if (n == 0) n = 1;
  hipError_t e = hipMalloc((void**)p, n * sizeof(T));
  if (e != hipSuccess) return fail(GPMDM_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  return GPMDM_OK;
}

template <typename T>
void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

inline long long cdiv(long long a, long long b) { return (a + b - 1) / b; }

}  // namespace gpmdm
