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

// The library's memory (memory.hip): device buffers are stream-ordered pool allocations made
// and released on a per-device lifecycle stream -- releasing one never synchronises the device
// (hipFree does) -- and pinned host buffers come from a size-class cache (hipHostFree also
// synchronises the device).  dfree's precondition: no launch still reads the buffer (the
// handle has waited for its own work), or use dfree_after(p, s) to order the release after
// stream s's work.
hipStream_t life_stream(int device);
hipStream_t life_stream_current();
int dev_alloc(void** p, size_t bytes);
void dev_free(void* p);
void dev_free_after(void* p, hipStream_t after);
int host_alloc(void** p, size_t bytes, unsigned flags);
void host_free(void* p);

template <typename T>
int dalloc(T** p, size_t n) {
  if (n == 0) n = 1;
  void* q = nullptr;
  const int rc = dev_alloc(&q, n * sizeof(T));
  *p = static_cast<T*>(q);
  return rc;
}

template <typename T>
void dfree(T*& p) {
  dev_free((void*)p);
  p = nullptr;
}

template <typename T>
void dfree_after(T*& p, hipStream_t after) {
  dev_free_after((void*)p, after);
  p = nullptr;
}

template <typename T>
int halloc(T** p, size_t n, unsigned flags) {
  void* q = nullptr;
  const int rc = host_alloc(&q, (n ? n : 1) * sizeof(T), flags);
  *p = static_cast<T*>(q);
  return rc;
}

template <typename T>
void hfree(T*& p) {
  host_free((void*)p);
  p = nullptr;
}

inline long long cdiv(long long a, long long b) { return (a + b - 1) / b; }

}  // namespace gpmdm
