// The library's memory and its lifecycle stream (DESIGN.md §1 "Lifecycle waits").
//
// hipFree, hipHostFree and hipFreeAsync of hipMalloc memory each wait for every stream of the
// device (measured: tools/microbench/sync_probe.hip, profiles/r06/lifecycle/sync_probe.txt), so
// a filter destroyed, rebound or re-imported while a bank steps on another stream would stall
// the host behind the bank's work.  Instead:
//  * device buffers are stream-ordered allocations from the device's default memory pool,
//    made and released on a library-owned non-blocking stream per device (the lifecycle
//    stream).  dfree releases a buffer in that stream's order: its caller has already waited
//    for every launch that reads the buffer (the handle's own read-out numbers, events and
//    side streams: capi_pf.hip quiesce) or orders the release after them (dfree_after, or a
//    hipStreamWaitEvent on the lifecycle stream);
//  * pinned host buffers are cached: a released buffer goes back to a free list of its size
//    class and is handed to the next request, never to hipHostFree (page-locked memory is
//    returned to the system when the process exits, as torch's host caching allocator does).
// Small lifecycle copies (init, import, tables) run on the lifecycle stream too, so they
// neither wait for nor hold up the legacy null stream's users.
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "status.h"

namespace gpmdm {

namespace {
std::mutex g_life_mu;
std::vector<hipStream_t> g_life;   // per device, made on first use

std::mutex g_host_mu;
std::map<std::pair<size_t, unsigned>, std::vector<void*>> g_host_free;    // (bytes, flags) -> free buffers
std::unordered_map<void*, std::pair<size_t, unsigned>> g_host_live;       // buffer -> its size class

size_t host_class(size_t bytes) {   // power-of-two size classes from 4 KiB
  size_t c = 4096;
  while (c < bytes) c <<= 1;
  return c;
}
}  // namespace

hipStream_t life_stream(int device) {
  std::lock_guard<std::mutex> lk(g_life_mu);
  if ((int)g_life.size() <= device) g_life.resize((size_t)device + 1, nullptr);
  if (!g_life[(size_t)device]) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    hipStream_t s = nullptr;
    if (hipSetDevice(device) == hipSuccess && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess)
      g_life[(size_t)device] = s;
    (void)hipSetDevice(cur);
  }
  return g_life[(size_t)device];
}

hipStream_t life_stream_current() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  return life_stream(dev);
}

int dev_alloc(void** p, size_t bytes) {
  *p = nullptr;
  hipStream_t s = life_stream_current();
  if (!s) return fail(GPMDM_E_HIP, "the library's lifecycle stream");
  hipError_t e = hipMallocAsync(p, bytes, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);   // complete before any other stream uses it
  if (e != hipSuccess) {
    *p = nullptr;
    (void)hipGetLastError();
    return fail(GPMDM_E_NOMEM, std::string("hipMallocAsync: ") + hipGetErrorString(e));
  }
  return GPMDM_OK;
}

static int device_of(void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    int cur = 0;
    (void)hipGetDevice(&cur);
    return cur;
  }
  return a.device;
}

void dev_free(void* p) {
  if (!p) return;
  hipStream_t s = life_stream(device_of(p));
  if (!s || hipFreeAsync(p, s) != hipSuccess) (void)hipGetLastError();
}

void dev_free_after(void* p, hipStream_t after) {
  if (!p) return;
  if (hipFreeAsync(p, after) != hipSuccess) (void)hipGetLastError();
}

int host_alloc(void** p, size_t bytes, unsigned flags) {
  *p = nullptr;
  const size_t c = host_class(bytes);
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    auto it = g_host_free.find({c, flags});
    if (it != g_host_free.end() && !it->second.empty()) {
      *p = it->second.back();
      it->second.pop_back();
      g_host_live[*p] = {c, flags};
      return GPMDM_OK;
    }
  }
  void* q = nullptr;
  if (hipHostMalloc(&q, c, flags) != hipSuccess) {
    (void)hipGetLastError();
    return fail(GPMDM_E_NOMEM, "hipHostMalloc");
  }
  std::lock_guard<std::mutex> lk(g_host_mu);
  g_host_live[q] = {c, flags};
  *p = q;
  return GPMDM_OK;
}

void host_free(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_host_mu);
  auto it = g_host_live.find(p);
  if (it == g_host_live.end()) return;
  g_host_free[it->second].push_back(p);
  g_host_live.erase(it);
}

}  // namespace gpmdm
