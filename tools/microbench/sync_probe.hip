// Which HIP runtime calls wait for unrelated device work?  A spin kernel (~150 ms) runs on a
// non-blocking stream A; each probed call is then timed on the host.  A call that returns in
// microseconds does not wait for A; one that takes ~150 ms synchronises with it.  Used to
// scope the library's lifecycle waits (DESIGN.md §1 "Lifecycle synchronisation").
//   hipcc --offload-arch=gfx950 -O2 tools/microbench/sync_probe.hip -o /tmp/sync_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("%s -> %s\n", #x, hipGetErrorString(e_));                            \
    }                                                                                  \
  } while (0)

__global__ void spin(unsigned long long ticks, double* out) {
  const unsigned long long t0 = wall_clock64();
  double acc = 0.0;
  while (wall_clock64() - t0 < ticks) acc += 1.0;
  if (threadIdx.x == 0 && acc < 0.0) out[blockIdx.x] = acc;   // never true: keeps the loop
}

int main() {
  int rate_khz = 0;
  CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  const unsigned long long ticks = (unsigned long long)rate_khz * 150;   // 150 ms
  hipStream_t A, B;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  double* dout = nullptr;
  CK(hipMalloc(&dout, 4096));
  std::vector<double> host(1 << 17, 1.0);   // 1 MiB pageable
  double* pinned = nullptr;
  CK(hipHostMalloc(&pinned, 1 << 20, 0));
  auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  auto probe = [&](const char* name, const std::function<void()>& f) {
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, A, ticks, dout);
    CK(hipGetLastError());
    const auto t0 = std::chrono::steady_clock::now();
    f();
    const auto t1 = std::chrono::steady_clock::now();
    const bool a_busy = hipStreamQuery(A) == hipErrorNotReady;
    std::printf("%-58s %9.3f ms   spin still running after: %s\n", name, ms(t0, t1), a_busy ? "yes" : "no");
    CK(hipDeviceSynchronize());
  };
  probe("(nothing)", [] {});
  double* p = nullptr;
  probe("hipMalloc 1 MiB", [&] { CK(hipMalloc(&p, 1 << 20)); });
  probe("hipFree 1 MiB", [&] { CK(hipFree(p)); });
  CK(hipMalloc(&p, 1 << 20));
  probe("hipMemcpy H2D 1 MiB pageable (null stream)", [&] { CK(hipMemcpy(p, host.data(), 1 << 20, hipMemcpyHostToDevice)); });
  probe("hipMemcpyAsync H2D pageable on B + sync B", [&] {
    CK(hipMemcpyAsync(p, host.data(), 1 << 20, hipMemcpyHostToDevice, B));
    CK(hipStreamSynchronize(B));
  });
  probe("hipMemcpyAsync H2D pinned on B + sync B", [&] {
    CK(hipMemcpyAsync(p, pinned, 1 << 20, hipMemcpyHostToDevice, B));
    CK(hipStreamSynchronize(B));
  });
  probe("hipMemcpyAsync D2H pageable on B + sync B", [&] {
    CK(hipMemcpyAsync(host.data(), p, 1 << 20, hipMemcpyDeviceToHost, B));
    CK(hipStreamSynchronize(B));
  });
  probe("hipMemset (null stream)", [&] { CK(hipMemset(p, 0, 1 << 20)); });
  probe("hipMemsetAsync on B + sync B", [&] {
    CK(hipMemsetAsync(p, 0, 1 << 20, B));
    CK(hipStreamSynchronize(B));
  });
  hipStream_t C = nullptr;
  probe("hipStreamCreateWithFlags(nonblocking)", [&] { CK(hipStreamCreateWithFlags(&C, hipStreamNonBlocking)); });
  probe("hipStreamDestroy", [&] { CK(hipStreamDestroy(C)); });
  hipEvent_t ev = nullptr;
  probe("hipEventCreateWithFlags", [&] { CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming)); });
  probe("hipEventDestroy", [&] { CK(hipEventDestroy(ev)); });
  double* hp = nullptr;
  probe("hipHostMalloc 1 MiB", [&] { CK(hipHostMalloc(&hp, 1 << 20, 0)); });
  probe("hipHostFree 1 MiB", [&] { CK(hipHostFree(hp)); });
  double* q = nullptr;
  probe("hipMallocAsync 1 MiB on B + sync B", [&] {
    CK(hipMallocAsync((void**)&q, 1 << 20, B));
    CK(hipStreamSynchronize(B));
  });
  probe("hipFreeAsync (hipMallocAsync memory) on B + sync B", [&] {
    CK(hipFreeAsync(q, B));
    CK(hipStreamSynchronize(B));
  });
  double* r = nullptr;
  CK(hipMalloc(&r, 1 << 20));
  probe("hipFreeAsync (hipMalloc memory) on B + sync B", [&] {
    CK(hipFreeAsync(r, B));
    CK(hipStreamSynchronize(B));
  });
  probe("hipDeviceSynchronize", [&] { CK(hipDeviceSynchronize()); });
  CK(hipFree(p));
  CK(hipFree(dout));
  CK(hipHostFree(pinned));
  std::printf("done\n");
  return 0;
}
