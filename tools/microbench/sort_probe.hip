// Cost of the ancestor-order sort (shard_order.hip) on gfx950: rocPRIM radix sort of P int
// keys < P with particle-index values, over all key bits and over only the top `b` bits
// (coarse ancestor buckets, one or two digit passes).  HIP events around 50 launches.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 sort_probe.hip -o sort_probe && ./sort_probe
#include <cstdio>
#include <cstring>
#include <vector>
#include <random>
#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  for (long long P : {100000ll, 200000ll, 400000ll, 800000ll}) {
    int bits = 1;
    while ((1ll << bits) < P) ++bits;
    std::vector<int> h(P);
    std::mt19937 g(1);
    std::uniform_int_distribution<int> U(0, (int)P - 1);
    for (auto& x : h) x = U(g);
    std::sort(h.begin(), h.end());
    for (auto& x : h) x = h[U(g)];                   // resample-like: many repeats, random order
    int *keys, *kout, *vout;
    CK(hipMalloc(&keys, P * 4));
    CK(hipMalloc(&kout, P * 4));
    CK(hipMalloc(&vout, P * 4));
    CK(hipMemcpy(keys, h.data(), P * 4, hipMemcpyHostToDevice));
    for (int lowbit : {0, bits - 12, bits - 8}) {
      size_t bytes = 0;
      CK(rocprim::radix_sort_pairs(nullptr, bytes, keys, kout, rocprim::counting_iterator<int>(0), vout, (size_t)P,
                                   (unsigned)lowbit, (unsigned)bits));
      void* tmp;
      CK(hipMalloc(&tmp, bytes));
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      for (int it = 0; it < 5; ++it)
        CK(rocprim::radix_sort_pairs(tmp, bytes, keys, kout, rocprim::counting_iterator<int>(0), vout, (size_t)P,
                                     (unsigned)lowbit, (unsigned)bits));
      CK(hipEventRecord(a, 0));
      for (int it = 0; it < 50; ++it)
        CK(rocprim::radix_sort_pairs(tmp, bytes, keys, kout, rocprim::counting_iterator<int>(0), vout, (size_t)P,
                                     (unsigned)lowbit, (unsigned)bits));
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("P=%lld bits [%d,%d): %.1f us per sort (temp %zu B)\n", P, lowbit, bits, ms * 1e3 / 50, bytes);
      CK(hipFree(tmp));
    }
    CK(hipFree(keys));
    CK(hipFree(kout));
    CK(hipFree(vout));
  }
  return 0;
}
