// Reproducer of the gfx950 store-data hazard (tests/test_isa_guard.py).
//
// Round 2's K* cache producer stored each lane's two A-fragment doubles with one 16-byte
// buffer_store_dwordx4 straight from the VGPRs the next sub-step's ds_read refilled;
// 0.33% of the stored values came out with a wrong low dword, nondeterministically, while
// two 8-byte stores of the same registers were exact.  This kernel isolates the pattern:
// per iteration each lane reads pattern A from LDS into v[0:3], stores v[0:3] to global
// memory, and the very next instruction refills v[0:3] from LDS with pattern B.  The
// stored data must be A.  Variants:
//   0: buffer_store_dwordx4, then ds_read_b128 at once        (the round-2 pattern)
//   1: buffer_store_dwordx4, s_nop 0, then ds_read_b128       (one wait state)
//   2: two buffer_store_dwordx2 of v[0:1], v[2:3], then ds_read_b128  (8-byte stores)
//   3: buffer_store_dwordx4, then v_mov_b32 x4 overwriting v[0:3] (a VALU write)
// Every lane checks its own stored values afterwards; the count of wrong dwords (and the
// lanes they hit) is printed per variant.  One run is recorded in profiles/r03/.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench/store_hazard.hip -o tools/microbench/store_hazard
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef unsigned v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned patA(unsigned it, unsigned lane, unsigned k) { return 0xA0000000u ^ (it * 977u) ^ (lane << 4) ^ k; }
__device__ __forceinline__ unsigned patB(unsigned it, unsigned lane, unsigned k) { return 0x5B000000u ^ (it * 131u) ^ (lane << 8) ^ (k << 2); }

template <int V>
__global__ __launch_bounds__(256) void k_store_hazard(unsigned* out, int iters) {
  __shared__ v4u lds[2][256];
  const unsigned tid = threadIdx.x, lane = tid & 63;
  const unsigned long long base = (unsigned long long)blockIdx.x * iters * 256;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(out + base * 4), (short)0, 0x7fffffff, 0x00020000);
  const unsigned a_addr = (unsigned)(size_t)&lds[0][tid];
  const unsigned b_addr = (unsigned)(size_t)&lds[1][tid];
  for (int it = 0; it < iters; ++it) {
    lds[0][tid] = (v4u){patA(it, lane, 0), patA(it, lane, 1), patA(it, lane, 2), patA(it, lane, 3)};
    lds[1][tid] = (v4u){patB(it, lane, 0), patB(it, lane, 1), patB(it, lane, 2), patB(it, lane, 3)};
    __syncthreads();
    const unsigned voff = ((unsigned)it * 256u + tid) * 16u;
    const unsigned voff8 = voff + 8u;
    // fixed registers v[40:43] (inline asm cannot name sub-registers of an operand)
#define HZ_READ_A "ds_read_b128 v[40:43], %0\n\ts_waitcnt lgkmcnt(0)\n\t"
#define HZ_READ_B "ds_read_b128 v[40:43], %3\n\ts_waitcnt lgkmcnt(0)"
#define HZ_ARGS : : "v"(a_addr), "v"(voff), "s"(rsrc), "v"(b_addr), "v"(voff8) : "v40", "v41", "v42", "v43", "memory"
    if constexpr (V == 0) {
      asm volatile(HZ_READ_A "buffer_store_dwordx4 v[40:43], %1, %2, 0 offen\n\t" HZ_READ_B HZ_ARGS);
    } else if constexpr (V == 1) {
      asm volatile(HZ_READ_A "buffer_store_dwordx4 v[40:43], %1, %2, 0 offen\n\ts_nop 0\n\t" HZ_READ_B HZ_ARGS);
    } else if constexpr (V == 2) {
      asm volatile(HZ_READ_A "buffer_store_dwordx2 v[40:41], %1, %2, 0 offen\n\t"
                   "buffer_store_dwordx2 v[42:43], %4, %2, 0 offen\n\t" HZ_READ_B HZ_ARGS);
    } else {
      asm volatile(HZ_READ_A "buffer_store_dwordx4 v[40:43], %1, %2, 0 offen\n\t"
                   "v_mov_b32 v40, %3\n\tv_mov_b32 v41, %3\n\tv_mov_b32 v42, %3\n\tv_mov_b32 v43, %3" HZ_ARGS);
    }
#undef HZ_READ_A
#undef HZ_READ_B
#undef HZ_ARGS
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 2048, iters = argc > 2 ? atoi(argv[2]) : 64;
  const size_t n = (size_t)blocks * iters * 256 * 4;
  unsigned* d;
  CK(hipMalloc(&d, n * 4));
  std::vector<unsigned> h(n);
  void (*kern[4])(unsigned*, int) = {k_store_hazard<0>, k_store_hazard<1>, k_store_hazard<2>, k_store_hazard<3>};
  const char* names[4] = {"dwordx4 + ds_read at once", "dwordx4 + s_nop 0 + ds_read", "2 x dwordx2 + ds_read",
                          "dwordx4 + VALU overwrite"};
  for (int v = 0; v < 4; ++v) {
    CK(hipMemset(d, 0, n * 4));
    hipLaunchKernelGGL(kern[v], dim3(blocks), dim3(256), 0, 0, d, iters);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
    size_t bad = 0, bad_lo = 0;
    unsigned long long lanes = 0;
    for (size_t b = 0; b < (size_t)blocks; ++b)
      for (int it = 0; it < iters; ++it)
        for (unsigned t = 0; t < 256; ++t)
          for (unsigned k = 0; k < 4; ++k) {
            const unsigned lane = t & 63;
            const unsigned want = 0xA0000000u ^ ((unsigned)it * 977u) ^ (lane << 4) ^ k;
            const unsigned got = h[((b * iters + it) * 256 + t) * 4 + k];
            if (got != want) {
              ++bad;
              if (k % 2 == 0) ++bad_lo;
              lanes |= 1ull << lane;
            }
          }
    printf("variant %d (%-28s): %zu of %zu dwords wrong (%zu low dwords), lanes mask %016llx\n", v, names[v], bad,
           n, bad_lo, lanes);
  }
  CK(hipFree(d));
  return 0;
}
