// Issue-sharing probe for gfx950: does FP64 MFMA (v_mfma_f64_16x16x4_f64) share its pipe with
// FP64 VALU, FP32 VALU, integer VALU, the f64 conversion/rounding/ldexp ops and LDS reads?
// Each kernel runs 8 independent MFMAs per iteration plus K ops of one kind (8 chains);
// compare with MFMA alone and the ops alone.  8 waves per CU (2 per SIMD), as gp_tile.
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench/mix_probe.hip -o tools/microbench/mix_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));

enum Op { NONE = 0, F64FMA, F32FMA, I32ADD, LDEXP, CVT, RNDNE, LDS, I64ADD, CNDMASK };

template <int OP, int NMFMA, int K>
__global__ void k_mix(double* out, int iters, double s) {
  __shared__ double lds[1024];
  for (int i = threadIdx.x; i < 1024; i += 256) lds[i] = i * s;
  __syncthreads();
  d4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = (d4){0, 0, 0, 0};
  const double a = s * threadIdx.x, b = s + threadIdx.x;
  double xd[8];
  float xf[8];
  int xi[8];
  long long xl[8];
  for (int i = 0; i < 8; ++i) {
    xd[i] = s * (threadIdx.x + i);
    xf[i] = (float)xd[i];
    xi[i] = threadIdx.x * 7 + i;
    xl[i] = (long long)threadIdx.x * 11 + i;
  }
  const double md = 1.0 + 1e-9 * s, cd = 1e-7;
  const float mf = 1.0f + 1e-6f * (float)s, cf = 1e-5f;
  const int ci = (int)(s * 3.0) | 1;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NMFMA; ++i) acc[i & 7] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i & 7], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < K / 8; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (OP == F64FMA) xd[i] = fma(xd[i], md, cd);
        if constexpr (OP == F32FMA) xf[i] = fmaf(xf[i], mf, cf);
        if constexpr (OP == I32ADD) xi[i] = (xi[i] + ci) ^ (xi[i] >> 3);
        if constexpr (OP == LDEXP) xd[i] = ldexp(xd[i], (j & 1) ? 1 : -1);
        if constexpr (OP == CVT) xi[i] += (int)(xd[i] + (double)xi[i]);
        if constexpr (OP == RNDNE) xd[i] = __builtin_rint(xd[i] * 0.75 + 0.3);
        if constexpr (OP == LDS) xd[i] += lds[(xi[i] + j * 8 + i + threadIdx.x) & 1023];
        if constexpr (OP == I64ADD) xl[i] = xl[i] + (xl[i] >> 5) + ci;
        if constexpr (OP == CNDMASK) xd[i] = (xi[i] & (1 << (j & 7))) ? xd[i] : 0.5 * s;
      }
    }
  }
  double t = 0;
  for (int i = 0; i < 8; ++i) {
    t += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if constexpr (OP == F64FMA || OP == LDEXP || OP == RNDNE || OP == LDS || OP == CNDMASK) t += xd[i];
    if constexpr (OP == F32FMA) t += xf[i];
    if constexpr (OP == I32ADD || OP == CVT) t += xi[i];
    if constexpr (OP == I64ADD) t += (double)xl[i];
  }
  if (t == 12345.678) out[0] = t;
}

template <typename F>
static float time_kernel(F launch, int reps = 5) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  launch();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  return best;
}

template <int OP, int K>
void row(const char* name, double* dout, int blocks, int iters, float t_mfma) {
  const float t_ops = time_kernel([&] { k_mix<OP, 0, K><<<blocks, 256>>>(dout, iters, 1.0); });
  const float t_mix = time_kernel([&] { k_mix<OP, 8, K><<<blocks, 256>>>(dout, iters, 1.0); });
  printf("%-10s K=%3d  ops alone %.3f ms  mfma+ops %.3f ms  (mfma alone %.3f; sum %.3f) -> overlap %.0f%%\n", name, K,
         t_ops, t_mix, t_mfma, t_ops + t_mfma, 100.0 * (t_ops + t_mfma - t_mix) / (t_ops > 1e-6 ? t_ops : 1));
}

int main() {
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  const int blocks = ncu * 2, iters = 2000;
  double* dout; CK(hipMalloc(&dout, 8));
  const float t_mfma = time_kernel([&] { k_mix<NONE, 8, 0><<<blocks, 256>>>(dout, iters, 1.0); });
  printf("mfma alone (8 per iter): %.3f ms = %.1f TF/s\n", t_mfma,
         (double)blocks * 4 * iters * 8 * 2.0 * 16 * 16 * 4 / t_mfma / 1e9);
  row<F64FMA, 16>("f64 fma", dout, blocks, iters, t_mfma);
  row<F64FMA, 64>("f64 fma", dout, blocks, iters, t_mfma);
  row<F32FMA, 64>("f32 fma", dout, blocks, iters, t_mfma);
  row<I32ADD, 64>("i32 add^", dout, blocks, iters, t_mfma);
  row<I64ADD, 32>("i64 add", dout, blocks, iters, t_mfma);
  row<LDEXP, 32>("ldexp f64", dout, blocks, iters, t_mfma);
  row<CVT, 32>("cvt", dout, blocks, iters, t_mfma);
  row<RNDNE, 32>("rndne", dout, blocks, iters, t_mfma);
  row<CNDMASK, 32>("cndmask", dout, blocks, iters, t_mfma);
  row<LDS, 32>("lds read", dout, blocks, iters, t_mfma);
  return 0;
}
