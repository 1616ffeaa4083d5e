// FP64 probe for gfx950: MFMA f64 16x16x4 fragment layout check and
// throughput of FP64 MFMA, FP64 VALU FMA, mixed issue and ocml exp(double).
// Standalone: hipcc --offload-arch=gfx950 -O3 fp64_probe.hip -o fp64_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));

// Layout probe: lane l supplies a[l], b[l]; result regs dumped per lane.
__global__ void k_layout(const double* a, const double* b, double* c) {
  int l = threadIdx.x;
  d4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[l], b[l], acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) c[l * 4 + r] = acc[r];
}

template <int NACC>
__global__ void k_mfma_rate(double* out, int iters, double s) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (d4){0, 0, 0, 0};
  double a = s * threadIdx.x, b = s + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double t = 0;
  for (int i = 0; i < NACC; ++i) t += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (t == 12345.678) out[0] = t;
}

template <int NCH>
__global__ void k_valu_rate(double* out, int iters, double s) {
  double x[NCH];
  for (int i = 0; i < NCH; ++i) x[i] = s * (threadIdx.x + i);
  double m = 1.0 + 1e-9 * s, c = 1e-7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) x[i] = fma(x[i], m, c);
  }
  double t = 0;
  for (int i = 0; i < NCH; ++i) t += x[i];
  if (t == 12345.678) out[0] = t;
}

// mixed: 16 MFMA accumulators + 8 VALU fma chains per iteration
__global__ void k_mixed(double* out, int iters, double s, int valu_per_iter) {
  d4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = (d4){0, 0, 0, 0};
  double a = s * threadIdx.x, b = s + threadIdx.x;
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = s * (threadIdx.x + i);
  double m = 1.0 + 1e-9 * s, c = 1e-7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = fma(x[i], m, c);
    }
  }
  double t = 0;
  for (int i = 0; i < 8; ++i) t += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3] + x[i];
  if (t == 12345.678) out[0] = t;
}

__global__ void k_exp_rate(double* out, int iters, double s) {
  double x[4];
  for (int i = 0; i < 4; ++i) x[i] = -s * (threadIdx.x + i) * 1e-3;
  double acc = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { acc += exp(x[i]); x[i] -= 1e-6; }
  }
  if (acc == 12345.678) out[0] = acc;
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

int main(int argc, char** argv) {
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  int ncu = prop.multiProcessorCount;
  printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, ncu, prop.clockRate);

  // ---- layout ----
  double ha[64], hb[64], hc[256];
  // assumed maps: A[i][k] at lane i + 16k ; B[k][j] at lane j + 16k
  double A[16][4], B[4][16];
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 4; ++k) A[i][k] = (i + 1) * 10 + k * 1000 + 0.5 * (i * k % 3);
  for (int k = 0; k < 4; ++k) for (int j = 0; j < 16; ++j) B[k][j] = (k == 0 ? 1 : 0) * (j + 1) + (k == 1 ? 0.25 * j * j : 0) + (k == 2 ? 1.0 / (j + 1) : 0) + (k == 3 ? -j : 0);
  for (int l = 0; l < 64; ++l) { ha[l] = A[l & 15][l >> 4]; hb[l] = B[l >> 4][l & 15]; }
  double *da, *db, *dc;
  CK(hipMalloc(&da, 64 * 8)); CK(hipMalloc(&db, 64 * 8)); CK(hipMalloc(&dc, 256 * 8));
  CK(hipMemcpy(da, ha, 64 * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, hb, 64 * 8, hipMemcpyHostToDevice));
  k_layout<<<1, 64>>>(da, db, dc);
  CK(hipMemcpy(hc, dc, 256 * 8, hipMemcpyDeviceToHost));
  int bad_a = 0, bad_b = 0;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
    // map A: row=(l>>4)+4r ; map B: row=(l>>4)*4+r ; col=l&15
    int col = l & 15;
    int rowA = (l >> 4) + 4 * r, rowB = (l >> 4) * 4 + r;
    double refA = 0, refB = 0;
    for (int k = 0; k < 4; ++k) { refA += A[rowA][k] * B[k][col]; refB += A[rowB][k] * B[k][col]; }
    if (fabs(refA - hc[l * 4 + r]) > 1e-9 * fabs(refA) + 1e-12) bad_a++;
    if (fabs(refB - hc[l * 4 + r]) > 1e-9 * fabs(refB) + 1e-12) bad_b++;
  }
  printf("layout: C row=(l>>4)+4r mismatches=%d ; C row=4*(l>>4)+r mismatches=%d\n", bad_a, bad_b);

  double* dout; CK(hipMalloc(&dout, 8));
  int iters = 2000;
  // MFMA rate: 4 waves/CU .. 8 waves/CU
  for (int wpc : {4, 8}) {
    int blocks = ncu * wpc / 4;
    float ms = time_kernel([&] { k_mfma_rate<8><<<blocks, 256>>>(dout, iters, 1.0); });
    double flops = (double)blocks * 4 * iters * 8 * 2.0 * 16 * 16 * 4;
    printf("mfma_f64 16x16x4  waves/CU=%d acc=8 : %.3f ms  %.2f TFLOP/s\n", wpc, ms, flops / ms / 1e9);
  }
  {
    int blocks = ncu * 2;
    float ms = time_kernel([&] { k_mfma_rate<1><<<blocks, 256>>>(dout, iters * 8, 1.0); });
    double flops = (double)blocks * 4 * iters * 8 * 2.0 * 16 * 16 * 4;
    printf("mfma_f64 16x16x4  waves/CU=8 acc=1 (dependent chain) : %.3f ms  %.2f TFLOP/s\n", ms, flops / ms / 1e9);
  }
  for (int wpc : {4, 8, 16}) {
    int blocks = ncu * wpc / 4;
    float ms = time_kernel([&] { k_valu_rate<8><<<blocks, 256>>>(dout, iters * 4, 1.0); });
    double flops = (double)blocks * 256 * iters * 4 * 8 * 2.0;
    printf("valu fma_f64 waves/CU=%d : %.3f ms  %.2f TFLOP/s\n", wpc, ms, flops / ms / 1e9);
  }
  {
    int blocks = ncu * 2;
    float ms = time_kernel([&] { k_mixed<<<blocks, 256>>>(dout, iters, 1.0, 64); });
    double mf = (double)blocks * 4 * iters * 8 * 2.0 * 16 * 16 * 4;
    double vf = (double)blocks * 256 * iters * 64 * 2.0;
    printf("mixed (8 mfma + 64 valu fma per iter) waves/CU=8 : %.3f ms  mfma %.2f TF + valu %.2f TF = %.2f TF\n",
           ms, mf / ms / 1e9, vf / ms / 1e9, (mf + vf) / ms / 1e9);
    float ms_m = time_kernel([&] { k_mfma_rate<8><<<blocks, 256>>>(dout, iters, 1.0); });
    printf("   (mfma alone same grid: %.3f ms)\n", ms_m);
  }
  for (int wpc : {8, 16}) {
    int blocks = ncu * wpc / 4;
    float ms = time_kernel([&] { k_exp_rate<<<blocks, 256>>>(dout, iters, 1.0); });
    double n = (double)blocks * 256 * iters * 4;
    printf("exp(double) waves/CU=%d : %.3f ms  %.2f Gexp/s\n", wpc, ms, n / ms / 1e6);
  }
  // Sustained rate (argv[1] = seconds, e.g. 0.5): one long launch at 8 waves/CU, so power
  // management has settled on its clock -- the practical ceiling for a multi-ms kernel.
  if (argc > 1) {
    const double secs = atof(argv[1]);
    const int blocks = ncu * 2;
    const int long_iters = (int)(iters * secs / 0.87e-3);
    hipEvent_t a0, a1; CK(hipEventCreate(&a0)); CK(hipEventCreate(&a1));
    CK(hipEventRecord(a0));
    k_mfma_rate<8><<<blocks, 256>>>(dout, long_iters, 1.0);
    CK(hipEventRecord(a1));
    CK(hipEventSynchronize(a1));
    float ms; CK(hipEventElapsedTime(&ms, a0, a1));
    const double flops = (double)blocks * 4 * long_iters * 8 * 2.0 * 16 * 16 * 4;
    printf("sustained mfma_f64 16x16x4 waves/CU=8, one %.0f ms launch: %.2f TFLOP/s\n", ms, flops / ms / 1e9);
  }
  return 0;
}
