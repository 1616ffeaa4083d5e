// Device-side GP factor: the setup step before the particle-filter path
// (_precompute_kernel_inverses, gpmdm.py:1284-1305), one GP block
// at a time (the observation GP, or one class block of the dynamics GP -- the reference
// builds the full masked Nx x Nx matrix, whose off-class blocks contribute exact zeros).
//
//   K = exp(-|x_i/l - x_j/l|^2) + a I + b I  [+ x~_i^T C^2 x~_j]  [+ c I]
//       (gpmdm.py:381-406 observation kernel; 408-434 dynamics kernel, 520-548 linear part;
//        the expansion form of the distance as gpmdm.py:508-515)
//   U = chol_upper(K)            rocSOLVER potrf
//   R = U^-1                     rocSOLVER trtri       (gpmdm.py:1287-1289: torch.inverse(U))
//   M = R R^T B                  two rocBLAS trmm      (beta = K_y^-1 Y, alpha_c = A_c Xout_c)
//
// Layout: the library is row-major; rocSOLVER/rocBLAS are column-major.  A row-major
// symmetric K is its own column-major image, so the column-major LOWER factor L (K = L L^T)
// is, read row-major, the upper factor U = L^T; the column-major inverse L^-1 read
// row-major is R = U^-1; and the column-major k x n image of a row-major n x k matrix is
// its transpose, so M^T = B^T R R^T is two right-side trmm with A = L^-1.
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <cmath>
#include <mutex>
#include <vector>

#include "common.h"
#include "status.h"

using namespace gpmdm;

namespace {

// Gram matrix of one GP block, row-major n x n (the sum order of the reference's torch
// expression: ((rbf + a) + b) + lin) + c).
__global__ __launch_bounds__(256) void k_gram(const double* __restrict__ Xs, const double* __restrict__ sq,
                                              const double* __restrict__ X, int n, int d,
                                              const double* __restrict__ lin_c2, double a, double b, double c,
                                              double* __restrict__ K) {
  const int j = blockIdx.x * 16 + (threadIdx.x & 15);
  const int i = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (i >= n || j >= n) return;
  double dot = 0.0;
  for (int k = 0; k < d; ++k) dot = fma(Xs[(long long)i * d + k], Xs[(long long)j * d + k], dot);
  double v = exp(-((sq[i] + sq[j]) - 2.0 * dot));
  if (i == j) v = (v + a) + b;
  if (lin_c2) {
    double l = 0.0;
    for (int k = 0; k < d; ++k) l = fma(lin_c2[k] * X[(long long)i * d + k], X[(long long)j * d + k], l);
    v += l + lin_c2[d];
  }
  if (i == j) v += c;
  K[(long long)i * n + j] = v;
}

// Zero the row-major strict lower triangle (the column-major upper part the solvers leave
// untouched).
__global__ __launch_bounds__(256) void k_zero_lower(double* R, int n) {
  const int j = blockIdx.x * 16 + (threadIdx.x & 15);
  const int i = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (i < n && j < i) R[(long long)i * n + j] = 0.0;
}

// Mirror the stored (column-major lower = row-major upper) triangle into the other one.
__global__ __launch_bounds__(256) void k_symmetrize_from_upper(double* A, int n) {
  const int j = blockIdx.x * 16 + (threadIdx.x & 15);
  const int i = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (i < n && j < i) A[(long long)i * n + j] = A[(long long)j * n + i];
}

// 2 sum_i log L_ii into *out (one block; the diagonal of a Cholesky factor).
__global__ __launch_bounds__(1024) void k_logdet_diag(const double* A, int n, double* out) {
  __shared__ double red[1024 / 64];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) s += log(A[(long long)i * n + i]);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < 1024 / 64; ++w) t += red[w];
    *out = 2.0 * t;
  }
}

struct Handle {
  rocblas_handle h = nullptr;
  ~Handle() {
    if (h) (void)rocblas_destroy_handle(h);
  }
};

#define RBCHK(expr)                                                                          \
  do {                                                                                       \
    rocblas_status st_ = (expr);                                                             \
    if (st_ != rocblas_status_success)                                                       \
      return fail(GPMDM_E_HIP, std::string(#expr) + ": " + rocblas_status_to_string(st_));   \
  } while (0)

struct DevBufs {
  double *Xs = nullptr, *sq = nullptr, *X = nullptr, *c2 = nullptr, *K = nullptr, *B0 = nullptr, *B1 = nullptr;
  int* info = nullptr;
  hipStream_t s = nullptr;   // the stream the buffers were used on (released after its work)
  ~DevBufs() {
    (void)hipStreamSynchronize(s);   // (an early error return may leave launches in flight)
    dfree(Xs); dfree(sq); dfree(X); dfree(c2); dfree(K); dfree(B0); dfree(B1); dfree(info);
  }
};

}  // namespace

extern "C" int gpmdm_gp_factor(int device, const double* X, int64_t n, int32_t d, const double* ls,
                               const double* lin_c2, double diag_a, double diag_b, double diag_c,
                               const double* B, int64_t k, double* R, double* M) {
  CHECK(X && ls && R, "null argument");
  CHECK(n >= 1 && n <= 46340, "n out of range (1..46340: n*n must fit rocBLAS' int32 indexing)");
  CHECK(d >= 1 && d <= kMaxD, "latent dimension out of range");
  CHECK(k >= 0 && (k == 0 || (B && M)), "right-hand side needs B and M");
  HIPCHK(hipSetDevice(device));
  const int N = (int)n;
  std::vector<double> xs((size_t)N * d), sq(N);
  for (long long i = 0; i < N; ++i) {
    double s = 0.0;
    for (int j = 0; j < d; ++j) {
      const double v = X[i * d + j] / ls[j];
      xs[i * d + j] = v;
      s += v * v;
    }
    sq[i] = s;
  }
  DevBufs b;
  TRY(dalloc(&b.Xs, xs.size()));
  TRY(dalloc(&b.sq, sq.size()));
  TRY(dalloc(&b.X, (size_t)N * d));
  TRY(dalloc(&b.K, (size_t)N * N));
  TRY(dalloc(&b.info, 1));
  HIPCHK(hipMemcpy(b.Xs, xs.data(), xs.size() * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b.sq, sq.data(), sq.size() * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b.X, X, (size_t)N * d * sizeof(double), hipMemcpyHostToDevice));
  if (lin_c2) {
    TRY(dalloc(&b.c2, (size_t)d + 1));
    HIPCHK(hipMemcpy(b.c2, lin_c2, (size_t)(d + 1) * sizeof(double), hipMemcpyHostToDevice));
  }
  Handle hd;
  RBCHK(rocblas_create_handle(&hd.h));
  hipStream_t s = nullptr;
  RBCHK(rocblas_set_stream(hd.h, s));
  const dim3 g2((unsigned)cdiv(N, 16), (unsigned)cdiv(N, 16));
  hipLaunchKernelGGL(k_gram, g2, dim3(256), 0, s, b.Xs, b.sq, b.X, N, (int)d, b.c2, diag_a, diag_b, diag_c, b.K);
  HIPCHK(hipGetLastError());
  int info = 0;
  RBCHK(rocsolver_dpotrf(hd.h, rocblas_fill_lower, N, b.K, N, b.info));
  HIPCHK(hipMemcpy(&info, b.info, sizeof(int), hipMemcpyDeviceToHost));
  if (info != 0)
    return fail(GPMDM_E_INVALID, "kernel matrix is not positive definite (potrf info=" + std::to_string(info) + ")");
  RBCHK(rocsolver_dtrtri(hd.h, rocblas_fill_lower, rocblas_diagonal_non_unit, N, b.K, N, b.info));
  HIPCHK(hipMemcpy(&info, b.info, sizeof(int), hipMemcpyDeviceToHost));
  if (info != 0) return fail(GPMDM_E_INVALID, "Cholesky factor is singular (trtri info=" + std::to_string(info) + ")");
  hipLaunchKernelGGL(k_zero_lower, g2, dim3(256), 0, s, b.K, N);
  HIPCHK(hipGetLastError());
  if (k > 0) {
    const int K = (int)k;
    TRY(dalloc(&b.B0, (size_t)N * K));
    TRY(dalloc(&b.B1, (size_t)N * K));
    HIPCHK(hipMemcpy(b.B0, B, (size_t)N * K * sizeof(double), hipMemcpyHostToDevice));
    const double one = 1.0;
    // column-major: T = B^T R = B^T (L^-1)^T ; M^T = T R^T = T L^-1   (A = L^-1, lower)
    RBCHK(rocblas_set_pointer_mode(hd.h, rocblas_pointer_mode_host));
    RBCHK(rocblas_dtrmm(hd.h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose,
                        rocblas_diagonal_non_unit, K, N, &one, b.K, N, b.B0, K, b.B1, K));
    RBCHK(rocblas_dtrmm(hd.h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_none,
                        rocblas_diagonal_non_unit, K, N, &one, b.K, N, b.B1, K, b.B0, K));
    HIPCHK(hipMemcpy(M, b.B0, (size_t)N * K * sizeof(double), hipMemcpyDeviceToHost));
  }
  HIPCHK(hipMemcpy(R, b.K, (size_t)N * N * sizeof(double), hipMemcpyDeviceToHost));
  return GPMDM_OK;
}

// One rocBLAS handle per device, created on first use (handle creation costs milliseconds;
// a training step at small N costs a few).  rocBLAS manages its own workspace on it.
rocblas_handle cached_handle(int device) {   // (also cutoff_image.hip)
  static std::mutex mu;
  static std::vector<rocblas_handle> handles;
  std::lock_guard<std::mutex> lock(mu);
  if ((int)handles.size() <= device) handles.resize(device + 1, nullptr);
  if (!handles[device] && rocblas_create_handle(&handles[device]) != rocblas_status_success) handles[device] = nullptr;
  return handles[device];
}

extern "C" int gpmdm_spd_inverse(int device, double* A, int64_t n, double* logdet, void* stream) {
  CHECK(A && logdet, "null argument");
  CHECK(n >= 1 && n <= 46340, "n out of range (1..46340: n*n must fit rocBLAS' int32 indexing)");
  *logdet = NAN;
  HIPCHK(hipSetDevice(device));
  rocblas_handle h = cached_handle(device);
  if (!h) return fail(GPMDM_E_HIP, "rocblas_create_handle failed");
  hipStream_t s = (hipStream_t)stream;
  RBCHK(rocblas_set_stream(h, s));
  const int N = (int)n;
  DevBufs b;
  b.s = s;
  TRY(dalloc(&b.info, 1));
  TRY(dalloc(&b.sq, 1));                                    // logdet scratch
  int info = 0;
  RBCHK(rocsolver_dpotrf(h, rocblas_fill_lower, N, A, N, b.info));
  HIPCHK(hipMemcpyAsync(&info, b.info, sizeof(int), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (info != 0)
    return fail(GPMDM_E_INVALID, "matrix is not positive definite (potrf info=" + std::to_string(info) + ")");
  hipLaunchKernelGGL(k_logdet_diag, dim3(1), dim3(1024), 0, s, A, N, b.sq);
  HIPCHK(hipGetLastError());
  RBCHK(rocsolver_dpotri(h, rocblas_fill_lower, N, A, N, b.info));
  const dim3 g2((unsigned)cdiv(N, 16), (unsigned)cdiv(N, 16));
  hipLaunchKernelGGL(k_symmetrize_from_upper, g2, dim3(256), 0, s, A, N);
  HIPCHK(hipGetLastError());
  double ld = NAN;
  HIPCHK(hipMemcpyAsync(&ld, b.sq, sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(&info, b.info, sizeof(int), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (info != 0) return fail(GPMDM_E_INVALID, "Cholesky factor is singular (potri info=" + std::to_string(info) + ")");
  *logdet = ld;
  return GPMDM_OK;
}
