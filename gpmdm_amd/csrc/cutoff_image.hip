// The observation-GP cutoff image built on the device from the model's own factor
// (gpmdm_model_build_obs_cutoff; SURVEY §8(f) row 1: the precompute feeding the path lives on
// the device, gpmdm.py:1284-1305).  The host path (gpmdm_model_set_obs_cutoff) needs K_y^-1 on
// the host -- 3.2 GB at configs[4] -- and packs it there; here:
//   1. R = U^-1 and M = K_y^-1 Y are read back out of the observation image the model already
//      holds (k_unpack_obs: the inverse of host_image.h ImagePacker::pack_block, a copy);
//   2. K_y^-1 = R R^T by rocBLAS dsyrk (the reference's Ky_inv = U^-1 U^-T, gpmdm.py:1289),
//      one triangle, read symmetrically by the packer;
//   3. tau, the spatial order, the K-step spheres and the row records on the host from X and
//      the column sums of M only (capi_model.hip cutoff_plan: O(N log N d) work on N x d);
//   4. the tile-major image by k_pack_cutoff: value for value host_image.h CutoffPacker::val
//      over the same perm (tests/test_gpu_obs_cutoff.py holds the two packers byte-equal).
// All on the library's lifecycle stream; no N x N matrix crosses PCIe.
#include <rocblas/rocblas.h>

#include "capi_internal.h"

rocblas_handle cached_handle(int device);   // precompute.hip

namespace gpmdm::capi {

// The doubles of column block J of a fragment-order image (host_image.h ImagePacker) back to
// R (n x n row-major, upper triangle) and M (n x n_m row-major).
__global__ void k_unpack_obs(const double* __restrict__ Bf, long long boff, long long nvals, int J, int n_rows,
                             int n_m, int coff, int nw, int ntw, double* __restrict__ R, double* __restrict__ M) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nvals) return;
  const int ws = 256 * ntw, nb = 16 * ntw * nw;
  const long long ks = q / ((long long)nw * ws);
  const int rem = (int)(q % ((long long)nw * ws));
  const int w = rem / ws, r2 = rem % ws;
  const int l = (r2 % 128) >> 1, v = 2 * (r2 / 128) + (r2 & 1);
  const int kk = v / ntw, nt = v % ntw;
  const long long row = ks * kBK + kk * 4 + (l >> 4);
  const long long col = (long long)J * nb + 16 * (nw * nt + w) + (l & 15) - coff;
  if (row >= n_rows || col < 0) return;
  const double x = Bf[boff + q];
  if (col < n_rows) {
    if (row <= col) R[row * n_rows + col] = x;
  } else if (col - n_rows < n_m) {
    M[row * n_m + (col - n_rows)] = x;
  }
}

// host_image.h CutoffPacker::pack_tile for tile t = blockIdx.y, K-step ks = blockIdx.x: the
// 256 doubles of Bt[toff[t] + 256 ks ..), lane j = 128 h + 2 l + e holding
// B[row = 16 ks + 4 (2h + e) + (l >> 4)][column l & 15 of tile t].  K: K^-1 column-major,
// upper triangle valid (dsyrk), read as K[min(a, b)][max(a, b)].
__global__ void k_pack_cutoff(const double* __restrict__ K, const double* __restrict__ M,
                              const long long* __restrict__ perm, const long long* __restrict__ toff,
                              int n_rows, int n_m, int T_R, double* __restrict__ Bt) {
  const int t = blockIdx.y, ks = blockIdx.x, j = threadIdx.x;
  const int kend = t < T_R ? t + 1 : T_R;
  if (ks >= kend) return;
  const int h = j >> 7, l = (j & 127) >> 1, e = j & 1;
  const long long row = (long long)ks * kBK + 4 * (2 * h + e) + (l >> 4);
  const int lc = l & 15;
  double v = 0.0;
  if (row < n_rows) {
    if (t < T_R) {
      const long long col = 16LL * t + lc;
      if (col < n_rows) {
        const long long bi = row / kBK, bj = col / kBK;
        if (bi <= bj) {
          const long long a = perm[row], b = perm[col];
          const double x = a <= b ? K[a + b * (long long)n_rows] : K[b + a * (long long)n_rows];
          v = bi < bj ? 2.0 * x : x;
        }
      }
    } else {
      const long long jm = 16LL * (t - T_R) + lc;
      if (jm < n_m) v = M[perm[row] * n_m + jm];
    }
  }
  Bt[toff[t] + 256LL * ks + j] = v;
}

}  // namespace gpmdm::capi

extern "C" int gpmdm_model_build_obs_cutoff(gpmdm_model_t m, double sigma2, const double* y_absmax, double* kinv_out,
                                            double* m_out) {
  CHECK(m && y_absmax, "null argument");
  CHECK(m->d <= 16, "the cutoff image is built for latent dimensions d <= 16");
  CHECK(ksteps((int)m->N) <= kMaxCutoffKs, "the cutoff image holds at most 65536 training rows");
  HIPCHK(hipSetDevice(m->device));
  hipStream_t ls = life_stream(m->device);
  CHECK(ls, "the library's lifecycle stream");
  const int N = (int)m->N, D = m->D;
  const GpImage& g = m->obs;
  double *R = nullptr, *K = nullptr, *Md = nullptr;
  long long* perm_d = nullptr;
  auto done = [&](int rc) {
    (void)hipStreamSynchronize(ls);
    dfree(R);
    dfree(K);
    dfree(Md);
    dfree(perm_d);
    return rc;
  };
  if (dalloc(&R, (size_t)N * N) || dalloc(&Md, (size_t)N * D)) return done(GPMDM_E_NOMEM);
  // 1. R and M out of the observation image (rows below the diagonal stay 0)
  if (hipMemsetAsync(R, 0, sizeof(double) * N * N, ls) != hipSuccess ||
      hipMemsetAsync(Md, 0, sizeof(double) * N * D, ls) != hipSuccess)
    return done(fail(GPMDM_E_HIP, "cutoff image: memset"));
  long long boff = 0;
  for (int J = 0; J < g.n_j; ++J) {
    const long long nv = (long long)ksteps(block_kmax(J, g.n_rows, g.geo.nb(), g.coff)) * g.geo.fs();
    hipLaunchKernelGGL(k_unpack_obs, dim3((unsigned)cdiv(nv, 256)), dim3(256), 0, ls, (const double*)g.Bf, boff, nv, J,
                       g.n_rows, g.n_m, g.coff, g.geo.nw, g.geo.ntw, R, Md);
    boff += nv;
  }
  if (hipGetLastError() != hipSuccess) return done(fail(GPMDM_E_HIP, "cutoff image: unpack launch"));
  std::vector<double> Mh((size_t)N * D);
  if (hipMemcpyAsync(Mh.data(), Md, sizeof(double) * N * D, hipMemcpyDeviceToHost, ls) != hipSuccess ||
      hipStreamSynchronize(ls) != hipSuccess)
    return done(fail(GPMDM_E_HIP, "cutoff image: M read-back"));
  // 3. the host half (tau, order, spheres, records, offsets)
  CutoffPlan pl;
  int rc = cutoff_plan(m, sigma2, Mh.data(), y_absmax, pl);
  if (rc) return done(rc);
  // 2. K^-1 = R R^T (column-major: A = R^T, K = A^T A; upper triangle)
  if (dalloc(&K, (size_t)N * N)) return done(GPMDM_E_NOMEM);
  rocblas_handle h = cached_handle(m->device);
  if (!h) return done(fail(GPMDM_E_HIP, "rocblas_create_handle failed"));
  const double one = 1.0, zero = 0.0;
  if (rocblas_set_stream(h, ls) != rocblas_status_success ||
      rocblas_dsyrk(h, rocblas_fill_upper, rocblas_operation_transpose, N, N, &one, R, N, &zero, K, N) !=
          rocblas_status_success)
    return done(fail(GPMDM_E_HIP, "cutoff image: rocblas_dsyrk"));
  dfree(R);                           // (released after the dsyrk in the lifecycle stream's order)
  if (kinv_out || m_out) {            // test aids: the K^-1 and M this image was packed from
    if (hipStreamSynchronize(ls) != hipSuccess) return done(fail(GPMDM_E_HIP, "cutoff image: dsyrk"));
    if (kinv_out) {
      std::vector<double> Kc((size_t)N * N);
      if (hipMemcpy(Kc.data(), K, sizeof(double) * N * N, hipMemcpyDeviceToHost) != hipSuccess)
        return done(fail(GPMDM_E_HIP, "cutoff image: K read-back"));
      for (long long i = 0; i < N; ++i)
        for (long long j = 0; j < N; ++j) kinv_out[i * N + j] = i <= j ? Kc[i + j * N] : Kc[j + i * N];
    }
    if (m_out) std::memcpy(m_out, Mh.data(), sizeof(double) * N * D);
  }
  // 4. the image
  if (dalloc(&perm_d, pl.perm.size()) ||
      hipMemcpyAsync(perm_d, pl.perm.data(), sizeof(long long) * pl.perm.size(), hipMemcpyHostToDevice, ls) != hipSuccess)
    return done(fail(GPMDM_E_HIP, "cutoff image: order upload"));
  rc = cutoff_install(m, pl, [&](double* Bt, const long long* toff) -> int {
    hipLaunchKernelGGL(k_pack_cutoff, dim3((unsigned)pl.T_R, (unsigned)(pl.T_R + pl.T_M)), dim3(256), 0, ls, K, Md,
                       perm_d, toff, N, D, pl.T_R, Bt);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ls));
    return GPMDM_OK;
  });
  return done(rc);
}
