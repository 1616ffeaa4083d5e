// Host-side construction of a GP's device image and the model-descriptor checks
// (plain C++17: no HIP; capi_model.hip uploads what this produces, and the host sanitizer test
// tests/test_host_asan.py builds it with -fsanitize=address,undefined).
//
// Fragment layout (consumed by gp_tile.h), for a tile shape (nw waves, each owning ntw
// column tiles of 16; nb = 16 ntw nw columns per block): column block J stores
// ksteps(block_kmax(J)) K-steps; each K-step holds nw waves x 256 ntw doubles, and inside a
// wave's share the value v = 2q + e of lane l sits at q*128 + 2l + e, where
// v = kk*ntw + nt is the B operand of MFMA sub-step kk (K=4) for column tile nt of wave w,
// whose 16 columns are interleaved with the other waves' tiles:
//   B[row = 16 ks + 4 kk + (l >> 4)][col = nb J + 16 (nw nt + w) + (l & 15)].
// A lane's 4 ntw values are therefore 16-byte loads, each wave-instruction reading one
// contiguous 1 KiB.  Rows below the diagonal of R are never stored (triangular skip).
//
// Dynamics images also carry H = (X~ C^2)^T B ((d+1) x cols, X~ = [Xin, 1], C^2 the linear
// kernel's coefficients, gpmdm.py:493-506): the linear kernel's share of K* B, seeded into
// the accumulators by MFMA.  Hf[((J kh_n + kh) nw + w) 64 ntw + ntw l + nt] =
//   H[row = 4 kh + (l >> 4)][col = nb J + 16 (nw nt + w) + (l & 15) - coff].
#pragma once

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <string>
#include <utility>
#include <vector>

#include "../../include/gpmdm_hip.h"
#include "geometry.h"

namespace gpmdm {

constexpr int kMaxClassesDesc = 32;

inline bool supported_d(int d) { return (d >= 1 && d <= 16) || d == 24 || d == 32; }

// "" if the descriptor is usable, else the reason (gpmdm_model_create's argument checks).
inline std::string check_model_desc(const gpmdm_model_desc* desc) {
  if (!desc) return "null argument";
  if (!(desc->N > 0 && desc->D > 0 && desc->C > 0)) return "N, D and C must be positive";
  if (!supported_d(desc->d)) return "latent dimension d must be 1..16, 24 or 32";
  if (desc->C > kMaxClassesDesc) return "at most 32 classes";
  if (desc->N >= (1ll << 30)) return "N too large";
  if (!(desc->X && desc->obs_R && desc->obs_beta && desc->y_lengthscales && desc->y_inv_lambda2 && desc->Nc &&
        desc->Xin && desc->dyn_R && desc->dyn_alpha && desc->x_lengthscales && desc->x_lin_coeff2 &&
        desc->x_inv_lambda2))
    return "null array in model descriptor";
  if (desc->tile_shape < GPMDM_TILE_DEFAULT || desc->tile_shape > GPMDM_TILE_32x512)
    return "tile_shape must be one of GPMDM_TILE_*";
  for (int c = 0; c < desc->C; ++c)
    if (desc->Nc[c] <= 0 || desc->Nc[c] >= (1ll << 30) || !desc->Xin[c] || !desc->dyn_R[c] || !desc->dyn_alpha[c])
      return "class " + std::to_string(c) + " has no dynamics rows";
  return "";
}

// One GP's image, packed block by block (the device image is streamed up per block so the
// host never holds a second copy of an N^2 matrix).
struct ImagePacker {
  int n_rows, d, n_m, coff, n_j;
  TileGeo geo;
  const double *X, *ls, *lin_c2, *R, *M;

  ImagePacker(int n_rows_, int d_, int n_m_, const double* X_, const double* ls_, const double* lin_c2_,
              const double* R_, const double* M_, TileGeo geo_)
      : n_rows(n_rows_), d(d_), n_m(n_m_), geo(geo_), X(X_), ls(ls_), lin_c2(lin_c2_), R(R_), M(M_) {
    coff = col_offset(n_rows + n_m, geo.nb());
    n_j = (n_rows + n_m + coff + geo.nb() - 1) / geo.nb();
  }

  // B = [triu(R) | M] (row-major inputs R: n_rows x n_rows, M: n_rows x n_m)
  double val(long long row, long long col) const {
    if (row >= n_rows || col < 0) return 0.0;
    if (col < n_rows) return row <= col ? R[row * n_rows + col] : 0.0;   // upper triangle of R
    const long long j = col - n_rows;
    return j < n_m ? M[row * n_m + j] : 0.0;
  }

  // Row records [Xs_i, |Xs_i|^2 * 64/ln2], Xs = X / ls: (d + 1) doubles per row, padded to
  // row_cap(n_rows) rows with Xs = 0 and |Xs|^2 = kPadSq (kernel value exactly 0).
  void records(std::vector<double>& rec) const {
    const int cap = row_cap(n_rows), rw = d + 1;
    rec.assign((size_t)cap * rw, 0.0);
    for (int i = n_rows; i < cap; ++i) rec[(size_t)i * rw + d] = kPadSq;
    for (long long i = 0; i < n_rows; ++i) {
      double s = 0.0;
      for (int j = 0; j < d; ++j) {
        const double v = X[i * d + j] / ls[j];
        rec[i * rw + j] = v;
        s += v * v;
      }
      rec[i * rw + d] = s * kLog2eX64;
    }
  }

  long long block_doubles(int J) const {
    return (long long)ksteps(block_kmax(J, n_rows, geo.nb(), coff)) * geo.fs();
  }
  long long total_doubles() const {
    long long t = 0;
    for (int J = 0; J < n_j; ++J) t += block_doubles(J);
    return t;
  }

  // Fragment-order B of column block J into dst[0, block_doubles(J)).
  void pack_block(int J, double* dst) const {
    const int nw = geo.nw, ntw = geo.ntw, nb = geo.nb(), ws = 256 * ntw;
    const int nks = ksteps(block_kmax(J, n_rows, nb, coff));
    for (int ks = 0; ks < nks; ++ks)
      for (int w = 0; w < nw; ++w) {
        double* o = dst + ((size_t)ks * nw + w) * ws;
        for (int l = 0; l < 64; ++l)
          for (int v = 0; v < 4 * ntw; ++v) {
            const int kk = v / ntw, nt = v % ntw;
            const long long row = (long long)ks * kBK + kk * 4 + (l >> 4);
            const long long col = (long long)J * nb + 16 * (nw * nt + w) + (l & 15) - coff;
            o[(v >> 1) * 128 + 2 * l + (v & 1)] = val(row, col);
          }
      }
  }

  // Dynamics GPs: H = (X~ C^2)^T B in fragment order (empty when lin_c2 is null).
  void linear(std::vector<double>& hf) const {
    hf.clear();
    if (!lin_c2) return;
    const int nw = geo.nw, ntw = geo.ntw, nb = geo.nb();
    const long long n_cols = (long long)n_rows + n_m;
    std::vector<double> H((size_t)(d + 1) * n_cols, 0.0);
    for (long long i = 0; i < n_rows; ++i)
      for (long long col = 0; col < n_cols; ++col) {
        const double b = val(i, col);
        if (b == 0.0) continue;
        for (int k = 0; k < d; ++k) H[k * n_cols + col] += lin_c2[k] * X[i * d + k] * b;
        H[(size_t)d * n_cols + col] += lin_c2[d] * b;
      }
    const int kh_n = lin_substeps(d);
    hf.assign((size_t)n_j * kh_n * nw * 64 * ntw, 0.0);
    for (int J = 0; J < n_j; ++J)
      for (int kh = 0; kh < kh_n; ++kh)
        for (int w = 0; w < nw; ++w)
          for (int l = 0; l < 64; ++l)
            for (int nt = 0; nt < ntw; ++nt) {
              const int row = 4 * kh + (l >> 4);
              const long long col = (long long)J * nb + 16 * (nw * nt + w) + (l & 15) - coff;
              if (row <= d && col >= 0 && col < n_cols)
                hf[(((size_t)J * kh_n + kh) * nw + w) * 64 * ntw + ntw * l + nt] = H[row * n_cols + col];
            }
  }
};

// ---------------------------------------------------------------------------------
// Observation-GP cutoff (opt-in, DESIGN.md §3 "Kernel-value cutoff"): kernel values below
// tau are flushed to exactly 0, so a K-step (16 training rows) whose values are all 0 for a
// particle tile contributes nothing, and its MFMAs are skipped.  Three host-side pieces:

// The training rows in a spatial order (recursive coordinate bisection of the scaled latents
// X / ls, leaves of kBK rows): K-steps of nearby points, so a compact particle tile is far
// from most K-steps.  Every leaf holds exactly kBK rows but the last.  Returns perm (image
// row -> training row).
inline void spatial_order_rec(const double* X, const double* ls, int d, long long* idx, long long n) {
  if (n <= kBK) return;
  int best = 0;
  double spread = -1.0;
  for (int j = 0; j < d; ++j) {
    double lo = 1e300, hi = -1e300;
    for (long long i = 0; i < n; ++i) {
      const double v = X[idx[i] * d + j] / ls[j];
      lo = v < lo ? v : lo;
      hi = v > hi ? v : hi;
    }
    if (hi - lo > spread) {
      spread = hi - lo;
      best = j;
    }
  }
  // stable sort of idx by the widest coordinate (ties by training row: deterministic)
  std::vector<std::pair<double, long long>> kv((size_t)n);
  for (long long i = 0; i < n; ++i) kv[(size_t)i] = {X[idx[i] * d + best] / ls[best], idx[i]};
  std::sort(kv.begin(), kv.end());
  for (long long i = 0; i < n; ++i) idx[i] = kv[(size_t)i].second;
  const long long leaves = (n + kBK - 1) / kBK;
  const long long left = ((leaves + 1) / 2) * kBK;   // a multiple of kBK: full leaves on the left
  spatial_order_rec(X, ls, d, idx, left);
  spatial_order_rec(X, ls, d, idx + left, n - left);
}
inline std::vector<long long> spatial_order(const double* X, const double* ls, long long n, int d) {
  std::vector<long long> idx((size_t)n);
  for (long long i = 0; i < n; ++i) idx[(size_t)i] = i;
  spatial_order_rec(X, ls, d, idx.data(), n);
  return idx;
}

// One bounding sphere per K-step of the image (rows in the order perm), in scaled
// coordinates: centre (d doubles) then radius, padded up to the radius of every row (a
// relative and absolute margin over the computed distances).
inline void kstep_spheres(const double* X, const double* ls, const long long* perm, long long n, int d,
                          std::vector<double>& out) {
  const long long nks = (n + kBK - 1) / kBK;
  out.assign((size_t)nks * (d + 1), 0.0);
  std::vector<double> c((size_t)d);
  for (long long k = 0; k < nks; ++k) {
    const long long r0 = k * kBK, r1 = (k + 1) * kBK < n ? (k + 1) * kBK : n;
    for (int j = 0; j < d; ++j) {
      double s = 0.0;
      for (long long r = r0; r < r1; ++r) s += X[perm[r] * d + j] / ls[j];
      c[(size_t)j] = s / (double)(r1 - r0);
    }
    double rad = 0.0;
    for (long long r = r0; r < r1; ++r) {
      double s = 0.0;
      for (int j = 0; j < d; ++j) {
        const double t = X[perm[r] * d + j] / ls[j] - c[(size_t)j];
        s += t * t;
      }
      rad = s > rad ? s : rad;
    }
    for (int j = 0; j < d; ++j) out[(size_t)k * (d + 1) + j] = c[(size_t)j];
    out[(size_t)k * (d + 1) + d] = std::sqrt(rad) * (1.0 + 1e-12) + 1e-12;
  }
}

// The cutoff image (obs_cutoff.h), tile-major: column tile t = 0 .. T_R - 1 holds the 16
// columns 16t .. 16t + 15 of the symmetric block form of K^-1 (upper block triangle, the
// off-diagonal 16 x 16 blocks doubled, rows and columns in the order perm; columns past N are
// zero), and needs K-steps 0 .. t (kend = t + 1); mean tile T_R + m holds columns 16m .. 16m + 15
// of M = K^-1 Y and needs every K-step (kend = T_R).  Column tiles and K-steps index the same
// 16-row groups, so the K-step sphere test also decides which R tiles a particle tile needs.
// Tile t's K-step ks is 2 KiB at toff[t] + 256 ks doubles: two halves of 1 KiB (sub-steps 0-1
// and 2-3), each one wave's 16-byte load with lane l at 16 l bytes:
//   Bt[toff[t] + 256 ks + 128 h + 2 l + e] = B[row = 16 ks + 4 (2h + e) + (l >> 4)][col of tile t, l & 15].
struct CutoffPacker {
  int n_rows, d, n_m, T_R, T_M;
  const double *X, *ls, *Kinv, *M;
  const long long* perm;   // image row -> training row

  CutoffPacker(int n_rows_, int d_, int n_m_, const double* X_, const double* ls_, const double* Kinv_,
               const double* M_, const long long* perm_)
      : n_rows(n_rows_), d(d_), n_m(n_m_), X(X_), ls(ls_), Kinv(Kinv_), M(M_), perm(perm_) {
    T_R = ksteps(n_rows);
    T_M = (n_m + 15) / 16;
  }
  int tiles() const { return T_R + T_M; }
  long long kend(int t) const { return t < T_R ? t + 1 : T_R; }
  std::vector<long long> offsets() const {
    std::vector<long long> o((size_t)tiles() + 1, 0);
    for (int t = 0; t < tiles(); ++t) o[(size_t)t + 1] = o[(size_t)t] + 256 * kend(t);
    return o;
  }
  // B[row][column l of tile t]
  double val(long long row, int t, int l) const {
    if (row >= n_rows) return 0.0;
    if (t < T_R) {
      const long long col = 16LL * t + l;
      if (col >= n_rows) return 0.0;
      const long long bi = row / kBK, bj = col / kBK;
      if (bi > bj) return 0.0;
      const double a = Kinv[perm[row] * n_rows + perm[col]];
      return bi < bj ? 2.0 * a : a;
    }
    const long long j = 16LL * (t - T_R) + l;
    return j < n_m ? M[perm[row] * n_m + j] : 0.0;
  }
  // tile t into dst[0, 256 kend(t))
  void pack_tile(int t, double* dst) const {
    for (long long ks = 0; ks < kend(t); ++ks)
      for (int l = 0; l < 64; ++l)
        for (int kk = 0; kk < 4; ++kk)
          dst[ks * 256 + (kk >> 1) * 128 + 2 * l + (kk & 1)] = val(ks * kBK + 4 * kk + (l >> 4), t, l & 15);
  }
  // row records in image-row order (as ImagePacker::records)
  void records(std::vector<double>& rec) const {
    const int cap = row_cap(n_rows), rw = d + 1;
    rec.assign((size_t)cap * rw, 0.0);
    for (int i = n_rows; i < cap; ++i) rec[(size_t)i * rw + d] = kPadSq;
    for (long long i = 0; i < n_rows; ++i) {
      double s = 0.0;
      for (int j = 0; j < d; ++j) {
        const double v = X[perm[i] * d + j] / ls[j];
        rec[(size_t)i * rw + j] = v;
        s += v * v;
      }
      rec[(size_t)i * rw + d] = s * kLog2eX64;
    }
  }
};

// The cutoff tau: every kernel value below it is flushed to 0.  Bounds:
//  * the quadratic form: flushing delta (0 <= delta_i <= tau) moves q = k^T K^-1 k by at most
//    (2 + e) e with e = sqrt(N) tau / sigma (|R^T k| = sqrt(q) <= 1, |R| <= 1 / sigma for
//    K_y = K + sigma^2 I), and 1 - q >= sigma^2 / (N + sigma^2) (lambda_max(K) <= N), so
//    tau_q = sigma h / (2.001 sqrt(N)), h = half an ulp of sigma^2 / (N + sigma^2), keeps the
//    change below half an ulp of the smallest possible 1 - q;
//  * each mean mu_j = sum_i k_i M_ij moves by at most tau |M_j|_1: tau_mu = min_j half an
//    ulp of max_i |Y_ij| / |M_j|_1 (below the resolution of the training observations).
// Returns min(tau_q, tau_mu).
inline double obs_cutoff_tau(long long N, double sigma2, const double* M, int D, const double* y_absmax) {
  const double vc_min = sigma2 / ((double)N + sigma2);
  const double h = 0.5 * (std::nextafter(vc_min, 1.0) - vc_min);
  double tau = std::sqrt(sigma2) * h / (2.001 * std::sqrt((double)N));
  for (int j = 0; j < D; ++j) {
    double m1 = 0.0;
    for (long long i = 0; i < N; ++i) m1 += std::fabs(M[i * D + j]);
    const double yj = y_absmax[j];
    if (m1 > 0.0 && yj > 0.0) {
      const double t = 0.5 * (std::nextafter(yj, 1e308) - yj) / m1;
      tau = t < tau ? t : tau;
    }
  }
  return tau;
}

}  // namespace gpmdm
