// Host sanitizer driver for the C ABI's host-side code (gpmdm_amd/csrc/host_image.h):
// descriptor validation and the MFMA-fragment image packing that gpmdm_model_create runs
// before any upload.  Built and run by tests/test_host_asan.py with
// -fsanitize=address,undefined; no HIP, no GPU.
//
// Packing check, independent of the layout formula: R and M are filled with distinct
// values, so a correct image is a permutation of exactly the non-zero entries of
// B = [triu(R) | M] plus zeros -- every distinct value must occur exactly once.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "host_image.h"

using namespace gpmdm;

static int failures = 0;
#define EXPECT(cond, ...)                  \
  do {                                     \
    if (!(cond)) {                         \
      std::printf("FAIL %s:%d ", __FILE__, __LINE__); \
      std::printf(__VA_ARGS__);            \
      std::printf("\n");                   \
      ++failures;                          \
    }                                      \
  } while (0)

static void check_packing(int n_rows, int n_m, int d, TileGeo geo, bool lin) {
  std::mt19937_64 rng(n_rows * 131 + n_m * 7 + d);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  std::vector<double> X((size_t)n_rows * d), ls(d), c2(d + 1), R((size_t)n_rows * n_rows), M((size_t)n_rows * n_m);
  for (auto& v : X) v = U(rng);
  for (auto& v : ls) v = 0.5 + std::fabs(U(rng));
  for (auto& v : c2) v = 0.1 + std::fabs(U(rng));
  // distinct non-zero values: value = 1 + linear index in [R | M]
  const long long ncols = (long long)n_rows + n_m;
  for (long long i = 0; i < n_rows; ++i) {
    for (long long j = 0; j < n_rows; ++j) R[i * n_rows + j] = 1.0 + (double)(i * ncols + j);
    for (long long j = 0; j < n_m; ++j) M[i * n_m + j] = 1.0 + (double)(i * ncols + n_rows + j);
  }
  const ImagePacker pk(n_rows, d, n_m, X.data(), ls.data(), lin ? c2.data() : nullptr, R.data(), M.data(), geo);
  EXPECT(pk.coff % 16 == 0 && pk.coff < geo.nb(), "coff %d", pk.coff);
  EXPECT((long long)pk.n_j * geo.nb() >= ncols + pk.coff, "n_j %d", pk.n_j);
  std::vector<double> img((size_t)pk.total_doubles());
  long long off = 0;
  for (int J = 0; J < pk.n_j; ++J) {
    pk.pack_block(J, img.data() + off);
    off += pk.block_doubles(J);
  }
  EXPECT(off == (long long)img.size(), "total %lld vs %zu", off, img.size());
  std::map<double, int> seen;
  for (double v : img)
    if (v != 0.0) ++seen[v];
  long long expected = 0;
  for (long long i = 0; i < n_rows; ++i)
    for (long long j = 0; j < ncols; ++j) {
      if (j < n_rows && i > j) continue;   // strictly lower R: never stored
      ++expected;
      const double v = 1.0 + (double)(i * ncols + j);
      auto it = seen.find(v);
      EXPECT(it != seen.end() && it->second == 1, "B[%lld][%lld] stored %d times", i, j,
             it == seen.end() ? 0 : it->second);
    }
  EXPECT((long long)seen.size() == expected, "%zu distinct values stored, %lld expected", seen.size(), expected);
  std::vector<double> rec;
  pk.records(rec);
  EXPECT(rec.size() == (size_t)row_cap(n_rows) * (d + 1), "record size");
  for (int i = n_rows; i < row_cap(n_rows); ++i) EXPECT(rec[(size_t)i * (d + 1) + d] == kPadSq, "pad row %d", i);
  for (int i = 0; i < n_rows; ++i) {
    double s2 = 0.0;
    for (int j = 0; j < d; ++j) s2 += (X[(size_t)i * d + j] / ls[j]) * (X[(size_t)i * d + j] / ls[j]);
    EXPECT(std::fabs(rec[(size_t)i * (d + 1) + d] - s2 * kLog2eX64) <= 1e-12 * (1.0 + s2 * kLog2eX64), "row %d", i);
  }
  if (lin) {
    std::vector<double> hf;
    pk.linear(hf);
    // H = (X~ C^2)^T triu-B: compare the sum of all entries (each H entry is stored once)
    double ref = 0.0;
    for (long long i = 0; i < n_rows; ++i)
      for (long long j = 0; j < ncols; ++j) {
        const double b = pk.val(i, j);
        double w = c2[d];
        for (int k = 0; k < d; ++k) w += c2[k] * X[i * d + k];
        ref += w * b;
      }
    double got = 0.0;
    for (double v : hf) got += v;
    EXPECT(std::fabs(got - ref) <= 1e-9 * std::fabs(ref), "H sum %.17g vs %.17g", got, ref);
  }
}

static void check_desc() {
  std::vector<double> a(64, 1.0);
  const double* pa = a.data();
  const double* ptrs[2] = {pa, pa};
  int64_t nc[2] = {3, 4};
  gpmdm_model_desc d{};
  EXPECT(check_model_desc(nullptr) == "null argument", "null desc");
  d.N = 8; d.D = 5; d.d = 3; d.C = 2; d.tile_shape = 0;
  EXPECT(check_model_desc(&d) == "null array in model descriptor", "null arrays");
  d.X = d.obs_R = d.obs_beta = d.y_lengthscales = d.y_inv_lambda2 = pa;
  d.x_lengthscales = d.x_lin_coeff2 = d.x_inv_lambda2 = pa;
  d.Nc = nc; d.Xin = ptrs; d.dyn_R = ptrs; d.dyn_alpha = ptrs;
  EXPECT(check_model_desc(&d).empty(), "valid: %s", check_model_desc(&d).c_str());
  d.d = 17;
  EXPECT(check_model_desc(&d).find("latent dimension") == 0, "d=17");
  d.d = 3; d.C = 33;
  EXPECT(check_model_desc(&d) == "at most 32 classes", "C=33");
  d.C = 2; d.N = 0;
  EXPECT(check_model_desc(&d).find("positive") != std::string::npos, "N=0");
  d.N = 8; d.tile_shape = 9;
  EXPECT(check_model_desc(&d).find("tile_shape") == 0, "tile shape");
  d.tile_shape = 0; nc[1] = 0;
  EXPECT(check_model_desc(&d) == "class 1 has no dynamics rows", "Nc=0");
}

// The cutoff image (gpmdm_model_set_obs_cutoff): spatial_order is a permutation whose
// K-steps are full leaves but the last; every row lies inside its K-step's sphere; the
// symmetric block image stores exactly 2 K^-1 off the diagonal blocks and K^-1 on them, in
// the permuted order, and nothing below the block diagonal; tau obeys its two bounds.
static void check_cutoff(int n, int D, int d) {
  std::mt19937_64 rng(n * 17 + d);
  std::normal_distribution<double> G(0.0, 3.0);
  std::vector<double> X((size_t)n * d), ls(d), S((size_t)n * n), M((size_t)n * D), ymax(D);
  for (auto& v : X) v = G(rng);
  for (int j = 0; j < d; ++j) ls[j] = 0.7 + 0.1 * j;
  for (long long i = 0; i < n; ++i)
    for (long long j = 0; j < n; ++j) S[i * n + j] = 1.0 + (double)(std::min(i, j) * n + std::max(i, j));   // symmetric
  for (auto& v : M) v = G(rng);
  for (auto& v : ymax) v = 1.0 + std::fabs(G(rng));
  const std::vector<long long> perm = spatial_order(X.data(), ls.data(), n, d);
  std::vector<int> hit(n, 0);
  for (long long r : perm) {
    EXPECT(r >= 0 && r < n, "perm value %lld", r);
    if (r >= 0 && r < n) ++hit[r];
  }
  for (int i = 0; i < n; ++i) EXPECT(hit[i] == 1, "row %d appears %d times", i, hit[i]);
  std::vector<double> sph;
  kstep_spheres(X.data(), ls.data(), perm.data(), n, d, sph);
  const long long nks = (n + kBK - 1) / kBK;
  EXPECT((long long)sph.size() == nks * (d + 1), "spheres %zu", sph.size());
  for (long long r = 0; r < n; ++r) {
    const long long k = r / kBK;
    double s = 0.0;
    for (int j = 0; j < d; ++j) {
      const double t = X[perm[r] * d + j] / ls[j] - sph[k * (d + 1) + j];
      s += t * t;
    }
    EXPECT(std::sqrt(s) <= sph[k * (d + 1) + d], "row %lld outside its sphere", r);
  }
  // the tile-major cutoff image: every tile's K-steps in place, every value where the
  // kernel (obs_cutoff.h) reads it
  CutoffPacker pk(n, d, D, X.data(), ls.data(), S.data(), M.data(), perm.data());
  EXPECT(pk.T_R == (int)nks && pk.T_M == (D + 15) / 16, "tiles %d %d", pk.T_R, pk.T_M);
  const std::vector<long long> off = pk.offsets();
  std::vector<double> img((size_t)off.back(), -7.0);
  for (int t = 0; t < pk.tiles(); ++t) {
    EXPECT(off[(size_t)t + 1] - off[(size_t)t] == 256 * pk.kend(t), "tile %d size", t);
    pk.pack_tile(t, img.data() + off[(size_t)t]);
  }
  for (double v : img) EXPECT(v != -7.0, "an image slot left unwritten%s", "");
  for (int t = 0; t < pk.tiles(); ++t)
    for (long long ks = 0; ks < pk.kend(t); ++ks)
      for (int l = 0; l < 64; ++l)
        for (int kk = 0; kk < 4; ++kk) {
          const long long i = ks * kBK + 4 * kk + (l >> 4);
          double want = 0.0;
          if (i < n) {
            if (t < pk.T_R) {
              const long long j = 16LL * t + (l & 15);
              if (j < n && i / kBK <= j / kBK) want = (i / kBK < j / kBK ? 2.0 : 1.0) * S[perm[i] * n + perm[j]];
            } else {
              const long long j = 16LL * (t - pk.T_R) + (l & 15);
              if (j < D) want = M[perm[i] * D + j];
            }
          }
          const double v = img[(size_t)(off[(size_t)t] + ks * 256 + (kk >> 1) * 128 + 2 * l + (kk & 1))];
          EXPECT(v == want, "tile %d ks %lld lane %d kk %d: %.17g vs %.17g", t, ks, l, kk, v, want);
        }
  // every value of the block upper triangle (and of M) is stored exactly once
  long long nz = 0;
  for (double v : img) nz += v != 0.0;
  long long want_nz = 0;
  for (long long i = 0; i < n; ++i) {
    for (long long j = 0; j < n; ++j) want_nz += (i / kBK <= j / kBK) && S[perm[i] * n + perm[j]] != 0.0;
    for (int j = 0; j < D; ++j) want_nz += M[perm[i] * D + j] != 0.0;
  }
  EXPECT(nz == want_nz, "non-zeros %lld vs %lld", nz, want_nz);
  std::vector<double> rec;
  pk.records(rec);
  EXPECT((long long)rec.size() == (long long)row_cap(n) * (d + 1), "records %zu", rec.size());
  const double sigma2 = 0.01;
  const double tau = obs_cutoff_tau(n, sigma2, M.data(), D, ymax.data());
  const double vc_min = sigma2 / (n + sigma2);
  const double e = std::sqrt((double)n) * tau / std::sqrt(sigma2);
  EXPECT(tau > 0.0 && (2.0 + e) * e <= 0.5 * (std::nextafter(vc_min, 1.0) - vc_min), "tau_q bound %.3g", tau);
  for (int j = 0; j < D; ++j) {
    double m1 = 0.0;
    for (int i = 0; i < n; ++i) m1 += std::fabs(M[(size_t)i * D + j]);
    EXPECT(tau * m1 <= 0.5 * (std::nextafter(ymax[j], 1e308) - ymax[j]), "tau_mu bound column %d", j);
  }
}

int main() {
  check_desc();
  const int cut[][3] = {{1, 2, 1}, {16, 3, 2}, {37, 5, 3}, {300, 7, 8}, {517, 4, 16}};
  for (const auto& c : cut) check_cutoff(c[0], c[1], c[2]);
  const TileGeo geos[] = {kGeo64x256, kGeo64x512, kGeo32x512, kGeo32x256, kGeo16x256};
  const int shapes[][3] = {{1, 1, 1}, {7, 3, 2}, {16, 62, 3}, {17, 5, 3}, {250, 62, 3}, {513, 8, 16}, {300, 3, 8}};
  for (const auto& g : geos)
    for (const auto& s : shapes)
      for (int lin = 0; lin < 2; ++lin) check_packing(s[0], s[1], s[2], g, lin != 0);
  if (failures) {
    std::printf("%d failures\n", failures);
    return 1;
  }
  std::printf("ok\n");
  return 0;
}
