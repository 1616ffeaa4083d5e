// Production tile variants built against a given gp_tile.h (code-generation A/B across
// source revisions: tools/microbench/tile_ab.sh).  Same driver as tile_bench.hip.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include GP_TILE_H   // -DGP_TILE_H='"<path>/gp_tile.h"': one header version per binary

using namespace gpmdm;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

#ifndef TB_D
#define TB_D 3
#endif
template <int VAR, int NW, int MT = 4, int NTW = 4>
void launch_var(const TileParams& p, hipStream_t s) {
  hipLaunchKernelGGL((k_gp_tile<TB_D, false, VAR, NW, MT, NTW>), dim3(p.n_j_max * p.tiles_ub), dim3(64 * NW), 0, s, p);
}

int main(int argc, char** argv) {
  // argv: P N D (defaults: the config-2 observation GP); d = TB_D at compile time
  const int P = argc > 1 ? atoi(argv[1]) : 100000;
  const int N = argc > 2 ? atoi(argv[2]) : 2000, D = argc > 3 ? atoi(argv[3]) : 62, d = TB_D;
  std::mt19937_64 rng(1);
  std::normal_distribution<double> nd(0.0, 1.0);
  const int cap = row_cap(N);   // padded like capi_model.hip build_image
  std::vector<double> hXs((size_t)cap * d, 0.0), hXsq(cap, kPadSq), hX((size_t)P * d);
  for (int i = 0; i < N; ++i) {
    double s = 0;
    for (int j = 0; j < d; ++j) { hXs[i * d + j] = 2.0 * nd(rng); s += hXs[i * d + j] * hXs[i * d + j]; }
    hXsq[i] = s;
  }
  for (auto& v : hX) v = 2.0 * nd(rng);
  std::vector<double> hRec((size_t)cap * (d + 1));
  for (int i = 0; i < cap; ++i) {
    for (int j = 0; j < d; ++j) hRec[(size_t)i * (d + 1) + j] = hXs[(size_t)i * d + j];
    hRec[(size_t)i * (d + 1) + d] = hXsq[i];
  }
  double *Xs, *Xsq, *Xrec, *Xrec128, *X, *q, *mu;
  CK(hipMalloc(&Xrec, hRec.size() * 8));
  CK(hipMemcpy(Xrec, hRec.data(), hRec.size() * 8, hipMemcpyHostToDevice));
  for (int i = 0; i < cap; ++i) hRec[(size_t)i * (d + 1) + d] *= 2.0;   // |Xs|^2 x 128/ln2 (VAR bit 22)
  CK(hipMalloc(&Xrec128, hRec.size() * 8));
  CK(hipMemcpy(Xrec128, hRec.data(), hRec.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&Xs, cap * d * 8)); CK(hipMalloc(&Xsq, cap * 8));
  CK(hipMalloc(&X, (size_t)P * d * 8)); CK(hipMalloc(&q, (size_t)P * (N + D + 4095) / 256 * 8)); CK(hipMalloc(&mu, (size_t)P * D * 8));
    CK(hipMemcpy(Xs, hXs.data(), cap * d * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(Xsq, hXsq.data(), cap * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(X, hX.data(), (size_t)P * d * 8, hipMemcpyHostToDevice));
  // geometries: {waves, particle tiles MT, column tiles per wave NTW}
  struct Geo { int nw, mt, ntw; };
  const Geo geos[] = {{4, 4, 4}, {8, 4, 4}, {4, 2, 8}, {4, 1, 16}, {4, 1, 8}, {4, 2, 6}};
  const int NGEO = sizeof(geos) / sizeof(geos[0]);
  TileParams pp[NGEO];
  int* tabs;
  CK(hipMalloc(&tabs, NGEO * 8 * sizeof(int)));
#if TB_D > 12
  const bool used[NGEO] = {false, true, true, false, false, false};
#else
  const bool used[NGEO] = {true, false, true, false, false, false};
#endif
  for (int v = 0; v < NGEO; ++v) {
    if (!used[v]) continue;
    const int nw = geos[v].nw, pt = 16 * geos[v].mt, nb = 16 * geos[v].ntw * nw, fs = nw * 256 * geos[v].ntw;
    const int ntiles = (P + pt - 1) / pt;
    int ht[5] = {0, P, 0, 0, ntiles};
    CK(hipMemcpy(tabs + 8 * v, ht, sizeof(ht), hipMemcpyHostToDevice));
    const int coff = getenv("TB_NO_COFF") ? 0 : col_offset(N + D, nb);
    const int n_j = (N + D + coff + nb - 1) / nb;
    long long total = 0;
    for (int J = 0; J < n_j; ++J) total += (long long)ksteps(block_kmax(J, N, nb, coff)) * fs;
    std::vector<double> hB(total);
    uint64_t st = 0x9e3779b97f4a7c15ull + v;   // cheap uniform values (timing only)
    for (auto& x : hB) { st = st * 6364136223846793005ull + 1442695040888963407ull; x = 0.01 * ((double)(st >> 11) * 0x1.0p-53 - 0.5); }
    double* B;
    CK(hipMalloc(&B, total * 8));
    CK(hipMemcpy(B, hB.data(), total * 8, hipMemcpyHostToDevice));
    TileParams& p = pp[v];
    p = TileParams{};
    p.seg[0].Xrec = Xrec; p.seg[0].Bf = B;
    p.seg[0].n_rows = N; p.seg[0].n_m = D; p.seg[0].n_j = n_j; p.seg[0].coff = coff;
    p.n_seg = 1; p.tiles_ub = ntiles; p.n_j_max = n_j; p.geo = TileGeo{nw, geos[v].mt, geos[v].ntw};
    int* tab = tabs + 8 * v;
    p.seg_pos_begin = tab; p.seg_pos_end = tab + 1; p.seg_out_base = tab + 2; p.seg_tile_start = tab + 3;
    p.X = X;
    for (int j = 0; j < d; ++j) p.ls[j] = 1.0;
    p.qpart = q; p.ld_q = P; p.mu = mu; p.ld_mu = D;
  }

  hipStream_t s = nullptr;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  typedef void (*L)(const TileParams&, hipStream_t);
  struct V { L fn; int pi; const char* name; };
#if TB_D > 12
  V vars[] = {{launch_var<0, 8>, 1, "64x512 (NW8)"}, {launch_var<131072, 4, 2, 8>, 2, "32x512 LDS coords"}};
#else
  V vars[] = {{launch_var<0, 4, 2, 8>, 2, "32x512 production"}, {launch_var<0, 4>, 0, "64x256"}};
#endif
  const int NV = sizeof(vars) / sizeof(vars[0]), ROUNDS = 7;
  std::vector<std::vector<float>> t(NV);
  for (int v = 0; v < NV; ++v) vars[v].fn(pp[vars[v].pi], s);
  CK(hipDeviceSynchronize());
  for (int r = 0; r < ROUNDS; ++r)
    for (int v = 0; v < NV; ++v) {
      CK(hipEventRecord(e0, s));
      for (int k = 0; k < 3; ++k) vars[v].fn(pp[vars[v].pi], s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms / 3);
    }
  // results check: every variant on the production geometry must write the same q partials
  {
    const size_t nq = (size_t)P * (pp[vars[0].pi].n_j_max);
    std::vector<double> q0(nq), q1(nq);
    CK(hipMemset(q, 0, nq * 8));
    vars[0].fn(pp[vars[0].pi], s);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(q0.data(), q, nq * 8, hipMemcpyDeviceToHost));
    for (int v = 1; v < NV; ++v) {
      if (vars[v].pi != vars[0].pi) continue;
      CK(hipMemset(q, 0, nq * 8));
      vars[v].fn(pp[vars[v].pi], s);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(q1.data(), q, nq * 8, hipMemcpyDeviceToHost));
      double md = 0, mx = 0;
      for (size_t i = 0; i < nq; ++i) { md = std::max(md, std::abs(q1[i] - q0[i])); mx = std::max(mx, std::abs(q0[i])); }
      printf("check %-30s max |q - q_production| = %.3g (max |q| %.3g)\n", vars[v].name, md, mx);
    }
  }
  // cross-revision bitwise check (tile_ab.sh): a hash of the production variant's q partials and means
  if (getenv("TB_QHASH") && *getenv("TB_QHASH")) {
    const size_t nq = (size_t)P * (pp[vars[0].pi].n_j_max), nm = (size_t)P * D;
    std::vector<double> q0(nq), m0(nm);
    CK(hipMemset(q, 0, nq * 8));
    CK(hipMemset(mu, 0, nm * 8));
    vars[0].fn(pp[vars[0].pi], s);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(q0.data(), q, nq * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(m0.data(), mu, nm * 8, hipMemcpyDeviceToHost));
    unsigned long long h = 1469598103934665603ull;   // FNV-1a over the bytes
    for (auto* v : {&q0, &m0})
      for (const unsigned char* c = (const unsigned char*)v->data(), *e = c + v->size() * 8; c < e; ++c)
        h = (h ^ *c) * 1099511628211ull;
    printf("qhash %016llx\n", h);
  }
  double rows = 0;   // per 16-column tile: rows up to its diagonal (or all, for mean tiles)
  for (int tc = 0; tc * 16 < N + D; ++tc) {
    const int hi = tc * 16 + 16;
    rows += (double)ksteps(hi <= N ? hi : N) * kBK;
  }
  const double fl = 2.0 * 16 * rows * P;
  for (int v = 0; v < NV; ++v) {
    std::sort(t[v].begin(), t[v].end());
    printf("%-30s median %.3f ms  min %.3f ms   (%.1f TF/s executed MFMA)\n", vars[v].name, t[v][ROUNDS / 2],
           t[v][0], fl / t[v][ROUNDS / 2] / 1e9);
  }
  return 0;
}
