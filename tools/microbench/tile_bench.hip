// A/B timing of k_gp_tile variants on the config-2 observation GP shape (N=2000, D=62,
// d=3, P=100k): template VAR bits (see gp_tile_lab.h) and NW (waves per workgroup).
// Variants run interleaved in one process (cdna_hip_programming.md §5.4 rule 24).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/microbench/tile_bench.hip -o tools/microbench/tile_bench
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "gp_tile_lab.h"

using namespace gpmdm;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

#ifndef TB_D
#define TB_D 3
#endif
template <int VAR, int NW, int MT = 4, int NTW = 4>
void launch_var(const LabParams& p, hipStream_t s) {
  hipLaunchKernelGGL((k_gp_tile_lab<TB_D, false, VAR, NW, MT, NTW>), dim3(p.n_j_max * p.tiles_ub), dim3(64 * NW), 0, s, p);
}

// K* cache pair (gp_tile_lab.h VAR bits 28/29): the full-K block generates and stores K*, the
// other blocks load it.  Chunked: particle tiles in CH chunks; producer of chunk k on the
// main stream, consumer of chunk k on a second stream after an event, so the producers'
// grid tail overlaps the consumers' work.
static hipStream_t g_s2 = nullptr;
static hipEvent_t g_ev[17];
static std::vector<LabParams> g_chunk[9];    // per chunk count: one LabParams per chunk
template <int NW, int MT, int NTW, int CH>
void launch_kc(const LabParams& p, hipStream_t s) {
  LabParams a = p, c = p;
  a.j_skip = 0;
  c.j_skip = 1;
  if (CH == 1) {
    hipLaunchKernelGGL((k_gp_tile_lab<TB_D, false, 268435456, NW, MT, NTW>), dim3(p.tiles_ub), dim3(64 * NW), 0, s, a);
    hipLaunchKernelGGL((k_gp_tile_lab<TB_D, false, 536870912, NW, MT, NTW>), dim3((p.n_j_max - 1) * p.tiles_ub), dim3(64 * NW), 0, s, c);
    return;
  }
  for (int k = 0; k < CH; ++k) {
    LabParams pa = g_chunk[CH][k], pc = g_chunk[CH][k];
    pa.j_skip = 0;
    pc.j_skip = 1;
    hipLaunchKernelGGL((k_gp_tile_lab<TB_D, false, 268435456, NW, MT, NTW>), dim3(pa.tiles_ub), dim3(64 * NW), 0, s, pa);
    hipEventRecord(g_ev[k], s);
    hipStreamWaitEvent(g_s2, g_ev[k], 0);
    hipLaunchKernelGGL((k_gp_tile_lab<TB_D, false, 536870912, NW, MT, NTW>), dim3((pc.n_j_max - 1) * pc.tiles_ub), dim3(64 * NW), 0, g_s2, pc);
  }
  hipEventRecord(g_ev[16], g_s2);
  hipStreamWaitEvent(s, g_ev[16], 0);
}

template <int NW, int MT, int NTW, int XV = 0>
void launch_kc_allcons(const LabParams& p, hipStream_t s) {   // producer, then consumers on every block
  LabParams a = p, c = p;
  a.j_skip = 0;
  c.j_skip = 0;
  hipLaunchKernelGGL((k_gp_tile_lab<TB_D, false, 268435456 | XV, NW, MT, NTW>), dim3(p.tiles_ub), dim3(64 * NW), 0, s, a);
  hipLaunchKernelGGL((k_gp_tile_lab<TB_D, false, 536870912 | XV, NW, MT, NTW>), dim3(p.n_j_max * p.tiles_ub), dim3(64 * NW), 0, s, c);
}
template <int NW, int MT, int NTW>
void launch_kc_allprod(const LabParams& p, hipStream_t s) {   // every block a producer (same values stored)
  LabParams a = p;
  a.j_skip = 0;
  hipLaunchKernelGGL((k_gp_tile_lab<TB_D, false, 268435456, NW, MT, NTW>), dim3(p.n_j_max * p.tiles_ub), dim3(64 * NW), 0, s, a);
}
template <int NW, int MT, int NTW>
void launch_kc_prod(const LabParams& p, hipStream_t s) {
  LabParams a = p;
  a.j_skip = 0;
  hipLaunchKernelGGL((k_gp_tile_lab<TB_D, false, 268435456, NW, MT, NTW>), dim3(p.tiles_ub), dim3(64 * NW), 0, s, a);
}
template <int NW, int MT, int NTW>
void launch_kc_cons(const LabParams& p, hipStream_t s) {
  LabParams c = p;
  c.j_skip = 1;
  hipLaunchKernelGGL((k_gp_tile_lab<TB_D, false, 536870912, NW, MT, NTW>), dim3((p.n_j_max - 1) * p.tiles_ub), dim3(64 * NW), 0, s, c);
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
  const Geo geos[] = {{4, 4, 4}, {8, 4, 4}, {4, 2, 8}, {4, 1, 16}, {4, 1, 8}, {4, 2, 6}, {8, 2, 8}, {4, 1, 4}, {4, 2, 4}};
  const int NGEO = sizeof(geos) / sizeof(geos[0]);
  LabParams pp[NGEO];
  int* tabs;
  CK(hipMalloc(&tabs, NGEO * 8 * sizeof(int)));
  for (int v = 0; v < NGEO; ++v) {
    const int nw = geos[v].nw, pt = 16 * geos[v].mt, nb = 16 * geos[v].ntw * nw, fs = nw * 256 * geos[v].ntw;
    const int ntiles = (P + pt - 1) / pt;
    int ht[5] = {0, P, 0, 0, ntiles};
    CK(hipMemcpy(tabs + 8 * v, ht, sizeof(ht), hipMemcpyHostToDevice));
    const int coff = getenv("TB_NO_COFF") ? 0 : col_offset(N + D, nb);
    const int n_j = (N + D + coff + nb - 1) / nb;
    long long total = 0;
    for (int J = 0; J < n_j; ++J) total += (long long)ksteps(block_kmax(J, N, nb, coff)) * fs;
    std::vector<double> hB(total);
    for (auto& x : hB) x = 0.01 * nd(rng);
    double* B;
    CK(hipMalloc(&B, total * 8));
    CK(hipMemcpy(B, hB.data(), total * 8, hipMemcpyHostToDevice));
    LabParams& p = pp[v];
    p = LabParams{};
    p.seg[0].Xs = Xs; p.seg[0].Xsq = Xsq; p.seg[0].Xrec = Xrec; p.seg[0].Bf = B;
    p.rec128 = Xrec128;
    p.seg[0].n_rows = N; p.seg[0].n_m = D; p.seg[0].n_j = n_j; p.seg[0].coff = coff;
    p.n_seg = 1; p.tiles_ub = ntiles; p.n_j_max = n_j; p.geo = TileGeo{nw, geos[v].mt, geos[v].ntw};
    int* tab = tabs + 8 * v;
    p.seg_pos_begin = tab; p.seg_pos_end = tab + 1; p.seg_out_base = tab + 2; p.seg_tile_start = tab + 3;
    p.X = X;
    for (int j = 0; j < d; ++j) p.ls[j] = 1.0;
    p.qpart = q; p.ld_q = P; p.mu = mu; p.ld_mu = D;
    if (v == 2) {                       // K* cache for the production geometry
      CK(hipMalloc(&p.kcache, (size_t)ntiles * ksteps(N) * 256 * geos[v].mt * 8));
      for (int CH = 2; CH <= 8; CH *= 2) {
        int* ct;
        CK(hipMalloc(&ct, CH * 8 * sizeof(int)));
        for (int k = 0; k < CH; ++k) {
          const int t0 = (int)((long long)ntiles * k / CH), t1 = (int)((long long)ntiles * (k + 1) / CH);
          int h[5] = {t0 * pt, std::min(P, t1 * pt), t0 * pt, 0, t1 - t0};
          CK(hipMemcpy(ct + 8 * k, h, sizeof(h), hipMemcpyHostToDevice));
          LabParams c = p;
          c.tiles_ub = t1 - t0;
          c.seg_pos_begin = ct + 8 * k; c.seg_pos_end = ct + 8 * k + 1; c.seg_out_base = ct + 8 * k + 2;
          c.seg_tile_start = ct + 8 * k + 3;
          c.kcache = p.kcache + (size_t)t0 * ksteps(N) * 256 * geos[v].mt;
          g_chunk[CH].push_back(c);
        }
      }
    }
  }

  hipStream_t s = nullptr;
  CK(hipStreamCreateWithFlags(&g_s2, hipStreamNonBlocking));
  for (int i = 0; i < 17; ++i) CK(hipEventCreateWithFlags(&g_ev[i], hipEventDisableTiming));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  typedef void (*L)(const LabParams&, hipStream_t);
  struct V { L fn; int pi; const char* name; };
#if defined(TB_SHAPES)
  // tile shapes on a small-row problem (the de-duplicated dynamics GP: a few thousand rows
  // against N_c ~ 1000 training rows): run as  tile_bench_shapes 7200 995 3
  V vars[] = {{launch_var<0, 4, 1, 4>, 7, "16x256"}, {launch_var<0, 4, 1, 8>, 4, "16x512"},
              {launch_var<0, 4, 2, 4>, 8, "32x256"}, {launch_var<0, 4, 2, 8>, 2, "32x512"},
              {launch_var<0, 4, 4, 4>, 0, "64x256"}};
#elif TB_D > 12
  V vars[] = {{launch_var<0, 4>, 0, "64x256"}, {launch_var<0, 8>, 1, "64x512 (NW8)"},
              {launch_var<0, 4, 2, 8>, 2, "32x512 (VGPR coords)"}, {launch_var<131072, 4, 2, 8>, 2, "32x512 LDS coords"},
              {launch_var<131072, 8>, 1, "64x512 LDS coords"}};
#else
  V vars[] = {{launch_var<0, 4, 2, 8>, 2, "32x512 production"},
              {launch_var<0, 8, 2, 8>, 6, "32x1024 NW8, sync every 2"},
              {launch_var<65536, 8, 2, 8>, 6, "32x1024 NW8, sync every 4"},
              {launch_var<65536 | 16, 8, 2, 8>, 6, "32x1024 NW8 sync 4, no gen"},
              {launch_var<65536 | 4096, 8, 2, 8>, 6, "32x1024 NW8 sync 4, gen interleaved"},
              {launch_var<65536 | 8192, 8, 2, 8>, 6, "32x1024 NW8 sync 4, gen split"},
              {launch_var<65536 | 2, 8, 2, 8>, 6, "32x1024 NW8 sync 4, cheap exp"},
              {launch_var<0, 4, 2, 8>, 2, "production again"},
              {launch_kc_allprod<4, 2, 8>, 2, "K* cache: every block produces"},
              {launch_kc<4, 2, 8, 1>, 2, "K* cache: producer + consumer"},
              {launch_kc_allcons<4, 2, 8>, 2, "K* cache: consumers on all J"},
              {launch_kc_prod<4, 2, 8>, 2, "K* cache: producer alone"},
              {launch_kc_cons<4, 2, 8>, 2, "K* cache: consumer alone"},
              {launch_var<16, 4, 2, 8>, 2, "no gen"}};
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
    const size_t nq = (size_t)P * (pp[2].n_j_max);
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
      size_t ndiff = 0, imax = 0;
      for (size_t i = 0; i < nq; ++i) {
        const double dd = std::abs(q1[i] - q0[i]);
        if (q1[i] != q0[i]) ++ndiff;
        if (dd > md) { md = dd; imax = i; }
        mx = std::max(mx, std::abs(q0[i]));
      }
      if (getenv("TB_KDUMP") && std::string(vars[v].name).find("all J") != std::string::npos) {
        std::vector<size_t> byJ(pp[2].n_j_max, 0), byX(8, 0), tiles;
        size_t tiles_bad = 0;
        for (size_t i = 0; i < nq; ++i)
          if (q1[i] != q0[i]) { ++byJ[i / P]; ++byX[((i % P) / 32) % 8]; }
        for (int tt = 0; tt < P / 32; ++tt) {
          bool b = false;
          for (int J = 0; J < pp[2].n_j_max; ++J) for (int k = 0; k < 32; ++k) { size_t i = (size_t)J * P + tt * 32 + k; b |= q1[i] != q0[i]; }
          tiles_bad += b;
        }
        printf("  by J:"); for (auto x : byJ) printf(" %zu", x);
        printf("  by tile%%8:"); for (auto x : byX) printf(" %zu", x);
        printf("  tiles with a difference: %zu of %d\n", tiles_bad, P / 32);
        std::vector<double> q2(nq);
        CK(hipMemset(q, 0, nq * 8));
        vars[v].fn(pp[vars[v].pi], s);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(q2.data(), q, nq * 8, hipMemcpyDeviceToHost));
        size_t nd2 = 0;
        for (size_t i = 0; i < nq; ++i) nd2 += q2[i] != q1[i];
        printf("  rerun of the same variant: %zu entries differ from the first run\n", nd2);
      }
      printf("check %-30s max |q - q_production| = %.3g (max |q| %.3g), %zu of %zu differ; worst [J=%zu, p=%zu] %.17g vs %.17g\n",
             vars[v].name, md, mx, ndiff, nq, imax / P, imax % P, q1[imax], q0[imax]);
    }
  }
  // K* cache contents after the producer alone vs the host value 2^(t/64) (TB_KDUMP)
  if (getenv("TB_KDUMP")) {
    const int nks = ksteps(N), MT = 2, NT = P / 32;
    for (int rep = 0; rep < 2; ++rep) {
    if (rep == 0) launch_kc_prod<4, 2, 8>(pp[2], s);
    else launch_kc_allcons<4, 2, 8>(pp[2], s);

    CK(hipDeviceSynchronize());
    std::vector<double> kc((size_t)NT * nks * 256 * MT);
    CK(hipMemcpy(kc.data(), pp[2].kcache, kc.size() * 8, hipMemcpyDeviceToHost));
    size_t bad = 0, shown = 0;
    for (int t = 0; t < NT; ++t)
      for (int ks = 0; ks < nks; ++ks)
        for (int kk = 0; kk < 4; ++kk)
          for (int l = 0; l < 64; ++l)
            for (int mt = 0; mt < MT; ++mt) {
              const int pi = t * 32 + mt * 16 + (l & 15), r = ks * 16 + kk * 4 + (l >> 4);
              double asq = 0, dot = 0;
              for (int j = 0; j < d; ++j) { asq += hX[(size_t)pi * d + j] * hX[(size_t)pi * d + j]; dot += hX[(size_t)pi * d + j] * hXs[(size_t)r * d + j]; }
              const double tt = -(asq * kLog2eX64 + hXsq[r]) + 2.0 * kLog2eX64 * dot;
              const double ex = std::exp2(tt / 64.0);
              const double got = kc[(((size_t)t * nks + ks) * 4 + kk) * 128 + l * 2 + mt];
              if (!(std::abs(got - ex) <= 1e-12 * std::abs(ex) + 1e-300)) {
                ++bad;
                if (shown++ < 3) printf("kdump bad t=%d ks=%d kk=%d lane=%d mt=%d got %.17g want %.17g\n", t, ks, kk, l, mt, got, ex);
              }
            }
    printf("kdump (%s): %zu bad of %zu\n", rep == 0 ? "producer alone" : "producer + consumers", bad, (size_t)NT * nks * 512);
    }
  }
  double rows = 0;   // per 16-column tile: rows up to its diagonal (or all, for mean tiles)
  for (int tc = 0; tc * 16 < N + D; ++tc) {
    const int hi = tc * 16 + 16;
    rows += (double)ksteps(hi <= N ? hi : N) * kBK;
  }
  const double fl = 2.0 * 16 * rows * P;
  // fullK variants (VAR bit 7): every 16-column tile runs all K-steps
  const double fl_full = 2.0 * 16 * ((N + D + 15) / 16) * (double)ksteps(N) * kBK * P;
  for (int v = 0; v < NV; ++v) {
    std::sort(t[v].begin(), t[v].end());
    const bool full = std::string(vars[v].name).find("fullK") != std::string::npos;
    printf("%-30s median %.3f ms  min %.3f ms   (%.1f TF/s executed MFMA)\n", vars[v].name, t[v][ROUNDS / 2],
           t[v][0], (full ? fl_full : fl) / t[v][ROUNDS / 2] / 1e9);
  }
  return 0;
}
