// Fused GP predictive tile for gfx950: kernel row generation + FP64 MFMA contraction.
//
// Replaces, for a tile of 128 particles x 128 columns:
//   observation GP  (gpmdm.py:955-959)  Ky* = exp(-|x*-X|^2/l^2),
//                   mean = Ky*^T beta, var-quadratic form = Ky*^T Ky^-1 Ky*
//   dynamics GP     (gpmdm.py:1061-1065) Kx* = RBF + linear kernel over the class-c rows,
//                   mean = Kx*^T alpha_c, quadratic form = Kx*^T A_c Kx*
// With K^-1 = R R^T (R = U^-1 from the reference's own Cholesky recipe, gpmdm.py:1286-1289)
// the quadratic form is |R^T k|^2; R is upper triangular, so column block J only needs
// training rows [0, (J+1)*NT): half the dense FLOPs.  B = [R | M] carries the mean
// weights M (beta or alpha_c) as extra columns, so one pass produces both.
//
// Per workgroup (256 threads, 4 waves as 2 (M) x 2 (N), each wave 64 x 64 = 4x4 MFMA
// 16x16 tiles of v_mfma_f64_16x16x4_f64):
//   K-step of 16 training rows: each thread generates 8 kernel values (exp in fp64) and
//   loads 4 x 16 B of B; they go to the other LDS buffer while the MFMAs of the current
//   step run (double-buffered, one barrier per step).
//   Epilogue: R columns -> per-row sum of squares (16-lane xor reduction) written as a
//   partial per (column block, wave column); mean columns -> written to mu.
// Workgroups are ordered heavy-first (largest column block first) so the triangular
// imbalance is absorbed by the dispatcher, and consecutive workgroups share a B panel
// (same J) so each XCD's L2 holds the panel its CUs stream.
#include "common.h"

namespace gpmdm {

template <int DI, bool DYN>
__global__ __launch_bounds__(256, (DI <= 12 ? 2 : 1)) void k_gp_tile(const TileParams prm) {
  __shared__ double As[2][kBK][kLDA];
  __shared__ double Bs[2][kBK][kLDB];

  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  const int J = prm.n_j_max - 1 - b / prm.tiles_ub;
  // tile index within this launch's segments (a launch may cover classes c0..c0+7)
  const int t = b - (b / prm.tiles_ub) * prm.tiles_ub + prm.seg_tile_start[0];

  int c = -1;
  for (int s = 0; s < prm.n_seg; ++s)
    if (t >= prm.seg_tile_start[s] && t < prm.seg_tile_start[s + 1]) c = s;
  c = __builtin_amdgcn_readfirstlane(c);
  if (c < 0) return;
  const SegDesc sg = prm.seg[c];
  if (J >= sg.n_j) return;

  const int seg_begin = prm.seg_pos_begin[c];
  const int pos0 = seg_begin + (t - prm.seg_tile_start[c]) * kPT;
  const int pos_end = prm.seg_pos_end[c];
  const int out_base = prm.seg_out_base[c] - seg_begin;   // out = out_base + pos

  // ---- particle coordinates of this thread's tile row ------------------------------
  const int m = tid & (kPT - 1);
  const int kh = __builtin_amdgcn_readfirstlane(tid >> 7);   // 0/1: even/odd K rows
  int pos = pos0 + m;
  if (pos >= pos_end) pos = pos0;                             // clamp (results unused)
  const int prow = prm.perm ? prm.perm[pos] : pos;
  double a[DI];
  double u[DYN ? DI : 1];
  double ubias = 0.0;
#pragma unroll
  for (int j = 0; j < DI; ++j) {
    const double x = prm.X[(long long)prow * DI + j];
    a[j] = x / prm.ls[j];
    if constexpr (DYN) u[j] = prm.lin_c2[j] * x;
  }
  if constexpr (DYN) ubias = prm.lin_c2[DI];

  const int n_rows = sg.n_rows;
  const double* __restrict__ Xs = sg.Xs;
  const double* __restrict__ Xl = sg.Xl;
  const double* __restrict__ Bg = sg.B + (long long)J * kNT;
  const long long ldb = sg.ld;

  auto gen = [&](int ks, double (&v)[8]) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int i = ks * kBK + kh + 2 * s;                    // wave-uniform row
      double val = 0.0;
      if (i < n_rows) {
        const double* xr = Xs + (long long)i * DI;
        double dist = 0.0;
#pragma unroll
        for (int j = 0; j < DI; ++j) {
          const double dd = a[j] - xr[j];
          dist = fma(dd, dd, dist);
        }
        val = exp(-dist);
        if constexpr (DYN) {
          const double* xl = Xl + (long long)i * DI;
          double l = ubias;
#pragma unroll
          for (int j = 0; j < DI; ++j) l = fma(u[j], xl[j], l);
          val += l;
        }
      }
      v[s] = val;
    }
  };
  const int brow = tid >> 6;          // 0..3
  const int bcol = (tid & 63) * 2;    // 2 doubles (16 B) per lane: one row per wave-instruction
  auto loadB = [&](int ks, double2 (&r)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long long row = (long long)ks * kBK + brow + 4 * q;
      r[q] = *reinterpret_cast<const double2*>(Bg + row * ldb + bcol);
    }
  };
  auto store = [&](int buf, const double (&v)[8], const double2 (&r)[4]) {
#pragma unroll
    for (int s = 0; s < 8; ++s) As[buf][kh + 2 * s][m] = v[s];
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<double2*>(&Bs[buf][brow + 4 * q][bcol]) = r[q];
  };

  // K range: column j of R needs rows i <= j; mean columns need every row.
  const int kmax = min(n_rows, (J + 1) * kNT);
  const int nks = (kmax + kBK - 1) / kBK;

  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;
  const int li = lane & 15, lk = lane >> 4;

  d4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};

  {
    double v[8];
    double2 r[4];
    gen(0, v);
    loadB(0, r);
    store(0, v, r);
  }
  __syncthreads();

  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    const bool more = ks + 1 < nks;
    double v[8];
    double2 r[4];
    if (more) {
      loadB(ks + 1, r);
      gen(ks + 1, v);
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      double af[4], bf[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) af[mt] = As[buf][kk * 4 + lk][wm * 64 + mt * 16 + li];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) bf[nt] = Bs[buf][kk * 4 + lk][wn * 64 + nt * 16 + li];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[mt], bf[nt], acc[mt][nt], 0, 0, 0);
    }
    if (more) store(buf ^ 1, v, r);
    __syncthreads();
  }

  // ---- epilogue --------------------------------------------------------------------
  // C/D layout of v_mfma_f64_16x16x4_f64: lane l, reg r -> row (l>>4) + 4r, col l&15.
  const int colw = J * kNT + wn * 64;
  const bool all_r = (J + 1) * kNT <= n_rows;
  if (J * kNT < n_rows) {
    double qs[4][4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double s = 0.0;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const double x = acc[mt][nt][r];
          const int col = colw + nt * 16 + li;
          if (all_r || col < n_rows) s = fma(x, x, s);
        }
        qs[mt][r] = s;
      }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double s = qs[mt][r];
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        s += __shfl_xor(s, 4);
        s += __shfl_xor(s, 8);
        qs[mt][r] = s;
      }
    if (li == 0) {
      double* qp = prm.qpart + (long long)(2 * J + wn) * prm.ld_q;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = pos0 + wm * 64 + mt * 16 + lk + 4 * r;
          if (p < pos_end) qp[out_base + p] = qs[mt][r];
        }
    }
  }
  if (!all_r) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int jm = colw + nt * 16 + li - n_rows;
      if (jm >= 0 && jm < sg.n_m) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int p = pos0 + wm * 64 + mt * 16 + lk + 4 * r;
            if (p < pos_end) prm.mu[(long long)(out_base + p) * prm.ld_mu + jm] = acc[mt][nt][r];
          }
      }
    }
  }
}

template <int DI>
static void launch_d(const TileParams& p, bool dyn, hipStream_t stream) {
  const dim3 grid((unsigned)(p.n_j_max * p.tiles_ub));
  if (dyn)
    hipLaunchKernelGGL((k_gp_tile<DI, true>), grid, dim3(256), 0, stream, p);
  else
    hipLaunchKernelGGL((k_gp_tile<DI, false>), grid, dim3(256), 0, stream, p);
}

void launch_gp_tile(const TileParams& p, int d, bool dyn, hipStream_t stream) {
  if (p.n_j_max <= 0 || p.tiles_ub <= 0) return;
  switch (d) {
#define GPMDM_D(n) case n: launch_d<n>(p, dyn, stream); break;
    GPMDM_D(1) GPMDM_D(2) GPMDM_D(3) GPMDM_D(4) GPMDM_D(5) GPMDM_D(6) GPMDM_D(7) GPMDM_D(8)
    GPMDM_D(9) GPMDM_D(10) GPMDM_D(11) GPMDM_D(12) GPMDM_D(13) GPMDM_D(14) GPMDM_D(15) GPMDM_D(16)
    GPMDM_D(24) GPMDM_D(32)
#undef GPMDM_D
    default: break;  // rejected by the host (d must be 1..16, 24 or 32)
  }
}

}  // namespace gpmdm
