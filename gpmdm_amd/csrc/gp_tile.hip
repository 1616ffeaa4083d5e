// Fused GP predictive tile for gfx950: kernel-row generation + FP64 MFMA contraction.
//
// Replaces, for a tile of 64 particles x 256 columns:
//   observation GP  (gpmdm.py:955-959)  Ky* = exp(-|x*-X|^2/l^2),
//                   mean = Ky*^T beta, var-quadratic form = Ky*^T Ky^-1 Ky*
//   dynamics GP     (gpmdm.py:1061-1065) Kx* = RBF + linear kernel over the class-c rows,
//                   mean = Kx*^T alpha_c, quadratic form = Kx*^T A_c Kx*
// The linear kernel (gpmdm.py:493-506) is rank d+1: k_lin(p, i) = x~_p^T C^2 x~_i with
// x~ = [x, 1], so its contribution to V = K* B is x~_p^T H with H = (X~ C^2)^T B, a
// (d+1)-row matrix precomputed on the host.  It is added to the accumulators after the K
// loop by ceil((d+1)/4) extra MFMA sub-steps, and the K loop generates only the RBF part
// (the same code as the observation GP).
// With K^-1 = R R^T (R = U^-1 from the reference's own Cholesky recipe, gpmdm.py:1286-1289)
// the quadratic form is |R^T k|^2.  R is upper triangular, so column block J only needs
// training rows [0, (J+1)*256), and each wave stops at its own 64 columns: about half the
// dense FLOPs.  B = [R | M] carries the mean weights M (beta or alpha_c) as extra columns,
// so one pass produces both.
//
// Workgroup = 4 waves; wave w owns the four 16-column tiles at columns
// 256J + 16(4t + w), t = 0..3 (interleaved, so all waves reach nearly the same K), for all
// 64 particles (4 x 4 tiles of v_mfma_f64_16x16x4_f64, 128 accumulator VGPRs).  A tile of R
// columns retires once K passes its diagonal: the K loop runs in phases with tiles
// [T0, T1) active, so no MFMA multiplies the zero triangle and no wave idles while its
// siblings (and the barrier) wait.  Per K-step of 16 training rows:
//   * K* tile (64 x 16) generated once per workgroup: each thread makes 4 values
//     (expansion-form distance as gpmdm.py:508-515, table-driven fp64 exp), stored to a
//     double-buffered LDS image that all 4 waves read as A fragments;
//   * B fragments stream from HBM/L2 straight into VGPRs (8 x 16 B per lane, one K-step
//     ahead): B is stored in fragment order, so no LDS round trip and no re-layout;
//   * one barrier per K-step.  Two workgroups per CU overlap each other's barriers.
// Workgroups are ordered heavy-first (column block J descending), which both balances the
// triangular work and makes concurrent workgroups share a B panel in each XCD's L2.
#include <type_traits>

#include "common.h"

namespace gpmdm {

// 2^(j/64), j = 0..63 (correctly rounded).
__constant__ double kExp2Tab[64] = {
    1.0, 1.0108892860517005, 1.0218971486541166, 1.0330248790212284,
    1.0442737824274138, 1.0556451783605572, 1.0671404006768237, 1.0787607977571199,
    1.0905077326652577, 1.102382583307841, 1.1143867425958924, 1.1265216186082418,
    1.1387886347566916, 1.1511892299529827, 1.1637248587775775, 1.1763969916502812,
    1.189207115002721, 1.202156731452703, 1.215247359980469, 1.22848053610687,
    1.241857812073484, 1.255380757024691, 1.2690509571917332, 1.2828700160787783,
    1.2968395546510096, 1.3109612115247644, 1.3252366431597413, 1.339667524053303,
    1.3542555469368927, 1.3690024229745905, 1.383909881963832, 1.3989796725383112,
    1.4142135623730951, 1.42961333839197, 1.4451808069770467, 1.460917794180647,
    1.4768261459394993, 1.4929077282912648, 1.5091644275934228, 1.5255981507445384,
    1.5422108254079407, 1.559004400237837, 1.5759808451078865, 1.593142151342267,
    1.6104903319492543, 1.6280274218573478, 1.645755478153965, 1.6636765803267364,
    1.681792830507429, 1.7001063537185235, 1.718619298122478, 1.7373338352737062,
    1.7562521603732995, 1.7753764925265212, 1.7947090750031072, 1.8142521755003989,
    1.8340080864093424, 1.8539791250833855, 1.8741676341103, 1.8945759815869656,
    1.9152065613971474, 1.9360617934922943, 1.9571441241754002, 1.978456026387951
};

// The kernel value is exp(x), x = -(|a|^2 + |b|^2) + 2 a.b (expansion form of
// gpmdm.py:508-515).  Every term arrives pre-multiplied by 64/ln2 (particle side in the
// kernel prologue, |b|^2 on the host), so the fma chain yields t = 64 x / ln2 directly and
// exp(x) = 2^(t/64): n = rint(t), f = t - n (exact, Sterbenz), 2^(f/64) - 1 by a degree-5
// polynomial in f (|f| <= 1/2, truncation < 2^-55), table 2^(j/64), ldexp.  No clamp is
// needed: v_cvt_i32_f64 saturates and ldexp underflows to 0 exactly like exp().
constexpr double kLog2eX64 = 92.33248261689366;   // 64 / ln 2 (host and device)

__device__ __forceinline__ double exp2_64(double t, const double* tab) {
  const double n = __builtin_rint(t);
  const double f = t - n;
  double p = fma(f, 1.2417843701716925e-12, 5.732851688640402e-10);
  p = fma(p, f, 2.1173137155464776e-07);
  p = fma(p, f, 5.86490495505617e-05);
  p = fma(p, f, 0.010830424696249145);
  p *= f;                                                          // 2^(f/64) - 1
  const int ni = (int)n;
  const double tj = tab[ni & 63];
  return ldexp(fma(tj, p, tj), ni >> 6);
}

// VAR: experiment switches for tools/microbench/tile_bench.hip (production uses 0).
//   bit 0: no tile retirement (every real tile runs to the block's last K-step)
//   bit 1: ablation -- replace the kernel-value generation by a cheap stand-in
//   bit 2: ablation -- generation reads no training rows (constant row)
//   bit 3: ablation -- no barrier in the K loop (wrong results; timing only)
//   bit 4: ablation -- no generation and no A stores at all (MFMA + B stream bound)
//   bit 5: ablation -- no B loads (B operands stay in registers)
//   bit 6: ablation -- no LDS A-fragment reads (A operands from registers)
//   bit 7: ablation -- every block runs the full K range (no triangular schedule)
template <int DI, bool DYN, int VAR = 0, int NW = 4>
__global__ __launch_bounds__(64 * NW, (DI <= 16 ? 2 : 1)) void k_gp_tile(const TileParams prm) {
  constexpr int NT = 64 * NW;                                // threads
  constexpr int NB = 64 * NW;                                // columns per block
  constexpr int FS = NW * 1024;                              // fragment doubles per K-step
  constexpr int GV = kBK / NW;                               // K* values per thread per K-step
  constexpr int RW = DI + 1;                                 // row record: Xs[DI], |Xs|^2
  constexpr int NRV = kBK * RW;                              // row values per K-step
  constexpr int RPT = (NRV + NT - 1) / NT;                   // row values per thread
  __shared__ double As[2][kBK][kLDA];
  __shared__ double RX[2][kBK][RW];
  __shared__ double tab[64];
  __shared__ double qred[NW][kPT];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x;
  const int J = prm.n_j_max - 1 - b / prm.tiles_ub;
  // tile index within this launch's segments (a launch may cover classes c0..c0+7)
  const int t = b - (b / prm.tiles_ub) * prm.tiles_ub + prm.seg_tile_start[0];

  int c = -1;
  for (int s = 0; s < prm.n_seg; ++s)
    if (t >= prm.seg_tile_start[s] && t < prm.seg_tile_start[s + 1]) c = s;
  c = __builtin_amdgcn_readfirstlane(c);
  if (c < 0) return;
  const int n_j = prm.seg[c].n_j;
  if (J >= n_j) return;
  const double* __restrict__ Xs = prm.seg[c].Xs;
  const double* __restrict__ Xsq = prm.seg[c].Xsq;
  const double* __restrict__ Bf = prm.seg[c].Bf;
  const int n_rows = prm.seg[c].n_rows;
  const int n_m = prm.seg[c].n_m;
  const int n_cols = n_rows + n_m;

  if (tid < 64) tab[tid] = kExp2Tab[tid];

  const int seg_begin = prm.seg_pos_begin[c];
  const int pos0 = seg_begin + (t - prm.seg_tile_start[c]) * kPT;
  const int pos_end = prm.seg_pos_end[c];
  const int out_base = prm.seg_out_base[c] - seg_begin;   // out = out_base + pos

  // ---- this thread's particle (generation role: particle m, rows w + 4s) ----------
  const int m = lane;
  int pos = pos0 + m;
  if (pos >= pos_end) pos = pos0;                          // clamp (results unused)
  const int prow = prm.perm ? prm.perm[pos] : pos;
  double a2[DI];                                           // 2 (x / l) (64 / ln 2)
  double asq = 0.0;
#pragma unroll
  for (int j = 0; j < DI; ++j) {
    const double x = prm.X[(long long)prow * DI + j];
    const double xs = x / prm.ls[j];
    asq = fma(xs, xs, asq);
    a2[j] = (2.0 * kLog2eX64) * xs;
  }
  asq *= kLog2eX64;                                        // |x / l|^2 (64 / ln 2)

  // ---- K ranges ------------------------------------------------------------------
  const int nks = (VAR & 128) ? ksteps(n_rows) : ksteps(block_kmax(J, n_rows, NB));
  // this wave's tiles: columns NB*J + 16(NW t + w) .. +15.  T1 = real tiles, kend[t] = the
  // K-step where tile t retires (R tile: past its last column's diagonal; tiles holding
  // mean columns: all rows).  kend is non-decreasing in t.
  int T1 = 0;
  int kend[4];
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) {
    const int c0 = J * NB + 16 * (NW * tt + w);
    const bool real = c0 < n_cols;
    if (real) T1 = tt + 1;
    const int hi = c0 + 16;
    int ke = (hi <= n_rows) ? ksteps(hi) : ksteps(n_rows);
    if constexpr (VAR & 129) ke = nks;
    kend[tt] = real ? (ke < nks ? ke : nks) : 0;
  }
  long long boff = 0;                                       // fragments of blocks < J
  for (int jj = 0; jj < J; ++jj) boff += (long long)ksteps(block_kmax(jj, n_rows, NB)) * FS;
  const double* __restrict__ Bw = Bf + boff + w * 1024 + lane * 2;
  // last K-step this wave multiplies (kend is non-decreasing over the real tiles; no
  // runtime indexing of kend[], which would put it in scratch)
  const int kmaxw = max(max(kend[0], kend[1]), max(kend[2], kend[3]));
  const int ks_last = (kmaxw > 0 ? kmaxw : 1) - 1;

  // Training rows of a K-step are staged through an LDS ring (RX) one step ahead with
  // vector loads, so generation reads them as LDS broadcasts: no scalar loads whose
  // lgkmcnt(0) waits would serialise with the A-fragment reads.
  const int last_row = n_rows - 1;
  auto load_rows = [&](int ks, double (&rr)[RPT]) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int idx = tid + NT * k;
      double v = 0.0;
      if (idx < NRV) {
        const int r = idx / RW, f = idx - (idx / RW) * RW;
        int i = ks * kBK + r;
        i = i < last_row ? i : last_row;
        v = f < DI ? Xs[(long long)i * DI + f] : Xsq[i];
      }
      rr[k] = v;
    }
  };
  auto store_rows = [&](int buf, const double (&rr)[RPT]) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int idx = tid + NT * k;
      if (idx < NRV) (&RX[buf][0][0])[idx] = rr[k];
    }
  };
  // Branch-free generation (rows past n_rows are zeroed after the fact).
  auto gen = [&](int ks, double (&v)[GV]) {
    const int rb = ks & 1;
#pragma unroll
    for (int s = 0; s < GV; ++s) {
      const int r = w + NW * s;
      const int i = ks * kBK + r;                          // wave-uniform training row
      const double* row = &RX[rb][r][0];
      double x;
      if constexpr (VAR & 4) {
        x = -(asq + 0.5 * i);
#pragma unroll
        for (int j = 0; j < DI; ++j) x = fma(a2[j], 0.25 * j, x);
      } else {
        x = -(asq + row[DI]);
#pragma unroll
        for (int j = 0; j < DI; ++j) x = fma(a2[j], row[j], x);
      }
      double val;
      if constexpr (VAR & 2) val = fma(x, 1e-3, 1.0);
      else val = exp2_64(x, tab);
      v[s] = i < n_rows ? val : 0.0;
    }
  };
  // B fragments: one register set, refilled sub-step by sub-step for the next K-step right
  // after the MFMAs that consumed it (so the prefetch needs no second set of registers).
  // The address is clamped to the wave's last K-step so no branch guards the loads.
  auto loadB_part = [&](int ks, int kk, double (&bb)[16]) {
    if constexpr (VAR & 32) {
#pragma unroll
      for (int q = 0; q < 4; ++q) bb[kk * 4 + q] = bb[kk * 4 + q] * 0.999 + 1e-3 * (ks & 1);
      return;
    }
    const double* src = Bw + (long long)(ks < ks_last ? ks : ks_last) * FS + kk * 256;
    const double2 x0 = *reinterpret_cast<const double2*>(src);
    const double2 x1 = *reinterpret_cast<const double2*>(src + 128);
    bb[kk * 4 + 0] = x0.x;
    bb[kk * 4 + 1] = x0.y;
    bb[kk * 4 + 2] = x1.x;
    bb[kk * 4 + 3] = x1.y;
  };
  auto store = [&](int buf, const double (&v)[GV]) {
#pragma unroll
    for (int s = 0; s < GV; ++s) As[buf][w + NW * s][m] = v[s];
  };

  const int li = lane & 15, lk = lane >> 4;
  d4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};

  // One K-step with tiles [T0, T1) active: generate K*(ks+1) and stage rows(ks+2), then per
  // sub-step kk: A fragments from LDS, MFMAs, refill B(ks+1) for kk.  (Generating for
  // ks+1 = nks is harmless: clamped rows, stored to a buffer never read again.)
  auto full_step = [&](auto t0c, auto t1c, int ks, double (&bb)[16]) {
    constexpr int T0 = decltype(t0c)::value, T1c = decltype(t1c)::value;
    const int buf = ks & 1;
    double v[GV];
    double rr[RPT];
    if constexpr (!(VAR & 16)) {
      load_rows(ks + 2, rr);
      gen(ks + 1, v);
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      double af[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        if constexpr (VAR & 64) af[mt] = asq + mt + kk + buf;
        else af[mt] = As[buf][kk * 4 + lk][mt * 16 + li];
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = T0; nt < T1c; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[mt], bb[kk * 4 + nt], acc[mt][nt], 0, 0, 0);
      loadB_part(ks + 1, kk, bb);
    }
    if constexpr (!(VAR & 16)) {
      store(buf ^ 1, v);
      store_rows(buf, rr);
    }
    if constexpr (!(VAR & 8)) __syncthreads();
  };

  double bb[16];
  if constexpr (VAR & 32) {
#pragma unroll
    for (int q = 0; q < 16; ++q) bb[q] = 1e-3 * q + lane;
  }
  {
    double rr[RPT];
    load_rows(0, rr);
    store_rows(0, rr);
    load_rows(1, rr);
    store_rows(1, rr);
  }
  __syncthreads();                                           // table + rows of steps 0, 1
  {
    double v[GV];
    gen(0, v);
    store(0, v);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) loadB_part(0, kk, bb);
  }
  __syncthreads();

  int ks = 0;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  // K-steps [ks, e) with tiles [T0, T1) active
  auto run_phase = [&](auto t0c, auto t1c, int e) {
    for (; ks < e; ++ks) full_step(t0c, t1c, ks, bb);
  };
  switch (T1) {
    case 4:
      run_phase(I0{}, I4{}, kend[0]);
      run_phase(I1{}, I4{}, kend[1]);
      run_phase(I2{}, I4{}, kend[2]);
      run_phase(I3{}, I4{}, kend[3]);
      break;
    case 3:
      run_phase(I0{}, I3{}, kend[0]);
      run_phase(I1{}, I3{}, kend[1]);
      run_phase(I2{}, I3{}, kend[2]);
      break;
    case 2:
      run_phase(I0{}, I2{}, kend[0]);
      run_phase(I1{}, I2{}, kend[1]);
      break;
    case 1:
      run_phase(I0{}, I1{}, kend[0]);
      break;
    default:
      break;
  }
  // the rest of the block's K range (other waves' tiles): generate only
  for (; ks < nks; ++ks) {
    double v[GV];
    double rr[RPT];
    load_rows(ks + 2, rr);
    gen(ks + 1, v);
    store((ks + 1) & 1, v);
    store_rows(ks & 1, rr);
    __syncthreads();
  }

  if constexpr (DYN) {
    // Linear-kernel share: acc += X~ H for this block.  A fragment: lane l holds
    // x~[particle mt*16 + (l&15)][4 kh + (l>>4)]; B fragment: Hf[J][kh][w][l][nt].
    constexpr int KH = (DI + 1 + 3) / 4;
    const double* __restrict__ Hw = prm.seg[c].Hf + ((long long)J * KH * NW + w) * 256 + lane * 4;
    int prw[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      int pp = pos0 + mt * 16 + li;
      if (pp >= pos_end) pp = pos0;
      prw[mt] = prm.perm ? prm.perm[pp] : pp;
    }
#pragma unroll
    for (int kh = 0; kh < KH; ++kh) {
      const int k = 4 * kh + lk;
      const double2 h0 = *reinterpret_cast<const double2*>(Hw + (long long)kh * NW * 256);
      const double2 h1 = *reinterpret_cast<const double2*>(Hw + (long long)kh * NW * 256 + 2);
      const double hb[4] = {h0.x, h0.y, h1.x, h1.y};
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const double xa = k < DI ? prm.X[(long long)prw[mt] * DI + (k < DI ? k : 0)] : (k == DI ? 1.0 : 0.0);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa, hb[nt], acc[mt][nt], 0, 0, 0);
      }
    }
  }

  // ---- epilogue --------------------------------------------------------------------
  // C/D layout of v_mfma_f64_16x16x4_f64: lane l, reg r -> row (l>>4) + 4r, col l&15.
  const bool has_r = J * NB < n_rows;
  if (has_r) {
    double qs[4][4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double s = 0.0;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const double x = acc[mt][nt][r];
          if (J * NB + 16 * (NW * nt + w) + li < n_rows) s = fma(x, x, s);
        }
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        s += __shfl_xor(s, 4);
        s += __shfl_xor(s, 8);
        qs[mt][r] = s;
      }
    if (li == 0) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) qred[w][mt * 16 + lk + 4 * r] = qs[mt][r];
    }
  }
  if ((J + 1) * NB > n_rows) {                                // mean columns
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int jm = J * NB + 16 * (NW * nt + w) + li - n_rows;
      if (jm >= 0 && jm < n_m) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int p = pos0 + mt * 16 + lk + 4 * r;
            if (p < pos_end) prm.mu[(long long)(out_base + p) * prm.ld_mu + jm] = acc[mt][nt][r];
          }
      }
    }
  }
  if (has_r) {
    __syncthreads();
    if (tid < kPT) {
      const int p = pos0 + tid;
      if (p < pos_end) {
        double q = 0.0;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) q += qred[ww][tid];
        prm.qpart[(long long)J * prm.ld_q + out_base + p] = q;
      }
    }
  }
}

template <int DI>
static void launch_d(const TileParams& p, bool dyn, hipStream_t stream) {
  const dim3 grid((unsigned)(p.n_j_max * p.tiles_ub));
  if (p.nw == 8) {
    if (dyn)
      hipLaunchKernelGGL((k_gp_tile<DI, true, 0, 8>), grid, dim3(512), 0, stream, p);
    else
      hipLaunchKernelGGL((k_gp_tile<DI, false, 0, 8>), grid, dim3(512), 0, stream, p);
  } else {
    if (dyn)
      hipLaunchKernelGGL((k_gp_tile<DI, true, 0, 4>), grid, dim3(256), 0, stream, p);
    else
      hipLaunchKernelGGL((k_gp_tile<DI, false, 0, 4>), grid, dim3(256), 0, stream, p);
  }
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
