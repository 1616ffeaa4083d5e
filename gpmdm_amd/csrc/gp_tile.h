#pragma once
// Fused GP predictive tile for gfx950: kernel-row generation + FP64 MFMA contraction.
//
// Replaces, for a tile of PT particles x NB columns (shapes in common.h: TileGeo):
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
// training rows up to its last column, and each 16-column tile stops at its own diagonal:
// about half the dense FLOPs.  B = [R | M] carries the mean weights M (beta or alpha_c) as
// extra columns, so one pass produces both.
//
// Workgroup = NW waves; wave w owns MT x NTW tiles of 16 x 16 (v_mfma_f64_16x16x4_f64,
// 128 accumulator VGPRs at MT x NTW = 16), its column tiles interleaved with the other
// waves' at columns NB J + 16 (NW t + w) so that all waves reach nearly the same K.  A tile
// of R columns retires once K passes its diagonal: the K loop runs in phases with tiles
// [T0, T1) active, so no MFMA multiplies the zero triangle.  Per K-step of 16 training rows:
//   * the K* tile (PT x 16) is generated once per workgroup (expansion-form distance as
//     gpmdm.py:508-515, table-driven fp64 exp), two K-steps ahead, into an LDS ring that
//     all waves read as A fragments; training rows are staged through a second LDS ring;
//   * B fragments stream from L2 straight into VGPRs by buffer loads (SGPR resource and
//     K-step offset, constant lane offset: no VALU address arithmetic), one K-step ahead;
//     B is stored in fragment order, so no LDS round trip and no re-layout;
//   * one barrier per two K-steps.  Two workgroups per CU overlap each other's barriers.
// Every VALU instruction costs MFMA issue time on gfx950 (tools/microbench/mix_probe), so
// the loop is written to minimise them (padded rows instead of masks, buffer addressing).
// Workgroups are ordered heavy-first (column block J descending), which both balances the
// triangular work and makes concurrent workgroups share a B panel in each XCD's L2.
// In the filter the observation GP's mean blocks reduce the likelihood partial sums
// (TileParams::spart) instead of storing the P x D mean.
#include <type_traits>

#include "common.h"

namespace gpmdm {

// 2^(j/64), j = 0..63 (correctly rounded).
static __constant__ double kExp2Tab[64] = {
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

// Geometry: NW waves; each wave owns MT x NTW tiles of 16 x 16 (16 MT particles x 16 NTW
// columns), so a workgroup covers PT = 16 MT particles x NB = 16 NTW NW columns.  K* costs
// the same per generated value whatever the geometry, so generation per MFMA falls as
// 1 / NB: (MT, NTW) = (4, 4) is 64 x 256, (2, 8) is 32 x 512 at the same accumulator
// count (128 VGPRs) and MFMA work per K-step, with half the K* values and A-fragment reads
// and twice the B fragments per K-step.
// FLAGS: kTileCoordLDS -- the particle coordinates are read from LDS in the generation
// instead of held in VGPRs (frees 2 d VGPRs: the 32-particle shapes above d = 12).
// The A/B variants measured against this kernel (other exp tables, barrier cadences, wave
// specialisation, the K* cache, ablations) live in tools/microbench/gp_tile_lab.h.
constexpr int kTileCoordLDS = 131072;
template <int I, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < E) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, E>(f);
  }
}

template <int DI, bool DYN, int FLAGS = 0, int NW = 4, int MT = 4, int NTW = 4>
__global__ __launch_bounds__(64 * NW, (DI <= 16 ? 2 : 1)) void k_gp_tile(const TileParams prm) {
  static_assert(MT == 1 || MT == 2 || MT == 4, "MT");
  static_assert(NTW == 4 || NTW == 6 || NTW == 8 || NTW == 16, "NTW");
  static_assert((FLAGS & ~kTileCoordLDS) == 0, "FLAGS");
  // B fragments in flight: BR sub-steps (a full K-step, 4, for NTW <= 8; 2 for NTW = 16,
  // whose full K-step of fragments would not fit next to 128 accumulator VGPRs)
  constexpr int BR = NTW >= 16 ? 2 : 4;
  // tiles retire in groups of RG (NTW = 16: 8 phase groups instead of 16, so the K loop has
  // 36 phase variants rather than 136; a group runs until its last tile's diagonal)
  constexpr int RG = NTW >= 16 ? 2 : 1;
  constexpr int NT = 64 * NW;                                // threads
  constexpr int PT = 16 * MT;                                // particles per tile
  constexpr int NB = 16 * NTW * NW;                          // columns per block
  constexpr int WS = 256 * NTW;                              // fragment doubles per wave per K-step
  constexpr int FS = NW * WS;                                // fragment doubles per K-step
  constexpr int NG = NT / PT;                                // generation row groups
  constexpr int GV = kBK / NG;                               // K* values per thread per K-step
  static_assert(GV * NG == kBK, "generation split");
  constexpr int LDA = PT + 16;                               // rows k, k+1 land 32 banks apart
  constexpr int RW = DI + 1;                                 // row record: Xs[DI], |Xs|^2
  constexpr int NRV = kBK * RW;                              // row values per K-step
  constexpr int RPT = (NRV + NT - 1) / NT;                   // row values per thread
  // LDS rings: one barrier per two K-steps (after odd ones), K* generated two K-steps ahead
  // into 4 slots, rows staged four ahead into 4 slots -- a slot is rewritten only after a
  // barrier that follows its last read, and read only after a barrier that follows its
  // write.  (One barrier per K-step: obs tile +0.6%; per four: no further gain, twice the
  // LDS -- tile_bench.)  General rule for S K-steps per barrier: lookahead LOOK >= S,
  // K* slots >= LOOK + S, row lookahead RA >= LOOK + S, row slots >= RA - LOOK + S.
  constexpr int SB = 2;                                      // K-steps per barrier
  constexpr int ASL = 2 * SB;                                // K* slots
  constexpr int RXS = 2 * SB;                                // row-record slots
  constexpr int LOOK = SB;                                   // generation lookahead (K-steps)
  constexpr int RA = 2 * SB;                                 // row staging lookahead
  __shared__ double As[ASL][kBK][LDA];
  __shared__ double RX[RXS][RPT * NT];                        // row records, then padding
  constexpr double kScale = kLog2eX64;
  // exp table 2^(j/64), one shared copy (lanes reading entries j and j + 32 in one lane
  // group conflict; a lane-replicated table removes the conflicts and costs more in
  // address arithmetic than they cost, tile_bench)
  __shared__ double tab[64];
  // read-out partials per block, or per 256-column half for the wide dynamics shape (epilogue)
  constexpr int NHS = (DYN && NW == 4 && NTW == 8) ? 2 : 1;
  __shared__ double qred[NHS * NW][PT];
  constexpr bool PLDS = (FLAGS & kTileCoordLDS) != 0;
  __shared__ double PA[PLDS ? PT : 1][PLDS ? DI + 1 : 1];
  __shared__ double sred[NHS * NW][PT];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x;
  // Dynamics launches size their grid by an upper bound (the de-duplicated row count is
  // only known on the device): the real tile count tu is read from the segment table and
  // workgroups map real-first -- J-major over the tu real tiles, heavy blocks first -- so
  // the empty workgroups trail the real work instead of sitting between the column blocks.
  // The observation GP's grid is exact (tu = tiles_ub).
  const int tu = DYN ? __builtin_amdgcn_readfirstlane(prm.seg_tile_start[prm.n_seg] - prm.seg_tile_start[0])
                     : prm.tiles_ub;
  if (DYN && (tu <= 0 || b >= prm.n_j_max * tu)) return;
  const int J = prm.n_j_max - 1 - b / tu;
  // tile index within this launch's segments (a launch may cover classes c0..c0+7)
  // segment tables live in device memory (the filter computes them on the device; the
  // predictive maps write theirs with k_seg_table).  A by-value table with a per-thread
  // select cost the d = 16 64x512 tile 6.7% through register allocation (tools/microbench/
  // tile_ab.sh: 760 -> 811 ms per config-5 launch)
  const int t = b - (b / tu) * tu + prm.seg_tile_start[0];

  int c = -1;
  for (int s = 0; s < prm.n_seg; ++s)
    if (t >= prm.seg_tile_start[s] && t < prm.seg_tile_start[s + 1]) c = s;
  c = __builtin_amdgcn_readfirstlane(c);
  if (c < 0) return;
  const int n_j = prm.seg[c].n_j;
  if (J >= n_j) return;
  const double* __restrict__ Xrec = prm.seg[c].Xrec;
  const double* __restrict__ Bf = prm.seg[c].Bf;
  const int n_rows = prm.seg[c].n_rows;
  const int n_m = prm.seg[c].n_m;
  const int n_cols = n_rows + n_m;
  const int coff = prm.seg[c].coff;

  for (int i = tid; i < 64; i += NT) tab[i] = kExp2Tab[i];

  const int seg_begin = prm.seg_pos_begin[c];
  const int pos0 = seg_begin + (t - prm.seg_tile_start[c]) * PT;
  const int pos_end = prm.seg_pos_end[c];
  const int out_base = prm.seg_out_base[c] - seg_begin;   // out = out_base + pos

  // ---- this thread's particle (generation role: particle m, rows g + NG s) ----------
  const int m = tid % PT;
  const int g = tid / PT;
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
    a2[j] = (2.0 * kScale) * xs;
  }
  asq *= kScale;                                           // |x / l|^2 (64 / ln 2)
  if constexpr (PLDS) {
    if (g == 0) {
#pragma unroll
      for (int j = 0; j < DI; ++j) PA[m][j] = a2[j];
    }
  }

  // ---- K ranges ------------------------------------------------------------------
  const int nks = ksteps(block_kmax(J, n_rows, NB, coff));
  // this wave's tiles: columns NB*J + 16(NW t + w) .. +15.  T1 = real tiles, kend[t] = the
  // K-step where tile t retires (R tile: past its last column's diagonal; tiles holding
  // mean columns: all rows).  kend is non-decreasing in t.
  int T1 = 0;
  int kend[NTW];
#pragma unroll
  for (int tt = 0; tt < NTW; ++tt) {
    const int c0 = J * NB + 16 * (NW * tt + w) - coff;    // front-padding tiles: c0 < 0
    const bool real = c0 >= 0 && c0 < n_cols;
    if (real) T1 = tt + 1;
    const int hi = c0 + 16;
    const int ke = (hi <= n_rows) ? ksteps(hi) : ksteps(n_rows);
    kend[tt] = real ? (ke < nks ? ke : nks) : 0;
  }
  long long boff = 0;                                       // fragments of blocks < J
  for (int jj = 0; jj < J; ++jj) boff += (long long)ksteps(block_kmax(jj, n_rows, NB, coff)) * FS;
  // B addressing: a buffer resource on this wave's share of block J (SGPRs), a per-lane
  // byte offset (VGPR, constant) and a wave-uniform K-step offset (SGPR), so the K loop
  // spends no VALU on 64-bit address arithmetic.
  const double* __restrict__ Bw = Bf + boff + w * WS;
  const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Bw, (short)0, 0x7fffffff, 0x00020000);
  const unsigned lane_off = (unsigned)lane * 16u;
  // last K-step this wave multiplies (kend is non-decreasing over the real tiles; no
  // runtime indexing of kend[], which would put it in scratch)
  int kmaxw = 0;
#pragma unroll
  for (int tt = 0; tt < NTW; ++tt) kmaxw = max(kmaxw, kend[tt]);
  const int ks_last = (kmaxw > 0 ? kmaxw : 1) - 1;

  // Training rows of a K-step are staged through an LDS ring (RX) with vector loads, so
  // generation reads them as LDS broadcasts: no scalar loads whose lgkmcnt(0) waits would
  // serialise with the A-fragment reads.
  // Branch-free: threads past the record count load a clamped (valid) address and store it
  // to a padding slot, so no exec-mask branch splits the K-step (the compiler otherwise
  // sinks the load into the conditional store and waits for it with vmcnt(0)).
  // Row records [Xs_i, |Xs_i|^2 64/ln2] (RW doubles per row, padded rows included) are one
  // contiguous array: buffer loads with a per-thread constant byte offset and a wave-uniform
  // K-step offset, no VALU address arithmetic per K-step.
  typedef unsigned v2u __attribute__((ext_vector_type(2)));
  const __amdgpu_buffer_rsrc_t rrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Xrec, (short)0, 0x7fffffff, 0x00020000);
  unsigned roff[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int idx = tid + NT * k;
    roff[k] = (unsigned)(idx < NRV ? idx : NRV - 1) * 8u;
  }
  auto load_rows = [&](int ks, double (&rr)[RPT]) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const v2u x = __builtin_amdgcn_raw_buffer_load_b64(rrsrc, roff[k], ks * (NRV * 8), 0);
      rr[k] = __builtin_bit_cast(double, (unsigned long long)x.x | ((unsigned long long)x.y << 32));
    }
  };
  auto store_rows = [&](int buf, const double (&rr)[RPT]) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) RX[buf][tid + NT * k] = rr[k];   // unconditional (padding slots)
  };
  // Branch-free generation.  The row arrays are padded to row_cap(n_rows) rows with
  // |Xs|^2 = kPadSq (2^28, geometry.h), so a padding row's exponent is about -2^28 x 64/ln2
  // (the float->int conversion is exact, ldexp underflows): its kernel value is exactly 0,
  // no masking per value.
  auto gen_one = [&](int rb, int s) -> double {
    const int r = g + NG * s;
    const double* row = &RX[rb][r * RW];
    double x = -(asq + row[DI]);
#pragma unroll
    for (int j = 0; j < DI; ++j) x = fma(PLDS ? PA[m][j] : a2[j], row[j], x);
    return exp2_64(x, tab);                                // padding rows: exactly 0
  };
  auto gen = [&](int rb, double (&v)[GV]) {
#pragma unroll
    for (int s = 0; s < GV; ++s) v[s] = gen_one(rb, s);
  };
  // B fragments: one register set, refilled sub-step by sub-step for the next K-step right
  // after the MFMAs that consumed it (so the prefetch needs no second set of registers).
  // The address is clamped to the wave's last K-step so no branch guards the loads.
  auto loadB_part = [&](int ks, int kk, int slot, double (&bb)[BR * NTW]) {
    const int kc = ks < ks_last ? ks : ks_last;
#pragma unroll
    for (int h = 0; h < NTW / 2; ++h) {
      typedef unsigned v4u __attribute__((ext_vector_type(4)));
      const int soff = (kc * FS + kk * (64 * NTW) + 128 * h) * 8;     // bytes, wave-uniform
      const v4u x = __builtin_amdgcn_raw_buffer_load_b128(brsrc, lane_off, soff, 0);
      bb[slot * NTW + 2 * h + 0] = __builtin_bit_cast(double, (unsigned long long)x.x | ((unsigned long long)x.y << 32));
      bb[slot * NTW + 2 * h + 1] = __builtin_bit_cast(double, (unsigned long long)x.z | ((unsigned long long)x.w << 32));
    }
  };
  auto store = [&](int buf, const double (&v)[GV]) {
#pragma unroll
    for (int s = 0; s < GV; ++s) As[buf][g + NG * s][m] = v[s];
  };

  const int li = lane & 15, lk = lane >> 4;
  d4 acc[MT][NTW];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};

  // One K-step with tiles [T0, T1) active: generate K*(ks+LOOK) and stage rows(ks+RA), then
  // per sub-step kk: A fragments from LDS, MFMAs, refill B(ks+1) for kk.  (Generating past
  // the last K-step is harmless: clamped rows, stored to a slot never read again.)
  auto full_step = [&](auto t0c, auto t1c, int ks, double (&bb)[BR * NTW]) {
    constexpr int T0 = decltype(t0c)::value, T1c = decltype(t1c)::value;
    const int buf = ks & (ASL - 1);
    const int gslot = (ks + LOOK) & (ASL - 1);
    const int rslot = (ks + RA) & (RXS - 1);
    const int grb = (ks + LOOK) & (RXS - 1);
    double v[GV];
    double rr[RPT];
    load_rows(ks + RA, rr);
    gen(grb, v);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      double af[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) af[mt] = As[buf][kk * 4 + lk][mt * 16 + li];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = T0; nt < T1c; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[mt], bb[(kk % BR) * NTW + nt], acc[mt][nt], 0, 0, 0);
      loadB_part(ks + (kk + BR) / 4, (kk + BR) % 4, kk % BR, bb);   // sub-step kk + BR
    }
    store(gslot, v);
    store_rows(rslot, rr);
    if (ks % SB == SB - 1) __syncthreads();
  };
  double bb[BR * NTW];
  {
    double rr[RPT];
#pragma unroll
    for (int j = 0; j < RA; ++j) {
      load_rows(j, rr);
      store_rows(j, rr);
    }
  }
  __syncthreads();                                           // table + rows of steps 0 .. RA-1
  {
    double v[GV];
#pragma unroll
    for (int j = 0; j < LOOK; ++j) {
      gen(j & (RXS - 1), v);
      store(j, v);
    }
#pragma unroll
    for (int kk = 0; kk < BR; ++kk) loadB_part(0, kk, kk, bb);
  }
  // Drain the prologue's loads (vmcnt(0)) so that the K loop's entry carries no pending
  // loads: otherwise the waitcnt pass merges the prologue's issue order into the loop
  // header and waits for every in-flight B fragment at sub-step 0 of each K-step.
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();

  int ks = 0;
  // K-steps [ks, kend[T0]) with tiles [T0, T1) active, for T0 = 0 .. T1-1
  // (groups of RG tiles: phase T0 = g0 RG runs until the group's last tile retires)
  static_for<1, NTW / RG + 1>([&](auto g1c) {
    constexpr int T1c = decltype(g1c)::value * RG;
    if ((T1 + RG - 1) / RG * RG == T1c) {
      static_for<0, T1c / RG>([&](auto g0c) {
        constexpr int T0 = decltype(g0c)::value * RG;
        int e = kend[T0];
        if constexpr (RG == 2) e = max(e, kend[T0 + 1]);
        for (; ks < e; ++ks) full_step(std::integral_constant<int, T0>{}, std::integral_constant<int, T1c>{}, ks, bb);
      });
    }
  });
  // the rest of the block's K range (other waves' tiles): generate only
  for (; ks < nks; ++ks) {
    double v[GV];
    double rr[RPT];
    load_rows(ks + RA, rr);
    gen((ks + LOOK) & (RXS - 1), v);
    store((ks + LOOK) & (ASL - 1), v);
    store_rows((ks + RA) & (RXS - 1), rr);
    if (ks % SB == SB - 1) __syncthreads();
  }

  if constexpr (DYN) {
    // Linear-kernel share: acc += X~ H for this block.  A fragment: lane l holds
    // x~[particle mt*16 + (l&15)][4 kh + (l>>4)]; B fragment: Hf[J][kh][w][l][nt].
    constexpr int KH = (DI + 1 + 3) / 4;
    const double* __restrict__ Hw = prm.seg[c].Hf + ((long long)J * KH * NW + w) * (64 * NTW) + lane * NTW;
    int prw[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      int pp = pos0 + mt * 16 + li;
      if (pp >= pos_end) pp = pos0;
      prw[mt] = prm.perm ? prm.perm[pp] : pp;
    }
#pragma unroll
    for (int kh = 0; kh < KH; ++kh) {
      const int k = 4 * kh + lk;
      double hb[NTW];
#pragma unroll
      for (int h = 0; h < NTW / 2; ++h) {
        const double2 hv = *reinterpret_cast<const double2*>(Hw + (long long)kh * NW * (64 * NTW) + 2 * h);
        hb[2 * h] = hv.x;
        hb[2 * h + 1] = hv.y;
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const double xa = k < DI ? prm.X[(long long)prw[mt] * DI + (k < DI ? k : 0)] : (k == DI ? 1.0 : 0.0);
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa, hb[nt], acc[mt][nt], 0, 0, 0);
      }
    }
  }

  // ---- epilogue --------------------------------------------------------------------
  // Read-out partials.  The dynamics GP's wide shape (4 waves x 8 column tiles: 32 x 512 and
  // its 16-row form) reduces each 256-column half of a block into its own partial in the
  // 16 x 256 shape's order, so the narrow and wide dynamics images give bitwise the same
  // outputs (tests/test_gpu_small_path.py, test_gpu_dedup.py); every other shape writes one
  // partial per block.  (The observation GP keeps one partial per block: the split moved
  // the d = 3 observation tile's register allocation and cost 0.5% of its launch time,
  // profiles/r04/split_epilogue_ab.txt.)
  constexpr int NH = NHS;
  if constexpr (NH == 1) {
    // C/D layout of v_mfma_f64_16x16x4_f64: lane l, reg r -> row (l>>4) + 4r, col l&15.
    const bool has_r = J * NB - coff < n_rows;
    const bool has_m = (J + 1) * NB - coff > n_rows;            // block holds mean columns
    const bool fused = prm.spart != nullptr;
    if (has_m) {
      if (!fused) {
  #pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          const int jm = J * NB + 16 * (NW * nt + w) + li - coff - n_rows;
          if (jm >= 0 && jm < n_m) {
  #pragma unroll
            for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int p = pos0 + mt * 16 + lk + 4 * r;
                if (p < pos_end)
                  prm.mu[(long long)(out_base + p) * prm.ld_mu + jm] = acc[mt][nt][r];
              }
          }
        }
      } else {
        // sum_j (z_j - mu_j)^2 lam2_j over this block's mean columns (gpmdm_pf.py:188-192 with
        // var_j = vc / lam2_j factored out; k_obs_ll finishes the likelihood).  A tile whose
        // particles share one filter (always, for a single filter) reads z_j once per column.
        const int Pf = (int)prm.Pf;
        const int f0 = pos0 / Pf, f1 = (min(pos0 + PT, pos_end) - 1) / Pf;   // wave-uniform
        double ss[MT][4];
  #pragma unroll
        for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
          for (int r = 0; r < 4; ++r) ss[mt][r] = 0.0;
  #pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          const int jm = J * NB + 16 * (NW * nt + w) + li - coff - n_rows;
          if (jm >= 0 && jm < n_m) {
            const double lam = prm.lam2[jm];
            if (f0 == f1) {
              const double zj = prm.z[(long long)f0 * n_m + jm];
  #pragma unroll
              for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const double t = zj - acc[mt][nt][r];
                  ss[mt][r] = fma(t * t, lam, ss[mt][r]);
                }
            } else {
  #pragma unroll
              for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
                for (int r = 0; r < 4; ++r) {
                  int p = pos0 + mt * 16 + lk + 4 * r;
                  p = p < pos_end ? p : pos0;
                  const double zz = prm.z[(long long)(p / Pf) * n_m + jm];
                  const double t = zz - acc[mt][nt][r];
                  ss[mt][r] = fma(t * t, lam, ss[mt][r]);
                }
            }
          }
        }
  #pragma unroll
        for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
          for (int r = 0; r < 4; ++r) {
            double v = ss[mt][r];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            if (li == 0) sred[w][mt * 16 + lk + 4 * r] = v;
          }
      }
      // mean columns do not enter the quadratic form
  #pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int col = J * NB + 16 * (NW * nt + w) + li - coff;
        if (col >= n_rows) {
  #pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[mt][nt] = (d4){0.0, 0.0, 0.0, 0.0};
        }
      }
    }
    if (has_r) {
      // Sum of squares over the block's R columns.  Front-padding columns (col < 0) have
      // B = 0, so V = 0 there: no mask (mean columns were zeroed above).
      double qs[MT][4];
  #pragma unroll
      for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
        for (int r = 0; r < 4; ++r) {
          double v = 0.0;
  #pragma unroll
          for (int nt = 0; nt < NTW; ++nt) v = fma(acc[mt][nt][r], acc[mt][nt][r], v);
          v += __shfl_xor(v, 1);
          v += __shfl_xor(v, 2);
          v += __shfl_xor(v, 4);
          v += __shfl_xor(v, 8);
          qs[mt][r] = v;
        }
      if (li == 0) {
  #pragma unroll
        for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
          for (int r = 0; r < 4; ++r) qred[w][mt * 16 + lk + 4 * r] = qs[mt][r];
      }
    }
    if (has_r || (has_m && fused)) {
      __syncthreads();
      if (tid < PT) {
        const int p = pos0 + tid;
        if (p < pos_end) {
          if (has_r) {
            double q = 0.0;
  #pragma unroll
            for (int ww = 0; ww < NW; ++ww) q += qred[ww][tid];
            prm.qpart[(long long)J * prm.ld_q + out_base + p] = q;
          }
          if (has_m && fused) {
            double sm = 0.0;
  #pragma unroll
            for (int ww = 0; ww < NW; ++ww) sm += sred[ww][tid];
            prm.spart[(long long)J * prm.ld_q + out_base + p] = sm;
          }
        }
      }
    }
  } else {
    // C/D layout of v_mfma_f64_16x16x4_f64: lane l, reg r -> row (l>>4) + 4r, col l&15.
    // Read-out partials: one per block, or -- the 4-wave shapes with 8 column tiles per wave
    // (32 x 512 and its 16-row form) -- one per 256-column half, each reduced exactly as the
    // 16 x 256 shape reduces the block holding the same columns (wave w's tiles w, w + 4, ...
    // of the half in order; lanes by xor 1, 2, 4, 8; waves in order) and stored at that
    // block's index: the 32 x 512 and 16 x 256 images give bitwise the same outputs.
    constexpr int NTH = NTW / NH;
    constexpr int HB = NB / NH;                                  // columns per partial
    const int pcoff = NH == 2 ? col_offset(n_cols, HB) : coff;   // the partial blocks' front padding
    int pj[NH];
    bool hr[NH], hm[NH];
    bool any_r = false, any_m = false;
  #pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int c0 = J * NB + HB * h - coff;                     // first real column of the part
      const bool real = c0 + HB > 0;                             // (a split block's first half
      pj[h] = real ? (c0 + pcoff) / HB : 0;                      //  may be front padding only)
      hr[h] = real && c0 < n_rows;
      hm[h] = real && c0 + HB > n_rows;                          // holds mean columns
      any_r = any_r || hr[h];
      any_m = any_m || hm[h];
    }
    const bool fused = prm.spart != nullptr;
    if (any_m) {
      if (!fused) {
  #pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          const int jm = J * NB + 16 * (NW * nt + w) + li - coff - n_rows;
          if (jm >= 0 && jm < n_m) {
  #pragma unroll
            for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int p = pos0 + mt * 16 + lk + 4 * r;
                if (p < pos_end)
                  prm.mu[(long long)(out_base + p) * prm.ld_mu + jm] = acc[mt][nt][r];
              }
          }
        }
      } else {
        // sum_j (z_j - mu_j)^2 lam2_j over this block's mean columns (gpmdm_pf.py:188-192 with
        // var_j = vc / lam2_j factored out; k_obs_ll finishes the likelihood).  A tile whose
        // particles share one filter (always, for a single filter) reads z_j once per column.
        const int Pf = (int)prm.Pf;
        const int f0 = pos0 / Pf, f1 = (min(pos0 + PT, pos_end) - 1) / Pf;   // wave-uniform
  #pragma unroll
        for (int h = 0; h < NH; ++h) {                          // one part at a time (registers)
          double ss[MT][4];
  #pragma unroll
          for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
            for (int r = 0; r < 4; ++r) ss[mt][r] = 0.0;
  #pragma unroll
          for (int nt = h * NTH; nt < (h + 1) * NTH; ++nt) {
            const int jm = J * NB + 16 * (NW * nt + w) + li - coff - n_rows;
            if (jm >= 0 && jm < n_m) {
              const double lam = prm.lam2[jm];
              if (f0 == f1) {
                const double zj = prm.z[(long long)f0 * n_m + jm];
  #pragma unroll
                for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    const double t = zj - acc[mt][nt][r];
                    ss[mt][r] = fma(t * t, lam, ss[mt][r]);
                  }
              } else {
  #pragma unroll
                for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    int p = pos0 + mt * 16 + lk + 4 * r;
                    p = p < pos_end ? p : pos0;
                    const double zz = prm.z[(long long)(p / Pf) * n_m + jm];
                    const double t = zz - acc[mt][nt][r];
                    ss[mt][r] = fma(t * t, lam, ss[mt][r]);
                  }
              }
            }
          }
  #pragma unroll
          for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
            for (int r = 0; r < 4; ++r) {
              double v = ss[mt][r];
              v += __shfl_xor(v, 1);
              v += __shfl_xor(v, 2);
              v += __shfl_xor(v, 4);
              v += __shfl_xor(v, 8);
              if (li == 0) sred[h * NW + w][mt * 16 + lk + 4 * r] = v;
            }
        }
      }
      // mean columns do not enter the quadratic form
  #pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int col = J * NB + 16 * (NW * nt + w) + li - coff;
        if (col >= n_rows) {
  #pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[mt][nt] = (d4){0.0, 0.0, 0.0, 0.0};
        }
      }
    }
    if (any_r) {
      // Sum of squares over the part's R columns.  Front-padding columns (col < 0) have
      // B = 0, so V = 0 there: no mask (mean columns were zeroed above).
  #pragma unroll
      for (int h = 0; h < NH; ++h) {
        if (!hr[h]) continue;
        double qs[MT][4];
  #pragma unroll
        for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
          for (int r = 0; r < 4; ++r) {
            double v = 0.0;
  #pragma unroll
            for (int nt = h * NTH; nt < (h + 1) * NTH; ++nt) v = fma(acc[mt][nt][r], acc[mt][nt][r], v);
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            qs[mt][r] = v;
          }
        if (li == 0) {
  #pragma unroll
          for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
            for (int r = 0; r < 4; ++r) qred[h * NW + w][mt * 16 + lk + 4 * r] = qs[mt][r];
        }
      }
    }
    if (any_r || (any_m && fused)) {
      __syncthreads();
      if (tid < PT) {
        const int p = pos0 + tid;
        if (p < pos_end) {
  #pragma unroll
          for (int h = 0; h < NH; ++h) {
            if (hr[h]) {
              double q = 0.0;
  #pragma unroll
              for (int ww = 0; ww < NW; ++ww) q += qred[h * NW + ww][tid];
              prm.qpart[(long long)pj[h] * prm.ld_q + out_base + p] = q;
            }
            if (hm[h] && fused) {
              double sm = 0.0;
  #pragma unroll
              for (int ww = 0; ww < NW; ++ww) sm += sred[h * NW + ww][tid];
              prm.spart[(long long)pj[h] * prm.ld_q + out_base + p] = sm;
            }
          }
        }
      }
    }
  }
}

template <int DI>
void launch_d(const TileParams& p, bool dyn, hipStream_t stream) {
  const dim3 grid((unsigned)(p.n_j_max * p.tiles_ub));
  const TileGeo g = p.geo;
  // 32 x 512 tiles above d = 12 (GPMDM_TILE_32x512, or wide dynamics images of such a
  // model): particle coordinates from LDS (VAR bit 17) -- in VGPRs they push the
  // 2-workgroup register budget into spills (config-5 shape, d = 16: 850 ms per launch vs
  // 1037 ms; the default 64 x 512 shape: 760 ms; profiles/r02/ablations/tb9, tb10)
  constexpr int kCoordVar = DI > 12 ? kTileCoordLDS : 0;
  if (dyn) {
    // dynamics images: narrow 16 x 256, wide = the observation GP's shape, or a model-wide
    // tile_shape (64 x 256 / 64 x 512)
    if (g.nw == 8)
      hipLaunchKernelGGL((k_gp_tile<DI, true, 0, 8>), grid, dim3(512), 0, stream, p);
    else if (g.mt == 2 && g.ntw == 8)
      hipLaunchKernelGGL((k_gp_tile<DI, true, kCoordVar, 4, 2, 8>), grid, dim3(256), 0, stream, p);
    else if (g.mt == 1)
      hipLaunchKernelGGL((k_gp_tile<DI, true, 0, 4, 1, 4>), grid, dim3(256), 0, stream, p);
    else
      hipLaunchKernelGGL((k_gp_tile<DI, true, 0, 4>), grid, dim3(256), 0, stream, p);
  } else if (g.mt == 2) {
    hipLaunchKernelGGL((k_gp_tile<DI, false, kCoordVar, 4, 2, 8>), grid, dim3(256), 0, stream, p);
  } else if (g.mt == 1 && g.ntw == 8) {
    // 16-row tiles over the 32 x 512 image (small filters, capi_model.hip obs_pick; d <= 12)
    if constexpr (DI <= 12) hipLaunchKernelGGL((k_gp_tile<DI, false, 0, 4, 1, 8>), grid, dim3(256), 0, stream, p);
  } else if (g.mt == 1 && g.ntw == 4) {
    // the 16 x 256 image of small models and filters (capi_model.hip obs_pick; d <= 12)
    if constexpr (DI <= 12) hipLaunchKernelGGL((k_gp_tile<DI, false, 0, 4, 1, 4>), grid, dim3(256), 0, stream, p);
  } else if (g.nw == 8) {
    hipLaunchKernelGGL((k_gp_tile<DI, false, 0, 8>), grid, dim3(512), 0, stream, p);
  } else {
    hipLaunchKernelGGL((k_gp_tile<DI, false, 0, 4>), grid, dim3(256), 0, stream, p);
  }
}

}  // namespace gpmdm
