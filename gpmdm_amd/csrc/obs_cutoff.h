#pragma once
// The observation GP with the opt-in kernel-value cutoff (GPMDM_PF(obs_cutoff=True);
// DESIGN.md §3 "Kernel-value cutoff"): map_x_to_y's variance and the filter's likelihood sum
// (gpmdm.py:923-963, gpmdm_pf.py:170-192) with every kernel value below tau replaced by 0.
//
// One workgroup per particle tile (PT particles), over the whole column range:
//  * the tile's bounding sphere is tested against every K-step's (16 training rows in the
//    image's spatial order, host_image.h): K-steps farther than the cutoff distance hold only
//    values below tau, i.e. zeros after the flush, and are dropped.  The active K-steps, in
//    ascending order, form the list klist;
//  * the R column tiles of the cutoff image are the same 16-row groups (host_image.h
//    CutoffPacker), so R tile t is needed only when K-step t is active (otherwise k_j = 0 on
//    all its columns for every particle of the tile): the tile list is klist followed by the
//    mean tiles.  R tile klist[i] needs list positions 0 .. i (its block triangle), a mean
//    tile every position;
//  * the tile list is cut into chunks of NW x NTW tiles (wave w: chunk tiles w, w + NW, ...),
//    and each chunk runs the dense kernel's K loop (gp_tile.h: generation two positions ahead
//    into an LDS ring, rows staged four ahead, B one position ahead in VGPRs, one barrier per
//    two positions, tiles retiring in phases) over list positions only: every chunk but the
//    first is full whatever the cloud (the partial one first, where it runs the fewest
//    positions), so the MFMAs per generated K-step stay those of the dense kernel however few
//    tiles are active;
//  * q = sum_j k_j V_j, V = K* B over the symmetric image, and S = sum_j (z_j - mu_j)^2 lam2_j
//    (mu = the mean tiles' V) are summed per column tile (its 16 columns by a DPP row
//    reduction) and then over the tiles in list order, by one thread per particle.  An R
//    tile's last list position is its own diagonal K-step, whose K* in the LDS ring are the
//    tile's k_j: its retired accumulators take the products V_j k_j there (no regeneration),
//    and every tile of the chunk is reduced after the chunk's K loop.
// Invariance: a K-step or R tile dropped for one tile composition contributes exact zeros to
// every particle of another composition that includes it (its values are flushed for that
// particle), and the sums run in increasing tile order, so a particle's q and S do not
// depend on which particles share its tile -- nor on the rank that evaluates it
// (tests/test_gpu_obs_cutoff.py: logical shards bitwise one rank).
#include "gp_tile.h"

namespace gpmdm {

// Sum over the 16 lanes of a row (lanes 16 r .. 16 r + 15) by DPP moves (VALU; no LDS traffic):
// quad swaps (xor 1, xor 2), then shifts by 4 and 8 within the row (lane l reads lane l + 4,
// l + 8).  Lane 16 r -- the only lane whose result is used -- receives ((q0 + q1) + (q2 + q3))
// over the row's quads, each quad ((v0 + v1) + (v2 + v3)): exactly the association of the
// xor-1/2/4/8 butterfly at that lane.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xF, 0xF, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32));
}
__device__ __forceinline__ double row16_sum(double v) {
  v += dpp_f64<0xB1>(v);    // quad_perm [1, 0, 3, 2]
  v += dpp_f64<0x4E>(v);    // quad_perm [2, 3, 0, 1]
  v += dpp_f64<0x104>(v);   // row_shl 4
  v += dpp_f64<0x108>(v);   // row_shl 8
  return v;
}

template <int DI, int NW, int MT, int NTW>
__global__ __launch_bounds__(64 * NW, 2) void k_obs_cutoff(const CutoffParams prm) {
  static_assert(NTW <= 8, "a full K-step of B fragments per tile in registers");
  // the generation reads the particle coordinates from LDS instead of VGPRs from d = 4: the
  // chunk loop keeps the epilogue's addresses live beside the accumulators and B fragments,
  // and 2 d VGPRs of coordinates push d >= 4 into spills (inside the K loop at d = 4)
  constexpr bool PLDS = DI > 3;
  constexpr int NT = 64 * NW;
  constexpr int PT = 16 * MT;
  constexpr int TPC = NW * NTW;                              // tiles per chunk
  constexpr int NG = NT / PT;
  constexpr int GV = kBK / NG;
  static_assert(GV * NG == kBK, "generation split");
  constexpr int LDA = (PT + 16) % 32 == 16 ? PT + 16 : PT + 32;
  constexpr int RW = DI + 1;
  constexpr int NRV = kBK * RW;
  constexpr int RPT = (NRV + NT - 1) / NT;
  constexpr int SB = 2, ASL = 2 * SB, RXS = 2 * SB, LOOK = SB, RA = 2 * SB;
  static_assert(TPC * PT <= ASL * kBK * LDA, "per-tile sums alias the K* ring");
  __shared__ double As[ASL][kBK][LDA];
  __shared__ double RX[RXS][RPT * NT];
  __shared__ double tab[64];
  __shared__ unsigned short klist[kMaxCutoffKs];
  // the tile's particles: a2 (2 x kScale x / l) and |x / l|^2 kScale; an odd row pitch so the
  // generation's per-particle reads (PLDS) hit distinct banks
  constexpr int PKW = (DI + 1) % 2 ? DI + 1 : DI + 2;
  __shared__ double PK[PT][PKW];
  __shared__ long long pfil[PT];
  __shared__ double tsph[DI + 1];
  __shared__ int wtot[NW];
  double* const ptile = &As[0][0][0];                         // [TPC][PT], after each chunk's K loop

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lk = lane >> 4;
  constexpr double kScale = kLog2eX64;
  for (int i = tid; i < 64; i += NT) tab[i] = kExp2Tab[i];

  // the workgroup's particle tile and part: whole tiles first, then the split tiles' second
  // parts (the longer ones in the balanced split's usual case), then their first parts
  int tile = (int)blockIdx.x, part = -1;                      // -1: the whole tile
  if (prm.chunk_grid) {
    part = 2 + tile / prm.n_split;
    tile -= (part - 2) * prm.n_split;
  } else if (tile >= prm.n_whole) {
    const int r = tile - prm.n_whole;
    part = r < prm.n_split ? 1 : 0;
    tile = prm.n_whole + (r < prm.n_split ? r : r - prm.n_split);
  }
  const int pos0 = prm.pos_begin + tile * PT;
  const int pos_end = prm.pos_end;
  const int T_R = prm.T_R;

  // ---- this thread's particle (generation role: particle m, rows g + NG s) -------------
  const int m = tid % PT;
  const int g = tid / PT;
  int pos = pos0 + m;
  if (pos >= pos_end) pos = pos0;                             // clamp (results unused)
  const long long prow = prm.perm ? prm.perm[pos] : pos;
  double a2[DI];
  double asq = 0.0;
#pragma unroll
  for (int j = 0; j < DI; ++j) {
    const double xs = prm.X[prow * DI + j] / prm.ls[j];
    asq = fma(xs, xs, asq);
    a2[j] = (2.0 * kScale) * xs;
  }
  asq *= kScale;
  if (g == 0) {
#pragma unroll
    for (int j = 0; j < DI; ++j) PK[m][j] = a2[j];
    PK[m][DI] = asq;
    pfil[m] = prow / prm.Pf;
  }
  __syncthreads();

  // ---- the active K-steps: the tile's bounding sphere (a2 units) against each K-step's ---
  if (tid < DI) {
    double c = 0.0;
    for (int p = 0; p < PT; ++p) c += PK[p][tid];
    tsph[tid] = c * (1.0 / PT);
  }
  __syncthreads();
  if (w == 0) {
    double r2 = 0.0;
    if (lane < PT) {
#pragma unroll
      for (int j = 0; j < DI; ++j) {
        const double t = PK[lane][j] - tsph[j];
        r2 = fma(t, t, r2);
      }
    }
    r2 = wave_max(r2);
    if (lane == 0) tsph[DI] = sqrt(r2) * (1.0 + 1e-12) + 1e-12;
  }
  __syncthreads();
  int n_act;
  {
    constexpr double kInv = 1.0 / (2.0 * kScale);
    const int per = (T_R + NT - 1) / NT;                      // <= 16 (T_R <= 4096, NT >= 256)
    const int k0 = tid * per, k1 = min(k0 + per, T_R);
    const double rt = tsph[DI] * kInv;
    unsigned bits = 0u;
    for (int k = k0; k < k1; ++k) {
      const double* sp = prm.ksph + (long long)k * (DI + 1);
      double d2 = 0.0;
#pragma unroll
      for (int j = 0; j < DI; ++j) {
        const double t = tsph[j] * kInv - sp[j];
        d2 = fma(t, t, d2);
      }
      const double gap = sqrt(d2) - rt - sp[DI];
      // inactive: every value of the K-step is exp(-|x - X_i|^2) < tau for every particle of
      // the tile, i.e. flushed (cut2's margin covers both tests' rounding)
      if (!(gap > 0.0 && gap * gap > prm.cut2)) bits |= 1u << (k - k0);
    }
    const int cnt = __builtin_popcount(bits);
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(incl, off);
      if (lane >= off) incl += y;
    }
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    int base = incl - cnt;
    n_act = 0;
    for (int ww = 0; ww < NW; ++ww) {
      base += ww < w ? wtot[ww] : 0;
      n_act += wtot[ww];
    }
    for (int k = k0, q = base; k < k1; ++k)
      if (bits >> (k - k0) & 1u) klist[q++] = (unsigned short)k;
    n_act = __builtin_amdgcn_readfirstlane(n_act);
  }
  __syncthreads();                                           // klist complete
  const int n_tiles = n_act + prm.T_M;
  // the chunks [c_lo, c_hi) of the tile list this workgroup runs (none: a second part of a
  // tile below two chunks; no early exit, which costs the K loop registers)
  int c_lo = 0, c_hi = (n_tiles + TPC - 1) / TPC;
  if (part >= 0) {
    // chunk grid (part 2 + cfe): chunk c = nc - 1 - cfe alone, as a split at c* = 1 -- chunk 0
    // the first part, a later one a second part; none past the list
    const bool cg = part >= 2;
    const int c = c_hi - 1 - (part - 2);
    const int cs = cg ? 1 : __builtin_amdgcn_readfirstlane(cutoff_split_chunk(n_act, prm.T_M, TPC));
    if (cg) part = c == 0 ? 0 : 1;
    if (part == 0) {
      c_hi = cs;
      if (tid == 0) prm.split[tile - prm.n_whole] = make_int2(n_act, cs);
    } else {
      c_lo = cg ? (c < 0 ? c_hi : c) : cs;
      if (cg && c >= 0) c_hi = c + 1;
    }
  }
  // (the second part's partials: list entry i of particle m at part[(i - r0) ld + o], r0 the
  // first chunk's size; uniform, so it stays out of the K loop's VGPRs)
  const bool second = part == 1;
  const int r0 = __builtin_amdgcn_readfirstlane(cutoff_chunk_begin(1, n_tiles, TPC));
  const long long pbase = __builtin_amdgcn_readfirstlane(pos0 - prm.pos_begin - prm.n_whole * PT);
  auto kat = [&](int i) -> int {                             // the K-step at list position i
    const int ii = i < n_act ? i : n_act - 1;
    return ii >= 0 ? __builtin_amdgcn_readfirstlane((int)klist[ii]) : 0;
  };

  // ---- row staging and K* generation (gp_tile.h's, over list positions) ----------------
  typedef unsigned v2u __attribute__((ext_vector_type(2)));
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)prm.Xrec, (short)0, 0x7fffffff, 0x00020000);
  // the image: one resource, 32-bit byte offsets (the host keeps it below 4 GiB)
  const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)prm.Bt, (short)0, -1, 0x00020000);
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
    for (int k = 0; k < RPT; ++k) RX[buf][tid + NT * k] = rr[k];
  };
  auto gen = [&](int rb, double (&v)[GV]) {
#pragma unroll
    for (int s = 0; s < GV; ++s) {
      const int r = g + NG * s;
      const double* row = &RX[rb][r * RW];
      double x = -(asq + row[DI]);
#pragma unroll
      for (int j = 0; j < DI; ++j) x = fma(PLDS ? PK[m][j] : a2[j], row[j], x);
      const double e = exp2_64(x, tab);
      v[s] = x < prm.t_cut ? 0.0 : e;                         // the cutoff: below tau, exactly 0
    }
  };
  auto store = [&](int buf, const double (&v)[GV]) {
#pragma unroll
    for (int s = 0; s < GV; ++s) As[buf][g + NG * s][m] = v[s];
  };

  d4 acc[MT][NTW];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
  __shared__ double qrun[PT], srun[PT];                       // running sums per particle
  if (tid < PT) {
    qrun[tid] = 0.0;
    srun[tid] = 0.0;
  }

  for (int c = c_lo; c < c_hi; ++c) {
    // ---- this wave's tiles of the chunk: list index i = c0 + NW nt + w < cend ----------
    // (the partial chunk first: cutoff_chunk_begin)
    const int c0 = __builtin_amdgcn_readfirstlane(cutoff_chunk_begin(c, n_tiles, TPC));
    const int cend = __builtin_amdgcn_readfirstlane(cutoff_chunk_begin(c + 1, n_tiles, TPC));
    // kend: list positions the tile multiplies; tb: byte offset of its data in the image (a
    // retired tile's prefetch past its diagonal reads the following tiles' data, never past
    // the image: every tile is followed by at least T_R K-steps of mean tiles)
    auto kend = [&](int nt) -> int {
      const int i = c0 + NW * nt + w;
      return i >= cend ? 0 : (i < n_act ? i + 1 : n_act);
    };
    unsigned tb[NTW];
    int T1 = 0;
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      const int i = c0 + NW * nt + w;
      const bool valid = i < cend;
      if (valid) T1 = nt + 1;
      const int t = !valid ? 0 : (i < n_act ? kat(i) : T_R + (i - n_act));
      tb[nt] = __builtin_amdgcn_readfirstlane((unsigned)(prm.toff[t] * 8));
    }
    const int last = cend - 1;
    const int npos = last < n_act ? last + 1 : n_act;          // list positions of this chunk
    // The K-steps of list positions [kb0, kb0 + 64) in a VGPR window (lane j: position kb0 + j):
    // in the K loop a K-step is one v_readlane, not an LDS round trip in front of the B loads
    // and the row staging (refilled every 64 - RA positions)
    int kb0 = 0, kw0 = 0;
    auto kwin = [&](int base) {
      kb0 = base;
      const int x0 = min(base + lane, n_act - 1);
      kw0 = x0 >= 0 ? (int)klist[x0] : 0;
    };
    auto katw = [&](int x) -> int {                          // kb0 <= x < kb0 + 64
      return __builtin_amdgcn_readlane(kw0, x - kb0);
    };
    kwin(0);
    // B fragments of list position i, sub-steps 2h, 2h + 1, for every tile (one contiguous
    // KiB per load instruction)
    auto loadB = [&](int i, int h, double (&bb)[4 * NTW]) {
      const unsigned kb = (unsigned)katw(i) * 2048u;
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const v4u x = __builtin_amdgcn_raw_buffer_load_b128(brsrc, (unsigned)lane * 16u, (int)(tb[nt] + kb + 1024u * h), 0);
        bb[(2 * h) * NTW + nt] = __builtin_bit_cast(double, (unsigned long long)x.x | ((unsigned long long)x.y << 32));
        bb[(2 * h + 1) * NTW + nt] = __builtin_bit_cast(double, (unsigned long long)x.z | ((unsigned long long)x.w << 32));
      }
    };
    auto step = [&](auto t0c, auto t1c, int i, bool retire, double (&bb)[4 * NTW]) {
      constexpr int T0 = decltype(t0c)::value, T1c = decltype(t1c)::value;
      const int buf = i & (ASL - 1);
      if (i + RA >= kb0 + 64) kwin(i);                       // (uniform; every 60 positions)
      double v[GV];
      double rr[RPT];
      load_rows(katw(i + RA), rr);
      gen((i + LOOK) & (RXS - 1), v);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        double af[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) af[mt] = As[buf][kk * 4 + lk][mt * 16 + li];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = T0; nt < T1c; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[mt], bb[kk * NTW + nt], acc[mt][nt], 0, 0, 0);
        if (kk & 1) loadB(i + 1, kk >> 1, bb);               // the next position's sub-steps
      }
      if (retire) {
        // tile T0's diagonal position: this K-step's rows are the tile's columns, so the K*
        // just multiplied are its k_j (the flushed values, as generated).  The tile's
        // accumulators are final from here on (it has retired), so they take the products
        // V_j k_j in place; their reduction over the 16 columns waits for the chunk's end,
        // with every other tile's (no reduction, no LDS partials, no extra barrier work
        // inside the K loop)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[mt][T0][r] *= As[buf][li][mt * 16 + lk + 4 * r];
      }
      store((i + LOOK) & (ASL - 1), v);
      store_rows((i + RA) & (RXS - 1), rr);
      if (i % SB == SB - 1) __syncthreads();
    };

    double bb[4 * NTW];
    {
      double rr[RPT];
#pragma unroll
      for (int j = 0; j < RA; ++j) {
        load_rows(katw(j), rr);
        store_rows(j, rr);
      }
    }
    __syncthreads();
    {
      double v[GV];
#pragma unroll
      for (int j = 0; j < LOOK; ++j) {
        gen(j & (RXS - 1), v);
        store(j, v);
      }
      loadB(0, 0, bb);
      loadB(0, 1, bb);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();

    int i = 0;
    static_for<1, NTW + 1>([&](auto t1c) {
      constexpr int T1c = decltype(t1c)::value;
      if (T1 == T1c) {
        static_for<0, T1c>([&](auto t0c) {
          constexpr int T0 = decltype(t0c)::value;
          const int e = kend(T0);
          const bool rt = c0 + NW * T0 + w < n_act;          // an R tile: retires at e - 1
          for (; i < npos && i < e; ++i)
            step(std::integral_constant<int, T0>{}, std::integral_constant<int, T1c>{}, i, rt && i == e - 1, bb);
        });
      }
    });
    for (; i < npos; ++i) {                                  // other waves' tiles: generate only
      if (i + RA >= kb0 + 64) kwin(i);
      double v[GV];
      double rr[RPT];
      load_rows(katw(i + RA), rr);
      gen((i + LOOK) & (RXS - 1), v);
      store((i + LOOK) & (ASL - 1), v);
      store_rows((i + RA) & (RXS - 1), rr);
      if (i % SB == SB - 1) __syncthreads();
    }
    if (prm.sp_stats && lane == 0) {
      unsigned run = 0;
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) run += (unsigned)kend(nt);
      atomicAdd(prm.sp_stats + 0, (unsigned long long)run * MT);
    }

    __syncthreads();                                         // every wave is done with As
    // ---- the chunk's per-tile sums into LDS (aliasing the K* ring), then in list order ------
    // R tiles: sum_j V_j k_j (the products formed at the diagonal); mean tiles:
    // (z_j - mu_j)^2 lam2_j over the tile's columns (gpmdm_pf.py:188-192 with var_j = vc / lam2_j
    // factored out; k_obs_ll finishes the likelihood); each reduced over its 16 columns (lanes li)
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      const int i2 = c0 + NW * nt + w;
      if (i2 >= cend) continue;                              // (wave-uniform)
      if (i2 < n_act) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int pr = mt * 16 + lk + 4 * r;
            const double v = row16_sum(acc[mt][nt][r]);
            if (li == 0) ptile[(NW * nt + w) * PT + pr] = v;
          }
      } else {
        const int jm = 16 * (i2 - n_act) + li;
        const bool real = jm < prm.n_m;
        const double lam = real ? prm.lam2[jm] : 0.0;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int pr = mt * 16 + lk + 4 * r;
            const double t = real ? prm.z[pfil[pr] * prm.n_m + jm] - acc[mt][nt][r] : 0.0;
            const double v = row16_sum((t * t) * lam);
            if (li == 0) ptile[(NW * nt + w) * PT + pr] = v;
          }
      }
    }
    __syncthreads();
    if (tid < PT) {
      const int ns = cend - c0;
      if (second) {                                          // a second part: the partials
        for (int s = 0; s < ns; ++s) prm.part[pbase + (long long)(c0 + s - r0) * prm.ld_part + tid] = ptile[s * PT + tid];
      } else {
        double qa = qrun[tid], sa = srun[tid];
        for (int s = 0; s < ns; ++s) {
          if (c0 + s < n_act)
            qa += ptile[s * PT + tid];
          else
            sa += ptile[s * PT + tid];
        }
        qrun[tid] = qa;
        srun[tid] = sa;
      }
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) acc[mt][nt] = (d4){0.0, 0.0, 0.0, 0.0};
    __syncthreads();                                         // before the next chunk's ring
  }

  if (part != 1 && tid < PT && pos0 + tid < pos_end) {
    prm.q[pos0 + tid - prm.pos_begin] = qrun[tid];
    prm.S[pos0 + tid - prm.pos_begin] = srun[tid];
  }
  if (prm.sp_stats && part != 1 && tid == 0) {
    {
      // the dense kernel's MFMA groups for this tile: every R tile to its diagonal, every
      // mean tile over all K-steps
      const unsigned long long dense = (unsigned long long)T_R * (T_R + 1) / 2 + (unsigned long long)prm.T_M * T_R;
      atomicAdd(prm.sp_stats + 1, dense * MT);
    }
  }
}

// 32-particle tiles of 4 waves x 8 column tiles up to d = 8, 64-particle tiles of 8 waves x 4
// above (the dense kernel's shapes; the particle coordinates push 32 x 512 into spills)
template <int DI>
bool launch_cut_d(const CutoffParams& p, hipStream_t s) {
  const long long n = (long long)p.pos_end - p.pos_begin;
  if (n <= 0) return true;
  constexpr int PT = DI <= 8 ? 32 : 64;
  // grid: the whole tiles, then two workgroups per split tile (capi_frame.hip sets n_whole +
  // n_split = the tile count)
  const unsigned grid = p.chunk_grid ? (unsigned)(p.n_chunk_max * p.n_split) : (unsigned)(p.n_whole + 2 * p.n_split);
  if (p.n_whole < 0 || p.n_split < 0 || (long long)(p.n_whole + p.n_split) * PT < n ||
      (long long)(p.n_whole + p.n_split - 1) * PT >= n || (p.n_split > 0 && (!p.part || !p.split)))
    return false;
  if (p.chunk_grid && (p.n_whole != 0 || p.n_split <= 0 || p.n_chunk_max <= 0 ||
                       (long long)p.n_chunk_max * cutoff_tile_list_chunk() < p.T_R + p.T_M))
    return false;
  if constexpr (DI <= 8)
    hipLaunchKernelGGL((k_obs_cutoff<DI, 4, 2, 8>), dim3(grid), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((k_obs_cutoff<DI, 8, 4, 4>), dim3(grid), dim3(512), 0, s, p);
  return true;
}

// workgroups of the cutoff kernel resident per CU at d
template <int DI>
int cut_blocks_per_cu_d() {
  int b = 0;
  hipError_t e;
  if constexpr (DI <= 8)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, reinterpret_cast<const void*>(&k_obs_cutoff<DI, 4, 2, 8>), 256, 0);
  else
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, reinterpret_cast<const void*>(&k_obs_cutoff<DI, 8, 4, 4>), 512, 0);
  return e == hipSuccess && b > 0 ? b : 1;
}

}  // namespace gpmdm
