#pragma once
// A/B laboratory of the fused GP tile (tools/microbench/tile_bench.hip): the production
// kernel of gpmdm_amd/csrc/gp_tile.h with every experiment switch measured against it
// (DESIGN.md §3 and profiles/r0*_ablations/).  VAR = 0 is the production path (plus the
// FLAGS of gp_tile.h at the same bit, 17); the other bits select the variants below.
// Not part of libgpmdm_hip.so.  Variants that needed data the library no longer carries
// (VAR bit 19: separate Xs / Xsq arrays) read the lab's own SegDesc fields below.
#include "../../gpmdm_amd/csrc/gp_tile.h"

namespace gpmdm {

struct LabSegDesc {               // SegDesc + the separate arrays of VAR bit 19
  const double* Xs;               // n_rows x d : training inputs / lengthscales
  const double* Xsq;              // n_rows     : |Xs_i|^2 * 64/ln2
  const double* Xrec;
  const double* Hf;
  const double* Bf;
  int n_rows;
  int n_m;
  int n_j;
  int coff;
};

struct LabParams {                // TileParams + the lab's extra inputs
  LabSegDesc seg[kMaxSeg];
  int n_seg;
  int tiles_ub;
  int n_j_max;
  TileGeo geo;
  const int* seg_pos_begin;
  const int* seg_pos_end;
  const int* seg_out_base;
  const int* seg_tile_start;
  const int* perm;
  const double* X;
  double ls[kMaxD];
  double* qpart;
  long long ld_q;
  double* mu;
  long long ld_mu;
  double* spart;
  const double* rec128;           // VAR bit 22: row records scaled by 128/ln2
  const double* z;
  const double* lam2;
  long long Pf;
  // K* cache (VAR bits 28/29): the full-K block's workgroups store each K-step's A
  // fragments here (tile-major, fragment order); the other blocks' workgroups, launched
  // after them, load them instead of generating K* again.
  double* kcache;
  int j_skip;                     // blocks skipped from the top: J = n_j_max - 1 - j_skip - b / tiles_ub
};

// 2^(j/128), j = 0..127 (correctly rounded).
static __constant__ double kExp2Tab128[128] = {
    1.0, 1.0054299011128027, 1.0108892860517005, 1.016378314910953,
    1.0218971486541166, 1.0274459491187637, 1.0330248790212284, 1.0386341019613787,
    1.0442737824274138, 1.0499440858006872, 1.0556451783605572, 1.061377227289262,
    1.0671404006768237, 1.0729348675259756, 1.0787607977571199, 1.0846183622133092,
    1.0905077326652577, 1.0964290818163769, 1.102382583307841, 1.1083684117236787,
    1.1143867425958924, 1.1204377524096067, 1.1265216186082418, 1.1326385195987192,
    1.1387886347566916, 1.1449721444318042, 1.1511892299529827, 1.1574400736337511,
    1.1637248587775775, 1.1700437696832502, 1.1763969916502812, 1.182784710984341,
    1.189207115002721, 1.1956643920398273, 1.202156731452703, 1.2086843236265816,
    1.215247359980469, 1.2218460329727576, 1.22848053610687, 1.2351510639369334,
    1.241857812073484, 1.2486009771892048, 1.255380757024691, 1.2621973503942507,
    1.2690509571917332, 1.275941778396392, 1.2828700160787783, 1.2898358734066657,
    1.2968395546510096, 1.3038812651919358, 1.3109612115247644, 1.318079601266064,
    1.3252366431597413, 1.3324325470831615, 1.339667524053303, 1.3469417862329458,
    1.3542555469368927, 1.3616090206382248, 1.3690024229745905, 1.3764359707545302,
    1.383909881963832, 1.3914243757719262, 1.3989796725383112, 1.4065759938190154,
    1.4142135623730951, 1.4218926021691656, 1.42961333839197, 1.4373759974489824,
    1.4451808069770467, 1.4530279958490526, 1.460917794180647, 1.4688504333369818,
    1.4768261459394993, 1.4848451658727524, 1.4929077282912648, 1.5010140696264256,
    1.5091644275934228, 1.5173590411982147, 1.5255981507445384, 1.533881997840956,
    1.5422108254079407, 1.550584877685, 1.559004400237837, 1.567469639965553,
    1.5759808451078865, 1.5845382652524937, 1.593142151342267, 1.6017927556826934,
    1.6104903319492543, 1.6192351351948637, 1.6280274218573478, 1.6368674497669644,
    1.645755478153965, 1.6546917676561943, 1.6636765803267364, 1.6727101796415966,
    1.681792830507429, 1.6909247992693053, 1.7001063537185235, 1.709337763100463,
    1.718619298122478, 1.7279512309618377, 1.7373338352737062, 1.746767386199169,
    1.7562521603732995, 1.7657884359332727, 1.7753764925265212, 1.785016611318935,
    1.7947090750031072, 1.804454167806624, 1.8142521755003989, 1.8241033854070534,
    1.8340080864093424, 1.843966568958626, 1.8539791250833855, 1.864046048397789,
    1.8741676341103, 1.8843441790323345, 1.8945759815869656, 1.9048633418176741,
    1.9152065613971474, 1.925605943636125, 1.9360617934922943, 1.9465744175792332,
    1.9571441241754002, 1.9677712232331759, 1.978456026387951, 1.9891988469672663
};

// 2^(j/256), j = 0..255 (correctly rounded).
static __constant__ double kExp2Tab256[256] = {
    1.0, 1.0027112750502025, 1.0054299011128027, 1.0081558981184175,
    1.0108892860517005, 1.0136300849514894, 1.016378314910953, 1.019133996077738,
    1.0218971486541166, 1.0246677928971357, 1.0274459491187637, 1.030231637686041,
    1.0330248790212284, 1.0358256936019572, 1.0386341019613787, 1.041450124688316,
    1.0442737824274138, 1.0471050958792898, 1.0499440858006872, 1.0527907730046264,
    1.0556451783605572, 1.0585073227945128, 1.061377227289262, 1.0642549128844645,
    1.0671404006768237, 1.0700337118202419, 1.0729348675259756, 1.075843889062791,
    1.0787607977571199, 1.0816856149932152, 1.0846183622133092, 1.0875590609177697,
    1.0905077326652577, 1.0934643990728858, 1.0964290818163769, 1.099401802630222,
    1.102382583307841, 1.1053714457017412, 1.1083684117236787, 1.1113735033448175,
    1.1143867425958924, 1.1174081515673693, 1.1204377524096067, 1.12347556733302,
    1.1265216186082418, 1.129575928566288, 1.1326385195987192, 1.1357094141578055,
    1.1387886347566916, 1.1418762039695616, 1.1449721444318042, 1.148076478840179,
    1.1511892299529827, 1.154310420590216, 1.1574400736337511, 1.1605782120274988,
    1.1637248587775775, 1.1668800369524817, 1.1700437696832502, 1.1732160801636373,
    1.1763969916502812, 1.1795865274628758, 1.182784710984341, 1.1859915656609938,
    1.189207115002721, 1.1924313825831512, 1.1956643920398273, 1.1989061670743806,
    1.202156731452703, 1.2054161090051239, 1.2086843236265816, 1.2119613992768012,
    1.215247359980469, 1.2185422298274085, 1.2218460329727576, 1.2251587936371455,
    1.22848053610687, 1.2318112847340759, 1.2351510639369334, 1.2384998981998165,
    1.241857812073484, 1.245224830175258, 1.2486009771892048, 1.2519862778663162,
    1.255380757024691, 1.2587844395497165, 1.2621973503942507, 1.2656195145788063,
    1.2690509571917332, 1.2724917033894028, 1.275941778396392, 1.2794012075056693,
    1.2828700160787783, 1.2863482295460256, 1.2898358734066657, 1.2933329732290895,
    1.2968395546510096, 1.3003556433796506, 1.3038812651919358, 1.3074164459346773,
    1.3109612115247644, 1.3145155879493546, 1.318079601266064, 1.3216532776031575,
    1.3252366431597413, 1.3288297242059544, 1.3324325470831615, 1.3360451382041458,
    1.339667524053303, 1.3432997311868353, 1.3469417862329458, 1.3505937158920345,
    1.3542555469368927, 1.3579273062129011, 1.3616090206382248, 1.365300717204012,
    1.3690024229745905, 1.3727141650876684, 1.3764359707545302, 1.380167867260238,
    1.383909881963832, 1.387662042298529, 1.3914243757719262, 1.3951969099662003,
    1.3989796725383112, 1.4027726912202048, 1.4065759938190154, 1.4103896082172707,
    1.4142135623730951, 1.4180478843204152, 1.4218926021691656, 1.4257477441054942,
    1.42961333839197, 1.433489413367789, 1.4373759974489824, 1.4412731191286257,
    1.4451808069770467, 1.449099089642035, 1.4530279958490526, 1.4569675544014438,
    1.460917794180647, 1.4648787441464057, 1.4688504333369818, 1.4728328908693675,
    1.4768261459394993, 1.4808302278224719, 1.4848451658727524, 1.488870989524397,
    1.4929077282912648, 1.4969554117672355, 1.5010140696264256, 1.5050837316234065,
    1.5091644275934228, 1.5132561874526098, 1.5173590411982147, 1.5214730189088146,
    1.5255981507445384, 1.529734466947287, 1.533881997840956, 1.5380407738316568,
    1.5422108254079407, 1.5463921831410214, 1.550584877685, 1.5547889397770887,
    1.559004400237837, 1.5632312899713576, 1.567469639965553, 1.5717194812923414,
    1.5759808451078865, 1.5802537626528246, 1.5845382652524937, 1.588834384317164,
    1.593142151342267, 1.597461597908627, 1.6017927556826934, 1.606135656416771,
    1.6104903319492543, 1.6148568142048607, 1.6192351351948637, 1.6236253270173289,
    1.6280274218573478, 1.632441451987275, 1.6368674497669644, 1.6413054476440063,
    1.645755478153965, 1.6502175739206177, 1.6546917676561943, 1.6591780921616162,
    1.6636765803267364, 1.6681872651305825, 1.6727101796415966, 1.6772453570178785,
    1.681792830507429, 1.6863526334483934, 1.6909247992693053, 1.6955093614893326,
    1.7001063537185235, 1.7047158096580513, 1.709337763100463, 1.713972247929926,
    1.718619298122478, 1.723278947746274, 1.7279512309618377, 1.732636182022311,
    1.7373338352737062, 1.7420442251551564, 1.746767386199169, 1.7515033530318782,
    1.7562521603732995, 1.761013843037584, 1.7657884359332727, 1.7705759740635547,
    1.7753764925265212, 1.7801900265154245, 1.785016611318935, 1.789856282321401,
    1.7947090750031072, 1.7995750249405351, 1.804454167806624, 1.809346539371032,
    1.8142521755003989, 1.8191711121586085, 1.8241033854070534, 1.8290490314048973,
    1.8340080864093424, 1.8389805867758937, 1.843966568958626, 1.8489660695104508,
    1.8539791250833855, 1.8590057724288205, 1.864046048397789, 1.8690999899412386,
    1.8741676341103, 1.8792490180565602, 1.8843441790323345, 1.8894531543909392,
    1.8945759815869656, 1.8997126981765553, 1.9048633418176741, 1.9100279502703899,
    1.9152065613971474, 1.9203992131630474, 1.925605943636125, 1.930826790987627,
    1.9360617934922943, 1.9413109895286405, 1.9465744175792332, 1.9518521162309783,
    1.9571441241754002, 1.9624504802089273, 1.9677712232331759, 1.9731063922552343,
    1.978456026387951, 1.9838201648502194, 1.9891988469672663, 1.9945921121709402
};

// exp2_64 on a lane-replicated table: entry j of this lane's copy at tabl[j * TREP].
template <int TREP>
__device__ __forceinline__ double exp2_64r(double t, const double* tabl) {
  const double n = __builtin_rint(t);
  const double f = t - n;
  double p = fma(f, 1.2417843701716925e-12, 5.732851688640402e-10);
  p = fma(p, f, 2.1173137155464776e-07);
  p = fma(p, f, 5.86490495505617e-05);
  p = fma(p, f, 0.010830424696249145);
  p *= f;                                                          // 2^(f/64) - 1
  const int ni = (int)n;
  const unsigned jj = __builtin_amdgcn_ubfe((unsigned)ni, 0u, 6u);   // ni & 63 (keeps v_lshl_add)
  const double tj = tabl[jj * TREP];
  return ldexp(fma(tj, p, tj), ni >> 6);
}

// Generalised table exp for the A/B variants (VAR bits 21-23): 2^(t / S) with S = 64 or 128
// table entries, the integer part of the exponent reduced by `ioff` (a per-particle integer
// folded out of t, see FOLD), and the final power of two applied by ldexp or by an integer
// add to the exponent field (clamped at 2^-1022: a value below that comes out as ~2^-1022
// instead of 0, which only ever multiplies zero-padded or negligible terms).
// S = 128: |f| <= 1/2 in units of 1/128, 2^(f/128) - 1 = f q(f) with q a degree-3 fit
// (least squares on Chebyshev nodes in long double; relative error 1.5e-16).
template <int S, bool IEXP>
__device__ __forceinline__ double exp2_gen(double t, const double* tab, int ioff) {
  const double n = __builtin_rint(t);
  const double f = t - n;
  double p;
  if constexpr (S == 128) {
    double q = fma(f, 3.583032206604434e-11, 2.6466431146364605e-08);
    q = fma(q, f, 1.4662262387641965e-05);
    q = fma(q, f, 0.00541521234812427);
    p = f * q;
  } else {
    p = fma(f, 1.2417843701716925e-12, 5.732851688640402e-10);
    p = fma(p, f, 2.1173137155464776e-07);
    p = fma(p, f, 5.86490495505617e-05);
    p = fma(p, f, 0.010830424696249145);
    p *= f;
  }
  const int ni = (int)n - ioff;
  constexpr int SH = S == 128 ? 7 : 6;
  const double tj = tab[ni & (S - 1)];
  const double r = fma(tj, p, tj);
  if constexpr (IEXP) {
    const int e = max(ni >> SH, -1022);
    return __hiloint2double(__double2hiint(r) + (e << 20), __double2loint(r));
  } else {
    return ldexp(r, ni >> SH);
  }
}

// exp(x) for t = x 256 / ln 2 <= ~0 (the kernel-value exponent, pre-scaled like exp2_64).
// Fewer and cheaper VALU ops than exp2_64 (FP64 VALU and FP64 MFMA share the SIMD's issue,
// tools/microbench/mix_probe.hip): no v_rndne/v_cvt/v_ldexp.
//   t >= -1022*256 (clamp: below that exp(x) < 2^-1022 and the result is 2^-1022-ish,
//     negligible next to the unit diagonal instead of an exact 0);
//   s = t + 1.5*2^52 rounds t to the nearest integer n, whose two's complement sits in the
//     low word of s; f = t - (s - 1.5*2^52), |f| <= 1/2 (exact);
//   2^(f/256) - 1 by a degree-4 Taylor polynomial (truncation < 4e-17);
//   2^(n/256) = table[n & 255] * 2^(n >> 8), the power of two added to the exponent field.
constexpr double kLog2eX256 = 4.0 * kLog2eX64;      // 256 / ln 2 (exactly 4x: rows arrive x64-scaled)
constexpr double kExpC1 = 0.0027076061740622863;   // (ln2/256)^k / k!
constexpr double kExpC2 = 3.6655655969101062e-06;
constexpr double kExpC3 = 3.3083026805413713e-09;
constexpr double kExpC4 = 2.239395190875157e-12;

__device__ __forceinline__ double exp2_256(double t, const double* tab) {
  t = fmax(t, -261632.0);
  const double s = t + 6755399441055744.0;
  const int ni = __double2loint(s);
  const double f = t - (s - 6755399441055744.0);
  double p = fma(f, kExpC4, kExpC3);
  p = fma(p, f, kExpC2);
  p = fma(p, f, kExpC1);
  p *= f;
  const double tj = tab[ni & 255];
  const double r = fma(tj, p, tj);
  return __hiloint2double(__double2hiint(r) + ((ni >> 8) << 20), __double2loint(r));
}

// exp2_64 without v_rndne/v_cvt/v_ldexp: the 64-entry table (lanes hitting one entry are
// LDS broadcasts) with the magic-number rounding and exponent-field insertion of exp2_256.
__device__ __forceinline__ double exp2_64m(double t, const double* tab) {
  t = fmax(t, -65408.0);                                    // -1022 * 64
  const double s = t + 6755399441055744.0;
  const int ni = __double2loint(s);
  const double f = t - (s - 6755399441055744.0);
  double p = fma(f, 1.2417843701716925e-12, 5.732851688640402e-10);
  p = fma(p, f, 2.1173137155464776e-07);
  p = fma(p, f, 5.86490495505617e-05);
  p = fma(p, f, 0.010830424696249145);
  p *= f;
  const double tj = tab[ni & 63];
  const double r = fma(tj, p, tj);
  return __hiloint2double(__double2hiint(r) + ((ni >> 6) << 20), __double2loint(r));
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
//   bit 8: exp2_256 (256-entry table, no rndne/cvt/ldexp) instead of exp2_64
//   bit 9: exp2_64m (64-entry table, no rndne/cvt/ldexp)
//   bit 10: A/B -- conditional row staging (only the NRV record threads load and store)
//   bit 11: A/B -- no vmcnt(0) drain after the prologue
//   bit 12: generation split across the sub-steps + sched_group_barrier MFMA/VALU interleave
//   bit 13: generation split across the sub-steps (no sched_group_barrier)
//   bit 14: A/B -- B fragments by flat global loads instead of buffer loads
//   bit 15: A/B -- one barrier per K-step (2-slot rings) instead of one per two K-steps
//   bit 16: A/B -- one barrier per four K-steps (8-slot rings)
//   bit 17: particle coordinates from LDS in the generation (see PLDS)
//   bit 18: A/B -- lane-replicated exp table (no LDS bank conflicts; one more integer
//           VALU per value for the address) instead of one shared 64-entry table
//           (measured: conflicts 16.4M -> 0 cycles per launch, time +0.4%)
//   bit 19: A/B -- training rows staged from the separate Xs / Xsq arrays by global loads
//           instead of row records by buffer loads (measured: records -1.1%)
//   bit 20: A/B -- K loop unrolled by 4 with compile-time ring slots (LDS offsets as
//           instruction immediates: -4.5 VALU per K-step, 2.7x code; measured: no gain)
//   bit 21: FOLD -- |x_p / l|^2 leaves the per-value exponent: its integer part (in table
//           units) is subtracted from the exponent as an integer, its fraction becomes a
//           per-particle factor c_p = 2^(-frac / S) applied to the tile's rows in the
//           epilogue (one fp64 add fewer per kernel value)
//   bit 22: 128-entry exp table with a degree-4 polynomial (one fp64 fma fewer per value;
//           the row records' |Xs|^2 must then be scaled by 128/ln2, TileParams::rec128)
//   bit 23: final power of two by an integer add to the exponent field (clamped) instead
//           of v_ldexp_f64
//   bit 24: three workgroups per CU (register cap 168: small shapes, e.g. 16x512, 32x384)
//   bit 25: GEN2 -- generate two K-steps' values (4 interleaved exp chains per thread) on
//           even K-steps and none on odd ones (same VALU, half the exposed chain latency)
//   bit 26: SPEC -- wave-specialised workgroup: NW/2 MFMA waves (the column geometry of an
//           NW/2-wave shape) and NW/2 producer waves that stage rows and generate K* two
//           K-steps ahead; no MFMA wave ever issues an exp chain (one workgroup per CU)
//   bit 27: PRIO -- s_setprio 1 around a K-step's MFMAs, 0 around its generation (the
//           SIMD arbiter then prefers the other wave's MFMAs while one wave generates)
//   bit 28: KPROD -- K* cache producer (launched on the full-K block only): as production,
//           and every A fragment the workgroup multiplies is also stored to prm.kcache
//           (wave w stores sub-step w of each K-step: one 1 KiB buffer store per K-step)
//   bit 29: KCONS -- K* cache consumer (the other blocks, launched after the producer): no
//           generation, no row staging, no LDS ring and no barrier in the K loop; the A
//           fragments stream from prm.kcache into VGPRs one K-step ahead, like B.  The
//           values are the producer's, so the results are bitwise production's.
//
// Geometry: NW waves; each wave owns MT x NTW tiles of 16 x 16 (16 MT particles x 16 NTW
// columns), so a workgroup covers PT = 16 MT particles x NB = 16 NTW NW columns.  K* costs
// the same per generated value whatever the geometry, so generation per MFMA falls as
// 1 / NB: (MT, NTW) = (4, 4) is 64 x 256, (2, 8) is 32 x 512 at the same accumulator
// count (128 VGPRs) and MFMA work per K-step, with half the K* values and A-fragment reads
// and twice the B fragments per K-step.
template <int DI, bool DYN, int VAR = 0, int NW = 4, int MT = 4, int NTW = 4>
__global__ __launch_bounds__(64 * NW, (DI <= 16 && !(VAR & 67108864) ? ((VAR & 16777216) ? 3 : 2) : 1)) void k_gp_tile_lab(const LabParams prm) {
  static_assert(MT == 1 || MT == 2 || MT == 4, "MT");
  static_assert(NTW == 4 || NTW == 6 || NTW == 8 || NTW == 16, "NTW");
  // B fragments in flight: BR sub-steps (a full K-step, 4, for NTW <= 8; 2 for NTW = 16,
  // whose full K-step of fragments would not fit next to 128 accumulator VGPRs)
  constexpr int BR = NTW >= 16 ? 2 : 4;
  // tiles retire in groups of RG (NTW = 16: 8 phase groups instead of 16, so the K loop has
  // 36 phase variants rather than 136; a group runs until its last tile's diagonal)
  constexpr int RG = NTW >= 16 ? 2 : 1;
  constexpr bool SPEC = (VAR & 67108864) != 0;
  static_assert(!SPEC || NW == 8, "SPEC: 4 MFMA + 4 producer waves");
  constexpr bool KPROD = (VAR & 268435456) != 0;
  constexpr bool KCONS = (VAR & 536870912) != 0;
  static_assert(!(KPROD && KCONS) && !((KPROD || KCONS) && (SPEC || DYN)), "K* cache: observation GP only");
  constexpr int NWM = SPEC ? NW / 2 : NW;                    // MFMA waves
  constexpr int NT = 64 * NW;                                // threads
  constexpr int NTG = SPEC ? 64 * (NW - NWM) : NT;           // generation / row-staging threads
  constexpr int PT = 16 * MT;                                // particles per tile
  constexpr int NB = 16 * NTW * NWM;                         // columns per block
  constexpr int WS = 256 * NTW;                              // fragment doubles per wave per K-step
  constexpr int FS = NWM * WS;                               // fragment doubles per K-step
  constexpr int NG = NTG / PT;                               // generation row groups
  constexpr int GV = kBK / NG;                               // K* values per thread per K-step
  static_assert(GV * NG == kBK, "generation split");
  constexpr int LDA = PT + 16;                               // rows k, k+1 land 32 banks apart
  constexpr int RW = DI + 1;                                 // row record: Xs[DI], |Xs|^2
  constexpr int NRV = kBK * RW;                              // row values per K-step
  constexpr int RPT = (NRV + NTG - 1) / NTG;                 // row values per thread
  // LDS rings.  Default: one barrier per two K-steps (after odd ones), K* generated
  // two K-steps ahead into 4 slots, rows staged four ahead into 4 slots -- a slot is
  // rewritten only after a barrier that follows its last read, and read only after a
  // barrier that follows its write.  VAR bit 15 (A/B): one barrier per K-step, K* one ahead
  // into 2 slots, rows two ahead into 2 slots.  (obs tile -0.6%, tile_bench; four K-steps
  // per barrier gains nothing more and doubles the LDS rings)
  // General rule for S K-steps per barrier (after steps with ks % S == S-1): lookahead
  // LOOK >= S, K* slots >= LOOK + S, row lookahead RA >= LOOK + S, row slots >= RA - LOOK + S.
  // VAR bit 16 (A/B): S = 4.
  constexpr int SB = (VAR & 32768) ? 1 : ((VAR & 65536) ? 4 : 2);   // K-steps per barrier
  constexpr int ASL = 2 * SB;                                // K* slots
  constexpr int RXS = 2 * SB;                                // row-record slots
  constexpr int LOOK = SB;                                   // generation lookahead (K-steps)
  constexpr int RA = 2 * SB;                                 // row staging lookahead
  __shared__ double As[ASL][kBK][LDA];
  __shared__ double RX[RXS][RPT * NTG];                       // row records, then padding
  constexpr bool E256 = (VAR & 256) != 0;
  constexpr bool FOLD = (VAR & 2097152) != 0;
  constexpr bool T128 = (VAR & 4194304) != 0;
  constexpr bool IEXP = (VAR & 8388608) != 0;
  constexpr bool GENX = FOLD || T128 || IEXP;                 // exp2_gen path
  constexpr int TS = T128 ? 128 : 64;                         // exp table entries (GENX)
  constexpr double kScale = E256 ? kLog2eX256 : (T128 ? 2.0 * kLog2eX64 : kLog2eX64);
  // exp table 2^(j/64).  Production: one shared copy (lanes reading entries j and j + 32
  // in one lane group conflict; the conflicts cost nothing measurable).  VAR bit 18:
  // replicated TREP times, lane l reading copy l mod TREP at double (j TREP + l mod TREP),
  // so a ds_read_b64 lane group (32 lanes, 64 banks of 4 B) hits 32 distinct bank pairs
  // (TREP = 32; 8-wave shapes 16 so two workgroups still fit a CU's 160 KiB).
  constexpr int TREP = (E256 || !(VAR & 262144)) ? 1 : (NW == 4 ? 32 : 16);
  __shared__ double tab[(E256 ? 256 : (T128 ? 128 : 64)) * TREP];
  __shared__ double csc[FOLD ? PT : 1];                       // FOLD: per-particle factor c_p
  __shared__ double qred[NW][PT];
  // VAR bit 17: particle coordinates read from LDS in the generation instead of held in
  // VGPRs (frees 2 d VGPRs: large d on the 32-particle shapes)
  constexpr bool PLDS = (VAR & 131072) != 0;
  __shared__ double PA[PLDS ? PT : 1][PLDS ? DI + 1 : 1];
  __shared__ double sred[NW][PT];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // SPEC: waves [0, NWM) multiply, waves [NWM, NW) stage rows and generate K*
  const bool producer = (!SPEC || w >= NWM) && !KCONS;     // KCONS: nothing to generate
  const bool consumer = !SPEC || w < NWM;
  const int gtid = SPEC ? (tid >= 64 * NWM ? tid - 64 * NWM : tid) : tid;   // generation-role index
  const int b = blockIdx.x;
  const int J = prm.n_j_max - 1 - ((KPROD || KCONS) ? prm.j_skip : 0) - b / prm.tiles_ub;
  // tile index within this launch's segments (a launch may cover classes c0..c0+7)
  // segment tables live in device memory (the filter computes them on the device; the
  // predictive maps write theirs with k_seg_table).  A by-value table with a per-thread
  // select cost the d = 16 64x512 tile 6.7% through register allocation (tools/microbench/
  // tile_ab.sh: 760 -> 811 ms per config-5 launch)
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
  const double* __restrict__ Xrec = prm.seg[c].Xrec;
  const double* __restrict__ Bf = prm.seg[c].Bf;
  const int n_rows = prm.seg[c].n_rows;
  const int n_m = prm.seg[c].n_m;
  const int n_cols = n_rows + n_m;
  const int coff = prm.seg[c].coff;

  if constexpr (E256) {
    for (int i = tid; i < 256; i += NT) tab[i] = kExp2Tab256[i];
  } else if constexpr (T128) {
    for (int i = tid; i < 128; i += NT) tab[i] = kExp2Tab128[i];
  } else {
    for (int i = tid; i < 64 * TREP; i += NT) tab[i] = kExp2Tab[i / TREP];
  }
  const double* tabl = tab + (TREP > 1 ? (tid & 63) % TREP : 0);   // this lane's copy

  const int seg_begin = prm.seg_pos_begin[c];
  const int pos0 = seg_begin + (t - prm.seg_tile_start[c]) * PT;
  const int pos_end = prm.seg_pos_end[c];
  const int out_base = prm.seg_out_base[c] - seg_begin;   // out = out_base + pos

  // ---- this thread's particle (generation role: particle m, rows g + NG s) ----------
  const int m = gtid % PT;
  const int g = gtid / PT;
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
  int aint = 0;                                            // FOLD: integer part of asq
  if constexpr (FOLD) {
    const double af = floor(asq);
    aint = (int)af;
    if (g == 0) csc[m] = exp2((af - asq) / (double)TS);    // 2^(-frac / S)
  }
  if constexpr (PLDS) {
    if (g == 0) {
#pragma unroll
      for (int j = 0; j < DI; ++j) PA[m][j] = a2[j];
    }
  }

  // ---- K ranges ------------------------------------------------------------------
  const int nks = (VAR & 128) ? ksteps(n_rows) : ksteps(block_kmax(J, n_rows, NB, coff));
  // this wave's tiles: columns NB*J + 16(NW t + w) .. +15.  T1 = real tiles, kend[t] = the
  // K-step where tile t retires (R tile: past its last column's diagonal; tiles holding
  // mean columns: all rows).  kend is non-decreasing in t.
  int T1 = 0;
  int kend[NTW];
#pragma unroll
  for (int tt = 0; tt < NTW; ++tt) {
    const int c0 = J * NB + 16 * (NWM * tt + w) - coff;   // front-padding tiles: c0 < 0
    const bool real = c0 >= 0 && c0 < n_cols;
    if (real) T1 = tt + 1;
    const int hi = c0 + 16;
    int ke = (hi <= n_rows) ? ksteps(hi) : ksteps(n_rows);
    if constexpr (VAR & 129) ke = nks;
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

  // K* cache (KPROD / KCONS): tile t's A fragments, K-step ks, sub-step kk, at doubles
  // ((ks 4 + kk) 64 + lane) MT of the tile's slab of ksteps(n_rows) K-steps.  Buffer
  // addressing as for B: SGPR resource and K-step offset, constant lane offset.
  typedef unsigned v2u __attribute__((ext_vector_type(2)));
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t krsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((KPROD || KCONS) ? prm.kcache + (long long)t * ksteps(n_rows) * (256 * MT) : Bw), (short)0,
      0x7fffffff, 0x00020000);
  const unsigned klane_off = (unsigned)lane * (unsigned)(MT * 8);
  double an[4 * MT];                                         // KCONS: the next K-step's A fragments
  auto loadA_part = [&](int ks, int kk) {
    const int kc = ks < ks_last ? ks : ks_last;
    const int soff = (kc * 4 + kk) * (64 * MT) * 8;
    if constexpr (MT == 1) {
      const v2u x = __builtin_amdgcn_raw_buffer_load_b64(krsrc, klane_off, soff, 0);
      an[kk] = __builtin_bit_cast(double, (unsigned long long)x.x | ((unsigned long long)x.y << 32));
    } else {
#pragma unroll
      for (int h = 0; h < MT / 2; ++h) {
        const v4u x = __builtin_amdgcn_raw_buffer_load_b128(krsrc, klane_off + 16u * h, soff, 0);
        an[kk * MT + 2 * h + 0] = __builtin_bit_cast(double, (unsigned long long)x.x | ((unsigned long long)x.y << 32));
        an[kk * MT + 2 * h + 1] = __builtin_bit_cast(double, (unsigned long long)x.z | ((unsigned long long)x.w << 32));
      }
    }
  };
  // 8-byte stores: 16-byte stores of these registers (refilled by the next sub-step's LDS
  // reads right behind the store) wrote a wrong low dword for 0.33% of the values
  auto storeA_part = [&](int ks, int kk, const double (&af)[MT]) {
    const int soff = (ks * 4 + kk) * (64 * MT) * 8;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const unsigned long long u = __builtin_bit_cast(unsigned long long, af[mt]);
      __builtin_amdgcn_raw_buffer_store_b64((v2u){(unsigned)u, (unsigned)(u >> 32)}, krsrc, klane_off + 8u * mt, soff, 0);
    }
  };

  // Training rows of a K-step are staged through an LDS ring (RX) one step ahead with
  // vector loads, so generation reads them as LDS broadcasts: no scalar loads whose
  // lgkmcnt(0) waits would serialise with the A-fragment reads.
  // Branch-free: threads past the record count load a clamped (valid) address and store it
  // to a padding slot, so no exec-mask branch splits the K-step (the compiler otherwise
  // sinks the load into the conditional store and waits for it with vmcnt(0)).
  // Row records [Xs_i, |Xs_i|^2 64/ln2] (RW doubles per row, padded rows included) are one
  // contiguous array: buffer loads with a per-thread constant byte offset and a wave-uniform
  // K-step offset, no VALU address arithmetic per K-step.
  constexpr bool RECB = !(VAR & 524288) && !E256;
  const __amdgpu_buffer_rsrc_t rrsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)(T128 ? prm.rec128 : Xrec), (short)0, 0x7fffffff, 0x00020000);
  unsigned roff[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int idx = gtid + NTG * k;
    roff[k] = (unsigned)(idx < NRV ? idx : NRV - 1) * 8u;
  }
  auto load_rows = [&](int ks, double (&rr)[RPT]) {
    if constexpr (RECB) {
      typedef unsigned v2u __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int k = 0; k < RPT; ++k) {
        const v2u x = __builtin_amdgcn_raw_buffer_load_b64(rrsrc, roff[k], ks * (NRV * 8), 0);
        rr[k] = __builtin_bit_cast(double, (unsigned long long)x.x | ((unsigned long long)x.y << 32));
      }
      return;
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      int idx = gtid + NTG * k;
      idx = idx < NRV ? idx : NRV - 1;
      const int r = idx / RW, f = idx - (idx / RW) * RW;
      int i = ks * kBK + r;
      const double* src = f < DI ? Xs + ((long long)i * DI + f) : Xsq + i;
      const double v = *src;
      rr[k] = (E256 && f == DI) ? 4.0 * v : v;
    }
  };
  auto store_rows = [&](int buf, const double (&rr)[RPT]) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      if constexpr (VAR & 1024) {
        if (gtid + NTG * k < NRV) RX[buf][gtid + NTG * k] = rr[k];
      } else {
        RX[buf][gtid + NTG * k] = rr[k];                    // unconditional (padding slots)
      }
    }
  };
  // Branch-free generation.  The row arrays are padded to row_cap(n_rows) rows with
  // |Xs|^2 = kPadSq, so the exponent of a padding row is ~ -1e300 and its kernel value is
  // exactly 0 (v_cvt_i32_f64 saturates, ldexp underflows): no masking per value.
  auto gen_one = [&](int ks, int rb, int s) -> double {
    const int r = g + NG * s;
    const double* row = &RX[rb][r * RW];
    double x;
    if constexpr (VAR & 4) {
      x = -(asq + 0.5 * (ks * kBK + r));
#pragma unroll
      for (int j = 0; j < DI; ++j) x = fma(a2[j], 0.25 * j, x);
    } else if constexpr (FOLD) {
      x = -row[DI];                                        // asq leaves via aint / csc
#pragma unroll
      for (int j = 0; j < DI; ++j) x = fma(PLDS ? PA[m][j] : a2[j], row[j], x);
    } else {
      x = -(asq + row[DI]);
#pragma unroll
      for (int j = 0; j < DI; ++j) x = fma(PLDS ? PA[m][j] : a2[j], row[j], x);
    }
    double val;
    if constexpr (VAR & 2) val = fma(x, 1e-3, 1.0);
    else if constexpr (GENX) val = exp2_gen<TS, IEXP>(x, tab, aint);
    else if constexpr (E256) val = exp2_256(x, tab);
    else if constexpr ((VAR & 512) != 0) val = exp2_64m(x, tab);
    else if constexpr (TREP > 1) val = exp2_64r<TREP>(x, tabl);
    else val = exp2_64(x, tab);
    return val;                                            // padding rows: exactly 0
  };
  auto gen = [&](int ks, int rb, double (&v)[GV]) {
#pragma unroll
    for (int s = 0; s < GV; ++s) v[s] = gen_one(ks, rb, s);
  };
  // B fragments: one register set, refilled sub-step by sub-step for the next K-step right
  // after the MFMAs that consumed it (so the prefetch needs no second set of registers).
  // The address is clamped to the wave's last K-step so no branch guards the loads.
  auto loadB_part = [&](int ks, int kk, int slot, double (&bb)[BR * NTW]) {
    if constexpr (VAR & 32) {
#pragma unroll
      for (int q = 0; q < NTW; ++q) bb[slot * NTW + q] = bb[slot * NTW + q] * 0.999 + 1e-3 * (ks & 1);
      return;
    }
    const int kc = ks < ks_last ? ks : ks_last;
    if constexpr ((VAR & 16384) != 0) {          // A/B: flat global loads (64-bit VGPR addresses)
      const double* src = Bw + (long long)kc * FS + kk * (64 * NTW) + lane * 2;
#pragma unroll
      for (int h = 0; h < NTW / 2; ++h) {
        const double2 x = *reinterpret_cast<const double2*>(src + 128 * h);
        bb[slot * NTW + 2 * h + 0] = x.x;
        bb[slot * NTW + 2 * h + 1] = x.y;
      }
      return;
    }
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

  // One K-step with tiles [T0, T1) active: generate K*(ks+1) and stage rows(ks+2), then per
  // sub-step kk: A fragments from LDS, MFMAs, refill B(ks+1) for kk.  (Generating for
  // ks+1 = nks is harmless: clamped rows, stored to a buffer never read again.)
  // VAR 4096/8192 (A/B): the K* values of step ks+1 are generated between the sub-steps'
  // MFMAs (value s after sub-step s*4/GV) instead of in one block; 4096 also pins an
  // MFMA/VALU interleave with sched_group_barrier so the generation's dependent chain
  // hides under the MFMA pipe.
  constexpr bool SPLIT = (VAR & (4096 | 8192)) != 0;
  // Static ring slots: with the default rings (ASL = RXS = 4) every slot a K-step touches is
  // a function of ks & 3, so the K loop runs four K-steps per iteration with compile-time
  // slots (SL = 0..3): LDS addresses are a constant per-lane base plus instruction
  // immediates, no VALU address arithmetic.  Steps before the first multiple of 4 and
  // after the last one use run-time slots (SL = -1).
  constexpr bool STATIC = SB == 2 && ASL == 4 && RXS == 4 && (VAR & 1048576) != 0;
  auto full_step = [&](auto t0c, auto t1c, auto slotc, int ks, double (&bb)[BR * NTW]) {
    constexpr int T0 = decltype(t0c)::value, T1c = decltype(t1c)::value, SL = decltype(slotc)::value;
    constexpr bool ST = SL >= 0;
    const int buf = ST ? SL : (ks & (ASL - 1));
    const int gslot = ST ? ((SL + LOOK) & (ASL - 1)) : ((ks + LOOK) & (ASL - 1));
    const int rslot = ST ? ((SL + RA) & (RXS - 1)) : ((ks + RA) & (RXS - 1));
    const int grb = ST ? ((SL + LOOK) & (RXS - 1)) : ((ks + LOOK) & (RXS - 1));
    double v[GV];
    double rr[RPT];
    constexpr bool GEN2 = (VAR & 33554432) != 0;
    double v2[GV];
    const bool gen_now = !GEN2 || (ks & 1) == 0;
    constexpr bool PRIO = (VAR & 134217728) != 0;
    if constexpr (!(VAR & 16) && !SPEC && !KCONS) {                // SPEC: producer waves generate
      load_rows(ks + RA, rr);
      if constexpr (PRIO) {
        // generation after the MFMAs, at low priority (below)
      } else if constexpr (GEN2) {
        if (gen_now) {                                  // K-steps ks+2 and ks+3 together
#pragma unroll
          for (int s2 = 0; s2 < GV; ++s2) {
            v[s2] = gen_one(ks + 2, (ks + 2) & (RXS - 1), s2);
            v2[s2] = gen_one(ks + 3, (ks + 3) & (RXS - 1), s2);
          }
        }
      } else if constexpr (!SPLIT) {
        gen(ks + LOOK, grb, v);
      }
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      double af[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if constexpr (VAR & 64) af[mt] = asq + mt + kk + buf;
        else if constexpr (KCONS) af[mt] = an[kk * MT + mt];
        else af[mt] = As[buf][kk * 4 + lk][mt * 16 + li];
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = T0; nt < T1c; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[mt], bb[(kk % BR) * NTW + nt], acc[mt][nt], 0, 0, 0);
      if constexpr (SPLIT && !(VAR & 16) && !SPEC && !KCONS) {
        constexpr int PER = 4 / GV > 0 ? 4 / GV : 1;
        if (kk % PER == 0) {
#pragma unroll
          for (int s = 0; s < GV; ++s)
            if (s == kk / PER) v[s] = gen_one(ks + LOOK, grb, s);
        }
      }
      if constexpr ((VAR & 4096) != 0) {
        constexpr int NM = MT * (T1c - T0);
#pragma unroll
        for (int q = 0; q < NM; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // 2 VALU
        }
      }
      loadB_part(ks + (kk + BR) / 4, (kk + BR) % 4, kk % BR, bb);   // sub-step kk + BR
      // KCONS: an[j] is reloaded one sub-step after its last MFMA read, not right behind it
      // (a reload issued directly after the MFMA that reads the registers gave
      // nondeterministic results: L1-hit loads of fragments the WG's other waves had just
      // fetched overtook the MFMA's operand read).  an[3] for step ks is loaded after step
      // ks's sub-step 0.
      if constexpr (KCONS) {
        if (kk == 0) loadA_part(ks, 3);
        else loadA_part(ks + 1, kk - 1);
      }
      if constexpr (KPROD) {
        if (w == kk) storeA_part(ks, kk, af);
      }
    }
    if constexpr (PRIO && !(VAR & 16) && !SPEC && !KCONS) {
      __builtin_amdgcn_s_setprio(0);
      gen(ks + LOOK, grb, v);
    }
    if constexpr (!(VAR & 16) && !SPEC && !KCONS) {
      if constexpr (GEN2) {
        if (gen_now) {
          store((ks + 2) & (ASL - 1), v);
          store((ks + 3) & (ASL - 1), v2);
        }
      } else {
        store(gslot, v);
      }
      store_rows(rslot, rr);
    }
    if constexpr (!(VAR & 8) && !KCONS) {
      if constexpr (ST) {
        if constexpr (SL % SB == SB - 1) __syncthreads();
      } else {
        if (ks % SB == SB - 1) __syncthreads();
      }
    }
  };
  // K-steps [ks, e) with tiles [T0, T1) active
  auto run_steps = [&](auto t0c, auto t1c, int& ks, const int e, double (&bb)[BR * NTW]) {
    using RT = std::integral_constant<int, -1>;
    if constexpr (STATIC) {
      for (; ks < e && (ks & 3); ++ks) full_step(t0c, t1c, RT{}, ks, bb);
      for (; ks + 4 <= e; ks += 4) {
        full_step(t0c, t1c, std::integral_constant<int, 0>{}, ks, bb);
        full_step(t0c, t1c, std::integral_constant<int, 1>{}, ks + 1, bb);
        full_step(t0c, t1c, std::integral_constant<int, 2>{}, ks + 2, bb);
        full_step(t0c, t1c, std::integral_constant<int, 3>{}, ks + 3, bb);
      }
    }
    for (; ks < e; ++ks) full_step(t0c, t1c, RT{}, ks, bb);
  };

  double bb[BR * NTW];
  if constexpr (VAR & 32) {
#pragma unroll
    for (int q = 0; q < BR * NTW; ++q) bb[q] = 1e-3 * q + lane;
  }
  if (producer) {
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
    if (producer) {
#pragma unroll
      for (int j = 0; j < LOOK; ++j) {
        gen(j, j & (RXS - 1), v);
        store(j, v);
      }
    }
    if (consumer) {
#pragma unroll
      for (int kk = 0; kk < BR; ++kk) loadB_part(0, kk, kk, bb);
      if constexpr (KCONS) {
#pragma unroll
        for (int kk = 0; kk < 3; ++kk) loadA_part(0, kk);   // sub-step 3: inside step 0
      }
    }
  }
  // Drain the prologue's loads (vmcnt(0)) so that the K loop's entry carries no pending
  // loads: otherwise the waitcnt pass merges the prologue's issue order into the loop
  // header and waits for every in-flight B fragment at sub-step 0 of each K-step.
  if constexpr (!(VAR & 2048)) __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();

  if constexpr (SPEC) {
    if (producer) {                                          // stage rows, generate K*: all K-steps
      for (int kp = 0; kp < nks; ++kp) {
        double v[GV];
        double rr[RPT];
        load_rows(kp + RA, rr);
        gen(kp + LOOK, (kp + LOOK) & (RXS - 1), v);
        store((kp + LOOK) & (ASL - 1), v);
        store_rows((kp + RA) & (RXS - 1), rr);
        if (kp % SB == SB - 1) __syncthreads();
      }
      // the epilogue's barrier (the MFMA waves' cross-wave reduction)
      const bool has_r0 = J * NB - coff < n_rows;
      const bool has_m0 = (J + 1) * NB - coff > n_rows;
      if (has_r0 || (has_m0 && prm.spart != nullptr)) __syncthreads();
      return;
    }
  }

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
        run_steps(std::integral_constant<int, T0>{}, std::integral_constant<int, T1c>{}, ks, e, bb);
      });
    }
  });
  // the rest of the block's K range (other waves' tiles): generate only
  for (; ks < nks && SPEC; ++ks)                             // SPEC: the producers generate
    if (ks % SB == SB - 1) __syncthreads();
  for (; ks < nks && !KCONS; ++ks) {
    if constexpr (KPROD) {                                   // this wave's sub-step of ks
      if (w < 4) {
        double af[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) af[mt] = As[ks & (ASL - 1)][w * 4 + lk][mt * 16 + li];
        storeA_part(ks, w, af);
      }
    }
    double v[GV];
    double rr[RPT];
    load_rows(ks + RA, rr);
    if constexpr ((VAR & 33554432) != 0) {             // GEN2: both K-steps on even ks
      if ((ks & 1) == 0) {
        double v2[GV];
#pragma unroll
        for (int s2 = 0; s2 < GV; ++s2) {
          v[s2] = gen_one(ks + 2, (ks + 2) & (RXS - 1), s2);
          v2[s2] = gen_one(ks + 3, (ks + 3) & (RXS - 1), s2);
        }
        store((ks + 2) & (ASL - 1), v);
        store((ks + 3) & (ASL - 1), v2);
      }
    } else {
      gen(ks + LOOK, (ks + LOOK) & (RXS - 1), v);
      store((ks + LOOK) & (ASL - 1), v);
    }
    store_rows((ks + RA) & (RXS - 1), rr);
    if (ks % SB == SB - 1) __syncthreads();
  }

  // FOLD: rows of V = K* B carry the per-particle factor c_p (row (l >> 4) + 4 r of tile mt)
  double cfold[MT][4];
  if constexpr (FOLD) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) cfold[mt][r] = csc[mt * 16 + (lane >> 4) + 4 * r];
    if constexpr (DYN) {                                   // before the linear-kernel share
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[mt][nt][r] *= cfold[mt][r];
    }
  }
  constexpr bool OFOLD = FOLD && !DYN;                     // obs: scale q and mean uses only
  if constexpr (DYN) {
    // Linear-kernel share: acc += X~ H for this block.  A fragment: lane l holds
    // x~[particle mt*16 + (l&15)][4 kh + (l>>4)]; B fragment: Hf[J][kh][w][l][nt].
    constexpr int KH = (DI + 1 + 3) / 4;
    const double* __restrict__ Hw = prm.seg[c].Hf + ((long long)J * KH * NWM + w) * (64 * NTW) + lane * NTW;
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
        const double2 hv = *reinterpret_cast<const double2*>(Hw + (long long)kh * NWM * (64 * NTW) + 2 * h);
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
  // C/D layout of v_mfma_f64_16x16x4_f64: lane l, reg r -> row (l>>4) + 4r, col l&15.
  const bool has_r = J * NB - coff < n_rows;
  const bool has_m = (J + 1) * NB - coff > n_rows;            // block holds mean columns
  const bool fused = prm.spart != nullptr;
  if (has_m) {
    if (!fused) {
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int jm = J * NB + 16 * (NWM * nt + w) + li - coff - n_rows;
        if (jm >= 0 && jm < n_m) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int p = pos0 + mt * 16 + lk + 4 * r;
              if (p < pos_end)
                prm.mu[(long long)(out_base + p) * prm.ld_mu + jm] = OFOLD ? cfold[mt][r] * acc[mt][nt][r] : acc[mt][nt][r];
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
        const int jm = J * NB + 16 * (NWM * nt + w) + li - coff - n_rows;
        if (jm >= 0 && jm < n_m) {
          const double lam = prm.lam2[jm];
          if (f0 == f1) {
            const double zj = prm.z[(long long)f0 * n_m + jm];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const double t = OFOLD ? fma(-cfold[mt][r], acc[mt][nt][r], zj) : zj - acc[mt][nt][r];
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
                const double t = OFOLD ? fma(-cfold[mt][r], acc[mt][nt][r], zz) : zz - acc[mt][nt][r];
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
      const int col = J * NB + 16 * (NWM * nt + w) + li - coff;
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
        if constexpr (OFOLD) v *= cfold[mt][r] * cfold[mt][r];
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
          for (int ww = 0; ww < NWM; ++ww) q += qred[ww][tid];
          prm.qpart[(long long)J * prm.ld_q + out_base + p] = q;
        }
        if (has_m && fused) {
          double sm = 0.0;
#pragma unroll
          for (int ww = 0; ww < NWM; ++ww) sm += sred[ww][tid];
          prm.spart[(long long)J * prm.ld_q + out_base + p] = sm;
        }
      }
    }
  }
}

}  // namespace gpmdm
