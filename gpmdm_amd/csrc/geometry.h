// Tile and column-block geometry of the fused GP tiles, shared by the host-side image
// packing (host_image.h, plain C++) and the kernels (gp_tile.h).  Everything here is
// constexpr: clang compiles constexpr functions for both host and device, so this header
// needs no HIP include and the packing code builds with any C++17 compiler (the host
// sanitizer test, tests/test_host_asan.py).
#pragma once

namespace gpmdm {

// ---------------------------------------------------------------------------------
// Fused GP tile geometry (see gp_tile.hip and DESIGN.md §3).
//   one workgroup = NW waves = 16 MT particles x 16 NTW NW columns of V = K* . B, where K*
//   (particles x training rows) is generated on the fly and B = [R | M] is the extended
//   weight matrix stored in MFMA-fragment order (each wave owns MT x NTW tiles of 16 x 16).
//   Shapes: 64x256 (NW 4, MT 4, NTW 4), 64x512 (8, 4, 4), 32x512 (4, 2, 8; the observation
//   GP default for d <= 12), 32x256 (4, 2, 4) and 16x256 (4, 1, 4; the dynamics GP default).
// ---------------------------------------------------------------------------------
constexpr int kBK = 16;           // training rows per K-step (4 x K=4 MFMA sub-steps)
constexpr int kMaxSeg = 8;        // segments (classes) per launch
constexpr int kMaxD = 32;         // latent dimension limit

// Tile shapes selectable per model (gpmdm_model_desc.tile_shape).
struct TileGeo {
  int nw, mt, ntw;
  constexpr int pt() const { return 16 * mt; }          // particles per tile
  constexpr int nb() const { return 16 * ntw * nw; }    // columns per block
  constexpr int fs() const { return nw * 256 * ntw; }   // fragment doubles per K-step
};
constexpr TileGeo kGeo64x256{4, 4, 4};
constexpr TileGeo kGeo64x512{8, 4, 4};
constexpr TileGeo kGeo32x512{4, 2, 8};
constexpr TileGeo kGeo32x256{4, 2, 4};
constexpr TileGeo kGeo16x256{4, 1, 4};

// Column-block geometry shared by the host (fragment layout) and the kernel.
// Columns are [R (n_rows) | M (n_m)].  The column space is padded at the FRONT by coff
// (a multiple of 16) so that the partial block is block 0, whose triangular K range is a
// single K-step, instead of a last block that needs every training row for a handful of
// mean columns.  Block J spans virtual columns [J nb, (J+1) nb) = real columns
// [J nb - coff, (J+1) nb - coff); its K range ends at min(n_rows, (J+1) nb - coff).
constexpr int block_kmax(int J, int n_rows, int nb, int coff) {
  const int hi = (J + 1) * nb - coff;
  return hi < n_rows ? hi : n_rows;
}
constexpr int col_offset(int n_cols, int nb) {
  const int r = n_cols % nb;
  return r ? ((nb - r) / 16) * 16 : 0;
}
constexpr int ksteps(int kmax) { return (kmax + kBK - 1) / kBK; }
// Rows the row records are padded to: the K loop stages rows up to eight K-steps past
// the last one it multiplies (A/B variants included).  Padding rows have Xs = 0 and
// |Xs|^2 = kPadSq (kernel value 0).
constexpr int row_cap(int n_rows) { return (ksteps(n_rows) + 8) * kBK; }
constexpr double kPadSq = 268435456.0;   // 2^28: exponent ~ -2^28 even x 128/ln2 scaled
                                        // (v_cvt_i32_f64 exact, ldexp underflows to 0)
// |Xs|^2 is stored pre-scaled by 64 / ln 2 for the tile kernel's exp2 (gp_tile.h)
constexpr double kLog2eX64 = 92.33248261689366;
// The observation GP's cutoff image: K-steps the sparse tile kernel can list (gp_tile.h).
constexpr int kMaxCutoffKs = 4096;
// Dynamics linear kernel: K=4 MFMA sub-steps covering the d+1 rows of H.
constexpr int lin_substeps(int d) { return (d + 1 + 3) / 4; }

}  // namespace gpmdm
