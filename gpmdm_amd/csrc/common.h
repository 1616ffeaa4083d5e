// Shared device helpers and launch declarations for libgpmdm_hip (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "geometry.h"

namespace gpmdm {

typedef double d4 __attribute__((ext_vector_type(4)));

struct SegDesc {                  // one GP: the observation GP, or the class-c dynamics GP
  const double* Xrec;             // row_cap(n_rows) x (d + 1): row records [Xs_i, |Xs_i|^2 * 64/ln2]
  const double* Hf;               // dyn only: H = (Xin C^2)^T B, (d+1) x cols, fragment order
  const double* Bf;               // B = [triu(R) | M] in fragment order (see capi_model.hip build_image)
  int n_rows;                     // training rows = R columns
  int n_m;                        // mean columns (D or d)
  int n_j;                        // column blocks
  int coff;                       // front padding of the column space (see col_offset)
};

struct TileParams {
  SegDesc seg[kMaxSeg];
  int n_seg;
  int tiles_ub;                   // grid = n_j_max * tiles_ub workgroups
  int n_j_max;
  TileGeo geo;                    // tile shape: fragment layout of B, particles per tile
  const int* seg_pos_begin;       // [n_seg]   first position (device)
  const int* seg_pos_end;         // [n_seg]
  const int* seg_out_base;        // [n_seg]   output row of the first position
  const int* seg_tile_start;      // [n_seg+1] prefix of tiles
  const int* perm;                // position -> particle row (nullptr: identity)
  const double* X;                // particle rows, n x d
  double ls[kMaxD];               // RBF lengthscales
  double* qpart;                  // [J][ld_q]: partial sums of (R^T k)^2 per column block
  long long ld_q;
  double* mu;                     // [out][ld_mu] mean columns (predictive maps)
  long long ld_mu;
  // Fused likelihood (particle filter, observation GP): instead of storing the mean, blocks
  // holding mean columns write spart[J][out] = sum_j (z_j - mu_j)^2 lam2_j over their mean
  // columns (z = the observation of the particle's filter, pos / Pf).
  double* spart;                  // nullptr: store mu
  const double* z;                // F x n_m
  const double* lam2;             // n_m: exp(y_log_lambdas)^2 = 1 / il2
  long long Pf;                   // particles per filter
};

void launch_gp_tile(const TileParams& p, int d, bool dyn, hipStream_t stream);

// The observation GP's kernel-value cutoff kernel (obs_cutoff.h).
struct CutoffParams {
  const double* X;           // particle states, d doubles each
  const int* perm;           // tile position -> particle (nullptr: identity)
  int pos_begin, pos_end;    // this launch's positions; outputs at pos - pos_begin
  double ls[kMaxD];          // observation GP lengthscales
  const double* Xrec;        // row records in image-row order, row_cap(n_rows) rows
  const double* Bt;          // the tile-major image
  const long long* toff;     // first double of each tile (T_R + T_M + 1)
  const double* ksph;        // per K-step bounding sphere: centre (d), radius
  int n_rows, n_m, T_R, T_M;
  double cut2;               // squared cutoff distance (scaled units), with rounding margin
  double t_cut;              // the flush threshold on the generation's exponent
  double* q;                 // per position: k^T K^-1 k
  double* S;                 // per position: sum_j (z_j - mu_j)^2 lam2_j
  const double* z;           // F x n_m observations
  const double* lam2;        // n_m
  long long Pf;              // particles per filter
  unsigned long long* sp_stats;   // MFMA groups run / the dense kernel's, or nullptr
  // split tiles (the grid's tail): particle tiles [n_whole, n_whole + n_split) run as two
  // workgroups each, chunks [0, c*) (q, S as a whole tile's, so far) and [c*, nc) (list entry
  // i's partial into part[(i - r0) * ld_part + o - n_whole * PT], r0 = the first chunk's
  // size; k_obs_ll chains them on)
  int n_whole, n_split;
  double* part;
  long long ld_part;
  int2* split;               // per split tile: (n_act, c*), written by its first workgroup
  // chunk grid (GPMDM_CUT_SPLIT_CHUNKS): every tile split at c* = 1 and every chunk its own
  // workgroup, n_chunk_max x n_split of them, chunk-major from each list's end (heavy first)
  int chunk_grid, n_chunk_max;
};
bool launch_obs_cutoff(const CutoffParams& p, int d, hipStream_t stream);   // false: bad shape
int cutoff_tile_particles(int d);   // PT of the cutoff kernel at d
int cutoff_tile_list_chunk();       // tpc: list entries per chunk
int cutoff_slots(int d);            // workgroups resident at once on the device (cached per d)

// First list entry of chunk c of a tile list of nt entries (obs_cutoff.h): the partial chunk
// first (nt - (nc - 1) tpc entries: the chunk that runs the fewest positions), then full ones
__host__ __device__ inline int cutoff_chunk_begin(int c, int nt, int tpc) {
  if (c <= 0) return 0;
  const int nc = (nt + tpc - 1) / tpc;
  return nt - (nc - c) * tpc;
}
// K-loop positions chunk c runs: up to its last R tile's diagonal, every active K-step once it
// holds a mean tile
__host__ __device__ inline int cutoff_chunk_positions(int c, int n_act, int T_M, int tpc) {
  const int last = cutoff_chunk_begin(c + 1, n_act + T_M, tpc) - 1;
  return last < n_act ? last + 1 : n_act;
}
// The split chunk c* of a split tile: the first chunk of its second workgroup, balancing the
// two workgroups' positions (plus a chunk's pipeline fill); nc (no second part) below two chunks
__host__ __device__ inline int cutoff_split_chunk(int n_act, int T_M, int tpc) {
  const int nc = (n_act + T_M + tpc - 1) / tpc;
  if (nc < 2) return nc;
  constexpr int kFill = 4;
  long long tot = 0;
  for (int c = 0; c < nc; ++c) tot += cutoff_chunk_positions(c, n_act, T_M, tpc) + kFill;
  long long pre = 0, best_v = tot;
  int best = 1;
  for (int c = 1; c < nc; ++c) {
    pre += cutoff_chunk_positions(c - 1, n_act, T_M, tpc) + kFill;
    const long long v = pre > tot - pre ? pre : tot - pre;
    if (v < best_v) {
      best_v = v;
      best = c;
    }
  }
  return best;
}

// ---------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11), counter = (index, frame, stream, sub).
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const unsigned hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const unsigned hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// 53-bit uniforms from two 32-bit words.
__device__ __forceinline__ double u01_co(unsigned hi, unsigned lo) {   // [0, 1)
  const unsigned long long x = (((unsigned long long)hi << 32) | lo) >> 11;
  return (double)x * 0x1.0p-53;
}
__device__ __forceinline__ double u01_oo(unsigned hi, unsigned lo) {   // (0, 1)
  const unsigned long long x = (((unsigned long long)hi << 32) | lo) >> 11;
  return ((double)x + 0.5) * 0x1.0p-53;
}

enum RngStream : unsigned { kStreamSwitch = 0, kStreamDyn = 1, kStreamResample = 2, kStreamSystematic = 3 };

// Order-preserving uint64 image of a double (atomicMax on doubles).
__device__ __forceinline__ unsigned long long ord_enc(double x) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double ord_dec(unsigned long long u) {
  const unsigned long long v = (u >> 63) ? (u & 0x7fffffffffffffffull) : ~u;
  return __longlong_as_double((long long)v);
}

// Publish a sequence number the host polls in mapped (fine-grained) host memory: a
// system-scope release store -- everything this thread's program order and the stream's
// earlier kernels wrote before it is visible to a host that observes the number with an
// acquire load (capi_internal.h gpmdm_pf::min_mapped).  A vector store with release semantics (the
// compiler emits the system-scope fence sequence in front of it); never a volatile plain store.
__device__ __forceinline__ void publish_seq(long long* p, long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wave (64-lane) reductions.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
  return v;
}

}  // namespace gpmdm
