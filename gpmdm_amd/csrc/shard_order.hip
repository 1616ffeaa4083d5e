// Ancestor-ordered shards for multi-rank filters.
//
// After a resample every rank holds the same replicated cloud; which particles a rank
// evaluates in the next frame is free (per-particle arithmetic and Philox draws depend on
// the particle index only, and the all-gather restores particle order).  Ranks therefore
// take contiguous slices of the particles ordered by resampling ancestor: a slice then
// covers a contiguous ancestor range, and the dynamics GP's ancestor de-duplication keeps
// ~1/R of the distinct (ancestor, class) keys per rank instead of nearly all of them.
//
// The order is a stable bucket sort of the slots on the bucket of their resampling uniform,
// b = floor(256 u_s).  The inverse-CDF search maps u monotonically to the ancestor, so a
// bucket's slots descend from one contiguous ancestor range and a rank's slice spans whole
// buckets except at its two ends -- the same locality as sorting on the ancestor itself, but
// computed from the draws alone (Philox, keyed by slot and frame): no ancestor array is
// read, nothing waits for the search.  Systematic resampling needs no pass at all (its
// uniforms, hence its ancestors, rise with the slot index: the identity order).  Every step
// is deterministic (block histograms, fixed-order scans, ranks counted in slot order), so
// every rank builds the same order.  Three launches, O(P):
//   k_ubucket_hist        per-block bucket histograms (2048 slots per block), bucket-major H[b][block]
//   k_ubucket_chunk_scan  exclusive scan of H inside 1024-entry chunks, chunk totals
//   k_ubucket_scatter     (each block first scans the chunk totals in LDS)
//                         own[offset(b, block) + rank of the slot among the block's bucket-b slots]
//                         = slot, and its inverse
// (rocPRIM's radix sort of such keys measured 145 us at P = 800k on MI355X,
// tools/microbench/sort_probe.hip.)
#include "pf_kernels.h"

namespace gpmdm {

namespace {

constexpr int kT = 256;           // threads per block = buckets
constexpr int kPer = 8;           // rounds of kT consecutive slots per block
constexpr int kBlk = kT * kPer;   // slots per block

// bucket of slot s's resampling uniform (k_resample's Philox draw, bit for bit)
__device__ __forceinline__ int ubucket(long long s, unsigned frame, uint2 key) {
  const uint4 r = philox4x32_10(make_uint4((unsigned)s, frame, kStreamResample, 0u), key);
  const int b = (int)(u01_co(r.x, r.y) * (double)kT);
  return b < kT - 1 ? b : kT - 1;
}

__global__ __launch_bounds__(kT) void k_ubucket_hist(long long P, unsigned frame, uint2 key, int nblk, int* H) {
  __shared__ int hist[kT];
  const int tid = threadIdx.x;
  hist[tid] = 0;
  __syncthreads();
  const long long s0 = (long long)blockIdx.x * kBlk + tid;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const long long s = s0 + (long long)k * kT;
    if (s < P) atomicAdd(&hist[ubucket(s, frame, key)], 1);
  }
  __syncthreads();
  H[(long long)tid * nblk + blockIdx.x] = hist[tid];
}

// Exclusive scan of H inside kChunk-entry chunks (in place), and each chunk's total.
constexpr int kChunk = 1024;                   // H entries per chunk (4 per thread)
constexpr int kMaxChunks = 4096;               // k_ubucket_scatter scans the chunk totals in LDS
__global__ __launch_bounds__(kT) void k_ubucket_chunk_scan(int* H, long long n, int* chunk_tot) {
  __shared__ int wtot[kT / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long base = (long long)blockIdx.x * kChunk + tid * 4;
  int v[4], t = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = base + k < n ? H[base + k] : 0;
    t += v[k];
  }
  int x = t;                                   // inclusive wave scan of the thread totals
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) wtot[w] = x;
  __syncthreads();
  int run = x - t;
  for (int u = 0; u < w; ++u) run += wtot[u];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (base + k < n) H[base + k] = run;
    run += v[k];
  }
  if (tid == kT - 1) chunk_tot[blockIdx.x] = run;
}

__global__ __launch_bounds__(kT) void k_ubucket_scatter(long long P, unsigned frame, uint2 key, int nblk,
                                                        const int* H, const int* chunk_tot, int nchunk,
                                                        int* own, int* inv) {
  constexpr int kW = kT / 64;
  constexpr int kCPer = kMaxChunks / kT;
  __shared__ int cnt[kW][kT];                  // this round's bucket counts per wave
  __shared__ int run[kT];                      // the block's earlier rounds' counts per bucket
  __shared__ int coff[kMaxChunks];             // exclusive prefix of the chunk totals
  __shared__ int wtot[kW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  {                                            // every block scans the (few) chunk totals itself
    int v[kCPer], t = 0;
#pragma unroll
    for (int k = 0; k < kCPer; ++k) {
      const int c = tid * kCPer + k;
      v[k] = c < nchunk ? chunk_tot[c] : 0;
      t += v[k];
    }
    int x = t;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    if (lane == 63) wtot[w] = x;
    __syncthreads();
    int e = x - t;
    for (int u = 0; u < w; ++u) e += wtot[u];
#pragma unroll
    for (int k = 0; k < kCPer; ++k) {
      coff[tid * kCPer + k] = e;
      e += v[k];
    }
  }
  run[tid] = 0;
  for (int k = 0; k < kPer; ++k) {
    const long long s = (long long)blockIdx.x * kBlk + (long long)k * kT + tid;
    const int b = s < P ? ubucket(s, frame, key) : -1;
    for (int i = tid; i < kW * kT; i += kT) (&cnt[0][0])[i] = 0;
    // rank among this wave's bucket-b slots (ballots over the bucket's 8 bits and validity)
    unsigned long long same = ~0ull;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool bit = (b >> j) & 1;
      const unsigned long long m = __ballot(bit);
      same &= bit ? m : ~m;
    }
    const unsigned long long valid = __ballot(b >= 0);
    same &= b >= 0 ? valid : ~valid;
    const int r_wave = __popcll(same & ((1ull << lane) - 1));
    __syncthreads();
    if (b >= 0 && r_wave == 0) cnt[w][b] = __popcll(same);   // one writer per (wave, bucket)
    __syncthreads();
    if (b >= 0) {
      int r = run[b] + r_wave;
      for (int v = 0; v < w; ++v) r += cnt[v][b];
      const long long h = (long long)b * nblk + blockIdx.x;
      const int pos = coff[h / kChunk] + H[h] + r;
      own[pos] = (int)s;
      inv[s] = pos;
    }
    __syncthreads();
    int t = 0;
    for (int v = 0; v < kW; ++v) t += cnt[v][tid];
    run[tid] += t;
  }
}

inline unsigned nblocks(long long n, long long b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

bool uniform_order_supported(long long P) {
  return nblocks((long long)kT * nblocks(P, kBlk), kChunk) <= (unsigned)kMaxChunks;   // P <= 33.5M
}

size_t uniform_order_temp_bytes(long long P) {
  const long long n = (long long)kT * nblocks(P, kBlk);
  return sizeof(int) * (size_t)(n + nblocks(n, kChunk));
}

int launch_uniform_order(long long P, unsigned frame, unsigned seed_lo, unsigned seed_hi, int* own, int* inv,
                         void* temp, size_t temp_bytes, hipStream_t s) {
  const int nblk = (int)nblocks(P, kBlk);
  const long long n = (long long)kT * nblk;
  const int nchunk = (int)nblocks(n, kChunk);
  if (temp_bytes < uniform_order_temp_bytes(P) || !uniform_order_supported(P)) return -1;
  int* H = static_cast<int*>(temp);
  int* chunk_tot = H + n;
  const uint2 key = make_uint2(seed_lo, seed_hi);   // filter_key(seed, 0): a single filter
  hipLaunchKernelGGL(k_ubucket_hist, dim3(nblk), dim3(kT), 0, s, P, frame, key, nblk, H);
  hipLaunchKernelGGL(k_ubucket_chunk_scan, dim3(nchunk), dim3(kT), 0, s, H, n, chunk_tot);
  hipLaunchKernelGGL(k_ubucket_scatter, dim3(nblk), dim3(kT), 0, s, P, frame, key, nblk, H, chunk_tot, nchunk,
                     own, inv);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace gpmdm
