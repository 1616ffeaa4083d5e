// Ancestor-ordered shards for multi-rank filters.
//
// After a resample every rank holds the same replicated cloud; which particles a rank
// evaluates in the next frame is free (per-particle arithmetic and Philox draws depend on
// the particle index only, and the all-gather restores particle order).  Ranks therefore
// take contiguous slices of the particles ordered by resampling ancestor: a slice then
// covers a contiguous ancestor range, and the dynamics GP's ancestor de-duplication keeps
// ~1/R of the distinct (ancestor, class) keys per rank instead of nearly all of them.
//
// The order is a stable bucket sort on the ancestor's bucket b = anc * 256 / P (256
// contiguous ancestor ranges; particle order inside a bucket).  Exact ancestor order is not
// needed: a rank's slice spans whole buckets except at its two ends, so at most the
// ancestors of two buckets are shared with neighbours.  Every step is deterministic (block
// histograms, fixed-order scans, ranks counted in particle order), so every rank computes
// the same order.  Four small launches, O(P):
//   k_bucket_hist     per-block bucket histograms, bucket-major H[b][block]
//   k_chunk_scan      exclusive scan of H inside 1024-entry chunks, chunk totals
//   k_chunk_offsets   one workgroup: exclusive scan of the chunk totals
//   k_bucket_scatter  own[start(b, block) + rank in block] = particle, and its inverse
// (rocPRIM's radix sort of the same keys measured 145 us at P = 800k on MI355X,
// tools/microbench/sort_probe.hip; this pass is a few us per launch.)
#include "pf_kernels.h"

namespace gpmdm {

namespace {

constexpr int kOB = 256;          // particles per block = buckets
constexpr int kChunk = 1024;      // H entries per scan chunk (4 per thread)

__device__ __forceinline__ int bucket_of(int anc, long long P) { return (int)(((long long)anc * kOB) / P); }

__global__ __launch_bounds__(kOB) void k_bucket_hist(const int* anc, long long P, int nblk, int* H) {
  __shared__ int hist[kOB];
  const int tid = threadIdx.x;
  hist[tid] = 0;
  __syncthreads();
  const long long s = (long long)blockIdx.x * kOB + tid;
  if (s < P) atomicAdd(&hist[bucket_of(anc[s], P)], 1);
  __syncthreads();
  H[(long long)tid * nblk + blockIdx.x] = hist[tid];
}

__global__ __launch_bounds__(256) void k_chunk_scan(int* H, long long n, int* chunk_tot) {
  __shared__ int part[256];
  const int tid = threadIdx.x;
  const long long base = (long long)blockIdx.x * kChunk + tid * 4;
  int v[4], run = 0;
  for (int k = 0; k < 4; ++k) {
    v[k] = base + k < n ? H[base + k] : 0;
    run += v[k];
  }
  part[tid] = run;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {          // Hillis-Steele inclusive scan
    const int x = tid >= off ? part[tid - off] : 0;
    __syncthreads();
    part[tid] += x;
    __syncthreads();
  }
  int e = tid ? part[tid - 1] : 0;
  for (int k = 0; k < 4; ++k) {
    if (base + k < n) H[base + k] = e;
    e += v[k];
  }
  if (tid == 255) chunk_tot[blockIdx.x] = part[255];
}

__global__ __launch_bounds__(1024) void k_chunk_offsets(int* chunk_tot, int nchunk) {
  __shared__ int part[1024];
  const int tid = threadIdx.x;
  const int per = (nchunk + 1023) / 1024;
  int s = 0;
  for (int i = 0; i < per; ++i) {
    const int c = tid * per + i;
    if (c < nchunk) s += chunk_tot[c];
  }
  part[tid] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int x = tid >= off ? part[tid - off] : 0;
    __syncthreads();
    part[tid] += x;
    __syncthreads();
  }
  int run = tid ? part[tid - 1] : 0;
  for (int i = 0; i < per; ++i) {
    const int c = tid * per + i;
    if (c < nchunk) {
      const int t = chunk_tot[c];
      chunk_tot[c] = run;
      run += t;
    }
  }
}

__global__ __launch_bounds__(kOB) void k_bucket_scatter(const int* anc, long long P, int nblk, const int* H,
                                                         const int* chunk_off, int* own, int* inv) {
  constexpr int kW = kOB / 64;
  __shared__ int cnt[kW][kOB];                        // bucket counts per wave
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long s = (long long)blockIdx.x * kOB + tid;
  const int b = s < P ? bucket_of(anc[s], P) : -1;
  for (int i = tid; i < kW * kOB; i += kOB) (&cnt[0][0])[i] = 0;
  // rank among this block's bucket-b particles, in particle order: lanes of this wave with
  // the same bucket (ballots over the bucket's 8 bits and its validity), then the earlier
  // waves' counts of that bucket -- deterministic, so every rank builds the same order
  unsigned long long same = ~0ull;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool bit = (b >> k) & 1;
    const unsigned long long m = __ballot(bit);
    same &= bit ? m : ~m;
  }
  const unsigned long long valid = __ballot(b >= 0);
  same &= b >= 0 ? valid : ~valid;
  const int r_wave = __popcll(same & ((1ull << lane) - 1));
  __syncthreads();
  if (b >= 0 && r_wave == 0) cnt[w][b] = __popcll(same);   // one writer per (wave, bucket)
  __syncthreads();
  if (b < 0) return;
  int r = r_wave;
  for (int v = 0; v < w; ++v) r += cnt[v][b];
  const long long h = (long long)b * nblk + blockIdx.x;
  const int pos = chunk_off[h / kChunk] + H[h] + r;
  own[pos] = (int)s;
  inv[s] = pos;
}

inline unsigned nblocks(long long n, int b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

size_t ancestor_order_temp_bytes(long long P) {
  const long long nblk = (P + kOB - 1) / kOB;
  const long long n = nblk * kOB;
  const long long nchunk = (n + kChunk - 1) / kChunk;
  return sizeof(int) * (size_t)(n + nchunk);
}

int launch_ancestor_order(const int* anc, int* own, int* inv, long long P, void* temp, size_t temp_bytes,
                          hipStream_t s) {
  const int nblk = (int)nblocks(P, kOB);
  const long long n = (long long)nblk * kOB;
  const int nchunk = (int)nblocks(n, kChunk);
  if (temp_bytes < ancestor_order_temp_bytes(P)) return -1;
  int* H = static_cast<int*>(temp);
  int* chunk = H + n;
  hipLaunchKernelGGL(k_bucket_hist, dim3(nblk), dim3(kOB), 0, s, anc, P, nblk, H);
  hipLaunchKernelGGL(k_chunk_scan, dim3(nchunk), dim3(256), 0, s, H, n, chunk);
  hipLaunchKernelGGL(k_chunk_offsets, dim3(1), dim3(1024), 0, s, chunk, nchunk);
  hipLaunchKernelGGL(k_bucket_scatter, dim3(nblk), dim3(kOB), 0, s, anc, P, nblk, H, chunk, own, inv);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace gpmdm
