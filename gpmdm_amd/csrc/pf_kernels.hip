// Particle-filter kernels around the fused GP tiles (gfx950).
//
//   k_switch        _propogate_markov_switching   gpmdm_pf.py:137-151
//   k_scan_counts   class counts, per-block offsets, this rank's class segments
//   k_group         stable class grouping (the order of gpmdm_pf.py:158-161)
//   k_dyn_finish    variance + sample mu + sqrt(var) eps   gpmdm.py:1062-1067, gpmdm_pf.py:167-168
//   k_obs_finish    variance + Gaussian log-likelihood      gpmdm.py:958-961, gpmdm_pf.py:188-192
//   k_obs_ll        the same from the tile kernel's fused partial sums (filter path)
//   k_norm_*        log_w = ll - max, w = exp / sum          gpmdm_pf.py:200-204
//   k_guide/k_resample  torch.multinomial(w, P, True) inverse CDF + gathers  gpmdm_pf.py:206-213
//                   and the read-out partial sums            gpmdm_pf.py:224-262, 302-312
//   k_readout       read-out totals
// All arithmetic is fp64; every reduction has a fixed order (bitwise run-to-run repeatable).
#include <cstdlib>

#include "common.h"
#include "pf_kernels.h"

namespace gpmdm {

constexpr int kB = 256;   // threads per block of the O(P) kernels
constexpr unsigned kMaxNormBlocks = 128;   // blocks per filter of k_norm_max

// ---------------------------------------------------------------------------------
// OWN: ancestor-ordered shards (thread i handles particle own[i]); the identity
// instantiation keeps p == i visible to the compiler (one-rank path unchanged).
template <bool OWN>
__global__ __launch_bounds__(kB) void k_switch(SwitchArgs a) {
  __shared__ int hist[kMaxClasses];
  const int tid = threadIdx.x;
  if (tid < a.C) hist[tid] = 0;
  const long long t = (long long)blockIdx.x * kB + tid;
  const long long i = a.base + t;                   // position in the ownership order
  long long dkey = -1;                              // de-duplication key (owner index)
  unsigned pid = 0;                                 // this thread's particle
  if (a.gmax_reset && t < a.F) a.gmax_reset[t] = ord_enc(-INFINITY);
  __syncthreads();
  if (t < a.n) {
    const long long p = OWN ? (long long)a.own[i] : i;
    pid = (unsigned)p;
    const int c0 = a.cls[p];
    const long long f = p / a.Pf;
    const uint2 key = filter_key(a.seed_lo, a.seed_hi, f);
    const unsigned pl = (unsigned)(p - f * a.Pf);
    int best = 0;
    double bestv = -INFINITY;
    for (int j = 0; j < a.C; j += 2) {
      double e0, e1 = 1.0;
      if (a.E) {
        e0 = a.E[p * a.C + j];
        if (j + 1 < a.C) e1 = a.E[p * a.C + j + 1];
      } else {
        const uint4 r = philox4x32_10(make_uint4(pl, a.frame, kStreamSwitch, (unsigned)(j >> 1)), key);
        e0 = -log(u01_oo(r.x, r.y));
        e1 = -log(u01_oo(r.z, r.w));
      }
      // torch.multinomial(p, 1) == argmax(p / E), first maximum (gpmdm_pf.py:150)
      const double v0 = a.T[c0 * a.C + j] / e0;
      if (v0 > bestv) { bestv = v0; best = j; }
      if (j + 1 < a.C) {
        const double v1 = a.T[c0 * a.C + j + 1] / e1;
        if (v1 > bestv) { bestv = v1; best = j + 1; }
      }
    }
    a.cls_new[p] = best;
    atomicAdd(&hist[best], 1);
    if (a.owner && i >= a.lo && i < a.hi) dkey = (long long)best * a.P + f * a.Pf + a.anc[p];
  }
  if (a.owner) {
    // Leader election: one atomicMin per distinct key per wave (its lowest lane), so a
    // collapsed cloud (every particle one ancestor) does not serialise P atomics on one
    // address.  The leader is deterministic; which particle leads does not change any value.
    const int lane = tid & 63;
    unsigned long long pending = __ballot(dkey >= 0);
    while (pending) {
      const int l0 = __ffsll((long long)pending) - 1;
      const unsigned lo32 = __shfl((unsigned)(dkey & 0xffffffffll), l0);
      const int hi32 = __shfl((int)(dkey >> 32), l0);
      const long long k0 = ((long long)hi32 << 32) | lo32;
      const unsigned long long same = __ballot(dkey == k0);
      if (lane == l0) atomicMin(&a.owner[k0], pid);
      pending &= ~same;
    }
  }
  __syncthreads();
  if (tid < a.C) a.blockcounts[(long long)blockIdx.x * a.C + tid] = hist[tid];
}

// ---------------------------------------------------------------------------------
// Exclusive scan of one int per thread over a 1024-thread workgroup: wave shuffles, the 16
// wave totals scanned by wave 0 -- two barriers instead of a 1024-wide Hillis-Steele's
// twenty (integer sums: any association gives the same result).  Returns the exclusive
// prefix of x; *total = the sum over the workgroup.  wtot / wpre: 16 ints of LDS each.
__device__ __forceinline__ int block1024_exclusive_scan(int x, int* wtot, int* wpre, int* total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int v = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(v, off);
    if (lane >= off) v += y;
  }
  if (lane == 63) wtot[w] = v;
  __syncthreads();
  if (w == 0) {
    int t = lane < 16 ? wtot[lane] : 0;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
      const int y = __shfl_up(t, off);
      if (lane >= off) t += y;
    }
    if (lane < 16) wpre[lane] = t;
  }
  __syncthreads();
  *total = wpre[15];
  return v - x + (w ? wpre[w - 1] : 0);
}

// One workgroup: exclusive scans of the per-block class counts, class starts, and the
// segments (grouped position ranges) of this rank's particle slice [lo, hi).
// (a device function: k_small_switch runs the same body inside its workgroup)
__device__ __forceinline__ void scan_counts_body(const ScanArgs& a) {
  __shared__ int wtot[16], wpre[16];
  __shared__ int tot[kMaxClasses];
  __shared__ int lo_cnt[kMaxClasses], hi_cnt[kMaxClasses];
  const int tid = threadIdx.x;
  const int nb = a.nb;
  const int chunk = (nb + 1023) / 1024;
  for (int c = 0; c < a.C; ++c) {
    int s = 0;
    for (int i = 0; i < chunk; ++i) {
      const int b = tid * chunk + i;
      if (b < nb) s += a.blockcounts[(long long)b * a.C + c];
    }
    int total;
    int run = block1024_exclusive_scan(s, wtot, wpre, &total);
    for (int i = 0; i < chunk; ++i) {
      const int b = tid * chunk + i;
      if (b < nb) {
        a.blockoff[(long long)b * a.C + c] = run;
        run += a.blockcounts[(long long)b * a.C + c];
      }
    }
    if (tid == 0) tot[c] = total;
  }
  __syncthreads();
  // counts of each class among particles [0, lo) and [0, hi)
  if (tid < a.C) { lo_cnt[tid] = 0; hi_cnt[tid] = 0; }
  __syncthreads();
  for (int which = 0; which < 2; ++which) {
    const long long bound = which ? a.hi : a.lo;
    const long long bb = bound / kB;
    const long long start = bb * kB;
    if (tid < kB && start + tid < bound) {
      const long long q = a.base + start + tid;
      const int cc = a.cls_new[a.own ? a.own[q] : q];
      atomicAdd(which ? &hi_cnt[cc] : &lo_cnt[cc], 1);
    }
    __syncthreads();
    if (tid < a.C) {
      const int base = bb < nb ? a.blockoff[bb * a.C + tid] : tot[tid];
      if (which) hi_cnt[tid] += base; else lo_cnt[tid] += base;
    }
    __syncthreads();
  }
  if (tid == 0) {
    int cs = 0, ob = 0, ts = 0;
    for (int c = 0; c < a.C; ++c) {
      a.class_start[c] = cs;
      a.counts[c] = tot[c];
      if (a.counts_host) a.counts_host[c] = tot[c];
      const int b0 = cs + lo_cnt[c], e0 = cs + hi_cnt[c];
      a.seg_pos_begin[c] = b0;
      a.seg_pos_end[c] = e0;
      a.seg_out_base[c] = ob;
      a.seg_tile_start[c] = ts;
      ob += e0 - b0;
      ts += (e0 - b0 + a.pt - 1) / a.pt;
      cs += tot[c];
    }
    if (a.counts_seq_host)              // the host waits on this number, not on an event
      publish_seq(a.counts_seq_host, a.counts_seq);   // (this thread wrote counts_host above)
    a.class_start[a.C] = cs;
    a.seg_tile_start[a.C] = ts;
  }
}
__global__ __launch_bounds__(1024) void k_scan_counts(ScanArgs a) { scan_counts_body(a); }

// ---------------------------------------------------------------------------------
template <bool OWN>
__global__ __launch_bounds__(kB) void k_group(GroupArgs a) {
  __shared__ int wcount[kB / 64][kMaxClasses];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long t = (long long)blockIdx.x * kB + tid;
  const long long i = a.base + t;                         // position in the ownership order
  const long long p = t < a.n ? (OWN ? (long long)a.own[i] : i) : -1;
  const int c = p >= 0 ? a.cls_new[p] : -1;
  int rank = 0;
  for (int k = 0; k < a.C; ++k) {
    const unsigned long long m = __ballot(c == k);
    if (c == k) rank = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wcount[w][k] = __popcll(m);
  }
  __syncthreads();
  if (c >= 0) {
    int off = a.class_start[c] + a.blockoff[(long long)blockIdx.x * a.C + c];
    for (int v = 0; v < w; ++v) off += wcount[v][c];
    a.perm[off + rank] = (int)p;
  }
}

// ---------------------------------------------------------------------------------
// Ancestor de-duplication of the dynamics GP.  After a resample, every
// offspring of one ancestor holds a bit-identical copy of its state, and the dynamics GP
// of (state, class) does not depend on anything else, so the tile kernel only needs one
// row per distinct (ancestor, new class) key of this rank's slice: its leader (the
// smallest particle index, k_switch's atomicMin).  Leaders are compacted in class-grouped
// position order, so leader rows of class c are contiguous and the tile kernel's segment
// tables keep their meaning.  Per-particle arithmetic is independent of which rows share a
// tile, so the results are bitwise those of the undeduplicated path.
__device__ __forceinline__ int lead_flag(const LeadArgs& a, long long pos) {
  if (pos >= a.npos) return 0;
  const long long p = a.perm[pos];
  // only this rank's slice registered owners, so owner == p also means "p is in the slice"
  const long long f = p / a.Pf;
  return a.owner[(long long)a.cls_new[p] * a.P + f * a.Pf + a.anc[p]] == (unsigned)p;
}

// flag | block-local exclusive count << 1, and leaders per block
__global__ __launch_bounds__(kB) void k_lead_flags(LeadArgs a) {
  __shared__ int wc[kB / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long pos = (long long)blockIdx.x * kB + tid;
  const int lf = lead_flag(a, pos);
  const unsigned long long m = __ballot(lf);
  const int excl = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) wc[w] = __popcll(m);
  __syncthreads();
  int base = 0;
  for (int v = 0; v < w; ++v) base += wc[v];
  if (pos < a.npos) a.lflag_scan[pos] = ((base + excl) << 1) | lf;
  if (tid == 0) {
    int t = 0;
    for (int v = 0; v < kB / 64; ++v) t += wc[v];
    a.lblock[blockIdx.x] = t;
  }
}

// One workgroup: lblock -> exclusive offsets (in place), then the leader segment tables.
__device__ __forceinline__ void lead_tables_body(const LeadArgs& a) {
  __shared__ int wtot[16], wpre[16];
  __shared__ int total;
  const int tid = threadIdx.x;
  const int nb = a.nb;
  const int chunk = (nb + 1023) / 1024;
  int s = 0;
  for (int i = 0; i < chunk; ++i) {
    const int b = tid * chunk + i;
    if (b < nb) s += a.lblock[b];
  }
  int tsum;
  int run = block1024_exclusive_scan(s, wtot, wpre, &tsum);
  for (int i = 0; i < chunk; ++i) {
    const int b = tid * chunk + i;
    if (b < nb) {
      const int cnt = a.lblock[b];
      a.lblock[b] = run;
      run += cnt;
    }
  }
  if (tid == 0) total = tsum;
  __syncthreads();
  if (tid == 0) {
    auto row = [&](long long x) { return x >= a.npos ? total : a.lblock[x / kB] + (a.lflag_scan[x] >> 1); };
    int ts = 0;
    for (int c = 0; c < a.C; ++c) {
      const int b0 = row(a.seg_pos_begin[c]), e0 = row(a.seg_pos_end[c]);
      a.lseg_pos_begin[c] = b0;
      a.lseg_pos_end[c] = e0;
      a.lseg_out_base[c] = b0;
      a.lseg_tile_start[c] = ts;
      ts += (e0 - b0 + a.pt - 1) / a.pt;
    }
    a.lseg_tile_start[a.C] = ts;
  }
}
__global__ __launch_bounds__(1024) void k_lead_tables(LeadArgs a) { lead_tables_body(a); }

__device__ __forceinline__ void lead_compact_row(const LeadArgs& a, long long pos, int first) {
  if (pos >= a.npos) return;
  const int v = a.lflag_scan[pos];
  if (!(v & 1)) return;
  const long long p = a.perm[pos];
  const int r = first + (v >> 1);
  const long long f = p / a.Pf;
  a.lperm[r] = (int)p;
  const long long key = (long long)a.cls_new[p] * a.P + f * a.Pf + a.anc[p];
  a.slot[key] = r;
  if (a.owner_reset) a.owner_reset[key] = 0xffffffffu;   // the next election's preset
}
__global__ __launch_bounds__(kB) void k_lead_compact(LeadArgs a) {
  lead_compact_row(a, (long long)blockIdx.x * kB + threadIdx.x, a.lblock[blockIdx.x]);
}

// k_lead_tables + k_lead_compact in one launch (nb <= kMaxLeadBlocks): block b's first leader
// row is the sum of the leader counts of blocks 0 .. b-1, which the block adds up itself
// (integers: any order gives k_lead_tables's prefix); block 0 also scans every block's count
// and writes the leader segment tables with k_lead_tables's row rule.  Same rows, same tables.
// Up to 1024 blocks (P <= 262,144 per launch): each block's prefix re-sum is O(nb) loads and
// block 0's table is 4 KB of static LDS in every block; above, the two launches (ADVICE r5:
// at nb = 8192 the re-sums were ~33M loads and a 32 KB table limited occupancy).
constexpr int kMaxLeadBlocks = 1024;
__global__ __launch_bounds__(kB) void k_lead_tables_compact(LeadArgs a) {
  __shared__ int red[kB / 64];
  __shared__ int pre[kMaxLeadBlocks];          // block 0: exclusive prefix of every block's count
  __shared__ int total_s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x, nb = a.nb;
  int s = 0;
  for (int bb = tid; bb < b; bb += kB) s += a.lblock[bb];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) red[w] = s;
  __syncthreads();
  int first = 0;
#pragma unroll
  for (int v = 0; v < kB / 64; ++v) first += red[v];
  if (b == 0) {
    // exclusive scan of the counts: per thread a chunk of consecutive blocks, then a
    // 256-wide scan of the chunk sums (wave shuffles + the four wave totals)
    const int chunk = (nb + kB - 1) / kB;
    int cs = 0;
    for (int i = 0; i < chunk; ++i) {
      const int bb = tid * chunk + i;
      if (bb < nb) cs += a.lblock[bb];
    }
    int incl = cs;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(incl, off);
      if (lane >= off) incl += y;
    }
    __syncthreads();                           // (red is reused)
    if (lane == 63) red[w] = incl;
    __syncthreads();
    int run = incl - cs;
    for (int v = 0; v < w; ++v) run += red[v];
    for (int i = 0; i < chunk; ++i) {
      const int bb = tid * chunk + i;
      if (bb < nb) {
        pre[bb] = run;
        run += a.lblock[bb];
      }
    }
    if (tid == kB - 1) total_s = run;
    __syncthreads();
    if (tid == 0) {
      const int total = total_s;
      auto row = [&](long long x) { return x >= a.npos ? total : pre[x / kB] + (a.lflag_scan[x] >> 1); };
      int ts = 0;
      for (int c = 0; c < a.C; ++c) {
        const int b0 = row(a.seg_pos_begin[c]), e0 = row(a.seg_pos_end[c]);
        a.lseg_pos_begin[c] = b0;
        a.lseg_pos_end[c] = e0;
        a.lseg_out_base[c] = b0;
        a.lseg_tile_start[c] = ts;
        ts += (e0 - b0 + a.pt - 1) / a.pt;
      }
      a.lseg_tile_start[a.C] = ts;
    }
  }
  lead_compact_row(a, (long long)b * kB + tid, first);
}


// ---------------------------------------------------------------------------------
// Small single-shard filters (all P <= kSmallSwitchP particles switched by one rank, no
// ownership order): one 1024-thread workgroup runs the switch, the class scan, the grouping
// and the leader compaction in one launch instead of seven (with the owner preset).  Every
// step is integer and deterministic (the leader of a key is its smallest particle index,
// whatever the order of the atomics; integer sums in any order are equal), the 256-thread
// blocks of k_switch / k_group / k_lead_* are the workgroup's quarters, and what the
// multi-kernel path reads back from its buffers is kept in LDS (the buffers are still
// written for the later stages), so every table is the multi-kernel path's exactly
// (tests/test_gpu_small_path.py).  The scans over at most four blocks are one thread per
// class (or one thread) instead of 1024-wide Hillis-Steele passes.
constexpr long long kSmallSwitchP = 1024;

__global__ __launch_bounds__(1024) void k_small_switch(SwitchArgs sa, ScanArgs sc, GroupArgs ga, LeadArgs la,
                                                       int dedup) {
  __shared__ int hist[4][kMaxClasses];        // block counts (blockcounts)
  __shared__ int boff[4][kMaxClasses];        // block offsets (blockoff)
  __shared__ int cstart[kMaxClasses];         // class_start
  __shared__ int lo_cnt[kMaxClasses], hi_cnt[kMaxClasses];
  __shared__ int segb[kMaxClasses], sege[kMaxClasses], sego[kMaxClasses], segt[kMaxClasses + 1];
  __shared__ int ctot[kMaxClasses];
  __shared__ int lsegb[kMaxClasses], lsege[kMaxClasses], lsegt[kMaxClasses + 1];
  __shared__ int wcount[4][4][kMaxClasses];
  __shared__ int wc[4][4];
  __shared__ int lblk[4];
  __shared__ int cls_s[kSmallSwitchP];        // cls_new
  __shared__ int anc_s[kSmallSwitchP];        // anc
  __shared__ int perm_s[kSmallSwitchP];       // perm
  __shared__ int lflag_s[kSmallSwitchP];      // lflag_scan
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, b = tid >> 8, wq = w & 3;
  const long long P = sa.P;
  const int C = sa.C;
  const int nb = (int)((P + kB - 1) / kB);
  if (dedup)
    for (long long i = tid; i < (long long)C * P; i += 1024) sa.owner[i] = 0xffffffffu;
  if (tid < 4 * kMaxClasses) hist[tid / kMaxClasses][tid % kMaxClasses] = 0;
  if (tid < kMaxClasses) { lo_cnt[tid] = 0; hi_cnt[tid] = 0; }
  if (sa.gmax_reset && tid < sa.F) sa.gmax_reset[tid] = ord_enc(-INFINITY);
  __threadfence();                            // the owner preset lands before the atomics
  __syncthreads();
  // ---- k_switch ----
  const long long p = tid;
  int best = -1;
  if (p < P) {
    const int c0 = sa.cls[p];
    const long long f = p / sa.Pf;
    const uint2 key = filter_key(sa.seed_lo, sa.seed_hi, f);
    const unsigned pl = (unsigned)(p - f * sa.Pf);
    best = 0;
    double bestv = -INFINITY;
    for (int j = 0; j < C; j += 2) {
      double e0, e1 = 1.0;
      if (sa.E) {
        e0 = sa.E[p * C + j];
        if (j + 1 < C) e1 = sa.E[p * C + j + 1];
      } else {
        const uint4 r = philox4x32_10(make_uint4(pl, sa.frame, kStreamSwitch, (unsigned)(j >> 1)), key);
        e0 = -log(u01_oo(r.x, r.y));
        e1 = -log(u01_oo(r.z, r.w));
      }
      const double v0 = sa.T[c0 * C + j] / e0;
      if (v0 > bestv) { bestv = v0; best = j; }
      if (j + 1 < C) {
        const double v1 = sa.T[c0 * C + j + 1] / e1;
        if (v1 > bestv) { bestv = v1; best = j + 1; }
      }
    }
    sa.cls_new[p] = best;
    cls_s[p] = best;
    atomicAdd(&hist[b][best], 1);
    if (dedup) {
      const int an = sa.anc[p];
      anc_s[p] = an;
      if (p >= sa.lo && p < sa.hi) atomicMin(&sa.owner[(long long)best * P + f * sa.Pf + an], (unsigned)p);
    }
  }
  __syncthreads();
  // ---- k_scan_counts ----
  if (tid < nb * C) sa.blockcounts[tid] = hist[tid / C][tid % C];   // block bb, class c: bb * C + c
  if (tid < C) {
    int run = 0;
    for (int bb = 0; bb < nb; ++bb) {
      boff[bb][tid] = run;
      sc.blockoff[(long long)bb * C + tid] = run;
      run += hist[bb][tid];
    }
    cstart[tid] = run;                         // class total, until the table pass
  }
  // class counts among positions [0, lo) and [0, hi): the partial block by atomics
  for (int which = 0; which < 2; ++which) {
    const long long bound = which ? sc.hi : sc.lo;
    const long long start = (bound / kB) * kB;
    if (tid < kB && start + tid < bound) atomicAdd(which ? &hi_cnt[cls_s[start + tid]] : &lo_cnt[cls_s[start + tid]], 1);
  }
  __syncthreads();
  if (tid == 0) {
    int cs = 0, ob = 0, ts = 0;
    for (int c = 0; c < C; ++c) {
      const int tot = cstart[c];
      const long long blo = sc.lo / kB, bhi = sc.hi / kB;
      const int lo = lo_cnt[c] + (blo < nb ? boff[blo][c] : tot);
      const int hi = hi_cnt[c] + (bhi < nb ? boff[bhi][c] : tot);
      cstart[c] = cs;
      ctot[c] = tot;
      const int b0 = cs + lo, e0 = cs + hi;
      segb[c] = b0;
      sege[c] = e0;
      sego[c] = ob;
      segt[c] = ts;
      ob += e0 - b0;
      ts += (e0 - b0 + sc.pt - 1) / sc.pt;
      cs += tot;
    }
    segt[C] = ts;
    hist[0][0] = cs;                           // (class_start[C]; hist is not read again)
  }
  __syncthreads();
  // the tables, one entry per lane (a one-thread loop of stores is vectorised into wide
  // stores, which tests/test_isa_guard.py rejects)
  if (tid < C) {
    sc.class_start[tid] = cstart[tid];
    sc.counts[tid] = ctot[tid];
    if (sc.counts_host) sc.counts_host[tid] = ctot[tid];
    sc.seg_pos_begin[tid] = segb[tid];
    sc.seg_pos_end[tid] = sege[tid];
    sc.seg_out_base[tid] = sego[tid];
    sc.seg_tile_start[tid] = segt[tid];
  } else if (tid == C) {
    sc.class_start[C] = hist[0][0];
    sc.seg_tile_start[C] = segt[C];
  }
  // ---- k_group ----
  {
    const int c = best;
    int rank = 0;
    for (int k = 0; k < C; ++k) {
      const unsigned long long m = __ballot(c == k);
      if (c == k) rank = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) wcount[b][wq][k] = __popcll(m);
    }
    __syncthreads();
    if (c >= 0) {
      int off = cstart[c] + boff[b][c];
      for (int v = 0; v < wq; ++v) off += wcount[b][v][c];
      ga.perm[off + rank] = (int)p;
      perm_s[off + rank] = (int)p;
    }
  }
  __syncthreads();
  if (!dedup) return;
  // ---- k_lead_flags ----
  {
    const long long pos = p;
    int lf = 0;
    if (pos < la.npos) {
      const long long q = perm_s[pos];
      const long long f = q / la.Pf;
      // the owners were set by this launch's atomics (at L2): read them past the L1
      lf = __hip_atomic_load(&la.owner[(long long)cls_s[q] * la.P + f * la.Pf + anc_s[q]], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT) == (unsigned)q;
    }
    const unsigned long long m = __ballot(lf);
    const int excl = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wc[b][wq] = __popcll(m);
    __syncthreads();
    int base = 0;
    for (int v = 0; v < wq; ++v) base += wc[b][v];
    if (pos < la.npos) {
      la.lflag_scan[pos] = ((base + excl) << 1) | lf;
      lflag_s[pos] = ((base + excl) << 1) | lf;
    }
    if (tid == 0) {                            // ---- k_lead_tables (one thread) ----
      int run = 0;
      for (int bb = 0; bb < nb; ++bb) {
        int t = 0;
        for (int v = 0; v < kB / 64; ++v) t += wc[bb][v];
        lblk[bb] = run;
        run += t;
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    int total = 0;
    for (int bb = 0; bb < nb; ++bb)
      for (int v = 0; v < kB / 64; ++v) total += wc[bb][v];
    auto row = [&](long long x) { return x >= la.npos ? total : lblk[x / kB] + (lflag_s[x] >> 1); };
    int ts = 0;
    for (int c = 0; c < C; ++c) {
      const int b0 = row(segb[c]), e0 = row(sege[c]);
      lsegb[c] = b0;
      lsege[c] = e0;
      lsegt[c] = ts;
      ts += (e0 - b0 + la.pt - 1) / la.pt;
    }
    lsegt[C] = ts;
  }
  __syncthreads();
  if (tid < C) {
    la.lseg_pos_begin[tid] = lsegb[tid];
    la.lseg_pos_end[tid] = lsege[tid];
    la.lseg_out_base[tid] = lsegb[tid];
    la.lseg_tile_start[tid] = lsegt[tid];
  } else if (tid == C) {
    la.lseg_tile_start[C] = lsegt[C];
  }
  // ---- k_lead_compact ----
  if (tid < nb) la.lblock[tid] = lblk[tid];
  if (p < la.npos) {
    const int v = lflag_s[p];
    if (v & 1) {
      const long long q = perm_s[p];
      const int r = lblk[b] + (v >> 1);
      const long long f = q / la.Pf;
      la.lperm[r] = (int)q;
      la.slot[(long long)cls_s[q] * la.P + f * la.Pf + anc_s[q]] = r;
    }
  }
}

// ---------------------------------------------------------------------------------
// Failure counters: one atomic per wave for the lanes that saw the event (events are rare;
// a collapsed or indefinite model can make every particle bad, hence the ballot).
__device__ __forceinline__ void count_event(unsigned* ctr, bool bad) {
  const unsigned long long b = __ballot(bad);
  if (b && (int)(threadIdx.x & 63) == __ffsll((long long)b) - 1) atomicAdd(ctr, (unsigned)__popcll(b));
}

// ---------------------------------------------------------------------------------
// out index o -> class segment
__device__ __forceinline__ int seg_of(const int* seg_out_base, int n_seg, int total, int o) {
  int c = 0;
  for (int s = 1; s < n_seg; ++s)
    if (o >= seg_out_base[s]) c = s;
  (void)total;
  return c;
}

__global__ __launch_bounds__(kB) void k_dyn_finish(DynFinishArgs a) {
  const long long o = (long long)blockIdx.x * kB + threadIdx.x;
  if (a.gmax_reset && o < a.F) a.gmax_reset[o] = ord_enc(-INFINITY);
  if (o < a.z_n) a.z_dst[o] = a.z_src[o];
  if (a.rows_out && o == 0) {
    int r = 0;
    for (int c = 0; c < a.n_rows_seg; ++c) r += a.rows_e[c] - a.rows_b[c];
    a.rows_out[0] = r;
    if (a.rows_host) a.rows_host[0] = r;
  }
  if (o >= a.n_out) return;
  const int c = a.seg_out_base ? seg_of(a.seg_out_base, a.n_seg, (int)a.n_out, (int)o) : 0;
  const long long pos = (a.seg_pos_begin ? a.seg_pos_begin[c] : 0) + (o - (a.seg_out_base ? a.seg_out_base[c] : 0));
  const long long p = a.perm ? a.perm[pos] : pos;
  long long r = o;                      // tile row holding this particle's GP outputs
  if (a.slot) r = a.slot[(long long)c * a.P + (p / a.Pf) * a.Pf + a.anc[p]];
  double q = 0.0;
  const int np = a.n_parts[c];
  for (int k = 0; k < np; ++k) q += a.qpart[(long long)k * a.ld_q + r];
  // k(x*, x*) of the dynamics kernel without noise: 1 + [x,1] diag(c^2) [x,1]^T (gpmdm.py:1100)
  const int d = a.d;
  double kd = 0.0;
  for (int j = 0; j < d; ++j) {
    const double x = a.X[p * d + j];
    kd = fma(a.lin_c2[j] * x, x, kd);
  }
  kd = 1.0 + (kd + a.lin_c2[d]);
  const double vc = kd - q;
  if (a.var_out) {                      // predictive map (map_x_dynamics_for_class)
    for (int j = 0; j < d; ++j) a.var_out[o * d + j] = vc * a.il2[j];
    return;
  }
  bool bad_state = false;
  // torch.normal(mean, std) = eps * std + mean (gpmdm_pf.py:167-168)
  for (int j = 0; j < d; j += 2) {
    double e0, e1 = 0.0;
    if (a.normals) {
      e0 = a.normals[pos * d + j];
      if (j + 1 < d) e1 = a.normals[pos * d + j + 1];
    } else {
      const long long f = p / a.Pf;
      const uint4 r = philox4x32_10(make_uint4((unsigned)(p - f * a.Pf), a.frame, kStreamDyn, (unsigned)(j >> 1)),
                                    filter_key(a.seed_lo, a.seed_hi, f));
      const double u1 = u01_oo(r.x, r.y), u2 = u01_co(r.z, r.w);
      const double rr = sqrt(-2.0 * log(u1));
      double sn, cs;
      sincos(6.283185307179586476925 * u2, &sn, &cs);
      e0 = rr * cs;
      e1 = rr * sn;
    }
    const double x0 = e0 * sqrt(vc * a.il2[j]) + a.mu[r * a.ld_mu + j];
    a.X_out[p * d + j] = x0;
    bad_state |= !isfinite(x0);
    if (j + 1 < d) {
      const double x1 = e1 * sqrt(vc * a.il2[j + 1]) + a.mu[r * a.ld_mu + j + 1];
      a.X_out[p * d + j + 1] = x1;
      bad_state |= !isfinite(x1);
    }
  }
  if (a.health) {
    count_event(a.health + kHealthDynVar, !(vc > 0.0));
    count_event(a.health + kHealthDynState, bad_state);
  }
}

// ---------------------------------------------------------------------------------
// One wave per particle: the D-term log-likelihood sum is spread over 64 lanes.
__global__ __launch_bounds__(kB) void k_obs_finish(ObsFinishArgs a) {
  const int lane = threadIdx.x & 63;
  const long long o = (long long)blockIdx.x * (kB / 64) + (threadIdx.x >> 6);
  double llv = -INFINITY;
  if (o < a.n_out) {
    double q = 0.0;
    for (int k = lane; k < a.n_parts; k += 64) q += a.qpart[(long long)k * a.ld_q + o];
    q = wave_sum(q);
    const double vc = 1.0 - q;                         // k(x*,x*) = 1 (gpmdm.py:991)
    const double* mu = a.mu + o * a.ld_mu;
    if (a.var_out) {
      for (int j = lane; j < a.D; j += 64) a.var_out[o * a.D + j] = vc * a.il2[j];
    } else {
      // ll = -1/2 sum[(z-mu)^2/var + log var] + sum(-log sqrt var) - D/2 ln(2pi)_f32
      const double* z = a.z + ((a.ll_offset + o) / a.Pf) * a.D;
      double s1 = 0.0, s2 = 0.0;
      for (int j = lane; j < a.D; j += 64) {
        const double var = vc * a.il2[j];
        const double t = z[j] - mu[j];
        s1 += t * t / var + log(var);
        s2 += -log(sqrt(var));
      }
      s1 = wave_sum(s1);
      s2 = wave_sum(s2);
      llv = -0.5 * s1 + s2 - a.ll_const;
      if (lane == 0) a.ll[a.ll_offset + o] = llv;
    }
  }
}

// Fused form of k_obs_finish for the filter (one thread per particle): the tile kernel
// left S = sum_j (z_j - mu_j)^2 lam2_j in spart, and with var_j = vc il2_j
//   ll = -1/2 sum_j[(z_j - mu_j)^2 / var_j + log var_j] + sum_j(-log sqrt var_j) - D/2 ln(2pi)_f32
//      = -1/2 S / vc - D log vc - sum_j log il2_j - D/2 ln(2pi)_f32
// (the reference's double count of log var kept, gpmdm_pf.py:188-192).
// (a device function: k_small_resample computes a deferred finish with the same code)
__device__ __forceinline__ double obs_ll_value(const ObsFinishArgs& a, long long o, double& vc) {
  double q = 0.0;
  for (int k = 0; k < a.n_parts; ++k) q += a.qpart[(long long)k * a.ld_q + o];
  double S = 0.0;
  for (int k = a.jm0; k < a.n_j; ++k) S += a.spart[(long long)k * a.ld_q + o];
  if (a.cut_part && o >= a.cut_o0) {
    // a split tile: its first part left q and S over list entries [0, tpc c*); the second
    // part's entries follow in list order (R tiles into q, then mean tiles into S), the whole
    // tile's running sums exactly
    const long long r = o - a.cut_o0;
    const int2 sp = a.cut_split[r / a.cut_pt];
    const int nt = sp.x + a.cut_tm;
    const int r0 = cutoff_chunk_begin(1, nt, a.cut_tpc);
    const double* pp = a.cut_part + r;
    int i = cutoff_chunk_begin(sp.y, nt, a.cut_tpc);
    for (; i + 8 <= nt; i += 8) {              // eight loads in flight, then the adds in order
      double v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = pp[(long long)(i + k - r0) * a.cut_ld];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (i + k < sp.x)
          q += v[k];
        else
          S += v[k];
      }
    }
    for (; i < nt; ++i) {
      const double v = pp[(long long)(i - r0) * a.cut_ld];
      if (i < sp.x)
        q += v;
      else
        S += v;
    }
  }
  vc = 1.0 - q;                                        // k(x*,x*) = 1 (gpmdm.py:991)
  return -0.5 * S / vc - a.D * log(vc) - a.sum_log_il2 - a.ll_const;
}

__global__ __launch_bounds__(kB) void k_obs_ll(ObsFinishArgs a) {
  const long long o = (long long)blockIdx.x * kB + threadIdx.x;
  unsigned long long key = 0;            // below ord_enc of any double
  if (o < a.n_out) {
    double vc;
    const double llv = obs_ll_value(a, o, vc);
    a.ll[a.own ? a.own[a.ll_offset + o] : a.ll_offset + o] = llv;
    if (a.health) {
      count_event(a.health + kHealthObsVar, !(vc > 0.0));
      count_event(a.health + kHealthObsLL, !isfinite(llv));
    }
    key = ord_enc(fmax(-INFINITY, llv));  // k_norm_max's value set: NaN ignored
  }
  if (a.bmax) {
    // the block's maximum as an integer key: the max of a set in ord_enc's total order
    // does not depend on how the set is split, so k_norm_exp_scan's max over the block
    // maxima is k_norm_max's atomicMax result exactly
    __shared__ unsigned long long wk[kB / 64];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned long long y = __shfl_xor(key, off);
      key = y > key ? y : key;
    }
    if ((threadIdx.x & 63) == 0) wk[threadIdx.x >> 6] = key;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long m = wk[0];
      for (int i = 1; i < kB / 64; ++i) m = wk[i] > m ? wk[i] : m;
      a.bmax[blockIdx.x] = m;
    }
  }
}

// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(kB) void k_norm_max(NormArgs a) {
  __shared__ double s[kB / 64];
  const long long f = blockIdx.y;
  // grid-stride over the filter's particles: at most kMaxNormBlocks atomics per filter
  // address (one per block; thousands of same-address atomics serialise at the L2)
  double v = -INFINITY;
  for (long long p = (long long)blockIdx.x * kB + threadIdx.x; p < a.P; p += (long long)gridDim.x * kB)
    v = fmax(v, a.ll[f * a.P + p]);
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = s[0];
    for (int i = 1; i < kB / 64; ++i) m = fmax(m, s[i]);
    atomicMax(a.gmax + f, ord_enc(m));
  }
}

// e = exp(ll - max); block-local inclusive scan of e; block sums.
__global__ __launch_bounds__(kB) void k_norm_exp_scan(NormArgs a) {
  __shared__ double wsum[kB / 64];
  __shared__ unsigned long long wk[kB / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long f = blockIdx.y;
  const long long p = (long long)blockIdx.x * kB + tid;
  double M;
  if (a.bmax) {
    // single filter: the maximum over k_obs_ll's block maxima (no k_norm_max launch); every
    // block computes it, block 0 publishes it for the resample and export
    unsigned long long key = 0;
    const int nk = a.nbmax ? a.nbmax : a.nb;
    for (int i = tid; i < nk; i += kB) key = a.bmax[i] > key ? a.bmax[i] : key;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned long long y = __shfl_xor(key, off);
      key = y > key ? y : key;
    }
    if (lane == 0) wk[w] = key;
    __syncthreads();
    key = wk[0];
    for (int i = 1; i < kB / 64; ++i) key = wk[i] > key ? wk[i] : key;
    if (blockIdx.x == 0 && tid == 0) a.gmax[f] = key;
    M = ord_dec(key);
  } else {
    M = ord_dec(a.gmax[f]);
  }
  const double e = p < a.P ? exp(a.ll[f * a.P + p] - M) : 0.0;
  if (p < a.P) a.e[f * a.P + p] = e;
  double x = e;                               // wave inclusive scan
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const double y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  double base = 0.0;
  for (int v = 0; v < w; ++v) base += wsum[v];
  x += base;
  if (p < a.P) a.local[f * a.P + p] = x;
  if (tid == kB - 1) a.blocksum[f * a.nb + blockIdx.x] = x;
}

// One workgroup per filter: exclusive scan of block sums, total S.
__global__ __launch_bounds__(1024) void k_norm_total(NormArgs a) {
  __shared__ double part[1024];
  const int tid = threadIdx.x;
  const int nb = a.nb;
  const long long f = blockIdx.x;
  const double* blocksum = a.blocksum + f * nb;
  double* blockoff = a.blockoff + f * nb;
  const int chunk = (nb + 1023) / 1024;
  double s = 0.0;
  for (int i = 0; i < chunk; ++i) {
    const int b = tid * chunk + i;
    if (b < nb) s += blocksum[b];
  }
  part[tid] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const double v = tid >= off ? part[tid - off] : 0.0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  double run = tid ? part[tid - 1] : 0.0;
  for (int i = 0; i < chunk; ++i) {
    const int b = tid * chunk + i;
    if (b < nb) {
      blockoff[b] = run;
      run += blocksum[b];
    }
  }
  if (tid == 1023) a.total[f] = part[1023];
}

// The normalised CDF of filter f at particle i: k_norm_exp_scan's block-local inclusive scan
// plus k_norm_total's block offset, over the total, the last bucket forced to 1 (torch:
// cumsum(w) / sum, gpmdm_pf.py:206-213).  Evaluated where the inverse-CDF searches read it
// (k_guide, k_sys_marks, k_resample) instead of stored by a CDF pass: the same expression on
// the same operands, so every value -- and every index -- is the stored CDF's, one dependent
// launch fewer per frame.
struct CdfView {
  const double* boff;
  const double* local;
  double S;
  long long P;
  __device__ __forceinline__ double operator[](long long i) const {
    return i == P - 1 ? 1.0 : (boff[i / kB] + local[i]) / S;
  }
};
__device__ __forceinline__ CdfView cdf_view(const ResampleArgs& a, long long f) {
  return CdfView{a.blockoff + f * a.nb, a.local + f * a.P, a.total[f], a.P};
}

// One thread per output slot s: inverse-CDF search, gather, read-out partials.
// identity=1 computes the read-outs of the current state without resampling (after init).
// Guide table for the inverse-CDF search: guide[b] = first i with cum[i] >= b / GB (P if
// none), for b = 0 .. GB + 2.  The queries b / GB are sorted, so neighbouring threads walk
// nearly the same binary-search path (cache-friendly, unlike the random uniforms).
//
// A wave's 64 queries are consecutive, so their answers lie between those of its first and
// last query: lanes 0-31 and 32-63 find those two by 32-way searches (32 independent probes
// per step: four steps span 10^6 particles, against 20 dependent loads of a binary search),
// then each lane searches the usually short range between them -- in registers when it holds
// at most 64 particles (a collapsed cloud's range is often a single particle).  For a monotone
// CDF every form returns the binary search's answer.
__global__ __launch_bounds__(kB) void k_guide(ResampleArgs a) {
  const long long f = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const long long b = (long long)blockIdx.x * kB + threadIdx.x;
  const long long nb = a.GB + 3;                       // queries b = 0 .. GB + 2
  const long long b0 = b - lane;                       // the wave's first query
  if (b0 >= nb) return;                                // (wave-uniform)
  const long long bl = b0 + 63 < nb - 1 ? b0 + 63 : nb - 1;   // its last query
  const CdfView cum = cdf_view(a, f);
  // two 32-way searches in lock step: half h finds the first index with cum >= t(h ? bl : b0)
  const int h = lane >> 5, k = lane & 31;
  const unsigned long long hm = h ? 0xffffffff00000000ull : 0x00000000ffffffffull;
  const double th = (double)(h ? bl : b0) / (double)a.GB;
  long long L = 0, H = a.P;
  while (__ballot(H - L > 32)) {
    const long long st = (H - L + 31) / 32;
    const bool live = H - L > 32;
    long long q = (L + (long long)(k + 1) * st < H ? L + (long long)(k + 1) * st : H) - 1;
    q = q > 0 ? q : 0;
    const long long c = __popcll(__ballot(live && cum[q] < th) & hm);
    if (live) {
      const long long nH = L + (c + 1) * st < H ? L + (c + 1) * st : H;
      L = L + c * st < H ? L + c * st : H;
      H = nH;
    }
  }
  {
    const long long q = L + k;
    L += __popcll(__ballot(q < H && cum[q] < th) & hm);
  }
  const long long A0 = __shfl(L, 0), A1 = __shfl(L, 32);
  const double t = (double)b / (double)a.GB;
  long long lo = A0, hi = A1;                          // this lane's answer is in [A0, A1]
  if (A1 - A0 <= 64) {
    // the range's CDF values in registers, one per lane; per lane a binary search over them
    const double v = A0 + lane < A1 ? cum[A0 + lane] : 0.0;
    int l = 0, r = (int)(A1 - A0);
    while (__ballot(r > l)) {
      const int m = l + (r - l) / 2;
      const double vm = __shfl(v, m < 63 ? m : 63);
      if (r > l) {
        if (vm < t) l = m + 1; else r = m;
      }
    }
    lo = A0 + l;
  } else {
    while (hi - lo > 0) {
      const long long mid = lo + (hi - lo) / 2;
      if (cum[mid] < t) lo = mid + 1; else hi = mid;
    }
  }
  if (b < nb) a.guide[f * nb + b] = (int)lo;
}

// ---------------------------------------------------------------------------------
// Systematic resampling by scan (north_star's scan-based systematic resampler).  Slot s
// draws u_s = (s + u0) / P; the search form gives slot s the first i with cum_i >= u_s, so
// particle i owns slots [S_{i-1}, S_i) with S_i = #{s : u_s <= cum_i} (u_s is monotone in
// s).  S_i comes from the closed form floor(cum_i P - u0) + 1, corrected against the same
// fp64 expression for u_s the search compares, so the indices are exactly the search's.
// Each particle with offspring marks the start of its run; an inclusive max-scan over the
// slots then fills every run with its particle: O(P) work, no per-slot search, no load
// imbalance when one ancestor takes most slots.
__device__ __forceinline__ double sys_u(long long s, double u0, long long P) {
  return ((double)s + u0) / (double)P;                      // exactly k_resample's expression
}
__device__ __forceinline__ long long sys_count(double c, double u0, long long P) {
  long long k = (long long)floor(c * (double)P - u0) + 1;    // estimate of #{s : u_s <= c}
  k = k < 0 ? 0 : (k > P ? P : k);
  while (k > 0 && sys_u(k - 1, u0, P) > c) --k;
  while (k < P && sys_u(k, u0, P) <= c) ++k;
  return k;
}
__device__ __forceinline__ double sys_u0(const ResampleArgs& a, long long f) {
  if (a.U) return a.U[0];
  const uint4 r = philox4x32_10(make_uint4(0u, a.frame, kStreamSystematic, 0u), filter_key(a.seed_lo, a.seed_hi, f));
  return u01_co(r.x, r.y);
}

// marks[s] = i where particle i's offspring start (-1 elsewhere: memset before)
__global__ __launch_bounds__(kB) void k_sys_marks(ResampleArgs a) {
  const long long f = blockIdx.y;
  const long long i = (long long)blockIdx.x * kB + threadIdx.x;
  if (i >= a.P) return;
  const double u0 = sys_u0(a, f);
  const CdfView cum = cdf_view(a, f);
  const long long lo = i > 0 ? sys_count(cum[i - 1], u0, a.P) : 0;
  const long long hi = sys_count(cum[i], u0, a.P);
  if (hi > lo) a.sys_mark[f * a.P + lo] = (int)i;
}

// block-local inclusive max-scan of the marks (in place) and the block maxima
__global__ __launch_bounds__(kB) void k_sys_scan(ResampleArgs a) {
  __shared__ int wmax[kB / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long f = blockIdx.y;
  const long long s = (long long)blockIdx.x * kB + tid;
  int x = s < a.P ? a.sys_mark[f * a.P + s] : -1;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off);
    if (lane >= off) x = max(x, y);
  }
  if (lane == 63) wmax[w] = x;
  __syncthreads();
  for (int v = 0; v < w; ++v) x = max(x, wmax[v]);
  if (s < a.P) a.sys_mark[f * a.P + s] = x;
  if (tid == kB - 1) a.sys_block[f * a.nb + blockIdx.x] = x;
}

// one workgroup per filter: exclusive max-scan of the block maxima (in place)
__global__ __launch_bounds__(1024) void k_sys_blocks(ResampleArgs a) {
  __shared__ int part[1024];
  const int tid = threadIdx.x;
  const long long f = blockIdx.x;
  int* blk = a.sys_block + f * a.nb;
  const int chunk = (a.nb + 1023) / 1024;
  int mx = -1;
  for (int i = 0; i < chunk; ++i) {
    const int b = tid * chunk + i;
    if (b < a.nb) mx = max(mx, blk[b]);
  }
  part[tid] = mx;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = tid >= off ? part[tid - off] : -1;
    __syncthreads();
    part[tid] = max(part[tid], v);
    __syncthreads();
  }
  int run = tid ? part[tid - 1] : -1;
  for (int i = 0; i < chunk; ++i) {
    const int b = tid * chunk + i;
    if (b < a.nb) {
      const int v = blk[b];
      blk[b] = run;
      run = max(run, v);
    }
  }
}

__global__ __launch_bounds__(kB) void k_resample(ResampleArgs a) {
  __shared__ double red[kB / 64][kMaxReadout];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long f = blockIdx.y;
  const long long s = (long long)blockIdx.x * kB + tid;   // slot within filter f
  const long long g0 = f * a.P;                            // filter f's first particle
  const uint2 key = filter_key(a.seed_lo, a.seed_hi, f);
  const int C = a.C, d = a.d;
  const int nq = C + 1 + d;
  const bool act = s < a.P;
  long long idx = 0;                                       // source, within filter f
  int cnew = -1;
  const double* xs = nullptr;                              // the source particle's state
  double e2 = 0.0, wv = 0.0;
  if (act) {
    if (a.identity) {
      idx = s;
    } else if (a.sys_mark) {                                // systematic by scan
      idx = max(a.sys_mark[g0 + s], a.sys_block[f * a.nb + blockIdx.x]);
    } else {
      double u;
      if (a.systematic) {                    // (search form; the filter resamples by scan)
        u = sys_u(s, sys_u0(a, f), a.P);
      } else if (a.U) {
        u = a.U[s];
      } else {
        const uint4 r = philox4x32_10(make_uint4((unsigned)s, a.frame, kStreamResample, 0u), key);
        u = u01_co(r.x, r.y);
      }
      const CdfView cum = cdf_view(a, f);
      // first index with cum >= u (torch's searchsorted), searched between two guide
      // entries that bracket it: t_lo = (q0 - 1) / GB <= u and t_hi = (q0 + 2) / GB > u for
      // q0 = floor(u GB) whatever its rounding, so the result is exactly that of a search
      // over [0, P]
      long long lo = 0, hi = a.P;
      if (a.GB > 0) {                           // guided (large P): bracket, then search
        const int* gd = a.guide + f * (a.GB + 3);
        const long long q0 = (long long)floor(u * (double)a.GB);
        lo = gd[q0 - 1 > 0 ? q0 - 1 : 0];
        hi = gd[q0 + 2 < a.GB + 2 ? q0 + 2 : a.GB + 2];
      }
      while (hi - lo > 0) {
        const long long mid = lo + (hi - lo) / 2;
        if (cum[mid] < u) lo = mid + 1; else hi = mid;
      }
      idx = lo;
    }
    if (a.rows) {                 // the exchanged row of particle idx, read in place
      const double* row = a.rows + (a.rows_inv ? (long long)a.rows_inv[g0 + idx] : g0 + idx) * a.rows_w;
      cnew = (int)row[0];
      xs = row + 1;
    } else {
      cnew = a.cls_src[g0 + idx];
      xs = a.X_src + (g0 + idx) * d;
    }
    if (!a.identity) {
      a.ridx[g0 + s] = (int)idx;
      a.cls_dst[g0 + s] = cnew;
    }
    // read-outs: post-resample class/state at slot s, pre-resample ll/log_w at slot s
    const double M = ord_dec(a.gmax[f]);
    const double llv = a.ll[g0 + s];
    const double lw = llv - M;
    e2 = exp((llv + lw) - M);                  // ll + log_w - max(ll + log_w); that max is M
    wv = a.e[g0 + s] / a.total[f];
  }
  if (!a.identity) {
    // The wave's 64 new states are one contiguous run of X_dst: lane l stores its elements
    // l, l + 64, ... of that run (8-byte stores, each instruction one contiguous 512 bytes)
    // from the source rows it finds through the owning lanes' pointers -- rows this wave has
    // just read.  Per-lane stores of d doubles at stride 8 d bytes ran at ~1 TB/s.
    const long long s0 = s - lane;                         // the wave's first slot
    const long long nv = a.P - s0 < 64 ? a.P - s0 : 64;   // its slots in range (wave-uniform)
    const long long n = nv * d;
    for (long long e = lane; e < 64LL * d; e += 64) {
      const int l2 = (int)(e / d), i2 = (int)(e - (long long)l2 * d);
      const double* src = (const double*)__shfl((long long)xs, l2);
      if (e < n) a.X_dst[(g0 + s0) * d + e] = src[i2];
    }
  }
  for (int k = 0; k < nq; ++k) {
    double v = 0.0;
    if (act) {
      if (k < C) v = (cnew == k) ? e2 : 0.0;
      else if (k == C) v = e2;
      else v = xs[k - C - 1] * wv;
    }
    v = wave_sum(v);
    if (lane == 0) red[w][k] = v;
  }
  __syncthreads();
  if (tid < nq) {
    double t = 0.0;
    for (int v = 0; v < kB / 64; ++v) t += red[v][tid];
    a.partials[(f * a.nb + blockIdx.x) * nq + tid] = t;
  }
}

// The all-gathered {ll} column (rows in position order: row r holds particle own[r]) into
// particle order, with each kRowsLL-particle block's maximum as an ord_enc key: the
// normaliser's maximum (gpmdm_pf.py:200) without k_norm_max, as k_obs_ll gives it to a
// single rank.  The maximum of a set in ord_enc's total order does not depend on how the
// set is split, so it is k_norm_max's result exactly.
constexpr int kRowsLLPer = 8;
constexpr long long kRowsLL = (long long)kRowsLLPer * kB;
__global__ __launch_bounds__(kB) void k_rows_ll(RowsLLArgs a) {
  __shared__ unsigned long long wk[kB / 64];
  unsigned long long key = 0;            // below ord_enc of any double
#pragma unroll
  for (int k = 0; k < kRowsLLPer; ++k) {
    const long long p = (long long)blockIdx.x * kRowsLL + (long long)k * kB + threadIdx.x;
    if (p < a.P) {
      const double v = a.rows[(a.inv ? (long long)a.inv[p] : p) * a.w];
      a.ll[p] = v;
      const unsigned long long kk = ord_enc(fmax(-INFINITY, v));   // k_norm_max's value set: NaN ignored
      key = kk > key ? kk : key;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long y = __shfl_xor(key, off);
    key = y > key ? y : key;
  }
  if ((threadIdx.x & 63) == 0) wk[threadIdx.x >> 6] = key;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = wk[0];
    for (int i = 1; i < kB / 64; ++i) m = wk[i] > m ? wk[i] : m;
    a.bmax[blockIdx.x] = m;
  }
}

// The read-out is in mapped host memory: publish its sequence number after it, so the host
// that sees the number sees the values -- gpmdm_pf_read then waits on host memory, and no
// event record sits between the read-out and the next frame's switch.  The protocol
// (DESIGN.md §1 "Mapped-memory handshake"):
//  * every other thread that wrote host memory in this kernel issues a system-scope fence
//    before the workgroup barrier (its stores are performed at system scope first);
//  * thread 0, after the barrier, publishes the number with a system-scope RELEASE store
//    (publish_seq): it orders thread 0's own stores, and everything that happens-before it
//    -- the other threads' fenced stores through the barrier, and every earlier kernel of
//    the stream (k_dyn_finish's row count) -- before the number;
//  * the host polls with ACQUIRE loads (gpmdm_pf::min_mapped), so its later plain loads of
//    the guarded values cannot be hoisted above the number.
// `stored`: this thread wrote host memory in this kernel (only those need the system-scope
// fence, whose L2 write-back costs ~3 us a wave; thread 0's release store includes its own).
__device__ inline void publish_readout(const ResampleArgs& a, long long f, int tid, bool stored) {
  if (!a.seq_host) return;              // (uniform over the workgroup)
  if (stored && tid != 0) __threadfence_system();
  __syncthreads();
  if (tid == 0) publish_seq(a.seq_host + f, a.seq);
}

__global__ __launch_bounds__(1024) void k_readout(ResampleArgs a) {
  __shared__ double red[8][16];
  __shared__ double tot[kMaxReadout];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nq = a.C + 1 + a.d;
  const long long f = blockIdx.x;
  const double* partials = a.partials + f * a.nb * nq;
  double* readout = a.readout + f * (a.C + a.d + 1);
  // eight read-out quantities per pass over the partials (every thread's loads in flight
  // together; per quantity the same thread-strided order as one quantity at a time)
  for (int k0 = 0; k0 < nq; k0 += 8) {
    double s[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) s[kk] = 0.0;
    for (long long b = tid; b < a.nb; b += 1024)
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
        if (k0 + kk < nq) s[kk] += partials[b * nq + k0 + kk];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const double v = wave_sum(s[kk]);
      if (lane == 0) red[kk][w] = v;
    }
    __syncthreads();
    if (tid < 8 && k0 + tid < nq) {
      double t = 0.0;
      for (int v = 0; v < 16; ++v) t += red[tid][v];
      tot[k0 + tid] = t;
    }
    __syncthreads();
  }
  // one value per lane, so every store is 8 bytes: a one-lane loop was vectorised into
  // 16-byte stores (the >8-byte store-data hazard; tests/test_isa_guard.py)
  const int nro = a.C + a.d + 1;
  if (tid < nro) {
    double v;
    if (tid < a.C) {                                     // class_probabilities
      double cl = 0.0;
      for (int c = 0; c < a.C; ++c) cl += tot[c];
      v = tot[tid] / cl;
    } else if (tid < a.C + a.d) {
      v = tot[tid + 1];                                  // current_state_mean
    } else {
      v = tot[a.C];                                      // log_likelihood()
    }
    readout[tid] = v;
    if (a.readout_host) a.readout_host[f * nro + tid] = v;
  }
  // the AUTO cutoff's counters of this frame, one per lane (8-byte stores: the ISA guard)
  const bool cst = a.cut_stats && f == 0 && tid < 2;
  if (cst) {
    a.cut_stats_host[tid] = a.cut_stats[tid];
    a.cut_stats[tid] = 0;
  }
  publish_readout(a, f, tid, tid < nro || cst);
}


// ---------------------------------------------------------------------------------
// Small filters (P <= kSmallP per filter, no guide table): one 1024-thread workgroup per
// filter runs normalise + CDF + resample + read-out in one launch instead of six -- at the
// notebook's P = 100 each launch of the multi-kernel path costs more than its work.  The
// arithmetic is the multi-kernel path's, association for association: the 256-thread
// blocks of k_norm_exp_scan / k_resample (and cdf_view's 256-particle blocks) are the
// workgroup's four 256-thread quarters (block b = waves 4b .. 4b+3, so every wave-level scan /
// sum sees the same lanes),
// k_norm_total / k_readout run as they are, and intermediates go through the same buffers;
// the max is exact in any order.  Systematic resampling takes the search form, whose indices
// the scan form reproduces exactly (k_sys_marks).  Results are bitwise those of the
// multi-kernel path (tests/test_gpu_small_path.py).
constexpr long long kSmallP = 1024;

__global__ __launch_bounds__(1024) void k_small_resample(NormArgs na, ResampleArgs a) {
  __shared__ double mx[16];
  __shared__ double wsum[4][4];
  // the values the multi-kernel path reads back from its buffers, kept here as written
  // (the buffers are still written for their other readers): M, block sums / offsets, S,
  // the read-out partials
  __shared__ double Msh, Ssh, bsum[4], boff[4];
  __shared__ double psh[4][kMaxReadout];
  __shared__ double cum_s[kSmallP];
  __shared__ double red[4][4][kMaxReadout];
  __shared__ double rred[8][16];
  __shared__ double tot[kMaxReadout];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = tid >> 8, wq = w & 3;                 // block of the multi-kernel path, its wave
  const long long f = blockIdx.x;
  const long long P = na.P;
  const int nb = na.nb;
  const long long p = tid;                            // = b * 256 + (tid & 255)
  const long long g0 = f * P;
  // the replay uniforms (host-mapped for small filters: a PCIe round trip) are loaded
  // here, ahead of the phases before the search, so their latency overlaps them
  const double u_pre = (a.U && !a.identity && p < P) ? a.U[a.systematic ? 0 : p] : 0.0;
  double llp;
  if (na.obs_pending) {
    // ---- k_obs_ll (deferred by the single-shard filter's weigh step): out index g0 + p ----
    double vc = 1.0, llv = 0.0;
    if (p < P) {
      llv = obs_ll_value(na.obs, g0 + p, vc);
      na.obs.ll[g0 + p] = llv;
    }
    if (na.obs.health) {
      count_event(na.obs.health + kHealthObsVar, p < P && !(vc > 0.0));
      count_event(na.obs.health + kHealthObsLL, p < P && !isfinite(llv));
    }
    llp = llv;
  } else {
    llp = p < P ? na.ll[g0 + p] : 0.0;
  }
  // ---- k_norm_max: the largest ll (NaN ignored, as fmax does) ----
  {
    double v = p < P ? llp : -INFINITY;
    v = fmax(-INFINITY, v);
    v = wave_max(v);
    if (lane == 0) mx[w] = v;
    __syncthreads();
    if (tid == 0) {
      double m = mx[0];
      for (int i = 1; i < 16; ++i) m = fmax(m, mx[i]);
      na.gmax[f] = ord_enc(m);
      Msh = ord_dec(ord_enc(m));
    }
    __syncthreads();
  }
  const double M = Msh;
  // ---- k_norm_exp_scan ----
  const double e = p < P ? exp(llp - M) : 0.0;
  if (p < P) na.e[g0 + p] = e;
  double e_incl;
  {
    double x = e;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const double y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[b][wq] = x;
    __syncthreads();
    double base = 0.0;
    for (int v = 0; v < wq; ++v) base += wsum[b][v];
    x += base;
    e_incl = x;
    if (p < P) na.local[g0 + p] = x;
    if ((tid & 255) == 255 && b < nb) {
      na.blocksum[f * nb + b] = x;
      bsum[b] = x;
    }
  }
  __syncthreads();
  // ---- k_norm_total ----
  // k_norm_total's 1024-wide Hillis-Steele scan over the nb <= 4 block sums (zeros
  // beyond): every addition past the first four slots adds an exact +0, so its values are
  // those of the same scan over four slots, computed here by one thread with the same
  // operand order (part[i] = part[i] + part[i - off]).
  if (tid == 0) {
    double h[4];
    for (int i = 0; i < 4; ++i) h[i] = i < nb ? bsum[i] : 0.0;
    for (int off = 1; off < 4; off <<= 1)
      for (int i = 3; i >= off; --i) h[i] = h[i] + h[i - off];
    for (int bb = 0; bb < 4; ++bb) boff[bb] = bb ? h[bb - 1] : 0.0;
    Ssh = h[3];
  }
  __syncthreads();
  const double S = Ssh;
  if (tid < nb) na.blockoff[f * nb + tid] = boff[tid];      // one 8-byte store per lane
  if (tid == 0) na.total[f] = S;
  // ---- the CDF (cdf_view's expression) ----
  if (p < P) cum_s[p] = p == P - 1 ? 1.0 : (boff[b] + e_incl) / S;
  __syncthreads();
  // ---- k_resample (slot s = p) ----
  const uint2 key = filter_key(a.seed_lo, a.seed_hi, f);
  const int C = a.C, d = a.d, nq = C + 1 + d;
  const bool act = p < P;
  long long idx = 0;
  int cnew = -1;
  double e2 = 0.0, wv = 0.0;
  if (act) {
    if (a.identity) {
      idx = p;
    } else {
      double u;
      if (a.systematic) {
        u = sys_u(p, a.U ? u_pre : sys_u0(a, f), P);
      } else if (a.U) {
        u = u_pre;
      } else {
        const uint4 r = philox4x32_10(make_uint4((unsigned)p, a.frame, kStreamResample, 0u), key);
        u = u01_co(r.x, r.y);
      }
      long long lo = 0, hi = P;
      while (hi - lo > 0) {
        const long long mid = lo + (hi - lo) / 2;
        if (cum_s[mid] < u) lo = mid + 1; else hi = mid;
      }
      idx = lo;
    }
    cnew = a.cls_src[g0 + idx];
    if (!a.identity) {
      a.ridx[g0 + p] = (int)idx;
      a.cls_dst[g0 + p] = cnew;
      if (a.cls_host) a.cls_host[g0 + p] = cnew;
      for (int j = 0; j < d; ++j) a.X_dst[(g0 + p) * d + j] = a.X_src[(g0 + idx) * d + j];
    }
    const double llv = llp;
    const double lw = llv - M;
    e2 = exp((llv + lw) - M);
    wv = e / S;
  }
  for (int k = 0; k < nq; ++k) {
    double v = 0.0;
    if (act) {
      if (k < C) v = (cnew == k) ? e2 : 0.0;
      else if (k == C) v = e2;
      else v = a.X_src[(g0 + idx) * d + (k - C - 1)] * wv;
    }
    v = wave_sum(v);
    if (lane == 0) red[b][wq][k] = v;
  }
  __syncthreads();
  if ((tid & 255) < nq && b < nb) {
    const int k = tid & 255;
    double t = 0.0;
    for (int v = 0; v < 4; ++v) t += red[b][v][k];
    a.partials[(f * nb + b) * nq + k] = t;
    psh[b][k] = t;
  }
  __syncthreads();
  // ---- k_readout ----
  double* readout = a.readout + f * (C + d + 1);
  for (int k0 = 0; k0 < nq; k0 += 8) {
    double sv[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) sv[kk] = 0.0;
    if (tid < nb)
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
        if (k0 + kk < nq) sv[kk] += psh[tid][k0 + kk];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const double v = wave_sum(sv[kk]);
      if (lane == 0) rred[kk][w] = v;
    }
    __syncthreads();
    if (tid < 8 && k0 + tid < nq) {
      double t = 0.0;
      for (int v = 0; v < 16; ++v) t += rred[tid][v];
      tot[k0 + tid] = t;
    }
    __syncthreads();
  }
  const int nro = C + d + 1;
  if (tid < nro) {
    double v;
    if (tid < C) {
      double cl = 0.0;
      for (int c = 0; c < C; ++c) cl += tot[c];
      v = tot[tid] / cl;
    } else if (tid < C + d) {
      v = tot[tid + 1];
    } else {
      v = tot[C];
    }
    readout[tid] = v;
    if (a.readout_host) a.readout_host[f * nro + tid] = v;
  }
  publish_readout(a, f, tid, true);   // (cls_host: any slot's thread)
}

// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(kB) void k_pack(PackArgs a) {
  const long long r = (long long)blockIdx.x * kB + threadIdx.x;
  if (r >= a.n) return;
  const long long p = a.own ? a.own[a.lo + r] : a.lo + r;
  const int lo = a.part == GPMDM_PACK_STATES ? 1 : 0;            // first column present
  const int hi = a.part == GPMDM_PACK_LL ? 1 : a.d + 2;           // one past the last
  double* o = a.buf + r * (hi - lo);                              // o[k - lo]: column k
  if (lo == 0) o[0] = a.ll[p];
  if (hi > 1) {
    o[1 - lo] = (double)a.cls[p];
    for (int j = 0; j < a.d; ++j) o[2 - lo + j] = a.X[p * a.d + j];
  }
}

// one thread per particle p, reading its row inv[p] (a gather: the writes stay coalesced;
// scattering the rows to own[r] made every write a partial-line write, 57 us at P = 800k)
__global__ __launch_bounds__(kB) void k_unpack(PackArgs a) {
  const long long p = (long long)blockIdx.x * kB + threadIdx.x;
  if (p >= a.n) return;
  const long long r = a.inv ? a.inv[p] : p;
  const int lo = a.part == GPMDM_PACK_STATES ? 1 : 0;
  const int hi = a.part == GPMDM_PACK_LL ? 1 : a.d + 2;
  const double* i = a.buf + r * (hi - lo);
  if (lo == 0) a.ll[p] = i[0];
  if (hi > 1) {
    a.cls[p] = (int)i[1 - lo];
    for (int j = 0; j < a.d; ++j) a.X[p * a.d + j] = i[2 - lo + j];
  }
}

// ---------------------------------------------------------------------------------
// predict(): class histogram of the current classes (k_switch's histogram without a switch)
__global__ __launch_bounds__(kB) void k_class_hist(const int* cls, long long P, int C, int* blockcounts) {
  __shared__ int hist[kMaxClasses];
  const int tid = threadIdx.x;
  if (tid < C) hist[tid] = 0;
  __syncthreads();
  const long long p = (long long)blockIdx.x * kB + tid;
  if (p < P) atomicAdd(&hist[cls[p]], 1);
  __syncthreads();
  if (tid < C) blockcounts[(long long)blockIdx.x * C + tid] = hist[tid];
}

__global__ __launch_bounds__(kB) void k_predict_scatter(const int* perm, const double* mu, double* mu_p,
                                                        long long P, int d) {
  const long long o = (long long)blockIdx.x * kB + threadIdx.x;
  if (o >= P) return;
  const long long p = perm[o];
  for (int j = 0; j < d; ++j) mu_p[p * d + j] = mu[o * d + j];
}

// One workgroup per filter: mean over the filter's particles, thread-strided partial sums
// combined in a fixed order.
__global__ __launch_bounds__(kB) void k_predict_mean(const double* mu_p, double* out, long long Pf, int d) {
  __shared__ double red[kB / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long f = blockIdx.x;
  for (int j = 0; j < d; ++j) {
    double s = 0.0;
    for (long long p = tid; p < Pf; p += kB) s += mu_p[(f * Pf + p) * d + j];
    s = wave_sum(s);
    if (lane == 0) red[w] = s;
    __syncthreads();
    if (tid == 0) {
      double t = 0.0;
      for (int v = 0; v < kB / 64; ++v) t += red[v];
      out[f * d + j] = t / (double)Pf;
    }
    __syncthreads();
  }
}

// One-segment table of a predictive map, written in stream order (no host-to-device copy
// of a host array per call): {pos_begin, pos_end, out_base, tile_start[0], tile_start[1]}.
__global__ void k_seg_table(int* t, int n, int tiles) {
  const int i = threadIdx.x;
  if (i < 5) t[i] = i == 1 ? n : (i == 4 ? tiles : 0);
}

// ---------------------------------------------------------------------------------
static inline unsigned nblk(long long n, int b) { return (unsigned)((n + b - 1) / b); }

void launch_seg_table(int* t, int n, int tiles, hipStream_t s) {
  hipLaunchKernelGGL(k_seg_table, dim3(1), dim3(64), 0, s, t, n, tiles);
}

void launch_class_hist(const int* cls, long long P, int C, int* blockcounts, hipStream_t s) {
  hipLaunchKernelGGL(k_class_hist, dim3(nblk(P, kB)), dim3(kB), 0, s, cls, P, C, blockcounts);
}
void launch_predict_mean(const int* perm, const double* mu, double* mu_p, double* out, long long P,
                         long long Pf, int F, int d, hipStream_t s) {
  hipLaunchKernelGGL(k_predict_scatter, dim3(nblk(P, kB)), dim3(kB), 0, s, perm, mu, mu_p, P, d);
  hipLaunchKernelGGL(k_predict_mean, dim3((unsigned)F), dim3(kB), 0, s, mu_p, out, Pf, d);
}

void launch_switch(const SwitchArgs& a, hipStream_t s) {
  if (a.own)
    hipLaunchKernelGGL(k_switch<true>, dim3(nblk(a.n > 0 ? a.n : 1, kB)), dim3(kB), 0, s, a);
  else
    hipLaunchKernelGGL(k_switch<false>, dim3(nblk(a.n > 0 ? a.n : 1, kB)), dim3(kB), 0, s, a);
}
void launch_scan_counts(const ScanArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, a);
}
void launch_group(const GroupArgs& a, hipStream_t s) {
  if (a.own)
    hipLaunchKernelGGL(k_group<true>, dim3(nblk(a.n > 0 ? a.n : 1, kB)), dim3(kB), 0, s, a);
  else
    hipLaunchKernelGGL(k_group<false>, dim3(nblk(a.n > 0 ? a.n : 1, kB)), dim3(kB), 0, s, a);
}
// switch + class scan + grouping (+ leader compaction with `la`): one launch for a small
// single-shard filter (k_small_switch, the same tables), the multi-kernel path otherwise.
// The owner preset of the leader election is part of either path.
bool launch_switch_group(const SwitchArgs& sa, const ScanArgs& sc, const GroupArgs& ga, const LeadArgs* la,
                         bool owner_preset, hipStream_t s) {
  static const bool no_small = std::getenv("GPMDM_NO_SMALL_PATH") != nullptr;
  if (!no_small && sa.P <= kSmallSwitchP && sa.n == sa.P && sa.base == 0 && !sa.own && sa.n > 0 &&
      (la == nullptr) == (sa.owner == nullptr) && (la == nullptr || la->npos == sa.P)) {
    LeadArgs l = la ? *la : LeadArgs{};
    hipLaunchKernelGGL(k_small_switch, dim3(1), dim3(1024), 0, s, sa, sc, ga, l, la ? 1 : 0);
    return true;
  }
  if (la && owner_preset) (void)hipMemsetAsync(sa.owner, 0xff, sizeof(unsigned) * (size_t)sa.C * sa.P, s);
  launch_switch(sa, s);
  launch_scan_counts(sc, s);
  launch_group(ga, s);
  if (la) launch_lead(*la, s);
  return false;
}
void launch_lead(const LeadArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_lead_flags, dim3((unsigned)a.nb), dim3(kB), 0, s, a);
  if (a.nb <= kMaxLeadBlocks) {
    hipLaunchKernelGGL(k_lead_tables_compact, dim3((unsigned)a.nb), dim3(kB), 0, s, a);
  } else {
    hipLaunchKernelGGL(k_lead_tables, dim3(1), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(k_lead_compact, dim3((unsigned)a.nb), dim3(kB), 0, s, a);
  }
}
void launch_dyn_finish(const DynFinishArgs& a, hipStream_t s) {
  if (a.n_out > 0) hipLaunchKernelGGL(k_dyn_finish, dim3(nblk(a.n_out, kB)), dim3(kB), 0, s, a);
}
void launch_obs_finish(const ObsFinishArgs& a, hipStream_t s) {
  if (a.n_out <= 0) return;
  if (a.spart)
    hipLaunchKernelGGL(k_obs_ll, dim3(nblk(a.n_out, kB)), dim3(kB), 0, s, a);
  else
    hipLaunchKernelGGL(k_obs_finish, dim3(nblk(a.n_out, kB / 64)), dim3(kB), 0, s, a);
}
void launch_normalise(const NormArgs& a, hipStream_t s) {
  const dim3 g(nblk(a.P, kB), (unsigned)a.F);
  const unsigned nbm = nblk(a.P, kB) < kMaxNormBlocks ? nblk(a.P, kB) : kMaxNormBlocks;
  if (!a.bmax) hipLaunchKernelGGL(k_norm_max, dim3(nbm, (unsigned)a.F), dim3(kB), 0, s, a);
  hipLaunchKernelGGL(k_norm_exp_scan, g, dim3(kB), 0, s, a);
  hipLaunchKernelGGL(k_norm_total, dim3((unsigned)a.F), dim3(1024), 0, s, a);
}
void launch_resample(const ResampleArgs& a, hipStream_t s) {
  if (!a.identity && a.sys_mark) {
    (void)hipMemsetAsync(a.sys_mark, 0xff, sizeof(int) * (size_t)a.P * a.F, s);   // -1: no run starts
    hipLaunchKernelGGL(k_sys_marks, dim3(nblk(a.P, kB), (unsigned)a.F), dim3(kB), 0, s, a);
    hipLaunchKernelGGL(k_sys_scan, dim3(nblk(a.P, kB), (unsigned)a.F), dim3(kB), 0, s, a);
    hipLaunchKernelGGL(k_sys_blocks, dim3((unsigned)a.F), dim3(1024), 0, s, a);
  } else if (!a.identity && a.GB > 0)
    hipLaunchKernelGGL(k_guide, dim3(nblk(a.GB + 3, kB), (unsigned)a.F), dim3(kB), 0, s, a);
  hipLaunchKernelGGL(k_resample, dim3(nblk(a.P, kB), (unsigned)a.F), dim3(kB), 0, s, a);
  hipLaunchKernelGGL(k_readout, dim3((unsigned)a.F), dim3(1024), 0, s, a);
}
// normalise + resample + read-out: one launch for small filters (k_small_resample, bitwise
// the multi-kernel path), the multi-kernel path otherwise (GPMDM_NO_SMALL_PATH=1 forces it)
bool small_resample_ok(const NormArgs& na, const ResampleArgs& ra) {
  static const bool no_small = std::getenv("GPMDM_NO_SMALL_PATH") != nullptr;
  return !no_small && na.P <= kSmallP && ra.GB == 0;
}

void launch_normalise_resample(const NormArgs& na, const ResampleArgs& ra, hipStream_t s) {
  if (small_resample_ok(na, ra)) {
    hipLaunchKernelGGL(k_small_resample, dim3((unsigned)na.F), dim3(1024), 0, s, na, ra);
    return;
  }
  if (na.obs_pending) launch_obs_finish(na.obs, s);
  launch_normalise(na, s);
  launch_resample(ra, s);
}
int rows_ll_blocks(long long P) { return (int)nblk(P, kRowsLL); }
void launch_rows_ll(const RowsLLArgs& a, hipStream_t s) {
  if (a.P > 0) hipLaunchKernelGGL(k_rows_ll, dim3(nblk(a.P, kRowsLL)), dim3(kB), 0, s, a);
}
void launch_pack(const PackArgs& a, hipStream_t s) {
  if (a.n > 0) hipLaunchKernelGGL(k_pack, dim3(nblk(a.n, kB)), dim3(kB), 0, s, a);
}
void launch_unpack(const PackArgs& a, hipStream_t s) {
  if (a.n > 0) hipLaunchKernelGGL(k_unpack, dim3(nblk(a.n, kB)), dim3(kB), 0, s, a);
}

}  // namespace gpmdm
