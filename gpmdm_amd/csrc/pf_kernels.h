// Argument blocks and launchers of the particle-filter kernels (pf_kernels.hip).
#pragma once

#include "../../include/gpmdm_hip.h"
#include "common.h"

namespace gpmdm {

constexpr int kMaxClasses = 32;
constexpr int kMaxReadout = kMaxClasses + 1 + kMaxD;

// Failure-detection counters (gpmdm_pf_health).  The filter keeps the
// reference's arithmetic -- a non-positive variance gives NaN log-likelihoods or states,
// as gpmdm_pf.py:167-168, 188-192 do -- and counts each event, per particle and step.
enum HealthCounter : int {
  kHealthObsVar = 0,      // observation-GP vc = 1 - k^T K_y^-1 k <= 0 (or NaN)
  kHealthObsLL = 1,       // non-finite log-likelihood
  kHealthDynVar = 2,      // dynamics-GP vc <= 0 (or NaN)
  kHealthDynState = 3,    // non-finite propagated state
  kHealthN = 4
};

// Filter banks: F independent filters of Pf particles each, stored filter-major
// (particle g = f * Pf + p).  The Philox key of filter f is seed + f and the counters use
// the in-filter index p, so filter f of a bank draws exactly what a single filter seeded
// with seed + f draws.
__device__ __forceinline__ uint2 filter_key(unsigned seed_lo, unsigned seed_hi, long long f) {
  const unsigned long long k = (((unsigned long long)seed_hi << 32) | seed_lo) + (unsigned long long)f;
  return make_uint2((unsigned)(k & 0xffffffffu), (unsigned)(k >> 32));
}

struct SwitchArgs {
  long long P;                    // all particles (F * Pf)
  long long base, n;              // positions [base, base + n) of the ownership order are switched
                                  // (all: 0, P; a multi-rank Philox rank: its slice)
  long long Pf;                   // particles per filter
  int C, F;
  unsigned frame, seed_lo, seed_hi;
  const int* cls;                 // P   current classes
  int* cls_new;                   // P   switched classes
  const double* T;                // C x C Markov matrix (device)
  const double* E;                // P x C Exp(1) draws (replay) or nullptr (philox)
  int* blockcounts;               // nb x C
  unsigned long long* gmax_reset; // F running maxima of the normaliser to reset (or nullptr)
  // ancestor de-duplication (nullptr: off).  Particles of this rank's slice [lo, hi) that
  // share a resampling ancestor and a new class have bit-identical dynamics-GP inputs; the
  // smallest such particle index becomes the key's leader: owner[c * P + ancestor] = min p.
  const int* anc;                 // P   in-filter ancestor index (resample source; identity after init)
  unsigned* owner;                // C x P, preset to 0xffffffff
  long long lo, hi;
  // ancestor-ordered shards (multi-rank philox; nullptr: identity): thread i handles particle
  // own[i], and this rank's slice is positions [lo, hi) of that order
  const int* own;
};

struct ScanArgs {
  int nb, C;                      // nb: blocks of k_switch's histogram
  int pt;                         // particles per dynamics-GP tile (seg_tile_start unit)
  long long lo, hi;               // this rank's particle slice (positions of the own order)
  const int* own;                 // ownership order (nullptr: identity)
  long long base;                 // position pos of the grouped range is particle own[base + pos]
  const int* blockcounts;
  const int* cls_new;
  int* blockoff;                  // nb x C
  int* class_start;               // C + 1
  int* counts;                    // C
  int* counts_host;               // C, or nullptr: the counts also into mapped host memory
  long long* counts_seq_host;     // mapped: `counts_seq` published after counts_host (k_scan_counts)
  long long counts_seq;
  int* seg_pos_begin;             // C
  int* seg_pos_end;               // C
  int* seg_out_base;              // C
  int* seg_tile_start;            // C + 1
};

struct GroupArgs {
  long long P;
  long long base, n;              // as SwitchArgs
  int C;
  const int* cls_new;
  const int* class_start;
  const int* blockoff;
  const int* own;                 // ownership order (nullptr: identity)
  int* perm;                      // grouped position -> particle
};

// Leader compaction over the class-grouped positions (ancestor de-duplication).
struct LeadArgs {
  long long P, Pf, lo, hi;        // P: all particles (key stride)
  long long npos;                 // grouped positions (P, or the rank's slice)
  int nb, C;
  int pt;                         // particles per dynamics-GP tile
  const int* perm;                // grouped position -> particle
  const int* cls_new;
  const int* anc;
  const unsigned* owner;
  const int* seg_pos_begin;       // [C] this rank's positions of class c (full grouping)
  const int* seg_pos_end;
  int* lflag_scan;                // P   block-local exclusive scan of the leader flags
  int* lblock;                    // nb  leaders per block of positions
  int* lseg_pos_begin;            // [C] leader rows of class c: [begin, end)
  int* lseg_pos_end;
  int* lseg_out_base;             // [C] (= begin: rows are their own output index)
  int* lseg_tile_start;           // [C + 1]
  int* lperm;                     // leader row -> particle
  int* slot;                      // C x P: key -> leader row
  unsigned* owner_reset;          // owner table to restore to 0xffffffff at each leader's key
                                  // (every registered key has one leader), or nullptr
};

struct DynFinishArgs {
  long long n_out;                // rows produced by the tile kernel
  long long Pf;                   // particles per filter (Philox key / counter split)
  int n_seg, d;
  unsigned frame, seed_lo, seed_hi;
  const int* seg_out_base;        // nullptr: single segment
  const int* seg_pos_begin;
  const int* perm;                // nullptr: identity
  int n_parts[kMaxClasses];       // q partials per segment
  const double* qpart;
  long long ld_q;
  const double* mu;
  long long ld_mu;
  const double* X;                // input rows (pre-dynamics states)
  double lin_c2[kMaxD + 1];
  double il2[kMaxD];              // exp(x_log_lambdas)^-2
  const double* normals;          // grouped-position-major draws (replay) or nullptr
  double* X_out;                  // PF: propagated states (P x d, particle index)
  double* var_out;                // predictive map: n x d variances (PF: nullptr)
  // ancestor de-duplication: the tile rows are leader rows, slot[c * P + g0 + anc[p]]
  const int* slot;                // nullptr: row = output index o
  const int* anc;
  long long P;
  unsigned* health;               // kHealth* counters (PF) or nullptr
  // PF bookkeeping done by output 0 / outputs < F (not by the switch, which may run ahead:
  // capi_frame.hip pre-switch): the normaliser maxima reset, and the row count of this dynamics
  // pass (sum over n_rows_seg segments of rows_e - rows_b) for gpmdm_pf_dyn_rows
  unsigned long long* gmax_reset; // F maxima, or nullptr
  int F;
  const int* rows_b;
  const int* rows_e;
  int n_rows_seg;
  int* rows_out;                  // or nullptr
  int* rows_host;                 // the same count into mapped host memory (the next frames'
                                  // tile-height choice, capi_frame.hip dyn_frame_geo), or nullptr
  // the frame's observation copied by outputs < z_n from host-mapped memory to the device
  // buffer the observation GP reads (no copy launch on the critical path), or z_n = 0
  const double* z_src;
  double* z_dst;
  long long z_n;
};

struct ObsFinishArgs {
  long long n_out;
  int n_parts, D;
  const double* qpart;
  long long ld_q;
  const double* mu;
  long long ld_mu;
  const double* z;                // F x D (device): observation of each filter
  long long Pf;                   // particles per filter (PF; predictive maps: unused)
  const double* il2;              // D  exp(y_log_lambdas)^-2 (device)
  double ll_const;                // 0.5 * D * ln(2 pi) in float32 (gpmdm_pf.py:5, 191)
  double* ll;                     // PF output (ll[ll_offset + o]) or nullptr
  long long ll_offset;
  const int* own;                 // PF ownership order: ll[own[ll_offset + o]] (nullptr: identity)
  double* var_out;                // predictive map output n x D, or nullptr
  // fused mode (the tile kernel wrote spart instead of mu): ll from q and S partials
  const double* spart;            // [J][ld_q] for J in [jm0, n_j), or nullptr
  int jm0, n_j;
  double sum_log_il2;             // sum_j log il2_j
  unsigned* health;               // kHealth* counters (PF) or nullptr
  // single filters: the maximum of each block's ll (ord_enc keys), which the normaliser
  // reads instead of running k_norm_max (nullptr: not produced)
  unsigned long long* bmax;
  // the cutoff kernel's split tiles (obs_cutoff.h): outputs from cut_o0 on chain their second
  // part's partials onto q and S in list order (nullptr: no split tiles)
  const double* cut_part;
  long long cut_ld, cut_o0;
  const int2* cut_split;
  int cut_pt, cut_tpc, cut_tm;
};

// Normalisation and resampling run per filter: grid (nb, F), nb blocks of 256 per filter.
struct NormArgs {
  long long P;                    // particles per filter
  int nb, F;
  const double* ll;               // F x P
  unsigned long long* gmax;       // F
  double* e;                      // exp(ll - max)
  double* local;                  // block-local inclusive scan of e
  double* blocksum;               // F x nb
  double* blockoff;               // F x nb
  double* total;                  // F: sum of e
  // a deferred likelihood finish (k_obs_ll) of a single-shard filter: the small-filter
  // kernel computes ll itself first, the multi-kernel path launches k_obs_ll first
  ObsFinishArgs obs;
  int obs_pending;
  // k_obs_ll's block maxima of ll (single filters, nb keys; k_rows_ll: nbmax keys): the
  // maximum without k_norm_max
  const unsigned long long* bmax;
  int nbmax;                      // keys in bmax (0: nb)
};

// k_rows_ll: the exchanged {ll} column into particle order + block maxima (single filters)
struct RowsLLArgs {
  long long P;
  const double* rows;             // column 0 of row r = ll of particle own[r]
  int w;                          // doubles per row
  const int* inv;                 // particle p's row (nullptr: p)
  double* ll;
  unsigned long long* bmax;       // rows_ll_blocks(P) keys
};
int rows_ll_blocks(long long P);
void launch_rows_ll(const RowsLLArgs& a, hipStream_t s);

struct ResampleArgs {
  long long P;                    // particles per filter
  int nb, F, C, d, systematic, identity;
  unsigned frame, seed_lo, seed_hi;
  const double* U;                // uniforms (replay, single filter) or nullptr
  // the normalised CDF is not stored: the searches evaluate it from the normaliser's
  // block-local scan and block offsets (cdf_view, pf_kernels.hip)
  const double* local;            // F x P
  const double* blockoff;         // F x nb
  const double* ll;
  const double* e;
  const double* total;
  const unsigned long long* gmax;
  const int* cls_src;
  const double* X_src;
  int* cls_dst;
  double* X_dst;
  int* ridx;                      // in-filter source index of each slot
  double* partials;               // F x nb x (C + 1 + d)
  double* readout;                // per filter: C posterior, d mean, 1 likelihood sum
  double* readout_host;           // the same into mapped host memory (small filters), or nullptr
  long long* seq_host;            // mapped: `seq` published after readout_host (or nullptr)
  long long seq;
  int* cls_host;                  // post-resample classes into mapped host memory (k_small_resample,
                                  // single replay filters: the next switch's counts on the host), or nullptr
  int* guide;                     // F x (GB + 3): guide[b] = first i with CDF_i >= b / GB
  long long GB;                   // guide buckets per filter
  // exchanged {class, state} rows read in place instead of cls_src / X_src (multi-rank
  // filters: row rows_inv[p] holds particle p, column 0 its class, 1..d its state), or nullptr
  const double* rows;
  int rows_w;
  const int* rows_inv;
  // systematic resampling by scan (no per-slot search): run starts of each particle's
  // offspring marked in sys_mark (F x P), block-local max-scan in place, block maxima
  // (F x nb) scanned; slot s's ancestor = max(local[s], block prefix).  nullptr: search.
  int* sys_mark;
  int* sys_block;
  // the observation cutoff's AUTO policy (gpmdm_pf_set_obs_cutoff mode 3): the cutoff kernel's
  // MFMA-group counters of this frame, copied by k_readout into mapped host memory (published
  // with the read-out) and reset; nullptr: not a cutoff frame of an AUTO filter
  unsigned long long* cut_stats;
  unsigned long long* cut_stats_host;
};

// Guide buckets per filter for the inverse-CDF search (P / 4: a resample search then spans
// ~4-8 particles instead of all P).  Below kGuideMinP the plain search over [0, P] is
// cheaper than building the table (P = 100k: 12.7 us plain vs 6.3 + 10.3 us guided;
// P = 800k: the guided search saves ~35 us per step).
constexpr long long kGuideMinP = 262144;
inline long long guide_buckets(long long P) { return P / 4 > 1 ? P / 4 : 1; }
inline long long guide_buckets_used(long long P) { return P >= kGuideMinP ? guide_buckets(P) : 0; }

struct PackArgs {
  long long n, lo;
  int d;
  const int* own;                 // row r holds particle own[lo + r] (nullptr: identity)
  const int* inv;                 // unpack: particle p's row is inv[p] (nullptr: identity)
  double* buf;
  int part;                       // GPMDM_PACK_*: {ll, class, X} | {class, X} | {ll}
  double* ll;
  int* cls;
  double* X;
};

// Ancestor-ordered shards (shard_order.hip): own = slots in stable order of the bucket
// floor(256 u) of their resampling uniform (Philox draw of `frame`, single filters), so each
// rank's contiguous slice of that order descends from a contiguous range of ancestors.
// Deterministic (identical on every rank).  temp: uniform_order_temp_bytes(P) of device memory.
size_t uniform_order_temp_bytes(long long P);
bool uniform_order_supported(long long P);   // P <= 33.5M (larger filters keep the identity order)
// inv: the inverse permutation, inv[own[r]] = r (particle p's exchanged row is inv[p])
int launch_uniform_order(long long P, unsigned frame, unsigned seed_lo, unsigned seed_hi, int* own, int* inv,
                         void* temp, size_t temp_bytes, hipStream_t s);

void launch_switch(const SwitchArgs& a, hipStream_t s);
void launch_scan_counts(const ScanArgs& a, hipStream_t s);
void launch_group(const GroupArgs& a, hipStream_t s);
void launch_lead(const LeadArgs& a, hipStream_t s);
void launch_dyn_finish(const DynFinishArgs& a, hipStream_t s);
void launch_obs_finish(const ObsFinishArgs& a, hipStream_t s);
void launch_normalise(const NormArgs& a, hipStream_t s);
void launch_resample(const ResampleArgs& a, hipStream_t s);
void launch_normalise_resample(const NormArgs& na, const ResampleArgs& ra, hipStream_t s);
bool small_resample_ok(const NormArgs& na, const ResampleArgs& ra);
// returns true when the one-workgroup small path ran (its owner preset leaves the table
// dirty); owner_preset = false skips the multi-kernel path's preset of a table that the last
// leader compaction restored (LeadArgs::owner_reset)
bool launch_switch_group(const SwitchArgs& sa, const ScanArgs& sc, const GroupArgs& ga, const LeadArgs* la,
                         bool owner_preset, hipStream_t s);
void launch_pack(const PackArgs& a, hipStream_t s);
// predict(): per-block class histogram of `cls` (blockcounts nb x C, nb = ceil(P / 256))
// single-segment tile table {0, n, 0, 0, tiles} at t[0..4] (predictive maps)
void launch_seg_table(int* t, int n, int tiles, hipStream_t s);
void launch_class_hist(const int* cls, long long P, int C, int* blockcounts, hipStream_t s);
// predict(): rows of mu (grouped order, perm: row -> particle) scattered to particle order,
// then per filter the mean over its Pf particles (fixed-order reduction) into out (F x d)
void launch_predict_mean(const int* perm, const double* mu, double* mu_p, double* out, long long P,
                         long long Pf, int F, int d, hipStream_t s);
void launch_unpack(const PackArgs& a, hipStream_t s);

}  // namespace gpmdm
