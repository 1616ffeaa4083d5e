// Internal interface of the C-ABI translation units (capi_*.hip): the model and filter
// handles (device layout, per-frame bookkeeping) and the helpers the units share.  Not part of
// the public ABI (include/gpmdm_hip.h).
//   capi_model.hip     models, predictive maps (gpmdm_model_*, gpmdm_predict_*), images
//   capi_pf.hip        filter and bank lifecycle, state import / export, settings, predict
//   capi_frame.hip     the per-frame launch sequence: switch, propagate, weigh, resample, read
//   capi_exchange.hip  the multi-rank exchange (pack / unpack, RCCL communicator, gathers)
//   capi_replay.hip    replay-draw staging (pinned buffers, staged normals, pre-switch)
#pragma once
#include <algorithm>
#include <chrono>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <dlfcn.h>
#include <functional>
#include <mutex>
#include <type_traits>

#include <rccl/rccl.h>   // types only: the entry points are resolved at run time (rccl())

#include "../../include/gpmdm_hip.h"
#include "common.h"
#include "host_image.h"
#include "pf_kernels.h"
#include "status.h"

static_assert(gpmdm::kMaxClassesDesc == gpmdm::kMaxClasses, "descriptor check and kernels agree on the class limit");

namespace gpmdm::capi {

// Rows from which a dynamics-GP predictive map uses the wide tile image (a throughput
// problem; below, the narrow tiles' shorter K loops win)
constexpr long long kWideRows = 4096;

// Single replay filters up to this size count their switched classes on the host
// (gpmdm_pf::cls_pin; the one-workgroup resampling kernel k_small_resample provides the
// classes).  The host loop is P x C fp64 divisions: ~1 us at the notebook's P = 100.
constexpr long long kHostCountsMaxP = 1024;

// One GP's device image: scaled inputs (+ squared norms) and B = [R | M] (+ H for the
// dynamics GPs) in MFMA-fragment order -- layout and packing in host_image.h.
struct GpImage {
  int n_rows = 0, n_m = 0, n_j = 0, coff = 0;
  bool dyn = false;       // a dynamics GP's image (linear-kernel rows H)
  TileGeo geo = kGeo64x256;
  double* Xrec = nullptr; // row_cap(n_rows) x (d + 1) row records (host_image.h)
  double* Hf = nullptr;   // dynamics only
  double* Bf = nullptr;

  void release() {
    dfree(Xrec);
    dfree(Hf);
    dfree(Bf);
  }
  SegDesc seg() const {
    SegDesc s{};
    s.Xrec = Xrec;
    s.Hf = Hf;
    s.Bf = Bf;
    s.n_rows = n_rows;
    s.n_m = n_m;
    s.n_j = n_j;
    s.coff = coff;
    return s;
  }
  // Read-out partials (gp_tile.h epilogue): one per column block, or for the dynamics GP's
  // wide shape (4 waves x 8 column tiles: 32 x 512) one per 256-column part, indexed as the
  // 16 x 256 image's blocks (front padding col_offset(n_cols, 256)) -- so the narrow and wide
  // dynamics images' partials are the same numbers in the same slots.
  bool split() const { return dyn && geo.nw == 4 && geo.ntw == 8; }
  int pnb() const { return split() ? geo.nb() / 2 : geo.nb(); }
  int pcoff() const { return split() ? col_offset(n_rows + n_m, pnb()) : coff; }
  int n_parts() const { return (int)cdiv(n_rows + pcoff(), pnb()); }              // parts holding R columns
  int n_pblocks() const { return (int)cdiv(n_rows + n_m + pcoff(), pnb()); }      // all parts
  int jm0() const { return (n_rows + pcoff()) / pnb(); }                          // first part with mean columns
  int tiles(long long n) const { return (int)cdiv(n, geo.pt()); }
};

int build_image(GpImage& g, int n_rows, int d, int n_m, const double* X, const double* ls,
                const double* lin_c2, const double* R, const double* M, TileGeo geo);

}  // namespace gpmdm::capi

using namespace gpmdm;
using namespace gpmdm::capi;

// =====================================================================================
struct gpmdm_model {
  // Reference count: the caller's handle plus one per filter built on the model, so a
  // filter keeps the device image it was built on alive until it is destroyed or rebound
  // (gpmdm_pf_set_model) even after the caller rebuilt the model (GPMDM.set_latents).
  std::atomic<int> refs{1};
  int device = 0;
  long long N = 0;
  int D = 0, d = 0, C = 0;
  std::vector<double> X;              // host copy, N x d
  std::vector<double> y_ls, x_ls, x_lin_c2, x_il2, y_il2;
  GpImage obs;
  // the observation GP in 16 x 256 tiles for small models and filters (obs_pick): at the
  // notebook's N = 500 and P = 100 the 512-column blocks leave a 32-K-step chain of wide
  // MFMA steps on a handful of CUs; 256-column blocks halve each chain (empty: not built)
  GpImage obs_small;
  std::vector<GpImage> dyn;           // narrow tiles (16x256): de-duplicated rows, small maps
  std::vector<GpImage> dynw;          // wide tiles (the observation GP's shape): every particle
                                      // (dedup off, predict), large maps; empty = same as dyn
  const std::vector<GpImage>& dyn_set(bool wide) const { return wide && !dynw.empty() ? dynw : dyn; }
  int dyn_parts_max() const {
    int mx = 0;
    for (auto& g : dyn) mx = std::max(mx, g.n_parts());
    for (auto& g : dynw) mx = std::max(mx, g.n_parts());
    return mx;
  }
  double* y_il2_dev = nullptr;
  double* y_lam2_dev = nullptr;   // 1 / il2 = exp(y_log_lambdas)^2
  double sum_log_il2 = 0.0;
  // Observation-GP cutoff image (gpmdm_model_set_obs_cutoff; empty: not set): K^-1's block
  // upper triangle and M over the training rows in a spatial order, tile-major
  // (host_image.h CutoffPacker, obs_cutoff.h), the K-step spheres, and the cutoff (tau; cut2 =
  // the squared scaled distance past which a value is below tau, with a margin; t_cut = ln tau
  // in the generation's exponent units)
  struct CutImage {
    int n_rows = 0, n_m = 0, T_R = 0, T_M = 0;
    double* Xrec = nullptr;
    double* Bt = nullptr;
    long long* toff = nullptr;
    double* sph = nullptr;
  } obs_cut;
  bool has_cutoff() const { return obs_cut.Bt != nullptr; }
  double cut_tau = 0.0, cut2 = 0.0, t_cut = 0.0;
  void release_cutoff() {
    dfree(obs_cut.Xrec);
    dfree(obs_cut.Bt);
    dfree(obs_cut.toff);
    dfree(obs_cut.sph);
    obs_cut = CutImage{};
  }

  // Lifecycle (DESIGN.md §1 "Lifecycle waits"): the filters built on the model --
  // gpmdm_model_set_obs_cutoff waits for each one's own last frame (quiesce) before it
  // replaces the cutoff image -- and one event per stream the predictive maps ran on, so the
  // images' release at the last reference is ordered after those launches on the lifecycle
  // stream (no device-wide wait either way).
  std::mutex life_mu;
  std::vector<gpmdm_pf*> users;
  std::vector<std::pair<hipStream_t, hipEvent_t>> uses;
  void add_user(gpmdm_pf* pf) {
    std::lock_guard<std::mutex> lk(life_mu);
    users.push_back(pf);
  }
  void remove_user(gpmdm_pf* pf) {
    std::lock_guard<std::mutex> lk(life_mu);
    users.erase(std::remove(users.begin(), users.end(), pf), users.end());
  }
  hipError_t note_use(hipStream_t s) {   // after a predictive map's launches on s
    std::lock_guard<std::mutex> lk(life_mu);
    for (auto& u : uses)
      if (u.first == s) return hipEventRecord(u.second, s);
    hipEvent_t ev = nullptr;
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) return e;
    uses.emplace_back(s, ev);
    return hipEventRecord(ev, s);
  }

  ~gpmdm_model() {
    (void)hipSetDevice(device);
    if (hipStream_t life = life_stream(device)) {
      for (auto& u : uses) (void)hipStreamWaitEvent(life, u.second, 0);
    }
    for (auto& u : uses) (void)hipEventDestroy(u.second);
    obs.release();
    obs_small.release();
    for (auto& g : dyn) g.release();
    for (auto& g : dynw) g.release();
    release_cutoff();
    dfree(y_il2_dev);
    dfree(y_lam2_dev);
  }
};

inline void model_release(gpmdm_model* m) {
  if (m && m->refs.fetch_sub(1) == 1) delete m;
}

// The observation launch's image and shape for filters of P particles each (all ranks;
// a bank: per filter) whose shard holds n rows.
// * Small models (N <= kSmallObsN, d <= 12) and filters (P <= kSmallObsP): the 16 x 256
//   image (model.obs_small).  Its column blocks differ from the default image's, so the
//   per-block partial sums combine in another order: results agree to rounding, not bit
//   for bit, and the choice depends on the per-filter P only (every rank of a sharded
//   filter, and a bank and its filters run alone, make the same one).  (Splitting the
//   default image's partials as the dynamics images do would make them bitwise, at 0.5% of
//   the d = 3 observation launch: gp_tile.h.)
//   GPMDM_OBS_IMAGE16=0 does not build the image.
// * Otherwise, with fewer 32-row tiles than one per CU per column block, 16-row tiles over
//   the same 32 x 512 image (the image's fragment layout depends on the waves and column
//   tiles only): each workgroup's MFMA chain halves and twice the CUs work; every output is
//   accumulated and reduced in the same order whatever the tile height, so results are
//   bitwise those of the default shape (tests/test_gpu_small_path.py).
//   GPMDM_OBS_SMALL_TILES=0 / 1 forces these 16-row tiles off / on (A/B).
constexpr long long kSmallObsN = 1024, kSmallObsP = 1024;

inline int obs_parts_max(const gpmdm_model* m) {
  return std::max(m->obs.n_parts(), m->obs_small.Bf ? m->obs_small.n_parts() : 0);
}
inline int obs_blocks_max(const gpmdm_model* m) {
  return std::max(m->obs.n_pblocks(), m->obs_small.Bf ? m->obs_small.n_pblocks() : 0);
}

struct gpmdm_pf {
  gpmdm_model* m = nullptr;
  // P = all particles = F filters x Pf (a single filter: F = 1, Pf = P)
  long long P = 0, Pf = 0, lo = 0, hi = 0, nloc = 0;
  int F = 1;
  int n_ranks = 1, rank = 0, rng_mode = 0, resample_mode = 0, nb = 0, nbf = 0;
  unsigned seed_lo = 0, seed_hi = 0, frame = 0;
  bool initialised = false, switched = false, propagated = false;
  bool dyn_done = false;             // gpmdm_pf_propagate_dynamics ran, gpmdm_pf_weigh not yet
  // replay filters whose caller draws the normals after the switch's class counts: the
  // switch launches the dynamics-GP tiles (they need no normals) before it waits for the
  // counts, so they run while the host draws; propagate then launches the finish only
  bool gemm_ahead = false;
  hipEvent_t cnt_done = nullptr;      // after the switch's class counts (replay, large filters)
  bool dedup = true;                  // ancestor de-duplication of the dynamics GP
  int dyn_tiles = GPMDM_DYN_TILES_AUTO;   // gpmdm_pf_set_dyn_tiles
  bool wide_dyn() const { return dyn_tiles == GPMDM_DYN_TILES_WIDE || (dyn_tiles == GPMDM_DYN_TILES_AUTO && !dedup); }
  bool dyn_wide_frame = false;        // this frame's dynamics image (set by the switch: dyn_frame_wide)
  // device state
  double *T = nullptr, *X = nullptr, *X_prop = nullptr, *ll = nullptr;
  int *cls = nullptr, *cls_new = nullptr, *perm = nullptr, *ridx = nullptr;
  int *blockcounts = nullptr, *blockoff = nullptr, *small = nullptr;   // small: class tables
  int *obs_tab = nullptr;            // [0, 5): the observation launch's segment table; [8, 13): the cutoff image's
  // the observation GP's kernel-value cutoff (gpmdm_pf_set_obs_cutoff): on, and the skip
  // statistics of the cutoff kernel (device: MFMA groups run, the dense kernel's count)
  bool obs_cutoff = false;
  unsigned long long* sp_stats = nullptr;
  bool sp_stats_on = false;
  // AUTO (gpmdm_pf_set_obs_cutoff mode 3; single-rank filters and banks with mapped
  // read-outs): the cutoff kernel while the reach it measured is low, the dense kernel
  // otherwise -- decided per frame from the last cutoff frame's MFMA-group fraction, with a
  // cutoff frame (a probe) at least every kCutAutoProbe frames.  The counters travel with the
  // read-out (k_readout -> cut_auto_host), so the decision is a function of the filter's own
  // trajectory: deterministic, but not rank-count invariant (multi-rank filters run mode 1).
  static constexpr int kCutAutoProbe = 8;
  static constexpr double kCutAutoMaxRun = 0.75;   // break-even: cutoff 0.65 vs dense 0.865 of peak
  bool cut_auto = false;
  unsigned long long* cut_auto_dev = nullptr;      // device counters {run, dense}
  unsigned long long* cut_auto_host = nullptr;     // mapped: the last cutoff frame's counters
  unsigned long long* cut_auto_hdev = nullptr;     // (its device view)
  bool cut_auto_pending = false;                   // a cutoff frame's counters are on their way
  long long cut_auto_seq = 0;                      // ... published with this read-out number
  double cut_auto_frac = -1.0;                     // the last measured fraction (< 0: none)
  long long cut_auto_probe = -(1LL << 40);         // the frame of the last cutoff frame
  bool cut_frame = false;                          // this frame's observation GP is the cutoff's
  bool cut_frame_auto = false;                     // ... an AUTO filter's (its counters go with the read-out)
  // the counters run on every cutoff frame of a one-rank filter with mapped read-outs (modes 1
  // and 3): AUTO's choice of kernel, and the split policy's choice of the chunk grid
  bool cut_measure_active() const {
    return obs_cutoff && !sp_stats_on && n_ranks == 1 && seq_pin != nullptr && cut_auto_dev != nullptr;
  }
  bool cut_auto_active() const { return cut_auto && cut_measure_active(); }
  static constexpr double kCutChunksMin = 0.5;     // GPMDM_CUT_SPLIT_AUTO: the chunk grid from this reach
  // the cutoff kernel's split tiles (capi_frame.hip): second parts' partials, (n_act, c*) per
  // split tile; grown on demand
  int cut_split_policy = GPMDM_CUT_SPLIT_AUTO;
  double* cut_part = nullptr;
  size_t cut_part_cap = 0;
  int2* cut_split = nullptr;
  int cut_split_cap = 0;
  // (grown inside a frame: the old buffers are released after the frame stream's earlier work)
  int ensure_cut_split(size_t n_part, int n_split, hipStream_t s) {
    if (n_part > cut_part_cap) {
      dfree_after(cut_part, s);
      cut_part_cap = 0;
      if (dalloc(&cut_part, n_part)) return fail(GPMDM_E_NOMEM, "cutoff split partials");
      cut_part_cap = n_part;
    }
    if (n_split > cut_split_cap) {
      dfree_after(cut_split, s);
      cut_split_cap = 0;
      if (dalloc(&cut_split, (size_t)n_split)) return fail(GPMDM_E_NOMEM, "cutoff split table");
      cut_split_cap = n_split;
    }
    return GPMDM_OK;
  }
  // likelihood finish deferred into the resampling launch (single-shard small filters:
  // k_small_resample computes ll first, one launch less per frame); flush_ll runs it for
  // any reader of ll that comes first
  bool ll_pending = false;
  ObsFinishArgs oa_pending{};
  const GpImage* obs_img = nullptr;   // the observation launch's image and shape (obs_pick)
  TileGeo obs_geo{};
  int* guide = nullptr;             // F x (GB + 3) inverse-CDF guide table
  int *sys_mark = nullptr, *sys_block = nullptr;   // systematic resampling by scan (pf_kernels.hip)
  // ancestor de-duplication: owner/slot are C x P keyed by (class, ancestor)
  unsigned* owner = nullptr;
  int *slot = nullptr, *lflag = nullptr, *lblock = nullptr, *ltab = nullptr, *lperm = nullptr;
  // ancestor-ordered shards (multi-rank philox filters, shard_order.hip): own = particles
  // in order of their resampling uniform's bucket; this rank evaluates positions [lo, hi)
  int* own = nullptr;
  int* own_inv = nullptr;            // own_inv[own[r]] = r
  unsigned char* own_tmp = nullptr;
  size_t own_tmp_bytes = 0;
  bool own_valid = false;
  bool shard_order = true;            // gpmdm_pf_set_shard_order
  // The order a resample installs depends only on (seed, frame), so the pre-switch computes
  // the next resample's order into own_next / inv_next behind the read-out (the GPU's gap
  // while the host takes the outputs); that resample swaps it in instead of computing it.
  int* own_next = nullptr;
  int* inv_next = nullptr;
  long long own_next_frame = -1;     // the frame own_next was computed for (-1: none)
  // (single-rank filters keep it only with the observation-GP cutoff: particles of one
  // resampling-ancestor range form compact tiles, which skip more of the cutoff's K-steps)
  bool order_wanted() const {
    return own && (n_ranks > 1 || obs_cutoff) && dedup && shard_order && resample_mode != GPMDM_RESAMPLE_SYSTEMATIC &&
           uniform_order_supported(P);
  }
  // Exchanged rows read in place (gpmdm_pf_unpack_part): the all-gathered {class, state} rows
  // are read by the resample's gathers through the ownership order (only the ancestors' rows
  // are ever touched) and the {ll} column by a launch inside the resample that also writes
  // the normaliser's block maxima, instead of two unpack passes over every particle.  Rows
  // are in position order (row r = particle own[r]); *_w = doubles per row.  flush_rows
  // writes them out for a reader that needs X_prop / cls_new / ll first (export).
  const double* rows_st = nullptr;   // column 0 = class, 1..d = state
  int rows_st_w = 0;
  const double* rows_ll = nullptr;   // column 0 = ll
  int rows_ll_w = 0;
  const int* rows_inv = nullptr;     // the ownership order the rows were gathered in (nullptr: identity)
  // observation upload through two pinned slots (a pageable hipMemcpyAsync is staged by the
  // runtime and stalls the launching thread); each slot's event guards its reuse
  double* zpin[2] = {nullptr, nullptr};
  const double* zdev[2] = {nullptr, nullptr};   // device views of zpin (small z read in place)
  double* rpin = nullptr;             // pinned read-out landing buffer (F x (C + d + 1))
  // replay-mode draws (E, normals, U) staged through pinned buffers: the caller's arrays are
  // free for reuse when the call returns, whatever the runtime does with pageable copies;
  // each buffer's event guards its reuse
  // Small draws (<= kZeroCopyBytes: the notebook's P = 100) are not copied at all: the
  // kernels read them from the mapped pinned buffer (a copy is a launch of its own, ~4 us
  // on the frame's critical path).  rep_src[k] is what the kernels read this frame; the
  // event, recorded after the consuming launches (draws_used), guards the buffer's reuse.
  double* rep_pin[3] = {nullptr, nullptr, nullptr};
  const double* rep_dev[3] = {nullptr, nullptr, nullptr};   // device view of rep_pin
  const double* rep_src[3] = {nullptr, nullptr, nullptr};
  hipEvent_t rep_ev[3] = {nullptr, nullptr, nullptr};
  static constexpr size_t kZeroCopyBytes = 32768;
  hipError_t upload_draws(int k, double* dst, const double* src, size_t n, hipStream_t s) {
    // the buffer's previous readers have run (kernels that read it in place: guarded by the
    // read-out number of the frame that read it, see draws_used)
    const bool in_place = sizeof(double) * n <= kZeroCopyBytes && rep_dev[k];
    hipError_t e = in_place && seq_pin ? wait_readout(ro_seq) : hipEventSynchronize(rep_ev[k]);
    if (e != hipSuccess) return e;
    // draws written straight into the staging buffer (gpmdm_pf_draw_buffers): no copy
    if (src != rep_pin[k]) std::memcpy(rep_pin[k], src, sizeof(double) * n);
    if (sizeof(double) * n <= kZeroCopyBytes && rep_dev[k]) {
      rep_src[k] = rep_dev[k];
      return hipSuccess;
    }
    rep_src[k] = dst;
    return hipMemcpyAsync(dst, rep_pin[k], sizeof(double) * n, hipMemcpyHostToDevice, s);
  }
  // after the launches that read buffer k: an event, unless they read it in place and the
  // frame's read-out number follows them (each event record between kernels idles the GPU
  // ~6 us; at the notebook's 0.11 ms frames that is 5%)
  hipError_t draws_used(int k, hipStream_t s) {
    if (seq_pin && rep_dev[k] && rep_src[k] == rep_dev[k]) return hipSuccess;
    return hipEventRecord(rep_ev[k], s);
  }
  int* cnt_pin = nullptr;             // class counts landing buffer (mapped; replay mode)
  // Host-side class counts (single small replay filters).  The per-class normals are drawn
  // on the host with shapes P_c x d after the switch, so the switch's class counts used to
  // cost a mid-frame stream synchronisation.  The switch is argmax_j T[c_p, j] / E[p, j]
  // (k_switch), and every input is on the host once the previous resample's classes are:
  // k_small_resample also writes them into mapped memory (cls_pin), so the host computes the
  // same counts with the same fp64 divisions and comparisons while the kernels run.  The
  // device's own counts still land in cnt_pin and are compared at the next synchronisation
  // (a mismatch is an error, never a silent divergence).
  int* cls_pin = nullptr;             // mapped: the current classes (valid when cls_host_ok)
  int* cls_pdev = nullptr;
  bool cls_host_ok = false;           // cls_pin holds the classes the next switch reads
  bool cls_ev_pending = false;        // ... once cls_ev (after the resample that wrote them) is done
  hipEvent_t cls_ev = nullptr;
  hipEvent_t cnt_ev = nullptr;        // after the switch whose device counts cnt_expect awaits
  std::vector<double> T_host;         // C x C
  int cnt_expect[kMaxClasses] = {0};
  bool cnt_check = false;             // compare cnt_pin with cnt_expect at the next sync
  // read-outs written by the resampling kernels straight into mapped host memory as well
  // (small read-out tables): gpmdm_pf_read then needs no copy launch, only the stream sync
  double* ro_pin = nullptr;
  double* ro_dev = nullptr;
  int* cnt_dev = nullptr;
  hipEvent_t zev[2] = {nullptr, nullptr};   // (unused: see zslot_free)
  // A z slot is written again two frames after its frame used it; its readers (k_dyn_finish,
  // the observation tiles, the likelihood finish) precede that frame's read-out, and the
  // resample of the frame in between has recorded ro_ev by then (the call order is enforced),
  // so ro_ev guards both slots -- no event record of its own between two kernels.
  hipError_t zslot_free() {
    if (seq_pin) return wait_readout(ro_seq);
    return ro_ev_ok ? hipEventSynchronize(ro_ev) : hipSuccess;
  }
  // Filters whose read-outs land in mapped memory (one number per filter of a bank) also get
  // their sequence numbers there (the read-out kernels publish them after the values:
  // publish_readout), and the host waits on them instead of on an event recorded behind the
  // read-out -- such a record idles the GPU ~6 us before the next frame's switch.
  long long* seq_pin = nullptr;
  long long* seq_dev = nullptr;
  // the last read-out's number (0: none launched); atomic because gpmdm_pf_draws_free may
  // run on a drawing thread while the frame's thread launches the next read-out
  std::atomic<long long> ro_seq{0};
  long long seq_min() const { return min_mapped(seq_pin, F); }   // (one number per filter)
  // The numbers are read with ACQUIRE loads: the device publishes each with a system-scope
  // release store after the values it guards (publish_seq, pf_kernels.hip), so a caller that
  // has seen a number >= its target may then read those values with plain loads -- the
  // acquire keeps the compiler (and the CPU) from moving them above the number's load.
  static long long min_mapped(const long long* p, long long n) {
    long long v = __atomic_load_n(p, __ATOMIC_ACQUIRE);
    for (long long f = 1; f < n; ++f) {
      const long long x = __atomic_load_n(p + f, __ATOMIC_ACQUIRE);
      v = x < v ? x : v;
    }
    return v;
  }
  // until every one of the n numbers at p is >= target (a number the device publishes after
  // the data it guards).  `s`: the stream the publishing kernel was launched on -- if the
  // number has not appeared after 60 s, that stream is drained and the number looked at once
  // more (an error, not a hang, if it is still missing).
  static hipError_t wait_mapped(const long long* p, long long n, long long target, hipStream_t s) {
    if (min_mapped(p, n) >= target) return hipSuccess;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 1;; ++it) {
      if (min_mapped(p, n) >= target) return hipSuccess;
      if ((it & 255) == 0) {
        std::this_thread::yield();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
          const hipError_t e = hipStreamSynchronize(s);
          if (e != hipSuccess) return e;
          return min_mapped(p, n) >= target ? hipSuccess : hipErrorUnknown;
        }
      } else {
        __builtin_ia32_pause();
      }
    }
  }
  hipStream_t ro_stream = nullptr;    // the stream of the last read-out (its number's publisher)
  hipStream_t cnt_stream = nullptr;   // the stream of the switch whose counts cseq guards
  hipError_t wait_readout(long long target) const { return wait_mapped(seq_pin, F, target, ro_stream); }
  hipError_t wait_counts() const { return wait_mapped(cseq_pin, 1, cseq, cnt_stream); }
  // the switch's class counts (replay filters): k_scan_counts publishes cseq after writing
  // them to cnt_pin, so the host's wait for them needs no event record behind the switch
  long long* cseq_pin = nullptr;
  long long* cseq_dev = nullptr;
  long long cseq = 0;
  bool pre_counts_seq = false;        // the pending pre-switch's counts come with cseq
  int zslot = 0;
  bool z_staged = false;              // zpin[zslot] holds the frame's z, k_dyn_finish copies it
  double *qdyn = nullptr, *mudyn = nullptr, *qobs = nullptr, *sobs = nullptr;
  int nparts_dyn_max = 0;
  // failure detection: kHealth* counters, device, zeroed at create
  unsigned* health = nullptr;
  // predict(): per-particle dynamics-GP means, lazily allocated
  double *pred_q = nullptr, *pred_mu = nullptr, *pred_mu_p = nullptr, *pred_out = nullptr;
  size_t pred_q_cap = 0;
  double *z = nullptr, *E = nullptr, *normals = nullptr, *U = nullptr;
  unsigned long long* gmax = nullptr;
  // single filters: k_obs_ll's per-block maxima of ll, read by the normaliser in place of
  // k_norm_max (bmax_ready: produced by this frame's weigh, not yet consumed)
  unsigned long long* bmax = nullptr;
  bool bmax_ready = false;
  unsigned long long* bmax_rows = nullptr;   // multi-rank filters: k_rows_ll's block maxima
  // the leader election's owner table is all 0xffffffff (the last compaction restored it)
  bool owner_clean = false;
  double *e = nullptr, *local = nullptr, *blocksum = nullptr, *blockoffw = nullptr, *total = nullptr,
         *partials = nullptr, *readout = nullptr;
  // library-driven exchange (gpmdm_pf_set_comm): an RCCL communicator of n_ranks ranks, a
  // library-owned stream for the collectives, and the packed rows.  pad = rows per rank in
  // the collective (the largest shard; ranks' shards differ by at most one row).  When the
  // shards are uneven (or GPMDM_COMM_PAD_ROWS asks for it) the gather lands in *_stage and
  // each rank's rows are copied down to their shard offset.
  ncclComm_t comm = nullptr;
  bool comm_loop = false;            // comm is an in-process loopback communicator (tests)
  hipStream_t cstream = nullptr;
  hipEvent_t cev[3] = {nullptr, nullptr, nullptr};
  long long pad = 0;
  bool padded = false;
  double *xs_send = nullptr, *xs_recv = nullptr, *xs_stage = nullptr;
  double *xl_send = nullptr, *xl_recv = nullptr, *xl_stage = nullptr;
  void release_comm() {
    if (cstream) (void)hipStreamSynchronize(cstream);
    double* bufs[] = {xs_send, xs_recv, xs_stage, xl_send, xl_recv, xl_stage};
    for (double* b : bufs) dfree(b);
    xs_send = xs_recv = xs_stage = xl_send = xl_recv = xl_stage = nullptr;
    for (auto& e : cev) {
      if (e) (void)hipEventDestroy(e);
      e = nullptr;
    }
    if (cstream) (void)hipStreamDestroy(cstream);
    cstream = nullptr;
    comm = nullptr;                    // the caller owns the communicator
    comm_loop = false;
  }
  // Pre-switch (Philox filters): the next frame's class switch needs no host input (its
  // draws are keyed by the frame counter), so the resample launches it right behind the
  // read-out; it runs while the host takes the frame's outputs, and gpmdm_pf_switch then
  // only consumes it.  Every later call that reads or rewrites the switch's tables, or must
  // see the filter between frames (predict, set_*, init), drops it first, and the next
  // gpmdm_pf_switch launches it again -- the same draws, bitwise the same tables.  The
  // normaliser-maximum reset and the dynamics row count moved out of the switch into
  // k_dyn_finish, so nothing a between-frames reader sees changes.  GPMDM_NO_PRESWITCH=1
  // turns it off (A/B).
  bool preswitch = true;
  bool preswitched = false;           // launched, not yet consumed by gpmdm_pf_switch
  // after the pre-switch: recorded on sw_stream only when another stream or the host must
  // wait for it (an event record between two kernels idles the GPU ~6 us; on the stream
  // itself the order already holds), so it covers whatever followed the pre-switch there too
  hipEvent_t sw_ev = nullptr;
  hipStream_t sw_stream = nullptr;
  // Replay filters pre-switch on the caller's request (gpmdm_pf_preswitch: the next frame's
  // Exp(1) draws are the caller's, drawn ahead on the host): the switch, its class counts into
  // mapped memory (cnt_pin, cnt_done after them) and the dynamics-GP tiles, all behind the
  // read-out.  gpmdm_pf_switch consumes it when handed the same E pointer.
  const double* pre_E = nullptr;
  bool pre_counts = false;            // the pre-switch's counts land in cnt_pin (cnt_done)
  hipStream_t up_stream = nullptr;    // its Exp(1) draws go up on this stream, beside the frame
  hipEvent_t up_ev = nullptr;         // still running on the caller's (the switch waits on it)
  hipEvent_t ndev_ev = nullptr;       // after the last dynamics finish (the device normals' reader)
  hipError_t make_up_stream() {
    if (up_stream) return hipSuccess;
    hipError_t e = hipStreamCreateWithFlags(&up_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&up_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ndev_ev, hipEventDisableTiming);
    return e;
  }
  // Replay normals copied to the device ahead of the propagate that reads them
  // (gpmdm_pf_stage_normals): the value ranges staged from nstage_ptr since the last propagate
  const double* nstage_ptr = nullptr;
  bool n_staged_frame = false;        // this frame's normals came fully staged
  std::vector<std::pair<long long, long long>> nstaged;
  bool normals_staged(const double* p, long long n) const {   // does the union cover [0, n)?
    if (p != nstage_ptr) return false;
    long long reach = 0;
    for (const auto& r : nstaged) {     // sorted by start
      if (r.first > reach) return false;
      reach = std::max(reach, r.second);
    }
    return reach >= n;
  }
  hipEvent_t ro_ev = nullptr;         // after the last read-out (gpmdm_pf_read waits on it)
  bool ro_ev_ok = false;
  int* rows_last() const { return small + 504; }   // rows of the last dynamics pass
  // Tile height of the dynamics pass on the 16 x 256 image: 16, 32 or 64 particle rows per
  // workgroup give bitwise the same results (same column blocks, same per-row association),
  // so the height is a pure schedule choice: short grids of few rows want 16-row tiles, long
  // grids 64-row ones (a B fragment feeds 4 row groups).  Chosen per frame from the row count
  // of the dynamics pass the last gpmdm_pf_read saw (k_dyn_finish writes it to rows_pin).
  int* rows_pin = nullptr;
  int* rows_pdev = nullptr;
  int rows_hint = 0;
  TileGeo dyn_geo_frame{};            // this frame's dynamics launch shape (set by the switch)
  // timing
  bool timing = false;
  std::vector<hipEvent_t> pool;
  struct Rec { int stage; hipEvent_t a, b; };
  std::vector<Rec> recs;

  // class tables of the step's grouping (small[0, 240)); predict() groups into its own
  // copy (small[256, 496), base 256) so the step's tables -- which gpmdm_pf_dyn_rows
  // reads -- survive a predict between steps
  int* class_start(int base = 0) const { return small + base; }
  int* counts(int base = 0) const { return small + base + 40; }
  int* seg_begin(int base = 0) const { return small + base + 80; }
  int* seg_end(int base = 0) const { return small + base + 120; }
  int* seg_out(int base = 0) const { return small + base + 160; }
  int* seg_tiles(int base = 0) const { return small + base + 200; }
  static constexpr int kPredictTables = 256;
  // leader segment tables (same shape as the full ones)
  int* lseg_begin() const { return ltab; }
  int* lseg_end() const { return ltab + 40; }
  int* lseg_out() const { return ltab + 80; }
  int* lseg_tiles() const { return ltab + 120; }
  const int* own_order() const { return own_valid ? own : nullptr; }

  ~gpmdm_pf() {
    // (gpmdm_pf_destroy has waited for the filter's own work: quiesce, capi_pf.hip; a handle
    // deleted by a failed create has launched nothing)
    if (m) (void)hipSetDevice(m->device);
    if (up_stream) (void)hipStreamSynchronize(up_stream);
    release_comm();
    double* ds[] = {T, X, X_prop, ll, qdyn, mudyn, qobs, sobs, z, E, normals, U,
                    e, local, blocksum, blockoffw, total, partials, readout,
                    pred_q, pred_mu, pred_mu_p, pred_out};
    for (double* p : ds) dfree(p);
    int* is[] = {cls, cls_new, perm, ridx, blockcounts, blockoff, small, obs_tab,
                 slot, lflag, lblock, ltab, lperm, guide, own, own_inv, own_next, inv_next, sys_mark, sys_block};
    for (int* p : is) dfree(p);
    dfree(own_tmp);
    dfree(gmax);
    dfree(sp_stats);
    dfree(cut_auto_dev);
    hfree(cut_auto_host);
    dfree(cut_part);
    dfree(cut_split);
    dfree(bmax);
    dfree(bmax_rows);
    dfree(owner);
    dfree(health);
    for (auto& r : recs) { pool.push_back(r.a); pool.push_back(r.b); }
    for (auto ev : pool) (void)hipEventDestroy(ev);
    hfree(rpin);
    hfree(cnt_pin);
    hfree(cseq_pin);
    hfree(rows_pin);
    hfree(cls_pin);
    if (cls_ev) (void)hipEventDestroy(cls_ev);
    if (cnt_ev) (void)hipEventDestroy(cnt_ev);
    if (sw_ev) (void)hipEventDestroy(sw_ev);
    if (ro_ev) (void)hipEventDestroy(ro_ev);
    if (cnt_done) (void)hipEventDestroy(cnt_done);
    if (up_ev) (void)hipEventDestroy(up_ev);
    if (ndev_ev) (void)hipEventDestroy(ndev_ev);
    if (up_stream) (void)hipStreamDestroy(up_stream);
    hfree(ro_pin);
    hfree(seq_pin);
    for (int k = 0; k < 2; ++k) {
      hfree(zpin[k]);
      if (zev[k]) (void)hipEventDestroy(zev[k]);
    }
    for (int k = 0; k < 3; ++k) {
      hfree(rep_pin[k]);
      if (rep_ev[k]) (void)hipEventDestroy(rep_ev[k]);
    }
    if (m) m->remove_user(this);
    model_release(m);
  }

  hipEvent_t ev() {
    if (!pool.empty()) { hipEvent_t x = pool.back(); pool.pop_back(); return x; }
    hipEvent_t x = nullptr;
    // timing-only events: no system-scope fence at record time (a fenced record left a
    // ~10 us bubble between the stages it separates)
    (void)hipEventCreateWithFlags(&x, hipEventDisableSystemFence);
    return x;
  }
  unsigned timing_mask = (1u << GPMDM_N_STAGES) - 1;   // gpmdm_pf_timing_stages
  void mark_begin(hipStream_t s, int stage, hipEvent_t& a) {
    a = nullptr;
    if (timing && (timing_mask >> stage & 1u)) { a = ev(); (void)hipEventRecord(a, s); }
  }
  void mark_end(hipStream_t s, int stage, hipEvent_t a) {
    if (!timing || !a) return;
    hipEvent_t b = ev();
    (void)hipEventRecord(b, s);
    recs.push_back({stage, a, b});
  }
};

namespace gpmdm::capi {
// shared helpers (defined in the unit named beside each)
void fill_tile_common(TileParams& tp, const gpmdm_model* m, bool dyn);
ResampleArgs resample_args(gpmdm_pf* pf);
NormArgs norm_args(gpmdm_pf* pf);
int flush_ll(gpmdm_pf* pf, hipStream_t s);
int drop_preswitch(gpmdm_pf* pf, hipStream_t s, bool host_wait);
int quiesce(gpmdm_pf* pf);
int quiesce_users(gpmdm_model* m);
int h2d(void* dst, const void* src, size_t bytes);
// the observation-GP cutoff image (capi_model.hip; packed on the host or the device)
struct CutoffPlan {
  std::vector<long long> perm, toff;
  std::vector<double> sph, rec;
  double tau = 0.0;
  int T_R = 0, T_M = 0;
};
int cutoff_plan(gpmdm_model* m, double sigma2, const double* M, const double* y_absmax, CutoffPlan& pl);
int cutoff_install(gpmdm_model* m, const CutoffPlan& pl, const std::function<int(double*, const long long*)>& fill);
int do_switch(gpmdm_pf* pf, const double* E, int64_t* class_counts, hipStream_t s, bool order_ahead = false, bool counts_ahead = false, bool e_uploaded = false);
int propagate_dynamics(gpmdm_pf* pf, const double* normals, hipStream_t s, bool zstage = false);
int weigh(gpmdm_pf* pf, const double* zh, hipStream_t s);
int propagate_exchange(gpmdm_pf* pf, const double* zh, const double* normals, hipStream_t s);
int flush_rows(gpmdm_pf* pf, hipStream_t s);
const GpImage& obs_pick(const gpmdm_model* m, long long P, long long n, TileGeo& geo);
}  // namespace gpmdm::capi

