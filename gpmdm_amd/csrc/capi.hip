// C ABI of libgpmdm_hip.so (include/gpmdm_hip.h): model and particle-filter handles,
// device memory layout, and the per-frame launch sequence.
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
#include <mutex>
#include <type_traits>

#include <rccl/rccl.h>   // types only: the entry points are resolved at run time (rccl())

#include "../../include/gpmdm_hip.h"
#include "common.h"
#include "host_image.h"
#include "pf_kernels.h"
#include "status.h"

using namespace gpmdm;

namespace gpmdm {
thread_local std::string g_err;
int fail(int code, const std::string& msg) {
  g_err = msg;
  // a failed HIP call stays this thread's "last error" until read: reported here, it must
  // not surface again in a later call's launch check (a refused hipSetDevice of a missing
  // device, say, in front of an unrelated filter's first hipGetLastError)
  if (code == GPMDM_E_HIP || code == GPMDM_E_NOMEM) (void)hipGetLastError();
  return code;
}
}  // namespace gpmdm

static_assert(kMaxClassesDesc == kMaxClasses, "descriptor check and kernels agree on the class limit");

// RCCL entry points, resolved from librccl.so.1 on the first call that needs a communicator
// (gpmdm_comm_*, gpmdm_pf_set_comm): a single-GPU user needs no RCCL at build or load time,
// and a process that already holds torch's RCCL gets that same library (same soname).
struct RcclApi {
  bool ok = false;
  std::string why;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*CommCount)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*CommUserRank)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*CommCuDevice)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

static const RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      api.why = std::string("RCCL is not available (librccl.so.1): ") + (e ? e : "");
      return;
    }
    bool all = true;
    auto get = [&](auto& fp, const char* name) {
      fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
      if (!fp) {
        all = false;
        api.why = std::string("librccl.so.1 lacks ") + name;
      }
    };
    get(api.AllGather, "ncclAllGather");
    get(api.CommCount, "ncclCommCount");
    get(api.CommUserRank, "ncclCommUserRank");
    get(api.CommCuDevice, "ncclCommCuDevice");
    get(api.CommInitRank, "ncclCommInitRank");
    get(api.CommInitAll, "ncclCommInitAll");
    get(api.GroupStart, "ncclGroupStart");
    get(api.GroupEnd, "ncclGroupEnd");
    get(api.CommDestroy, "ncclCommDestroy");
    get(api.GetUniqueId, "ncclGetUniqueId");
    get(api.GetErrorString, "ncclGetErrorString");
    api.ok = all;
  });
  return api;
}

#define RCCL_OR_FAIL()                                                      \
  do {                                                                     \
    if (!rccl().ok) return fail(GPMDM_E_HIP, rccl().why);                  \
  } while (0)

namespace {

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

template <typename T>
int upload(T** dst, const std::vector<T>& v) {
  TRY(dalloc(dst, v.size()));
  HIPCHK(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return GPMDM_OK;
}

int build_image(GpImage& g, int n_rows, int d, int n_m, const double* X, const double* ls,
                const double* lin_c2, const double* R, const double* M, TileGeo geo) {
  const ImagePacker pk(n_rows, d, n_m, X, ls, lin_c2, R, M, geo);
  g.geo = geo;
  g.dyn = lin_c2 != nullptr;
  g.n_rows = n_rows;
  g.n_m = n_m;
  g.coff = pk.coff;
  g.n_j = pk.n_j;
  std::vector<double> rec, hf;
  pk.records(rec);
  TRY(upload(&g.Xrec, rec));
  if (lin_c2) {
    pk.linear(hf);
    TRY(upload(&g.Hf, hf));
  }
  TRY(dalloc(&g.Bf, (size_t)pk.total_doubles()));
  long long off = 0;
  std::vector<double> buf;
  for (int J = 0; J < g.n_j; ++J) {
    buf.assign((size_t)pk.block_doubles(J), 0.0);
    pk.pack_block(J, buf.data());
    HIPCHK(hipMemcpy(g.Bf + off, buf.data(), buf.size() * sizeof(double), hipMemcpyHostToDevice));
    off += (long long)buf.size();
  }
  return GPMDM_OK;
}

}  // namespace

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

  ~gpmdm_model() {
    obs.release();
    obs_small.release();
    for (auto& g : dyn) g.release();
    for (auto& g : dynw) g.release();
    dfree(y_il2_dev);
    dfree(y_lam2_dev);
  }
};

static void model_release(gpmdm_model* m) {
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

static int obs_parts_max(const gpmdm_model* m) {
  return std::max(m->obs.n_parts(), m->obs_small.Bf ? m->obs_small.n_parts() : 0);
}
static int obs_blocks_max(const gpmdm_model* m) {
  return std::max(m->obs.n_pblocks(), m->obs_small.Bf ? m->obs_small.n_pblocks() : 0);
}
static const GpImage& obs_pick(const gpmdm_model* m, long long P, long long n, TileGeo& geo) {
  if (m->obs_small.Bf && P <= kSmallObsP) {
    geo = m->obs_small.geo;
    return m->obs_small;
  }
  const TileGeo g = m->obs.geo;
  geo = g;
  if (g.nw == 4 && g.mt == 2 && g.ntw == 8 && m->d <= 12) {
    static const char* env = std::getenv("GPMDM_OBS_SMALL_TILES");
    bool small = (long long)m->obs.n_j * cdiv(n, g.pt()) <= 256;
    if (env) small = env[0] == '1';
    if (small) geo = TileGeo{4, 1, 8};
  }
  return m->obs;
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
  int *obs_tab = nullptr;
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
  bool order_wanted() const {
    return own && dedup && shard_order && resample_mode != GPMDM_RESAMPLE_SYSTEMATIC && uniform_order_supported(P);
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
         *cum = nullptr, *partials = nullptr, *readout = nullptr;
  // library-driven exchange (gpmdm_pf_set_comm): an RCCL communicator of n_ranks ranks, a
  // library-owned stream for the collectives, and the packed rows.  pad = rows per rank in
  // the collective (the largest shard; ranks' shards differ by at most one row).  When the
  // shards are uneven (or GPMDM_COMM_PAD_ROWS asks for it) the gather lands in *_stage and
  // each rank's rows are copied down to their shard offset.
  ncclComm_t comm = nullptr;
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
    if (preswitched) (void)hipDeviceSynchronize();   // a pre-switch may still use the buffers
    if (up_stream) (void)hipStreamSynchronize(up_stream);
    release_comm();
    double* ds[] = {T, X, X_prop, ll, qdyn, mudyn, qobs, sobs, z, E, normals, U,
                    e, local, blocksum, blockoffw, total, cum, partials, readout,
                    pred_q, pred_mu, pred_mu_p, pred_out};
    for (double* p : ds) dfree(p);
    int* is[] = {cls, cls_new, perm, ridx, blockcounts, blockoff, small, obs_tab,
                 slot, lflag, lblock, ltab, lperm, guide, own, own_inv, own_next, inv_next, sys_mark, sys_block};
    for (int* p : is) dfree(p);
    dfree(own_tmp);
    dfree(gmax);
    dfree(bmax);
    dfree(bmax_rows);
    dfree(owner);
    dfree(health);
    for (auto& r : recs) { pool.push_back(r.a); pool.push_back(r.b); }
    for (auto ev : pool) (void)hipEventDestroy(ev);
    if (rpin) (void)hipHostFree(rpin);
    if (cnt_pin) (void)hipHostFree(cnt_pin);
    if (cseq_pin) (void)hipHostFree(cseq_pin);
    if (rows_pin) (void)hipHostFree(rows_pin);
    if (cls_pin) (void)hipHostFree(cls_pin);
    if (cls_ev) (void)hipEventDestroy(cls_ev);
    if (cnt_ev) (void)hipEventDestroy(cnt_ev);
    if (sw_ev) (void)hipEventDestroy(sw_ev);
    if (ro_ev) (void)hipEventDestroy(ro_ev);
    if (cnt_done) (void)hipEventDestroy(cnt_done);
    if (up_ev) (void)hipEventDestroy(up_ev);
    if (ndev_ev) (void)hipEventDestroy(ndev_ev);
    if (up_stream) (void)hipStreamDestroy(up_stream);
    if (ro_pin) (void)hipHostFree(ro_pin);
    if (seq_pin) (void)hipHostFree(seq_pin);
    for (int k = 0; k < 2; ++k) {
      if (zpin[k]) (void)hipHostFree(zpin[k]);
      if (zev[k]) (void)hipEventDestroy(zev[k]);
    }
    for (int k = 0; k < 3; ++k) {
      if (rep_pin[k]) (void)hipHostFree(rep_pin[k]);
      if (rep_ev[k]) (void)hipEventDestroy(rep_ev[k]);
    }
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

// =====================================================================================
extern "C" {

const char* gpmdm_last_error(void) { return g_err.c_str(); }
const char* gpmdm_version(void) { return "gpmdm_hip 0.1.0 (gfx950, fp64 MFMA)"; }

int gpmdm_model_create(const gpmdm_model_desc* desc, int device, gpmdm_model_t* out) {
  CHECK(out, "null argument");
  *out = nullptr;
  {
    const std::string why = check_model_desc(desc);   // host_image.h
    CHECK(why.empty(), why);
  }
  HIPCHK(hipSetDevice(device));
  auto* m = new gpmdm_model();
  m->device = device;
  m->N = desc->N;
  m->D = desc->D;
  m->d = desc->d;
  m->C = desc->C;
  const int d = m->d;
  m->X.assign(desc->X, desc->X + desc->N * d);
  m->y_ls.assign(desc->y_lengthscales, desc->y_lengthscales + d);
  m->y_il2.assign(desc->y_inv_lambda2, desc->y_inv_lambda2 + m->D);
  m->x_ls.assign(desc->x_lengthscales, desc->x_lengthscales + d);
  m->x_lin_c2.assign(desc->x_lin_coeff2, desc->x_lin_coeff2 + d + 1);
  m->x_il2.assign(desc->x_inv_lambda2, desc->x_inv_lambda2 + d);
  // tile shapes: the observation GP defaults to 32x512 (half the kernel-value generation per
  // MFMA of 64x256, tools/microbench/tile_bench.hip); the dynamics GPs use 64-particle tiles
  // (their class-grouped tile starts are computed on the device in 64s, pf_kernels.hip)
  // (above d = 12 the 32x512 shape's registers spill -- launch_d then reads its particle
  // coordinates from LDS -- and 64x512 (8 waves) is the best shape: config 5, d = 16,
  // 760 ms per launch vs 850 ms for 32x512 with LDS coordinates, tile_ab.sh).  The dynamics
  // GPs run few rows (ancestor de-duplication) against short triangular blocks: their time
  // is the K loop of the heaviest blocks, which narrow particle tiles shorten (64 -> 32 ->
  // 16 particles: dyn GEMM 0.215 -> 0.163 -> 0.150 ms per step at config 2).  Evaluating
  // every particle (de-duplication off, GPMDM_PF.predict, large predictive maps) is a
  // throughput problem like the observation GP's, so the dynamics GPs get a second image in
  // the observation GP's shape (half the kernel-value generation per MFMA of 16x256 and
  // 40% fewer generated rows; config 2, 100k rows: see DESIGN.md §3).
  TileGeo obs_geo = d <= 12 ? kGeo32x512 : kGeo64x512, dyn_geo = kGeo16x256;
  TileGeo dynw_geo = obs_geo;
  switch (desc->tile_shape) {
    case GPMDM_TILE_DEFAULT: break;
    case GPMDM_TILE_64x256: obs_geo = dyn_geo = dynw_geo = kGeo64x256; break;
    case GPMDM_TILE_64x512: obs_geo = dyn_geo = dynw_geo = kGeo64x512; break;
    case GPMDM_TILE_32x512: obs_geo = kGeo32x512; break;
    default: break;   // rejected by check_model_desc
  }
  int rc = build_image(m->obs, (int)m->N, d, m->D, desc->X, desc->y_lengthscales, nullptr,
                       desc->obs_R, desc->obs_beta, obs_geo);
  if (rc) { delete m; return rc; }
  {
    const char* e = std::getenv("GPMDM_OBS_IMAGE16");       // "0": not built (A/B, tests)
    if (m->N <= kSmallObsN && d <= 12 && obs_geo.nw == kGeo32x512.nw && obs_geo.mt == kGeo32x512.mt &&
        obs_geo.ntw == kGeo32x512.ntw && !(e && e[0] == '0')) {
      rc = build_image(m->obs_small, (int)m->N, d, m->D, desc->X, desc->y_lengthscales, nullptr,
                       desc->obs_R, desc->obs_beta, kGeo16x256);
      if (rc) { delete m; return rc; }
    }
  }
  m->dyn.resize(m->C);
  const bool two = dynw_geo.nw != dyn_geo.nw || dynw_geo.mt != dyn_geo.mt || dynw_geo.ntw != dyn_geo.ntw;
  if (two) m->dynw.resize(m->C);
  for (int c = 0; c < m->C; ++c) {
    rc = build_image(m->dyn[c], (int)desc->Nc[c], d, d, desc->Xin[c], desc->x_lengthscales,
                     m->x_lin_c2.data(),
                     desc->dyn_R[c], desc->dyn_alpha[c], dyn_geo);
    if (rc) { delete m; return rc; }
    if (two) {
      rc = build_image(m->dynw[c], (int)desc->Nc[c], d, d, desc->Xin[c], desc->x_lengthscales,
                       m->x_lin_c2.data(), desc->dyn_R[c], desc->dyn_alpha[c], dynw_geo);
      if (rc) { delete m; return rc; }
    }
  }
  rc = dalloc(&m->y_il2_dev, m->D);
  if (rc) { delete m; return rc; }
  if (hipMemcpy(m->y_il2_dev, m->y_il2.data(), m->D * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
    delete m;
    return fail(GPMDM_E_HIP, "upload y_inv_lambda2");
  }
  {
    std::vector<double> lam2(m->D);
    for (int j = 0; j < m->D; ++j) {
      lam2[j] = 1.0 / m->y_il2[j];
      m->sum_log_il2 += std::log(m->y_il2[j]);
    }
    rc = dalloc(&m->y_lam2_dev, m->D);
    if (rc) { delete m; return rc; }
    if (hipMemcpy(m->y_lam2_dev, lam2.data(), m->D * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
      delete m;
      return fail(GPMDM_E_HIP, "upload lambda^2");
    }
  }
  *out = m;
  return GPMDM_OK;
}

int gpmdm_model_destroy(gpmdm_model_t m) {
  model_release(m);   // freed once the last filter built on it is gone
  return GPMDM_OK;
}

// ------------------------------------------------------------------------------------
static void fill_tile_common(TileParams& tp, const gpmdm_model* m, bool dyn) {
  const int d = m->d;
  for (int j = 0; j < d; ++j) tp.ls[j] = dyn ? m->x_ls[j] : m->y_ls[j];
}

// The predictive maps' per-call scratch is released in stream order on every exit after
// its allocation, a failed launch included (the launch error is what the call reports).
static int finish_scratch(double* q, hipStream_t s) {
  const hipError_t launch = hipGetLastError();
  const hipError_t freed = hipFreeAsync(q, s);
  if (launch != hipSuccess) return fail(GPMDM_E_HIP, std::string("predictive-map launch: ") + hipGetErrorString(launch));
  if (freed != hipSuccess) return fail(GPMDM_E_HIP, std::string("hipFreeAsync: ") + hipGetErrorString(freed));
  return GPMDM_OK;
}

int gpmdm_predict_obs(gpmdm_model_t m, const double* Xs, int64_t n, double* mu, double* var, void* stream) {
  CHECK(m, "null model");
  CHECK(n >= 0 && n < (1ll << 31), "bad n");
  if (n == 0) return GPMDM_OK;
  CHECK(Xs && mu && var, "null buffer");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipSetDevice(m->device));
  const int nparts = m->obs.n_parts();
  // per-call scratch on the caller's stream (stream-ordered allocation: calls on different
  // streams never share it), freed in stream order after the finish kernel
  double* q = nullptr;
  HIPCHK(hipMallocAsync((void**)&q, sizeof(double) * ((size_t)nparts * n + 4), s));
  TileParams tp{};
  tp.seg[0] = m->obs.seg();
  tp.n_seg = 1;
  tp.geo = m->obs.geo;
  tp.tiles_ub = m->obs.tiles(n);
  tp.n_j_max = m->obs.n_j;
  int* tab = reinterpret_cast<int*>(q + (size_t)nparts * n);   // segment table after q
  launch_seg_table(tab, (int)n, m->obs.tiles(n), s);
  tp.seg_pos_begin = tab + 0;
  tp.seg_pos_end = tab + 1;
  tp.seg_out_base = tab + 2;
  tp.seg_tile_start = tab + 3;
  tp.perm = nullptr;
  tp.X = Xs;
  fill_tile_common(tp, m, false);
  tp.qpart = q;
  tp.ld_q = n;
  tp.mu = mu;
  tp.ld_mu = m->D;
  launch_gp_tile(tp, m->d, false, s);
  ObsFinishArgs fa{};
  fa.n_out = n;
  fa.n_parts = nparts;
  fa.D = m->D;
  fa.qpart = q;
  fa.ld_q = n;
  fa.mu = mu;
  fa.ld_mu = m->D;
  fa.il2 = m->y_il2_dev;
  fa.var_out = var;
  launch_obs_finish(fa, s);
  return finish_scratch(q, s);
}

int gpmdm_predict_dyn(gpmdm_model_t m, int c, const double* Xs, int64_t n, double* mu, double* var, void* stream) {
  CHECK(m, "null model");
  CHECK(c >= 0 && c < m->C, "class index out of range");
  CHECK(n >= 0 && n < (1ll << 31), "bad n");
  if (n == 0) return GPMDM_OK;
  CHECK(Xs && mu && var, "null buffer");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipSetDevice(m->device));
  const GpImage& g = m->dyn_set(n >= kWideRows)[c];
  const int nparts = g.n_parts();
  double* q = nullptr;                 // per-call scratch, stream-ordered (see gpmdm_predict_obs)
  HIPCHK(hipMallocAsync((void**)&q, sizeof(double) * ((size_t)nparts * n + 4), s));
  TileParams tp{};
  tp.seg[0] = g.seg();
  tp.n_seg = 1;
  tp.geo = g.geo;
  tp.tiles_ub = g.tiles(n);
  tp.n_j_max = g.n_j;
  int* tab = reinterpret_cast<int*>(q + (size_t)nparts * n);   // segment table after q
  launch_seg_table(tab, (int)n, g.tiles(n), s);
  tp.seg_pos_begin = tab + 0;
  tp.seg_pos_end = tab + 1;
  tp.seg_out_base = tab + 2;
  tp.seg_tile_start = tab + 3;
  tp.X = Xs;
  fill_tile_common(tp, m, true);
  tp.qpart = q;
  tp.ld_q = n;
  tp.mu = mu;
  tp.ld_mu = m->d;
  launch_gp_tile(tp, m->d, true, s);
  DynFinishArgs fa{};
  fa.n_out = n;
  fa.n_seg = 1;
  fa.d = m->d;
  fa.n_parts[0] = nparts;
  fa.qpart = q;
  fa.ld_q = n;
  fa.mu = mu;
  fa.ld_mu = m->d;
  fa.X = Xs;
  for (int j = 0; j <= m->d; ++j) fa.lin_c2[j] = m->x_lin_c2[j];
  for (int j = 0; j < m->d; ++j) fa.il2[j] = m->x_il2[j];
  fa.var_out = var;
  launch_dyn_finish(fa, s);
  return finish_scratch(q, s);
}

// ------------------------------------------------------------------------------------
static int pf_create(gpmdm_model_t m, const double* T, int64_t F, int64_t Pf, int rng_mode, uint64_t seed,
                     int resample_mode, int n_ranks, int rank, gpmdm_pf_t* out) {
  CHECK(m && T && out, "null argument");
  *out = nullptr;
  CHECK(Pf >= 1 && F >= 1 && F <= 65535 && F * Pf < (1ll << 31) - 256, "num_particles out of range");
  CHECK(F == 1 || (rng_mode == GPMDM_RNG_PHILOX && n_ranks == 1),
        "filter banks use device (philox) draws on one rank; shard filters, not particles");
  const long long P = F * Pf;
  CHECK(rng_mode == GPMDM_RNG_REPLAY || rng_mode == GPMDM_RNG_PHILOX, "bad rng mode");
  CHECK(resample_mode == GPMDM_RESAMPLE_MULTINOMIAL || resample_mode == GPMDM_RESAMPLE_SYSTEMATIC,
        "bad resample mode");
  CHECK(n_ranks >= 1 && rank >= 0 && rank < n_ranks, "bad rank");
  HIPCHK(hipSetDevice(m->device));
  auto* pf = new gpmdm_pf();
  pf->m = m;
  m->refs.fetch_add(1);   // released by ~gpmdm_pf
  pf->P = P;
  pf->Pf = Pf;
  pf->F = (int)F;
  pf->n_ranks = n_ranks;
  pf->rank = rank;
  pf->lo = P * rank / n_ranks;
  pf->hi = P * (rank + 1) / n_ranks;
  pf->nloc = pf->hi - pf->lo;
  pf->rng_mode = rng_mode;
  pf->resample_mode = resample_mode;
  pf->seed_lo = (unsigned)(seed & 0xffffffffu);
  pf->seed_hi = (unsigned)(seed >> 32);
  pf->nb = (int)cdiv(P, 256);
  pf->nbf = (int)cdiv(Pf, 256);
  const int C = m->C, d = m->d, D = m->D;
  const int maxparts = m->dyn_parts_max();
  pf->nparts_dyn_max = maxparts;
  const long long nl = std::max(pf->nloc, 1ll);
  int rc = 0;
#define ALLOC(ptr, n) do { rc = dalloc(&pf->ptr, (size_t)(n)); if (rc) { delete pf; return rc; } } while (0)
  ALLOC(T, C * C);
  ALLOC(X, P * d);
  ALLOC(X_prop, P * d);
  ALLOC(ll, P);
  ALLOC(cls, P);
  ALLOC(cls_new, P);
  ALLOC(perm, P);
  ALLOC(ridx, P);
  ALLOC(blockcounts, (long long)pf->nb * C);
  ALLOC(blockoff, (long long)pf->nb * C);
  ALLOC(small, 512);
  ALLOC(obs_tab, 8);
  ALLOC(owner, (long long)C * P);
  ALLOC(slot, (long long)C * P);
  ALLOC(lflag, P);
  ALLOC(lblock, pf->nb);
  ALLOC(ltab, 200);
  ALLOC(lperm, P);
  ALLOC(qdyn, (long long)maxparts * nl);
  ALLOC(mudyn, nl * d);
  ALLOC(qobs, (long long)obs_parts_max(m) * nl);
  ALLOC(sobs, (long long)obs_blocks_max(m) * nl);   // fused likelihood partials (no mean stored)
  ALLOC(z, F * D);
  if (rng_mode == GPMDM_RNG_REPLAY) {
    ALLOC(E, P * C);
    ALLOC(normals, P * d);
    ALLOC(U, P);
  }
  ALLOC(gmax, F);
  if (F == 1 && n_ranks == 1) ALLOC(bmax, pf->nb);
  if (F == 1 && n_ranks > 1) ALLOC(bmax_rows, rows_ll_blocks(P));
  ALLOC(e, P);
  ALLOC(local, P);
  ALLOC(blocksum, F * pf->nbf);
  ALLOC(blockoffw, F * pf->nbf);
  ALLOC(total, F);
  ALLOC(cum, P);
  ALLOC(guide, guide_buckets_used(Pf) > 0 ? F * (guide_buckets(Pf) + 3) : 1);
  ALLOC(partials, F * pf->nbf * (C + 1 + d));
  ALLOC(readout, F * (C + d + 1));
  ALLOC(health, kHealthN);
  if (resample_mode == GPMDM_RESAMPLE_SYSTEMATIC) {
    ALLOC(sys_mark, P);
    ALLOC(sys_block, F * pf->nbf);
  }
  if (n_ranks > 1 && rng_mode == GPMDM_RNG_PHILOX) {
    pf->own_tmp_bytes = std::max<size_t>(uniform_order_temp_bytes(P), 1);
    ALLOC(own, P);
    ALLOC(own_inv, P);
    ALLOC(own_next, P);
    ALLOC(inv_next, P);
    ALLOC(own_tmp, pf->own_tmp_bytes);
  }
#undef ALLOC
  for (int k = 0; k < 2; ++k) {
    void* zv = nullptr;
    if (hipHostMalloc((void**)&pf->zpin[k], sizeof(double) * F * D, hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipEventCreateWithFlags(&pf->zev[k], hipEventDisableTiming) != hipSuccess ||
        hipHostGetDevicePointer(&zv, pf->zpin[k], 0) != hipSuccess) {
      delete pf;
      return fail(GPMDM_E_NOMEM, "pinned observation buffer");
    }
    pf->zdev[k] = (const double*)zv;
  }
  if (hipHostMalloc((void**)&pf->rpin, sizeof(double) * F * (C + d + 1)) != hipSuccess) {
    delete pf;
    return fail(GPMDM_E_NOMEM, "pinned read-out buffer");
  }
  if (sizeof(double) * F * (C + d + 1) <= 32768) {
    void* rv = nullptr;
    if (hipHostMalloc((void**)&pf->ro_pin, sizeof(double) * F * (C + d + 1),
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(&rv, pf->ro_pin, 0) != hipSuccess) {
      delete pf;
      return fail(GPMDM_E_NOMEM, "mapped read-out buffer");
    }
    pf->ro_dev = (double*)rv;
    void* sv = nullptr;
    if (hipHostMalloc((void**)&pf->seq_pin, sizeof(long long) * F, hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer(&sv, pf->seq_pin, 0) != hipSuccess) {
      delete pf;
      return fail(GPMDM_E_NOMEM, "mapped read-out number");
    }
    for (long long f = 0; f < F; ++f) pf->seq_pin[f] = 0;
    pf->seq_dev = (long long*)sv;
  }
  {
    void* rv = nullptr;
    if (hipHostMalloc((void**)&pf->rows_pin, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(&rv, pf->rows_pin, 0) != hipSuccess) {
      delete pf;
      return fail(GPMDM_E_NOMEM, "mapped row-count buffer");
    }
    pf->rows_pdev = (int*)rv;
    *pf->rows_pin = 0;
  }
  if (rng_mode == GPMDM_RNG_REPLAY) {
    const long long n[3] = {P * C, P * d, P};      // E, normals, U
    // mapped, coherent (fine-grained): kernels may read the small draws in place
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    for (int k = 0; k < 3; ++k) {
      void* dv = nullptr;
      if (hipHostMalloc((void**)&pf->rep_pin[k], sizeof(double) * n[k], fl) != hipSuccess ||
          hipEventCreateWithFlags(&pf->rep_ev[k], hipEventDisableTiming) != hipSuccess ||
          hipHostGetDevicePointer(&dv, pf->rep_pin[k], 0) != hipSuccess) {
        delete pf;
        return fail(GPMDM_E_NOMEM, "pinned replay-draw buffer");
      }
      pf->rep_dev[k] = (const double*)dv;
    }
    void* cv = nullptr;
    if (hipHostMalloc((void**)&pf->cnt_pin, sizeof(int) * kMaxClasses, fl) != hipSuccess ||
        hipHostGetDevicePointer(&cv, pf->cnt_pin, 0) != hipSuccess) {
      delete pf;
      return fail(GPMDM_E_NOMEM, "pinned class-count buffer");
    }
    pf->cnt_dev = (int*)cv;
    void* qv = nullptr;
    if (hipHostMalloc((void**)&pf->cseq_pin, sizeof(long long), fl) != hipSuccess ||
        hipHostGetDevicePointer(&qv, pf->cseq_pin, 0) != hipSuccess) {
      delete pf;
      return fail(GPMDM_E_NOMEM, "mapped class-count number");
    }
    *pf->cseq_pin = 0;
    pf->cseq_dev = (long long*)qv;
    if (F == 1 && n_ranks == 1 && P <= kHostCountsMaxP) {
      void* lv = nullptr;
      if (hipHostMalloc((void**)&pf->cls_pin, sizeof(int) * P, fl) != hipSuccess ||
          hipHostGetDevicePointer(&lv, pf->cls_pin, 0) != hipSuccess ||
          hipEventCreateWithFlags(&pf->cls_ev, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&pf->cnt_ev, hipEventDisableTiming) != hipSuccess) {
        delete pf;
        return fail(GPMDM_E_NOMEM, "pinned class buffer");
      }
      pf->cls_pdev = (int*)lv;
      pf->T_host.assign(T, T + (size_t)C * C);
    }
  }
  if (rng_mode == GPMDM_RNG_REPLAY && hipEventCreateWithFlags(&pf->cnt_done, hipEventDisableTiming) != hipSuccess) {
    delete pf;
    return fail(GPMDM_E_HIP, "filter events");
  }
  if (hipEventCreateWithFlags(&pf->sw_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&pf->ro_ev, hipEventDisableTiming) != hipSuccess) {
    delete pf;
    return fail(GPMDM_E_HIP, "filter events");
  }
  pf->preswitch = rng_mode == GPMDM_RNG_PHILOX && std::getenv("GPMDM_NO_PRESWITCH") == nullptr;
  pf->obs_img = &obs_pick(m, pf->Pf, pf->nloc, pf->obs_geo);
  const int tab[5] = {(int)pf->lo, (int)pf->hi, 0, 0, (int)cdiv(pf->nloc, pf->obs_geo.pt())};
  if (hipMemcpy(pf->obs_tab, tab, sizeof(tab), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(pf->T, T, sizeof(double) * C * C, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(pf->health, 0, sizeof(unsigned) * kHealthN) != hipSuccess ||
      hipMemset(pf->small, 0, sizeof(int) * 512) != hipSuccess) {
    delete pf;
    return fail(GPMDM_E_HIP, "upload of particle-filter tables failed");
  }
  *out = pf;
  return GPMDM_OK;
}

int gpmdm_pf_create(gpmdm_model_t m, const double* T, int64_t P, int rng_mode, uint64_t seed,
                    int resample_mode, int n_ranks, int rank, gpmdm_pf_t* out) {
  return pf_create(m, T, 1, P, rng_mode, seed, resample_mode, n_ranks, rank, out);
}

int gpmdm_bank_create(gpmdm_model_t m, const double* T, int64_t n_filters, int64_t P, uint64_t seed,
                      int resample_mode, gpmdm_pf_t* out) {
  return pf_create(m, T, n_filters, P, GPMDM_RNG_PHILOX, seed, resample_mode, 1, 0, out);
}

int gpmdm_pf_draw_buffers(gpmdm_pf_t pf, double** exp_draws, double** normals, double** uniforms) {
  CHECK(pf, "null handle");
  CHECK(pf->rng_mode == GPMDM_RNG_REPLAY, "draw buffers belong to replay filters");
  if (exp_draws) *exp_draws = pf->rep_pin[0];
  if (normals) *normals = pf->rep_pin[1];
  if (uniforms) *uniforms = pf->rep_pin[2];
  return GPMDM_OK;
}

int gpmdm_pf_draws_free(gpmdm_pf_t pf, int which) {
  CHECK(pf, "null handle");
  CHECK(pf->rng_mode == GPMDM_RNG_REPLAY, "draw buffers belong to replay filters");
  CHECK(which >= 0 && which < 3, "which: 0 exp draws, 1 normals, 2 uniforms");
  HIPCHK(hipSetDevice(pf->m->device));
  HIPCHK(hipEventSynchronize(pf->rep_ev[which]));
  if (pf->seq_pin && pf->rep_dev[which] && pf->rep_src[which] == pf->rep_dev[which]) {
    HIPCHK(pf->wait_readout(pf->ro_seq));   // last read in place: guarded by the read-out number (draws_used)
    // a replay pre-switch launched after that read-out reads the Exp(1) draws in place too:
    // its class counts (published after its switch) follow that read
    if (which == 0 && pf->preswitched && pf->pre_counts)
      HIPCHK(pf->pre_counts_seq ? pf->wait_counts() : hipEventSynchronize(pf->cnt_done));
  }
  return GPMDM_OK;
}

int gpmdm_pf_shape(gpmdm_pf_t pf, int64_t* n_filters, int64_t* P) {
  CHECK(pf, "null handle");
  if (n_filters) *n_filters = pf->F;
  if (P) *P = pf->Pf;
  return GPMDM_OK;
}

int gpmdm_pf_destroy(gpmdm_pf_t pf) {
  delete pf;
  return GPMDM_OK;
}

static ResampleArgs resample_args(gpmdm_pf* pf) {
  const gpmdm_model* m = pf->m;
  ResampleArgs ra{};
  ra.P = pf->Pf;
  ra.nb = pf->nbf;
  ra.F = pf->F;
  ra.C = m->C;
  ra.d = m->d;
  ra.systematic = pf->resample_mode == GPMDM_RESAMPLE_SYSTEMATIC;
  ra.frame = pf->frame;
  ra.seed_lo = pf->seed_lo;
  ra.seed_hi = pf->seed_hi;
  ra.cum = pf->cum;
  ra.ll = pf->ll;
  ra.e = pf->e;
  ra.total = pf->total;
  ra.gmax = pf->gmax;
  ra.cls_src = pf->cls_new;
  ra.X_src = pf->X_prop;
  ra.cls_dst = pf->cls;
  ra.X_dst = pf->X;
  ra.ridx = pf->ridx;
  ra.partials = pf->partials;
  ra.readout = pf->readout;
  ra.readout_host = pf->ro_dev;
  ra.guide = pf->guide;
  ra.GB = guide_buckets_used(pf->Pf);   // 0: plain search
  ra.sys_mark = pf->sys_mark;           // systematic: by scan, no search
  ra.sys_block = pf->sys_block;
  return ra;
}

static NormArgs norm_args(gpmdm_pf* pf) {
  NormArgs na{};
  na.P = pf->Pf;
  na.nb = pf->nbf;
  na.F = pf->F;
  na.ll = pf->ll;
  na.gmax = pf->gmax;
  na.e = pf->e;
  na.local = pf->local;
  na.blocksum = pf->blocksum;
  na.blockoff = pf->blockoffw;
  na.total = pf->total;
  na.cum = pf->cum;
  if (pf->ll_pending) {
    na.obs = pf->oa_pending;
    na.obs_pending = 1;
  }
  if (pf->bmax_ready) na.bmax = pf->bmax;
  return na;
}

static int flush_ll(gpmdm_pf* pf, hipStream_t s) {
  if (!pf->ll_pending) return GPMDM_OK;
  launch_obs_finish(pf->oa_pending, s);
  pf->ll_pending = false;
  HIPCHK(hipGetLastError());
  return GPMDM_OK;
}

// Undo a pre-switch before a call that reads or rewrites the switch's tables or needs the
// filter between frames: the caller's stream (or, with none, the host) waits for it, and
// the next gpmdm_pf_switch launches the switch again (same draws: the same tables).
static int drop_preswitch(gpmdm_pf* pf, hipStream_t s, bool host_wait) {
  if (!pf->preswitched) return GPMDM_OK;
  if (host_wait || s != pf->sw_stream) HIPCHK(hipEventRecord(pf->sw_ev, pf->sw_stream));   // (see sw_ev)
  if (host_wait)
    HIPCHK(hipEventSynchronize(pf->sw_ev));
  else if (s != pf->sw_stream)
    HIPCHK(hipStreamWaitEvent(s, pf->sw_ev, 0));
  pf->preswitched = false;
  pf->switched = false;
  pf->gemm_ahead = pf->pre_counts = false;   // (a replay pre-switch's tiles are redone too)
  return GPMDM_OK;
}

// The device's class counts of the last host-counted switch (checked by the next one, after
// the resample that followed it): they must equal the host's (same inputs, same fp64
// operations); a difference is reported as an error, never used.
static int check_counts(gpmdm_pf* pf) {
  if (!pf->cnt_check) return GPMDM_OK;
  // done: it precedes the resample already waited for (whose read-out number follows it)
  HIPCHK(pf->seq_pin ? pf->wait_readout(pf->ro_seq) : hipEventSynchronize(pf->cnt_ev));
  pf->cnt_check = false;
  for (int c = 0; c < pf->m->C; ++c)
    if (pf->cnt_pin[c] != pf->cnt_expect[c])
      return fail(GPMDM_E_STATE, "host and device class counts of the switch differ");
  return GPMDM_OK;
}

int gpmdm_pf_init(gpmdm_pf_t pf, const double* states, const int64_t* classes) {
  CHECK(pf && states && classes, "null argument");
  gpmdm_model* m = pf->m;
  HIPCHK(hipSetDevice(m->device));
  TRY(drop_preswitch(pf, nullptr, true));
  pf->bmax_ready = false;
  const long long P = pf->P;
  std::vector<int> c32(P);
  for (long long i = 0; i < P; ++i) {
    CHECK(classes[i] >= 0 && classes[i] < m->C, "class id out of range");
    c32[i] = (int)classes[i];
  }
  HIPCHK(hipMemcpy(pf->X, states, sizeof(double) * P * m->d, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(pf->cls, c32.data(), sizeof(int) * P, hipMemcpyHostToDevice));
  if (pf->cls_pin) {
    std::memcpy(pf->cls_pin, c32.data(), sizeof(int) * P);
    pf->cls_host_ok = true;
    pf->cls_ev_pending = false;
  }
  for (long long i = 0; i < P; ++i) c32[i] = (int)(i % pf->Pf);   // no shared ancestors yet
  HIPCHK(hipMemcpy(pf->ridx, c32.data(), sizeof(int) * P, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(pf->ll, 0, sizeof(double) * P));
  const std::vector<unsigned long long> neg(pf->F, 0x000fffffffffffffull);   // ord_enc(-inf)
  HIPCHK(hipMemcpy(pf->gmax, neg.data(), sizeof(unsigned long long) * pf->F, hipMemcpyHostToDevice));
  // read-outs of the initial state: ll = log_w = 0, w = 1/P (gpmdm_pf.py:102-104)
  ResampleArgs ra = resample_args(pf);
  ra.identity = 1;
  ra.cls_src = pf->cls;
  ra.X_src = pf->X;
  launch_normalise_resample(norm_args(pf), ra, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(pf->ro_ev, nullptr));
  HIPCHK(hipDeviceSynchronize());
  pf->ro_ev_ok = true;
  if (pf->seq_pin) pf->ro_seq = pf->seq_min();   // (synchronised: nothing to wait for)
  pf->initialised = true;
  pf->own_valid = false;               // no ancestors yet: identity ownership
  pf->rows_st = pf->rows_ll = nullptr;
  pf->switched = pf->propagated = pf->dyn_done = pf->ll_pending = pf->gemm_ahead = false;
  return GPMDM_OK;
}

// Restore an exported state (gpmdm_pf.py:78-82, 100-104): particles, ancestors, ll and the
// weights, then the read-outs of that state from the restored values themselves -- the
// identity resampling pass reads ll, max(ll) and e / total, so with e = w and total = 1 it
// reads w as the exporter's read-out read e / S (export's w is that same division), and
// the read-outs equal the exporter's bit for bit.  The next frame's normalisation
// recomputes e and the total from its own ll (weights are not recursive, gpmdm_pf.py:198).
int gpmdm_pf_import(gpmdm_pf_t pf, const double* states, const int64_t* classes, const double* ll,
                    const double* log_w, const double* w, const int64_t* ridx, int64_t frame) {
  CHECK(pf && states && classes && ll && log_w && w, "null argument");
  gpmdm_model* m = pf->m;
  HIPCHK(hipSetDevice(m->device));
  TRY(drop_preswitch(pf, nullptr, true));
  if (pf->switched || pf->dyn_done || pf->propagated) return fail(GPMDM_E_STATE, "import between switch and resample");
  CHECK(frame < (1ll << 32), "frame out of range");
  const long long P = pf->P, Pf = pf->Pf;
  const int F = pf->F;
  std::vector<int> c32(P), r32(P);
  for (long long i = 0; i < P; ++i) {
    CHECK(classes[i] >= 0 && classes[i] < m->C, "class id out of range");
    c32[i] = (int)classes[i];
    if (ridx) CHECK(ridx[i] >= 0 && ridx[i] < Pf, "resample index out of range");
    r32[i] = ridx ? (int)ridx[i] : (int)(i % Pf);
  }
  // max(ll) per filter as k_norm_max takes it (fmax: NaN ignored), and log_w = ll - max
  std::vector<unsigned long long> gm(F);
  for (int f = 0; f < F; ++f) {
    double M = -INFINITY;
    for (long long i = f * Pf; i < (f + 1) * Pf; ++i) M = std::fmax(M, ll[i]);
    for (long long i = f * Pf; i < (f + 1) * Pf; ++i) {
      const double lw = ll[i] - M;
      CHECK(std::memcmp(&lw, &log_w[i], sizeof(double)) == 0 || (std::isnan(lw) && std::isnan(log_w[i])),
            "log_w is not ll - max(ll) of its filter");
    }
    unsigned long long u;
    std::memcpy(&u, &M, sizeof(u));
    gm[f] = (u >> 63) ? ~u : (u | 0x8000000000000000ull);   // ord_enc (common.h)
  }
  const std::vector<double> ones(F, 1.0);
  HIPCHK(hipMemcpy(pf->X, states, sizeof(double) * P * m->d, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(pf->cls, c32.data(), sizeof(int) * P, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(pf->ridx, r32.data(), sizeof(int) * P, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(pf->ll, ll, sizeof(double) * P, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(pf->e, w, sizeof(double) * P, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(pf->total, ones.data(), sizeof(double) * F, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(pf->gmax, gm.data(), sizeof(unsigned long long) * F, hipMemcpyHostToDevice));
  if (pf->cls_pin) {
    std::memcpy(pf->cls_pin, c32.data(), sizeof(int) * P);
    pf->cls_host_ok = true;
    pf->cls_ev_pending = false;
  }
  pf->bmax_ready = false;
  pf->ll_pending = false;
  pf->cnt_check = false;
  if (frame >= 0) pf->frame = (unsigned)frame;
  ResampleArgs ra = resample_args(pf);
  ra.identity = 1;
  ra.cls_src = pf->cls;
  ra.X_src = pf->X;
  launch_resample(ra, nullptr);
  HIPCHK(hipGetLastError());
  // the next frame's shards: the identity order (the exporter's uniforms are not part of the
  // state; the ownership order changes which rank evaluates a particle, never its values)
  pf->own_valid = false;
  pf->rows_st = pf->rows_ll = nullptr;
  HIPCHK(hipEventRecord(pf->ro_ev, nullptr));
  HIPCHK(hipDeviceSynchronize());
  pf->ro_ev_ok = true;
  if (pf->seq_pin) pf->ro_seq = pf->seq_min();   // (synchronised: nothing to wait for)
  pf->initialised = true;
  pf->switched = pf->propagated = pf->dyn_done = pf->gemm_ahead = false;
  return GPMDM_OK;
}

static void launch_dyn_gemm(gpmdm_pf* pf, hipStream_t s);

// Rows from which an AUTO de-duplicated pass runs on the wide image instead of the narrow
// one -- only where the two give bitwise the same results (the 32 x 512 wide image reduces
// each 256-column half in the 16 x 256 order: d <= 12), so the choice, made per rank from
// its last read frame's rows, never changes a result.  GPMDM_DYN_WIDE_ROWS overrides (tests:
// test_gpu_small_path.py forces every de-duplicated pass wide and compares bit for bit).
constexpr int kDynWideRows = 32768;   // ~equal at 25k rows, wide 5% ahead at 100k (profiles/r04/dyn)

static bool dyn_frame_wide(const gpmdm_pf* pf) {
  if (pf->dyn_tiles != GPMDM_DYN_TILES_AUTO || !pf->dedup) return pf->wide_dyn();
  const gpmdm_model* m = pf->m;
  // (the per-half reduction that makes the images bitwise equal exists for d <= 12 only)
  if (m->d > 12 || m->dynw.empty() || !m->dynw[0].split() || m->dyn[0].geo.nw != 4 || m->dyn[0].geo.ntw != 4)
    return false;
  static const char* env = std::getenv("GPMDM_DYN_WIDE_ROWS");
  static const long long thr = env ? std::atoll(env) : kDynWideRows;
  return pf->rows_hint >= thr;
}

// The frame's dynamics launch shape: the image's own (the 16 x 256 image at 32 or 64 rows per
// workgroup lost at every row count measured, profiles/r04/dyn, and was removed).
static TileGeo dyn_frame_geo(const gpmdm_pf* pf) { return pf->m->dyn_set(pf->dyn_wide_frame)[0].geo; }

// counts_ahead (replay pre-switch): the class counts into mapped memory with cnt_done after
// them, and the dynamics-GP tiles launched behind, without waiting.
static int do_switch(gpmdm_pf* pf, const double* E, int64_t* class_counts, hipStream_t s, bool order_ahead = false,
                     bool counts_ahead = false, bool e_uploaded = false) {
  gpmdm_model* m = pf->m;
  const int C = m->C;
  if (pf->rng_mode == GPMDM_RNG_REPLAY && !e_uploaded) {
    CHECK(E, "replay mode needs the Exp(1) switch draws");
    HIPCHK(pf->upload_draws(0, pf->E, E, (size_t)pf->P * C, s));
  }
  hipEvent_t t0;
  pf->mark_begin(s, GPMDM_STAGE_SWITCH, t0);
  // (the owner preset of the leader election is launch_switch_group's)
  // Multi-rank Philox filters switch and group only their own slice (the classes of the
  // other particles arrive with the all-gather); otherwise all P (replay draws are indexed
  // by the global class grouping).
  const bool sl = pf->n_ranks > 1 && pf->rng_mode == GPMDM_RNG_PHILOX;
  const long long base = sl ? pf->lo : 0, nsw = sl ? pf->nloc : pf->P;
  const int nbs = (int)std::max<long long>(cdiv(nsw, 256), 1);
  SwitchArgs sa{};
  sa.P = pf->P;
  sa.base = base;
  sa.n = nsw;
  sa.Pf = pf->Pf;
  sa.F = pf->F;
  sa.C = C;
  sa.frame = pf->frame;
  sa.seed_lo = pf->seed_lo;
  sa.seed_hi = pf->seed_hi;
  sa.cls = pf->cls;
  sa.cls_new = pf->cls_new;
  sa.T = pf->T;
  sa.E = pf->rng_mode == GPMDM_RNG_REPLAY ? pf->rep_src[0] : nullptr;
  sa.blockcounts = pf->blockcounts;
  sa.gmax_reset = nullptr;             // k_dyn_finish resets the maxima (the switch may run ahead)
  if (pf->dedup && pf->nloc > 0) {
    sa.anc = pf->ridx;
    sa.owner = pf->owner;
    sa.lo = pf->lo;
    sa.hi = pf->hi;
  }
  sa.own = pf->own_order();
  pf->dyn_wide_frame = dyn_frame_wide(pf);
  pf->dyn_geo_frame = dyn_frame_geo(pf);
  ScanArgs sc{};
  sc.nb = nbs;
  sc.C = C;
  sc.pt = pf->dyn_geo_frame.pt();      // tile unit of the dynamics pass
  sc.lo = sl ? 0 : pf->lo;
  sc.hi = sl ? pf->nloc : pf->hi;
  sc.own = pf->own_order();
  sc.base = base;
  sc.blockcounts = pf->blockcounts;
  sc.cls_new = pf->cls_new;
  sc.blockoff = pf->blockoff;
  sc.class_start = pf->class_start();
  sc.counts = pf->counts();
  sc.seg_pos_begin = pf->seg_begin();
  sc.seg_pos_end = pf->seg_end();
  sc.seg_out_base = pf->seg_out();
  sc.seg_tile_start = pf->seg_tiles();
  GroupArgs ga{};
  ga.P = pf->P;
  ga.base = base;
  ga.n = nsw;
  ga.C = C;
  ga.cls_new = pf->cls_new;
  ga.class_start = pf->class_start();
  ga.blockoff = pf->blockoff;
  ga.own = pf->own_order();
  ga.perm = pf->perm;
  LeadArgs la{};
  if (pf->dedup && pf->nloc > 0) {
    la.P = pf->P;
    la.Pf = pf->Pf;
    la.lo = pf->lo;
    la.hi = pf->hi;
    la.npos = nsw;
    la.nb = nbs;
    la.C = C;
    la.pt = pf->dyn_geo_frame.pt();
    la.perm = pf->perm;
    la.cls_new = pf->cls_new;
    la.anc = pf->ridx;
    la.owner = pf->owner;
    la.seg_pos_begin = pf->seg_begin();
    la.seg_pos_end = pf->seg_end();
    la.lflag_scan = pf->lflag;
    la.lblock = pf->lblock;
    la.lseg_pos_begin = pf->lseg_begin();
    la.lseg_pos_end = pf->lseg_end();
    la.lseg_out_base = pf->lseg_out();
    la.lseg_tile_start = pf->lseg_tiles();
    la.lperm = pf->lperm;
    la.slot = pf->slot;
    la.owner_reset = pf->owner;        // restores the preset for the next election
  }
  sc.counts_host = (class_counts || counts_ahead) ? pf->cnt_dev : nullptr;   // the counts straight to the host
  if (sc.counts_host && pf->cseq_pin) {
    sc.counts_seq_host = pf->cseq_dev;
    sc.counts_seq = pf->cseq + 1;
  }
  // the counts on the host (cls_pin): no wait for this switch
  // (GPMDM_NO_HOST_COUNTS=1: the device counts and the synchronisation, for A/B tests)
  static const bool no_host_counts = std::getenv("GPMDM_NO_HOST_COUNTS") != nullptr;
  const bool host_counts =
      class_counts && pf->rng_mode == GPMDM_RNG_REPLAY && pf->cls_host_ok && !sl && !no_host_counts;
  if (host_counts) {
    if (pf->cls_ev_pending) {          // the resample that wrote cls_pin (normally done: read)
      // (k_small_resample writes cls_pin before the read-out number it publishes)
      HIPCHK(pf->seq_pin ? pf->wait_readout(pf->ro_seq) : hipEventSynchronize(pf->cls_ev));
      pf->cls_ev_pending = false;
    }
    TRY(check_counts(pf));
    int cnt[kMaxClasses] = {0};
    for (long long p = 0; p < pf->P; ++p) {  // k_switch's argmax, the same fp64 operations
      const double* Tr = pf->T_host.data() + (size_t)pf->cls_pin[p] * C;
      const double* Ep = E + p * C;
      int best = 0;
      double bestv = -INFINITY;
      for (int j = 0; j < C; ++j) {
        const double v = Tr[j] / Ep[j];
        if (v > bestv) { bestv = v; best = j; }
      }
      ++cnt[best];
    }
    for (int c = 0; c < C; ++c) pf->cnt_expect[c] = cnt[c];
  }
  const bool small_path = launch_switch_group(sa, sc, ga, sa.owner ? &la : nullptr, !pf->owner_clean, s);
  // (the one-launch small switch writes the counts without the number: an event then)
  const bool counts_by_seq = sc.counts_seq_host && !small_path;
  if (counts_by_seq) {
    pf->cseq = sc.counts_seq;
    pf->cnt_stream = s;
  }
  if (sa.owner) pf->owner_clean = !small_path;   // the small path presets in-kernel, leaves it dirty
  if (order_ahead) {
    // (pre-switch) the next resample's ownership order: its uniforms are keyed by the
    // frame, so it is known now; timed with the switch
    if (launch_uniform_order(pf->P, pf->frame, pf->seed_lo, pf->seed_hi, pf->own_next, pf->inv_next, pf->own_tmp,
                             pf->own_tmp_bytes, s) != 0)
      return fail(GPMDM_E_HIP, "ownership-order pass failed");
    pf->own_next_frame = (long long)pf->frame;
  }
  pf->mark_end(s, GPMDM_STAGE_SWITCH, t0);
  HIPCHK(hipGetLastError());
  if (pf->rng_mode == GPMDM_RNG_REPLAY) HIPCHK(pf->draws_used(0, s));
  if (counts_ahead) {
    if (!counts_by_seq) HIPCHK(hipEventRecord(pf->cnt_done, s));
    if (pf->nloc > 0) {
      launch_dyn_gemm(pf, s);
      HIPCHK(hipGetLastError());
      pf->gemm_ahead = true;
    }
    pf->pre_counts = true;
    pf->pre_counts_seq = counts_by_seq;
  } else if (host_counts) {
    if (!pf->seq_pin) HIPCHK(hipEventRecord(pf->cnt_ev, s));
    pf->cnt_check = true;
    for (int c = 0; c < C; ++c) class_counts[c] = pf->cnt_expect[c];
  } else if (class_counts) {
    int tmp[kMaxClasses];
    const int* src = pf->cnt_pin;
    if (!sc.counts_host) {
      HIPCHK(hipMemcpyAsync(tmp, pf->counts(), sizeof(int) * C, hipMemcpyDeviceToHost, s));
      src = tmp;
    }
    if (pf->cnt_done && pf->nloc > 0) {
      // the dynamics-GP tiles need the switch's tables, not the normals the caller draws
      // from these counts: they run while it draws (propagate launches the finish only)
      if (!counts_by_seq) HIPCHK(hipEventRecord(pf->cnt_done, s));
      launch_dyn_gemm(pf, s);
      HIPCHK(hipGetLastError());
      pf->gemm_ahead = true;
      HIPCHK(counts_by_seq ? pf->wait_counts() : hipEventSynchronize(pf->cnt_done));
    } else {
      HIPCHK(hipStreamSynchronize(s));
    }
    for (int c = 0; c < C; ++c) class_counts[c] = src[c];
  }
  pf->switched = true;
  return GPMDM_OK;
}

int gpmdm_pf_switch(gpmdm_pf_t pf, const double* E, int64_t* class_counts, void* stream) {
  CHECK(pf, "null handle");
  if (!pf->initialised) return fail(GPMDM_E_STATE, "particle filter not initialised");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipSetDevice(pf->m->device));
  if (pf->preswitched && pf->rng_mode == GPMDM_RNG_REPLAY && E != pf->pre_E)
    TRY(drop_preswitch(pf, s, false));   // other draws than the pre-switch's: switch again
  if (pf->preswitched) {               // launched by the last resample / gpmdm_pf_preswitch: consume it
    if (s != pf->sw_stream) {
      HIPCHK(hipEventRecord(pf->sw_ev, pf->sw_stream));
      HIPCHK(hipStreamWaitEvent(s, pf->sw_ev, 0));
    }
    pf->preswitched = false;
    if (class_counts && pf->pre_counts) {
      // the counts, not the tiles behind them
      HIPCHK(pf->pre_counts_seq ? pf->wait_counts() : hipEventSynchronize(pf->cnt_done));
      for (int c = 0; c < pf->m->C; ++c) class_counts[c] = pf->cnt_pin[c];
    } else if (class_counts) {
      int tmp[kMaxClasses];
      HIPCHK(hipMemcpyAsync(tmp, pf->counts(), sizeof(int) * pf->m->C, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      for (int c = 0; c < pf->m->C; ++c) class_counts[c] = tmp[c];
    }
    pf->pre_counts = false;
    return GPMDM_OK;
  }
  return do_switch(pf, E, class_counts, s);
}

int gpmdm_pf_stage_normals(gpmdm_pf_t pf, const double* normals, int64_t begin, int64_t end, void* stream) {
  CHECK(pf, "null handle");
  if (pf->rng_mode != GPMDM_RNG_REPLAY) return fail(GPMDM_E_STATE, "staged normals are replay draws");
  const long long n = (long long)pf->P * pf->m->d;
  CHECK(normals && begin >= 0 && begin <= end && end <= n, "bad normals range");
  if (begin == end || sizeof(double) * (size_t)n <= gpmdm_pf::kZeroCopyBytes) return GPMDM_OK;   // (small: read in place)
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipSetDevice(pf->m->device));
  const size_t bytes = sizeof(double) * (size_t)(end - begin);
  if (normals != pf->rep_pin[1]) {    // into the staging buffer once its previous readers have run
    HIPCHK(hipEventSynchronize(pf->rep_ev[1]));
    std::memcpy(pf->rep_pin[1] + begin, normals + begin, bytes);
  }
  HIPCHK(pf->make_up_stream());
  // on the side stream, after the device copy's last reader (ndev_ev: the last dynamics
  // finish), so a copy staged between frames runs beside the frame still on `stream`
  HIPCHK(hipStreamWaitEvent(pf->up_stream, pf->ndev_ev, 0));
  HIPCHK(hipMemcpyAsync(pf->normals + begin, pf->rep_pin[1] + begin, bytes, hipMemcpyHostToDevice, pf->up_stream));
  HIPCHK(hipEventRecord(pf->up_ev, pf->up_stream));
  HIPCHK(hipStreamWaitEvent(s, pf->up_ev, 0));
  HIPCHK(pf->draws_used(1, pf->up_stream));   // the staging buffer's reader: the copy
  if (pf->nstage_ptr != normals) {
    pf->nstage_ptr = normals;
    pf->nstaged.clear();
  }
  pf->nstaged.emplace_back((long long)begin, (long long)end);
  std::sort(pf->nstaged.begin(), pf->nstaged.end());
  return GPMDM_OK;
}

int gpmdm_pf_preswitch(gpmdm_pf_t pf, const double* E, void* stream) {
  CHECK(pf, "null handle");
  if (!pf->initialised) return fail(GPMDM_E_STATE, "particle filter not initialised");
  if ((pf->switched && !pf->preswitched) || pf->dyn_done || pf->propagated)
    return fail(GPMDM_E_STATE, "preswitch inside a step");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipSetDevice(pf->m->device));
  if (pf->rng_mode == GPMDM_RNG_PHILOX) {
    if (pf->preswitched) return GPMDM_OK;   // (the resample's)
    TRY(do_switch(pf, nullptr, nullptr, s));
  } else {
    CHECK(E, "replay mode needs the Exp(1) switch draws");
    TRY(drop_preswitch(pf, s, false));   // an earlier pre-switch's draws are replaced
    HIPCHK(pf->make_up_stream());
    // the draws go up beside the frame still running on `stream` (upload_draws first waits
    // for the last switch, the device copy's only reader); the switch waits for them
    HIPCHK(pf->upload_draws(0, pf->E, E, (size_t)pf->P * pf->m->C, pf->up_stream));
    HIPCHK(hipEventRecord(pf->up_ev, pf->up_stream));
    HIPCHK(hipStreamWaitEvent(s, pf->up_ev, 0));
    TRY(do_switch(pf, E, nullptr, s, false, pf->cnt_done != nullptr, true));
    pf->pre_E = E;
  }
  pf->sw_stream = s;
  pf->preswitched = true;
  return GPMDM_OK;
}

// The dynamics-GP tile launches of this rank's rows (per class, segments of at most kMaxSeg
// classes per launch): narrow tiles for the de-duplicated rows, the wide image when every
// particle is evaluated.  They need the switch's tables only, not the normals.
static void launch_dyn_gemm(gpmdm_pf* pf, hipStream_t s) {
  gpmdm_model* m = pf->m;
  const int C = m->C, d = m->d;
  const long long nl = pf->nloc;
  const std::vector<GpImage>& dset = m->dyn_set(pf->dyn_wide_frame);
  hipEvent_t t0;
  pf->mark_begin(s, GPMDM_STAGE_DYN_GEMM, t0);
  for (int c0 = 0; c0 < C; c0 += kMaxSeg) {
    const int ns = std::min(kMaxSeg, C - c0);
    TileParams tp{};
    int njm = 0;
    for (int k = 0; k < ns; ++k) {
      tp.seg[k] = dset[c0 + k].seg();
      njm = std::max(njm, dset[c0 + k].n_j);
    }
    tp.n_seg = ns;
    tp.geo = pf->dyn_geo_frame;      // tile starts computed on the device in units of pt
    // an upper bound (the leaders' tile count is known on the device only): the empty
    // workgroups map last and exit at once (an exact grid read back measured no faster,
    // DESIGN.md §3 "Dynamics tiles")
    tp.tiles_ub = (int)(cdiv(nl, tp.geo.pt()) + ns);
    tp.n_j_max = njm;
    if (pf->dedup) {                  // one row per (ancestor, class) leader
      tp.seg_pos_begin = pf->lseg_begin() + c0;
      tp.seg_pos_end = pf->lseg_end() + c0;
      tp.seg_out_base = pf->lseg_out() + c0;
      tp.seg_tile_start = pf->lseg_tiles() + c0;
      tp.perm = pf->lperm;
    } else {
      tp.seg_pos_begin = pf->seg_begin() + c0;
      tp.seg_pos_end = pf->seg_end() + c0;
      tp.seg_out_base = pf->seg_out() + c0;
      tp.seg_tile_start = pf->seg_tiles() + c0;
      tp.perm = pf->perm;
    }
    tp.X = pf->X;
    fill_tile_common(tp, m, true);
    tp.qpart = pf->qdyn;
    tp.ld_q = nl;
    tp.mu = pf->mudyn;
    tp.ld_mu = d;
    launch_gp_tile(tp, d, true, s);
  }
  pf->mark_end(s, GPMDM_STAGE_DYN_GEMM, t0);
}

// _propogate_dynamics for this rank's particles (gpmdm_pf.py:153-168): the dynamics GP per
// class (de-duplicated rows or every particle) and the new states X_prop.
// zstage: the frame's observation, already in the mapped staging slot zpin[zslot] (the
// one-call propagate): k_dyn_finish copies it to pf->z, and weigh skips its copy launch.
static int propagate_dynamics(gpmdm_pf* pf, const double* normals, hipStream_t s, bool zstage = false) {
  gpmdm_model* m = pf->m;
  const int C = m->C, d = m->d;
  if (pf->rng_mode == GPMDM_RNG_REPLAY) {
    CHECK(normals, "replay mode needs the dynamics normals");
    pf->n_staged_frame = pf->normals_staged(normals, (long long)pf->P * d);
    if (pf->n_staged_frame)
      pf->rep_src[1] = pf->normals;    // every value already copied (gpmdm_pf_stage_normals)
    else
      HIPCHK(pf->upload_draws(1, pf->normals, normals, (size_t)pf->P * d, s));
    pf->nstage_ptr = nullptr;
    pf->nstaged.clear();
  }
  const long long nl = pf->nloc;
  if (nl > 0) {
    const std::vector<GpImage>& dset = m->dyn_set(pf->dyn_wide_frame);
    if (!pf->gemm_ahead) launch_dyn_gemm(pf, s);   // (replay: launched by the switch already)
    pf->gemm_ahead = false;
    hipEvent_t t0;
    pf->mark_begin(s, GPMDM_STAGE_DYN_FINISH, t0);
    DynFinishArgs fa{};
    fa.n_out = nl;
    fa.Pf = pf->Pf;
    fa.n_seg = C;
    fa.d = d;
    fa.frame = pf->frame;
    fa.seed_lo = pf->seed_lo;
    fa.seed_hi = pf->seed_hi;
    fa.seg_out_base = pf->seg_out();
    fa.seg_pos_begin = pf->seg_begin();
    fa.perm = pf->perm;
    for (int c = 0; c < C; ++c) fa.n_parts[c] = dset[c].n_parts();
    fa.qpart = pf->qdyn;
    fa.ld_q = nl;
    fa.mu = pf->mudyn;
    fa.ld_mu = d;
    fa.X = pf->X;
    for (int j = 0; j <= d; ++j) fa.lin_c2[j] = m->x_lin_c2[j];
    for (int j = 0; j < d; ++j) fa.il2[j] = m->x_il2[j];
    fa.normals = pf->rng_mode == GPMDM_RNG_REPLAY ? pf->rep_src[1] : nullptr;
    fa.X_out = pf->X_prop;
    if (pf->dedup) {
      fa.slot = pf->slot;
      fa.anc = pf->ridx;
      fa.P = pf->P;
    }
    fa.health = pf->health;
    fa.gmax_reset = pf->gmax;
    fa.F = pf->F;
    fa.rows_b = pf->dedup ? pf->lseg_begin() : pf->seg_begin();
    fa.rows_e = pf->dedup ? pf->lseg_end() : pf->seg_end();
    fa.n_rows_seg = C;
    fa.rows_out = pf->rows_last();
    fa.rows_host = pf->rows_pdev;
    if (zstage) {
      fa.z_src = pf->zdev[pf->zslot];
      fa.z_dst = pf->z;
      fa.z_n = (long long)m->D * pf->F;
      pf->z_staged = true;
    }
    launch_dyn_finish(fa, s);
    pf->mark_end(s, GPMDM_STAGE_DYN_FINISH, t0);
  } else {
    // no particles on this rank: the maxima reset and row count k_dyn_finish would do
    static const unsigned long long kNegInf[1] = {0x000fffffffffffffull};   // ord_enc(-inf)
    for (int f = 0; f < pf->F; ++f)
      HIPCHK(hipMemcpyAsync(pf->gmax + f, kNegInf, sizeof(kNegInf), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(pf->rows_last(), 0, sizeof(int), s));
  }
  HIPCHK(hipGetLastError());
  if (pf->rng_mode == GPMDM_RNG_REPLAY) {
    // the staging buffer's readers: the side-stream copies when staged (they recorded
    // rep_ev[1] themselves), else the copy / the in-place reads above (one record fewer
    // between the dynamics finish and the observation GP when staged)
    if (!pf->n_staged_frame) HIPCHK(pf->draws_used(1, s));
    if (pf->ndev_ev) HIPCHK(hipEventRecord(pf->ndev_ev, s));
  }
  pf->dyn_done = true;
  pf->switched = false;
  return GPMDM_OK;
}

// _update_weights' likelihoods for this rank's particles (gpmdm_pf.py:170-192): uploads z,
// runs the observation GP tile and the likelihood finish.
static int weigh(gpmdm_pf* pf, const double* zh, hipStream_t s) {
  gpmdm_model* m = pf->m;
  const int d = m->d, D = m->D;
  hipEvent_t t0;
  // z: a small shard's tiles read it in place from the mapped staging slot (no copy launch);
  // otherwise it is copied once (every tile holding mean columns reads it)
  const int zk = pf->zslot;
  const bool zmap = pf->nloc <= 4096 && sizeof(double) * D * pf->F <= 32768;
  const double* zsrc = pf->z;
  if (pf->z_staged) {                  // staged by gpmdm_pf_propagate, copied by k_dyn_finish
    pf->z_staged = false;
    pf->zslot ^= 1;
  } else {
    HIPCHK(pf->zslot_free());
    std::memcpy(pf->zpin[zk], zh, sizeof(double) * D * pf->F);
    if (zmap)
      zsrc = pf->zdev[zk];
    else
      HIPCHK(hipMemcpyAsync(pf->z, pf->zpin[zk], sizeof(double) * D * pf->F, hipMemcpyHostToDevice, s));
    pf->zslot ^= 1;
  }
  const long long nl = pf->nloc;
  if (nl > 0) {
    // ---- observation GP + likelihood over particles [lo, hi) ----
    pf->mark_begin(s, GPMDM_STAGE_OBS_GEMM, t0);
    TileParams tp{};
    const GpImage& oi = *pf->obs_img;
    tp.seg[0] = oi.seg();
    tp.n_seg = 1;
    tp.geo = pf->obs_geo;
    tp.tiles_ub = (int)cdiv(nl, pf->obs_geo.pt());
    tp.n_j_max = oi.n_j;
    tp.seg_pos_begin = pf->obs_tab + 0;
    tp.seg_pos_end = pf->obs_tab + 1;
    tp.seg_out_base = pf->obs_tab + 2;
    tp.seg_tile_start = pf->obs_tab + 3;
    tp.perm = pf->own_order();           // positions [lo, hi) of the ownership order
    tp.X = pf->X_prop;
    fill_tile_common(tp, m, false);
    tp.qpart = pf->qobs;
    tp.ld_q = nl;
    tp.spart = pf->sobs;
    tp.z = zsrc;
    tp.lam2 = m->y_lam2_dev;
    tp.Pf = pf->Pf;
    launch_gp_tile(tp, d, false, s);
    pf->mark_end(s, GPMDM_STAGE_OBS_GEMM, t0);
    pf->mark_begin(s, GPMDM_STAGE_OBS_FINISH, t0);
    ObsFinishArgs oa{};
    oa.n_out = nl;
    oa.n_parts = oi.n_parts();
    oa.D = D;
    oa.qpart = pf->qobs;
    oa.ld_q = nl;
    oa.spart = pf->sobs;
    oa.jm0 = oi.jm0();                   // first part with mean columns
    oa.n_j = oi.n_pblocks();
    oa.sum_log_il2 = m->sum_log_il2;
    oa.z = zsrc;
    oa.Pf = pf->Pf;
    oa.il2 = m->y_il2_dev;
    oa.ll_const = (double)((float)(0.5 * D) * (float)1.8378770351409912);
    oa.ll = pf->ll;
    oa.ll_offset = pf->lo;
    oa.own = pf->own_order();
    oa.health = pf->health;
    pf->ll_pending = false;
    pf->bmax_ready = false;
    if (pf->n_ranks == 1 && !oa.own && oa.ll_offset == 0 && small_resample_ok(norm_args(pf), resample_args(pf))) {
      pf->oa_pending = oa;             // computed by the resampling launch (or flush_ll)
      pf->ll_pending = true;
    } else {
      if (pf->bmax && !oa.own && oa.ll_offset == 0) {   // single filter: the maxima for k_norm_exp_scan
        oa.bmax = pf->bmax;
        pf->bmax_ready = true;
      }
      launch_obs_finish(oa, s);
    }
    pf->mark_end(s, GPMDM_STAGE_OBS_FINISH, t0);
  }
  HIPCHK(hipGetLastError());
  pf->propagated = true;
  pf->dyn_done = false;
  return GPMDM_OK;
}

static int pack_part(gpmdm_pf* pf, double* send, int part, hipStream_t s);
static int unpack_part(gpmdm_pf* pf, const double* recv, int part, hipStream_t s);

static int nccl_fail(ncclResult_t r, const char* what) {
  return fail(GPMDM_E_HIP, std::string(what) + ": " + (rccl().ok ? rccl().GetErrorString(r) : "RCCL missing"));
}

// rows [0, pad) of every rank's send buffer -> recv (even shards) or the staging buffer
// (uneven shards), on cstream: the collective only (inside an ncclGroupStart/End a
// host-driven copy would be enqueued before the grouped collective itself)
static int gather_rows(gpmdm_pf* pf, const double* send, double* recv, double* stage, int width) {
  const size_t cnt = (size_t)pf->pad * width;
  const ncclResult_t r = rccl().AllGather(send, pf->padded ? stage : recv, cnt, ncclDouble, pf->comm, pf->cstream);
  if (r != ncclSuccess) return nccl_fail(r, "ncclAllGather");
  return GPMDM_OK;
}

// uneven shards: each rank k's rows of the staging buffer down to [lo_k, hi_k) of recv
static int gather_copy_down(gpmdm_pf* pf, double* recv, const double* stage, int width) {
  if (!pf->padded) return GPMDM_OK;
  const size_t cnt = (size_t)pf->pad * width;
  for (int k = 0; k < pf->n_ranks; ++k) {
    const long long lo = pf->P * k / pf->n_ranks, hi = pf->P * (k + 1) / pf->n_ranks;
    if (hi > lo)
      HIPCHK(hipMemcpyAsync(recv + lo * width, stage + (size_t)k * cnt, sizeof(double) * (hi - lo) * width,
                            hipMemcpyDeviceToDevice, pf->cstream));
  }
  return GPMDM_OK;
}

// The library's exchange (gpmdm_pf_set_comm) in stages, the schedule of gpmdm_amd/pf.py's
// process-group path: {class, state} all-gathered on the library stream while the
// observation GP runs on the caller's stream, then {ll}; the caller's stream waits for both
// gathers before unpacking (replaces the reference's single-process hand-over to
// normalise / resample, gpmdm_pf.py:194-213).  One rank per process runs them in sequence
// (propagate_exchange); one process driving several devices runs each stage for every
// rank and groups the collectives (gpmdm_pf_propagate_multi).
static int exch_states(gpmdm_pf* pf, const double* normals, hipStream_t s) {
  TRY(propagate_dynamics(pf, normals, s));
  TRY(pack_part(pf, pf->xs_send, GPMDM_PACK_STATES, s));
  HIPCHK(hipEventRecord(pf->cev[0], s));
  HIPCHK(hipStreamWaitEvent(pf->cstream, pf->cev[0], 0));
  return GPMDM_OK;
}
static int exch_ll(gpmdm_pf* pf, const double* zh, hipStream_t s) {
  TRY(weigh(pf, zh, s));
  TRY(pack_part(pf, pf->xl_send, GPMDM_PACK_LL, s));
  HIPCHK(hipEventRecord(pf->cev[1], s));
  HIPCHK(hipStreamWaitEvent(pf->cstream, pf->cev[1], 0));
  return GPMDM_OK;
}
static int exch_finish(gpmdm_pf* pf, hipStream_t s) {
  HIPCHK(hipEventRecord(pf->cev[2], pf->cstream));
  HIPCHK(hipStreamWaitEvent(s, pf->cev[2], 0));
  TRY(unpack_part(pf, pf->xs_recv, GPMDM_PACK_STATES, s));
  TRY(unpack_part(pf, pf->xl_recv, GPMDM_PACK_LL, s));
  return GPMDM_OK;
}

static int propagate_exchange(gpmdm_pf* pf, const double* zh, const double* normals, hipStream_t s) {
  const int d = pf->m->d;
  TRY(exch_states(pf, normals, s));
  TRY(gather_rows(pf, pf->xs_send, pf->xs_recv, pf->xs_stage, d + 1));
  TRY(gather_copy_down(pf, pf->xs_recv, pf->xs_stage, d + 1));
  TRY(exch_ll(pf, zh, s));
  TRY(gather_rows(pf, pf->xl_send, pf->xl_recv, pf->xl_stage, 1));
  TRY(gather_copy_down(pf, pf->xl_recv, pf->xl_stage, 1));
  return exch_finish(pf, s);
}

int gpmdm_pf_propagate(gpmdm_pf_t pf, const double* zh, const double* normals, void* stream) {
  CHECK(pf && zh, "null argument");
  if (!pf->switched || pf->preswitched) return fail(GPMDM_E_STATE, "propagate called before switch");
  if (pf->rng_mode == GPMDM_RNG_REPLAY) CHECK(normals, "replay mode needs the dynamics normals");
  HIPCHK(hipSetDevice(pf->m->device));
  if (pf->comm) return propagate_exchange(pf, zh, normals, (hipStream_t)stream);
  // a large shard's z goes through k_dyn_finish (no copy launch before the observation GP)
  const int D = pf->m->D;
  const bool zstage = pf->nloc > 4096 && pf->nloc >= (long long)D * pf->F;
  if (zstage) {
    HIPCHK(pf->zslot_free());
    std::memcpy(pf->zpin[pf->zslot], zh, sizeof(double) * D * pf->F);
  }
  const int rc = propagate_dynamics(pf, normals, (hipStream_t)stream, zstage);
  if (rc) {
    pf->z_staged = false;
    return rc;
  }
  return weigh(pf, zh, (hipStream_t)stream);
}

// One stage's all-gathers of every rank's filter driven by this thread, grouped (a single
// thread that drives several ranks must group their collectives), then the copy-downs.
static int group_gather(gpmdm_pf* const* pfs, int n, bool states) {
  ncclResult_t e = rccl().GroupStart();
  if (e != ncclSuccess) return nccl_fail(e, "ncclGroupStart");
  int rc = GPMDM_OK;
  for (int i = 0; i < n && rc == GPMDM_OK; ++i) {
    gpmdm_pf* pf = pfs[i];
    rc = states ? gather_rows(pf, pf->xs_send, pf->xs_recv, pf->xs_stage, pf->m->d + 1)
                : gather_rows(pf, pf->xl_send, pf->xl_recv, pf->xl_stage, 1);
  }
  e = rccl().GroupEnd();
  if (rc != GPMDM_OK) return rc;
  if (e != ncclSuccess) return nccl_fail(e, "ncclGroupEnd");
  for (int i = 0; i < n; ++i) {
    gpmdm_pf* pf = pfs[i];
    HIPCHK(hipSetDevice(pf->m->device));
    TRY(states ? gather_copy_down(pf, pf->xs_recv, pf->xs_stage, pf->m->d + 1)
               : gather_copy_down(pf, pf->xl_recv, pf->xl_stage, 1));
  }
  return GPMDM_OK;
}

int gpmdm_pf_propagate_multi(gpmdm_pf_t* pfs, int n, const double* zh, const double* normals,
                             void* const* streams) {
  CHECK(pfs && zh && streams && n >= 1, "null argument");
  RCCL_OR_FAIL();
  for (int i = 0; i < n; ++i) {
    gpmdm_pf* pf = pfs[i];
    CHECK(pf, "null handle");
    CHECK(pf->comm, "gpmdm_pf_propagate_multi needs every filter's communicator (gpmdm_pf_set_comm)");
    CHECK(pf->n_ranks == n && pf->rank == i, "filter i must be rank i of n");
    if (!pf->switched || pf->preswitched) return fail(GPMDM_E_STATE, "propagate called before switch");
    if (pf->rng_mode == GPMDM_RNG_REPLAY) CHECK(normals, "replay mode needs the dynamics normals");
  }
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(pfs[i]->m->device));
    TRY(exch_states(pfs[i], normals, (hipStream_t)streams[i]));
  }
  TRY(group_gather(pfs, n, true));
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(pfs[i]->m->device));
    TRY(exch_ll(pfs[i], zh, (hipStream_t)streams[i]));
  }
  TRY(group_gather(pfs, n, false));
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(pfs[i]->m->device));
    TRY(exch_finish(pfs[i], (hipStream_t)streams[i]));
  }
  return GPMDM_OK;
}

int gpmdm_pf_set_comm(gpmdm_pf_t pf, void* rccl_comm, int flags) {
  CHECK(pf, "null handle");
  CHECK((flags & ~GPMDM_COMM_PAD_ROWS) == 0, "bad flags");
  TRY(drop_preswitch(pf, nullptr, true));
  CHECK(!pf->switched && !pf->propagated, "set_comm between switch and resample");
  HIPCHK(hipSetDevice(pf->m->device));
  pf->release_comm();
  if (!rccl_comm) return GPMDM_OK;
  CHECK(pf->F == 1, "filter banks shard filters, not particles: no communicator");
  RCCL_OR_FAIL();
  ncclComm_t comm = (ncclComm_t)rccl_comm;
  int n = 0, r = 0, dev = -1;
  ncclResult_t e = rccl().CommCount(comm, &n);
  if (e != ncclSuccess) return nccl_fail(e, "ncclCommCount");
  e = rccl().CommUserRank(comm, &r);
  if (e != ncclSuccess) return nccl_fail(e, "ncclCommUserRank");
  e = rccl().CommCuDevice(comm, &dev);
  if (e != ncclSuccess) return nccl_fail(e, "ncclCommCuDevice");
  CHECK(n == pf->n_ranks && r == pf->rank, "communicator size/rank differ from the filter's n_ranks/rank");
  CHECK(dev == pf->m->device, "communicator is on another device than the model");
  const int d = pf->m->d;
  const long long mx = cdiv(pf->P, pf->n_ranks);            // largest shard
  pf->padded = (pf->P % pf->n_ranks) != 0 || (flags & GPMDM_COMM_PAD_ROWS);
  pf->pad = mx + ((flags & GPMDM_COMM_PAD_ROWS) ? 1 : 0);
  const long long rows = pf->pad * pf->n_ranks;
  int rc = 0;
  auto fail_out = [&](int code) { pf->release_comm(); return code; };
  if ((rc = dalloc(&pf->xs_send, (size_t)pf->pad * (d + 1))) || (rc = dalloc(&pf->xl_send, (size_t)pf->pad)) ||
      (rc = dalloc(&pf->xs_recv, (size_t)pf->P * (d + 1))) || (rc = dalloc(&pf->xl_recv, (size_t)pf->P)))
    return fail_out(rc);
  if (pf->padded &&
      ((rc = dalloc(&pf->xs_stage, (size_t)rows * (d + 1))) || (rc = dalloc(&pf->xl_stage, (size_t)rows))))
    return fail_out(rc);
  // padding rows of the send buffers travel but are dropped: keep them defined
  if (hipMemset(pf->xs_send, 0, sizeof(double) * pf->pad * (d + 1)) != hipSuccess ||
      hipMemset(pf->xl_send, 0, sizeof(double) * pf->pad) != hipSuccess ||
      hipStreamCreateWithFlags(&pf->cstream, hipStreamNonBlocking) != hipSuccess)
    return fail_out(fail(GPMDM_E_HIP, "communicator stream / buffers"));
  for (auto& ev : pf->cev)
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
      return fail_out(fail(GPMDM_E_HIP, "communicator events"));
  pf->comm = comm;
  return GPMDM_OK;
}

int gpmdm_comm_unique_id(void* id) {
  CHECK(id, "null argument");
  RCCL_OR_FAIL();
  ncclUniqueId u;
  const ncclResult_t e = rccl().GetUniqueId(&u);
  if (e != ncclSuccess) return nccl_fail(e, "ncclGetUniqueId");
  static_assert(sizeof(ncclUniqueId) == GPMDM_COMM_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id, &u, sizeof(u));
  return GPMDM_OK;
}

int gpmdm_comm_init(int n_ranks, int rank, const void* id, int device, void** comm) {
  CHECK(id && comm && n_ranks >= 1 && rank >= 0 && rank < n_ranks, "bad argument");
  *comm = nullptr;
  RCCL_OR_FAIL();
  HIPCHK(hipSetDevice(device));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  const ncclResult_t e = rccl().CommInitRank(&c, n_ranks, u, rank);
  if (e != ncclSuccess) return nccl_fail(e, "ncclCommInitRank");
  *comm = c;
  return GPMDM_OK;
}

int gpmdm_comm_init_all(int n, const int* devices, void** comms) {
  CHECK(n >= 1 && devices && comms, "bad argument");
  RCCL_OR_FAIL();
  std::vector<ncclComm_t> c((size_t)n, nullptr);
  const ncclResult_t e = rccl().CommInitAll(c.data(), n, devices);
  if (e != ncclSuccess) return nccl_fail(e, "ncclCommInitAll");
  for (int i = 0; i < n; ++i) comms[i] = c[(size_t)i];
  return GPMDM_OK;
}

int gpmdm_comm_destroy(void* comm) {
  if (!comm) return GPMDM_OK;
  RCCL_OR_FAIL();
  const ncclResult_t e = rccl().CommDestroy((ncclComm_t)comm);
  return e == ncclSuccess ? GPMDM_OK : nccl_fail(e, "ncclCommDestroy");
}

int gpmdm_pf_propagate_dynamics(gpmdm_pf_t pf, const double* normals, void* stream) {
  CHECK(pf, "null handle");
  if (!pf->switched || pf->preswitched)
    return fail(GPMDM_E_STATE, "propagate_dynamics called before switch");
  if (pf->rng_mode == GPMDM_RNG_REPLAY) CHECK(normals, "replay mode needs the dynamics normals");
  HIPCHK(hipSetDevice(pf->m->device));
  return propagate_dynamics(pf, normals, (hipStream_t)stream);
}

int gpmdm_pf_weigh(gpmdm_pf_t pf, const double* zh, void* stream) {
  CHECK(pf && zh, "null argument");
  if (!pf->dyn_done) return fail(GPMDM_E_STATE, "weigh called before propagate_dynamics");
  HIPCHK(hipSetDevice(pf->m->device));
  return weigh(pf, zh, (hipStream_t)stream);
}

int gpmdm_pf_exchange_width(gpmdm_pf_t pf, int64_t* width, int64_t* lo, int64_t* hi) {
  CHECK(pf, "null handle");
  if (width) *width = pf->m->d + 2;
  if (lo) *lo = pf->lo;
  if (hi) *hi = pf->hi;
  return GPMDM_OK;
}

int gpmdm_pf_pack(gpmdm_pf_t pf, double* send, void* stream) {
  return gpmdm_pf_pack_part(pf, send, GPMDM_PACK_ALL, stream);
}

int gpmdm_pf_unpack(gpmdm_pf_t pf, const double* recv, void* stream) {
  return gpmdm_pf_unpack_part(pf, recv, GPMDM_PACK_ALL, stream);
}

int gpmdm_pf_pack_part(gpmdm_pf_t pf, double* send, int part, void* stream) {
  CHECK(pf && send, "null argument");
  CHECK(part >= GPMDM_PACK_ALL && part <= GPMDM_PACK_LL, "part must be GPMDM_PACK_*");
  HIPCHK(hipSetDevice(pf->m->device));
  return pack_part(pf, send, part, (hipStream_t)stream);
}

static int pack_part(gpmdm_pf* pf, double* send, int part, hipStream_t s) {
  TRY(flush_ll(pf, s));
  PackArgs a{};
  a.n = pf->nloc;
  a.lo = pf->lo;
  a.d = pf->m->d;
  a.own = pf->own_order();
  a.buf = send;
  a.part = part;
  a.ll = pf->ll;
  a.cls = pf->cls_new;
  a.X = pf->X_prop;
  launch_pack(a, s);
  HIPCHK(hipGetLastError());
  return GPMDM_OK;
}

int gpmdm_pf_unpack_part(gpmdm_pf_t pf, const double* recv, int part, void* stream) {
  CHECK(pf && recv, "null argument");
  CHECK(part >= GPMDM_PACK_ALL && part <= GPMDM_PACK_LL, "part must be GPMDM_PACK_*");
  HIPCHK(hipSetDevice(pf->m->device));
  return unpack_part(pf, recv, part, (hipStream_t)stream);
}

static int launch_unpack_rows(gpmdm_pf* pf, const double* recv, int part, const int* inv, hipStream_t s) {
  PackArgs a{};
  a.n = pf->P;
  a.lo = 0;
  a.d = pf->m->d;
  a.inv = inv;
  a.buf = const_cast<double*>(recv);
  a.part = part;
  a.ll = pf->ll;
  a.cls = pf->cls_new;
  a.X = pf->X_prop;
  launch_unpack(a, s);
  HIPCHK(hipGetLastError());
  return GPMDM_OK;
}

// Exchanged rows are read in place by the next resample (gpmdm_pf.rows_*) when it runs the
// multi-kernel path (the one-workgroup small path reads the unpacked arrays).
static bool rows_in_place(gpmdm_pf* pf) {
  return pf->F == 1 && !small_resample_ok(norm_args(pf), resample_args(pf));
}

static int unpack_part(gpmdm_pf* pf, const double* recv, int part, hipStream_t s) {
  const int* inv = pf->own_valid ? pf->own_inv : nullptr;
  if (!rows_in_place(pf)) return launch_unpack_rows(pf, recv, part, inv, s);
  const int d = pf->m->d;
  const int w = part == GPMDM_PACK_ALL ? d + 2 : (part == GPMDM_PACK_STATES ? d + 1 : 1);
  if (part != GPMDM_PACK_LL) {
    pf->rows_st = recv + (part == GPMDM_PACK_ALL ? 1 : 0);
    pf->rows_st_w = w;
  }
  if (part != GPMDM_PACK_STATES) {
    pf->rows_ll = recv;
    pf->rows_ll_w = w;
  }
  pf->rows_inv = inv;
  return GPMDM_OK;
}

// Write rows held in place out to cls_new / X_prop / ll, for a reader that comes before the
// resample (export).
static int flush_rows(gpmdm_pf* pf, hipStream_t s) {
  const int d = pf->m->d;
  if (pf->rows_st && pf->rows_st_w == d + 2) {            // one {ll, class, state} buffer
    TRY(launch_unpack_rows(pf, pf->rows_st - 1, GPMDM_PACK_ALL, pf->rows_inv, s));
    if (pf->rows_ll == pf->rows_st - 1) pf->rows_ll = nullptr;
  } else if (pf->rows_st) {
    TRY(launch_unpack_rows(pf, pf->rows_st, GPMDM_PACK_STATES, pf->rows_inv, s));
  }
  if (pf->rows_ll) {
    if (pf->rows_ll_w == d + 2)
      TRY(launch_unpack_rows(pf, pf->rows_ll, GPMDM_PACK_ALL, pf->rows_inv, s));
    else
      TRY(launch_unpack_rows(pf, pf->rows_ll, GPMDM_PACK_LL, pf->rows_inv, s));
  }
  pf->rows_st = pf->rows_ll = nullptr;
  return GPMDM_OK;
}

int gpmdm_pf_resample(gpmdm_pf_t pf, const double* uniforms, void* stream) {
  CHECK(pf, "null handle");
  if (!pf->propagated) return fail(GPMDM_E_STATE, "resample called before propagate");
  gpmdm_model* m = pf->m;
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipSetDevice(m->device));
  const bool sys = pf->resample_mode == GPMDM_RESAMPLE_SYSTEMATIC;
  if (pf->rng_mode == GPMDM_RNG_REPLAY) {
    CHECK(uniforms, "replay mode needs the resampling uniforms");
    if (pf->up_stream) {
      // (a filter that pre-switches) beside the observation GP still running on `stream`:
      // host-to-device copies share one engine in submission order, so a copy queued on
      // `stream` behind the GP would hold the next frame's draws (queued on up_stream after
      // it) back until the GP ends.  upload_draws first waits for the last resample.
      HIPCHK(pf->upload_draws(2, pf->U, uniforms, sys ? 1 : (size_t)pf->P, pf->up_stream));
      HIPCHK(hipEventRecord(pf->up_ev, pf->up_stream));
      HIPCHK(hipStreamWaitEvent(s, pf->up_ev, 0));
    } else {
      HIPCHK(pf->upload_draws(2, pf->U, uniforms, sys ? 1 : (size_t)pf->P, s));
    }
  }
  hipEvent_t t0;
  pf->mark_begin(s, GPMDM_STAGE_RESAMPLE, t0);
  ResampleArgs ra = resample_args(pf);
  if (pf->seq_pin) {                   // the read-out's number, published after it
    ra.seq_host = pf->seq_dev;
    ra.seq = ++pf->ro_seq;
    pf->ro_stream = s;
  }
  ra.U = pf->rng_mode == GPMDM_RNG_REPLAY ? pf->rep_src[2] : nullptr;
  NormArgs na = norm_args(pf);
  const bool small = small_resample_ok(na, ra);
  if (small || !pf->bmax_rows) TRY(flush_rows(pf, s));    // (unpack_part holds rows only for this path)
  if (pf->rows_ll) {                   // the exchanged ll column, and its maximum for the normaliser
    RowsLLArgs la{};
    la.P = pf->P;
    la.rows = pf->rows_ll;
    la.w = pf->rows_ll_w;
    la.inv = pf->rows_inv;
    la.ll = pf->ll;
    la.bmax = pf->bmax_rows;
    launch_rows_ll(la, s);
    na.bmax = pf->bmax_rows;
    na.nbmax = rows_ll_blocks(pf->P);
  }
  if (pf->rows_st) {                   // the gathers read the exchanged rows in place
    ra.rows = pf->rows_st;
    ra.rows_w = pf->rows_st_w;
    ra.rows_inv = pf->rows_inv;
  }
  pf->rows_st = pf->rows_ll = nullptr;
  const bool cls_host = pf->cls_pin && small;
  if (cls_host) ra.cls_host = pf->cls_pdev;
  launch_normalise_resample(na, ra, s);
  pf->bmax_ready = false;
  pf->cls_host_ok = cls_host;
  if (cls_host) {
    if (!pf->seq_pin) HIPCHK(hipEventRecord(pf->cls_ev, s));
    pf->cls_ev_pending = true;
  }
  pf->ll_pending = false;
  if (pf->rng_mode == GPMDM_RNG_REPLAY) HIPCHK(pf->draws_used(2, s));
  // next frame's ownership order (identical on every rank: the same draws), after the
  // gathers that read this frame's rows through the current one; systematic uniforms rise
  // with the slot, so the identity order already groups the slots by ancestor
  pf->own_valid = false;
  if (pf->order_wanted()) {
    if (pf->own_next_frame == (long long)pf->frame) {
      // computed behind the last read-out (the kernels above already hold the old pointers)
      std::swap(pf->own, pf->own_next);
      std::swap(pf->own_inv, pf->inv_next);
    } else if (launch_uniform_order(pf->P, pf->frame, pf->seed_lo, pf->seed_hi, pf->own, pf->own_inv, pf->own_tmp,
                                    pf->own_tmp_bytes, s) != 0) {
      return fail(GPMDM_E_HIP, "ownership-order pass failed");
    }
    pf->own_valid = true;
  }
  pf->own_next_frame = -1;
  pf->mark_end(s, GPMDM_STAGE_RESAMPLE, t0);
  HIPCHK(hipGetLastError());
  if (!pf->seq_pin) {                  // (else the read-out kernel publishes its number)
    HIPCHK(hipEventRecord(pf->ro_ev, s));
    pf->ro_ev_ok = true;
  }
  pf->frame += 1;
  pf->propagated = false;
  if (pf->preswitch) {                 // the next frame's switch, behind the read-out
    TRY(do_switch(pf, nullptr, nullptr, s, pf->order_wanted()));
    pf->sw_stream = s;
    pf->preswitched = true;
  }
  return GPMDM_OK;
}

int gpmdm_pf_step(gpmdm_pf_t pf, const double* zh, const double* E, const double* normals,
                  const double* uniforms, void* stream) {
  CHECK(pf, "null handle");
  CHECK(pf->n_ranks == 1 || pf->comm, "gpmdm_pf_step on several ranks needs a communicator (gpmdm_pf_set_comm) "
        "or the staged calls switch/propagate/pack/unpack/resample");
  TRY(gpmdm_pf_switch(pf, E, nullptr, stream));
  TRY(gpmdm_pf_propagate(pf, zh, normals, stream));
  TRY(gpmdm_pf_resample(pf, uniforms, stream));
  return GPMDM_OK;
}

int gpmdm_pf_read(gpmdm_pf_t pf, double* post, double* mean, double* lik, void* stream) {
  CHECK(pf, "null handle");
  if (!pf->initialised) return fail(GPMDM_E_STATE, "particle filter not initialised");
  const gpmdm_model* m = pf->m;
  HIPCHK(hipSetDevice(m->device));
  hipStream_t s = (hipStream_t)stream;
  const int nr = m->C + m->d + 1;
  const double* src = pf->ro_pin;      // written by the read-out kernels themselves
  if (!src) {
    HIPCHK(hipMemcpyAsync(pf->rpin, pf->readout, sizeof(double) * pf->F * nr, hipMemcpyDeviceToHost, s));
    src = pf->rpin;
    HIPCHK(hipStreamSynchronize(s));
  } else if (pf->seq_pin) {
    HIPCHK(pf->wait_readout(pf->ro_seq));     // not the stream: a pre-switch may follow
  } else if (pf->ro_ev_ok) {
    HIPCHK(hipEventSynchronize(pf->ro_ev));   // not the stream: a pre-switch may follow
  } else {
    HIPCHK(hipStreamSynchronize(s));
  }
  pf->rows_hint = __atomic_load_n(pf->rows_pin, __ATOMIC_RELAXED);   // its dynamics pass has run (the read-out follows it)
  for (int f = 0; f < pf->F; ++f) {
    const double* b = src + (size_t)f * nr;
    if (post) std::memcpy(post + (size_t)f * m->C, b, sizeof(double) * m->C);
    if (mean) std::memcpy(mean + (size_t)f * m->d, b + m->C, sizeof(double) * m->d);
    if (lik) lik[f] = b[m->C + m->d];
  }
  return GPMDM_OK;
}

int gpmdm_pf_export(gpmdm_pf_t pf, double* states, int64_t* classes, double* ll, double* log_w,
                    double* w, int64_t* ridx, void* stream) {
  CHECK(pf, "null handle");
  const gpmdm_model* m = pf->m;
  HIPCHK(hipSetDevice(m->device));
  hipStream_t s = (hipStream_t)stream;
  TRY(flush_ll(pf, s));
  TRY(flush_rows(pf, s));
  HIPCHK(hipStreamSynchronize(s));
  const long long P = pf->P;
  if (states) HIPCHK(hipMemcpy(states, pf->X, sizeof(double) * P * m->d, hipMemcpyDeviceToHost));
  std::vector<int> tmp(P);
  if (classes) {
    HIPCHK(hipMemcpy(tmp.data(), pf->cls, sizeof(int) * P, hipMemcpyDeviceToHost));
    for (long long i = 0; i < P; ++i) classes[i] = tmp[i];
  }
  if (ridx) {
    HIPCHK(hipMemcpy(tmp.data(), pf->ridx, sizeof(int) * P, hipMemcpyDeviceToHost));
    for (long long i = 0; i < P; ++i) ridx[i] = tmp[i];
  }
  std::vector<double> l(P);
  HIPCHK(hipMemcpy(l.data(), pf->ll, sizeof(double) * P, hipMemcpyDeviceToHost));
  if (ll) std::memcpy(ll, l.data(), sizeof(double) * P);
  std::vector<unsigned long long> gm(pf->F);
  std::vector<double> S(pf->F);
  HIPCHK(hipMemcpy(gm.data(), pf->gmax, sizeof(unsigned long long) * pf->F, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(S.data(), pf->total, sizeof(double) * pf->F, hipMemcpyDeviceToHost));
  if (w) HIPCHK(hipMemcpy(w, pf->e, sizeof(double) * P, hipMemcpyDeviceToHost));
  for (int f = 0; f < pf->F; ++f) {
    const unsigned long long v = (gm[f] >> 63) ? (gm[f] & 0x7fffffffffffffffull) : ~gm[f];
    double M;
    std::memcpy(&M, &v, sizeof(M));
    for (long long i = f * pf->Pf; i < (f + 1) * pf->Pf; ++i) {
      if (log_w) log_w[i] = l[i] - M;
      if (w) w[i] /= S[f];
    }
  }
  return GPMDM_OK;
}

int gpmdm_pf_set_dedup(gpmdm_pf_t pf, int enable) {
  CHECK(pf, "null handle");
  TRY(drop_preswitch(pf, nullptr, true));
  if (pf->switched || pf->dyn_done) return fail(GPMDM_E_STATE, "set_dedup between switch and propagate");
  pf->dedup = enable != 0;
  return GPMDM_OK;
}

int gpmdm_pf_set_dyn_tiles(gpmdm_pf_t pf, int mode) {
  CHECK(pf, "null handle");
  CHECK(mode == GPMDM_DYN_TILES_AUTO || mode == GPMDM_DYN_TILES_NARROW || mode == GPMDM_DYN_TILES_WIDE,
        "mode must be GPMDM_DYN_TILES_*");
  TRY(drop_preswitch(pf, nullptr, true));
  if (pf->switched || pf->dyn_done) return fail(GPMDM_E_STATE, "set_dyn_tiles between switch and propagate");
  pf->dyn_tiles = mode;
  return GPMDM_OK;
}

int gpmdm_pf_set_shard_order(gpmdm_pf_t pf, int enable) {
  CHECK(pf, "null handle");
  TRY(drop_preswitch(pf, nullptr, true));
  if (pf->switched || pf->dyn_done || pf->propagated) return fail(GPMDM_E_STATE, "set_shard_order inside a step");
  pf->shard_order = enable != 0;
  if (!pf->shard_order) pf->own_valid = false;
  return GPMDM_OK;
}

int gpmdm_pf_dyn_rows(gpmdm_pf_t pf, int64_t* rows, void* stream) {
  CHECK(pf && rows, "null argument");
  HIPCHK(hipSetDevice(pf->m->device));
  hipStream_t s = (hipStream_t)stream;
  int r = 0;                           // k_dyn_finish's count of the last pass's rows
  HIPCHK(hipMemcpyAsync(&r, pf->rows_last(), sizeof(int), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  *rows = r;
  return GPMDM_OK;
}

int gpmdm_pf_enable_timing(gpmdm_pf_t pf, int enable) {
  CHECK(pf, "null handle");
  pf->timing = enable != 0;
  return GPMDM_OK;
}

int gpmdm_pf_timing_stages(gpmdm_pf_t pf, unsigned mask) {
  CHECK(pf, "null handle");
  pf->timing_mask = mask & ((1u << GPMDM_N_STAGES) - 1);
  return GPMDM_OK;
}

int gpmdm_pf_stage_times(gpmdm_pf_t pf, double* ms, int64_t* launches) {
  CHECK(pf, "null handle");
  HIPCHK(hipSetDevice(pf->m->device));
  double acc[GPMDM_N_STAGES] = {0};
  int64_t n[GPMDM_N_STAGES] = {0};
  for (auto& r : pf->recs) {
    HIPCHK(hipEventSynchronize(r.b));
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, r.a, r.b));
    acc[r.stage] += t;
    n[r.stage] += 1;
    pf->pool.push_back(r.a);
    pf->pool.push_back(r.b);
  }
  pf->recs.clear();
  if (ms) std::memcpy(ms, acc, sizeof(acc));
  if (launches) std::memcpy(launches, n, sizeof(n));
  return GPMDM_OK;
}

int gpmdm_pf_frame(gpmdm_pf_t pf, int64_t* frame) {
  CHECK(pf && frame, "null argument");
  *frame = pf->frame;
  return GPMDM_OK;
}

int gpmdm_pf_set_model(gpmdm_pf_t pf, gpmdm_model_t m) {
  CHECK(pf && m, "null argument");
  TRY(drop_preswitch(pf, nullptr, true));
  if (pf->switched || pf->dyn_done || pf->propagated) return fail(GPMDM_E_STATE, "set_model inside a step");
  gpmdm_model* old = pf->m;
  if (m == old) return GPMDM_OK;
  CHECK(m->C == old->C && m->d == old->d && m->D == old->D,
        "the new model's (C, d, D) differ from the filter's");
  CHECK(m->device == old->device, "the new model lives on another device");
  HIPCHK(hipSetDevice(m->device));
  // buffers shaped by the model's column blocks
  const int maxparts = m->dyn_parts_max();
  const long long nl = std::max(pf->nloc, 1ll);
  double *qdyn = nullptr, *qobs = nullptr, *sobs = nullptr;
  int rc = dalloc(&qdyn, (size_t)maxparts * nl);
  if (!rc) rc = dalloc(&qobs, (size_t)obs_parts_max(m) * nl);
  if (!rc) rc = dalloc(&sobs, (size_t)obs_blocks_max(m) * nl);
  TileGeo og{};
  const GpImage* oimg = &obs_pick(m, pf->Pf, pf->nloc, og);
  const int tab[5] = {(int)pf->lo, (int)pf->hi, 0, 0, (int)cdiv(pf->nloc, og.pt())};
  if (!rc && hipMemcpy(pf->obs_tab, tab, sizeof(tab), hipMemcpyHostToDevice) != hipSuccess)
    rc = fail(GPMDM_E_HIP, "upload of the observation tile table");
  if (rc) {
    dfree(qdyn);
    dfree(qobs);
    dfree(sobs);
    return rc;
  }
  HIPCHK(hipDeviceSynchronize());    // launches in flight may still read the old buffers
  dfree(pf->qdyn);
  dfree(pf->qobs);
  dfree(pf->sobs);
  dfree(pf->pred_q);
  pf->pred_q_cap = 0;
  pf->qdyn = qdyn;
  pf->qobs = qobs;
  pf->sobs = sobs;
  pf->nparts_dyn_max = maxparts;
  pf->obs_geo = og;
  pf->obs_img = oimg;
  m->refs.fetch_add(1);
  pf->m = m;
  model_release(old);
  return GPMDM_OK;
}

int gpmdm_pf_health(gpmdm_pf_t pf, int64_t* counts, int reset, void* stream) {
  CHECK(pf, "null handle");
  HIPCHK(hipSetDevice(pf->m->device));
  hipStream_t s = (hipStream_t)stream;
  TRY(flush_ll(pf, s));
  unsigned h[kHealthN];
  HIPCHK(hipMemcpyAsync(h, pf->health, sizeof(h), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (counts)
    for (int k = 0; k < kHealthN; ++k) counts[k] = h[k];
  if (reset) HIPCHK(hipMemsetAsync(pf->health, 0, sizeof(h), s));
  return GPMDM_OK;
}

int gpmdm_pf_predict(gpmdm_pf_t pf, double* mean, void* stream) {
  CHECK(pf && mean, "null argument");
  if (!pf->initialised) return fail(GPMDM_E_STATE, "particle filter not initialised");
  HIPCHK(hipSetDevice(pf->m->device));
  TRY(drop_preswitch(pf, (hipStream_t)stream, false));   // predict rewrites the grouping scratch
  if (pf->switched || pf->dyn_done || pf->propagated) return fail(GPMDM_E_STATE, "predict inside a step");
  gpmdm_model* m = pf->m;
  HIPCHK(hipSetDevice(m->device));
  hipStream_t s = (hipStream_t)stream;
  const int C = m->C, d = m->d;
  const long long P = pf->P;
  const size_t qn = (size_t)pf->nparts_dyn_max * P;
  if (pf->pred_q_cap < qn) {
    dfree(pf->pred_q);
    TRY(dalloc(&pf->pred_q, qn));
    pf->pred_q_cap = qn;
  }
  if (!pf->pred_mu) {
    TRY(dalloc(&pf->pred_mu, (size_t)P * d));
    TRY(dalloc(&pf->pred_mu_p, (size_t)P * d));
    TRY(dalloc(&pf->pred_out, (size_t)pf->F * d));
  }
  // group the current particles by their current class (perm / block tables are the
  // switch's scratch, rebuilt by the next switch; the class tables are predict's own)
  const int tb = gpmdm_pf::kPredictTables;
  const int nbs = (int)cdiv(P, 256);
  launch_class_hist(pf->cls, P, C, pf->blockcounts, s);
  ScanArgs sc{};
  sc.nb = nbs;
  sc.C = C;
  sc.pt = m->dyn_set(true)[0].geo.pt();
  sc.lo = 0;
  sc.hi = P;
  sc.blockcounts = pf->blockcounts;
  sc.cls_new = pf->cls;
  sc.blockoff = pf->blockoff;
  sc.class_start = pf->class_start(tb);
  sc.counts = pf->counts(tb);
  sc.seg_pos_begin = pf->seg_begin(tb);
  sc.seg_pos_end = pf->seg_end(tb);
  sc.seg_out_base = pf->seg_out(tb);
  sc.seg_tile_start = pf->seg_tiles(tb);
  launch_scan_counts(sc, s);
  GroupArgs ga{};
  ga.P = P;
  ga.n = P;
  ga.C = C;
  ga.cls_new = pf->cls;
  ga.class_start = pf->class_start(tb);
  ga.blockoff = pf->blockoff;
  ga.perm = pf->perm;
  launch_group(ga, s);
  // each class's dynamics-GP mean (gpmdm.py:1032-1068), rows in grouped order
  for (int c0 = 0; c0 < C; c0 += kMaxSeg) {
    const int ns = std::min(kMaxSeg, C - c0);
    TileParams tp{};
    int njm = 0;
    for (int k = 0; k < ns; ++k) {
      tp.seg[k] = m->dyn_set(true)[c0 + k].seg();
      njm = std::max(njm, m->dyn_set(true)[c0 + k].n_j);
    }
    tp.n_seg = ns;
    tp.geo = m->dyn_set(true)[c0].geo;
    tp.tiles_ub = (int)(cdiv(P, tp.geo.pt()) + ns);
    tp.n_j_max = njm;
    tp.seg_pos_begin = pf->seg_begin(tb) + c0;
    tp.seg_pos_end = pf->seg_end(tb) + c0;
    tp.seg_out_base = pf->seg_out(tb) + c0;
    tp.seg_tile_start = pf->seg_tiles(tb) + c0;
    tp.perm = pf->perm;
    tp.X = pf->X;
    fill_tile_common(tp, m, true);
    tp.qpart = pf->pred_q;
    tp.ld_q = P;
    tp.mu = pf->pred_mu;
    tp.ld_mu = d;
    launch_gp_tile(tp, d, true, s);
  }
  launch_predict_mean(pf->perm, pf->pred_mu, pf->pred_mu_p, pf->pred_out, P, pf->Pf, pf->F, d, s);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(pf->rpin, pf->pred_out, sizeof(double) * pf->F * d, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  std::memcpy(mean, pf->rpin, sizeof(double) * pf->F * d);
  return GPMDM_OK;
}

}  // extern "C"
