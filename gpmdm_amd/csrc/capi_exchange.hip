// C ABI, multi-rank exchange: pack / unpack of the {class, state} and {ll}
// rows, the library-driven exchange over an RCCL communicator (gpmdm_pf_set_comm,
// gpmdm_comm_*), the staged calls propagate_dynamics / weigh, and rows read in place by the
// resample (replaces the single-process hand-over of gpmdm_pf.py:194-213).
#include <condition_variable>

#include "capi_internal.h"

namespace gpmdm::capi {

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

static int pack_part(gpmdm_pf* pf, double* send, int part, hipStream_t s);

static int unpack_part(gpmdm_pf* pf, const double* recv, int part, hipStream_t s);

static int nccl_fail(ncclResult_t r, const char* what) {
  return fail(GPMDM_E_HIP, std::string(what) + ": " + (rccl().ok ? rccl().GetErrorString(r) : "RCCL missing"));
}

// ---- In-process loopback transport (gpmdm_comm_init_loopback; tests only) ----------------
// The exchange's collectives with the same call pattern and stream semantics as RCCL's, for
// R ranks held by one process -- also R ranks on ONE device, which RCCL refuses -- so the
// library's multi-rank exchange (uneven shards, staging + copy-down, grouped collectives,
// several streams) runs at R > 1 on a one-GPU box.  An all-gather registers each rank's
// (send, recv, stream) and an event on that stream (its send rows are final there); the last
// rank to arrive enqueues, on every rank's stream, a wait for every rank's event, the R
// device copies into that rank's recv, and an event; then every stream waits for every
// other rank's copies, so no rank's stream runs past the collective before all rows have
// landed everywhere (RCCL's completion semantics).  A rank that arrives earlier returns at
// once inside a group (loop_group_start/end: one thread driving every rank) and otherwise
// blocks on the host until the last rank has enqueued the copies (one thread per rank).
struct LoopGroup {
  int n = 0;
  std::vector<int> dev;
  std::vector<hipEvent_t> ready, done;
  struct Slot {
    const void* send = nullptr;
    void* recv = nullptr;
    hipStream_t s = nullptr;
    bool in = false;
  };
  std::vector<Slot> slot;
  size_t bytes = 0;
  int arrived = 0, refs = 0, err = GPMDM_OK;
  unsigned long long gen = 0;
  std::string why;
  std::mutex mu;
  std::condition_variable cv;
};
struct LoopComm {
  LoopGroup* g;
  int rank;
};

static std::mutex g_loop_mu;
static std::vector<LoopComm*> g_loop_live;   // the live loopback communicators
static thread_local int t_loop_depth = 0;   // loop_group_start nesting on this thread
static thread_local std::vector<std::pair<LoopGroup*, unsigned long long>> t_loop_pending;

static LoopComm* as_loop(void* comm) {
  std::lock_guard<std::mutex> lk(g_loop_mu);
  for (LoopComm* c : g_loop_live)
    if (c == comm) return c;
  return nullptr;
}

// until collective `gen` of g has been enqueued by its last rank (120 s: an error, not a hang)
static int loop_wait(LoopGroup& g, std::unique_lock<std::mutex>& lk, unsigned long long gen) {
  if (!g.cv.wait_for(lk, std::chrono::seconds(120), [&] { return g.gen != gen; }))
    return fail(GPMDM_E_STATE, "loopback all-gather: not every rank joined the collective within 120 s");
  return g.err == GPMDM_OK ? GPMDM_OK : fail(g.err, g.why);
}

// the last rank's half: copies and completion edges on every rank's stream (lock held)
static int loop_run(LoopGroup& g) {
  auto hip = [&](hipError_t e, const char* what) {
    if (e == hipSuccess) return GPMDM_OK;
    g.why = std::string("loopback all-gather: ") + what + ": " + hipGetErrorString(e);
    return GPMDM_E_HIP;
  };
  int rc = GPMDM_OK;
  for (int j = 0; j < g.n && rc == GPMDM_OK; ++j) {
    if ((rc = hip(hipSetDevice(g.dev[(size_t)j]), "hipSetDevice"))) break;
    const LoopGroup::Slot& dj = g.slot[(size_t)j];
    for (int k = 0; k < g.n && rc == GPMDM_OK; ++k)
      rc = hip(hipStreamWaitEvent(dj.s, g.ready[(size_t)k], 0), "hipStreamWaitEvent");
    for (int k = 0; k < g.n && rc == GPMDM_OK && g.bytes; ++k)
      rc = hip(hipMemcpyAsync(static_cast<char*>(dj.recv) + (size_t)k * g.bytes, g.slot[(size_t)k].send, g.bytes,
                              hipMemcpyDefault, dj.s),
               "hipMemcpyAsync");
    if (rc == GPMDM_OK) rc = hip(hipEventRecord(g.done[(size_t)j], dj.s), "hipEventRecord");
  }
  for (int j = 0; j < g.n && rc == GPMDM_OK; ++j) {
    if ((rc = hip(hipSetDevice(g.dev[(size_t)j]), "hipSetDevice"))) break;
    for (int k = 0; k < g.n && rc == GPMDM_OK; ++k)
      if (k != j) rc = hip(hipStreamWaitEvent(g.slot[(size_t)j].s, g.done[(size_t)k], 0), "hipStreamWaitEvent");
  }
  return rc;
}

static int loop_all_gather(LoopComm* c, const void* send, void* recv, size_t bytes, hipStream_t s) {
  LoopGroup& g = *c->g;
  int cur = 0;
  HIPCHK(hipGetDevice(&cur));
  std::unique_lock<std::mutex> lk(g.mu);
  LoopGroup::Slot& me = g.slot[(size_t)c->rank];
  if (me.in) return fail(GPMDM_E_STATE, "loopback all-gather: a rank entered a collective twice");
  if (g.arrived > 0 && bytes != g.bytes) return fail(GPMDM_E_INVALID, "loopback all-gather: ranks differ in size");
  g.bytes = bytes;
  HIPCHK(hipSetDevice(g.dev[(size_t)c->rank]));
  HIPCHK(hipEventRecord(g.ready[(size_t)c->rank], s));
  me = {send, recv, s, true};
  const unsigned long long gen = g.gen;
  if (++g.arrived == g.n) {
    g.err = loop_run(g);
    for (auto& sl : g.slot) sl = LoopGroup::Slot{};
    g.arrived = 0;
    ++g.gen;
    g.cv.notify_all();
    (void)hipSetDevice(cur);
    return g.err == GPMDM_OK ? GPMDM_OK : fail(g.err, g.why);
  }
  (void)hipSetDevice(cur);
  if (t_loop_depth > 0) {
    t_loop_pending.emplace_back(&g, gen);
    return GPMDM_OK;
  }
  return loop_wait(g, lk, gen);
}

static void loop_group_start() { ++t_loop_depth; }

static int loop_group_end() {
  if (t_loop_depth > 0 && --t_loop_depth > 0) return GPMDM_OK;
  std::vector<std::pair<LoopGroup*, unsigned long long>> pend;
  pend.swap(t_loop_pending);
  int rc = GPMDM_OK;
  for (auto& [g, gen] : pend) {
    std::unique_lock<std::mutex> lk(g->mu);
    const int r = loop_wait(*g, lk, gen);
    if (rc == GPMDM_OK) rc = r;
  }
  return rc;
}

static void loop_unref(LoopGroup* g) {
  bool last = false;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    last = --g->refs == 0;
  }
  if (!last) return;
  for (int k = 0; k < g->n; ++k) {
    (void)hipSetDevice(g->dev[(size_t)k]);
    if (g->ready[(size_t)k]) (void)hipEventDestroy(g->ready[(size_t)k]);
    if (g->done[(size_t)k]) (void)hipEventDestroy(g->done[(size_t)k]);
  }
  delete g;
}

// ---- the exchange's collectives, through RCCL or the loopback ------------------------------

// rows [0, pad) of every rank's send buffer -> recv (even shards) or the staging buffer
// (uneven shards), on cstream: the collective only (inside an ncclGroupStart/End a
// host-driven copy would be enqueued before the grouped collective itself)
static int gather_rows(gpmdm_pf* pf, const double* send, double* recv, double* stage, int width) {
  const size_t cnt = (size_t)pf->pad * width;
  if (pf->comm_loop)
    return loop_all_gather(reinterpret_cast<LoopComm*>(pf->comm), send, pf->padded ? stage : recv,
                           sizeof(double) * cnt, pf->cstream);
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

int propagate_exchange(gpmdm_pf* pf, const double* zh, const double* normals, hipStream_t s) {
  const int d = pf->m->d;
  TRY(exch_states(pf, normals, s));
  TRY(gather_rows(pf, pf->xs_send, pf->xs_recv, pf->xs_stage, d + 1));
  TRY(gather_copy_down(pf, pf->xs_recv, pf->xs_stage, d + 1));
  TRY(exch_ll(pf, zh, s));
  TRY(gather_rows(pf, pf->xl_send, pf->xl_recv, pf->xl_stage, 1));
  TRY(gather_copy_down(pf, pf->xl_recv, pf->xl_stage, 1));
  return exch_finish(pf, s);
}

// One stage's all-gathers of every rank's filter driven by this thread, grouped (a single
// thread that drives several ranks must group their collectives), then the copy-downs.
static int group_gather(gpmdm_pf* const* pfs, int n, bool states) {
  const bool loop = pfs[0]->comm_loop;
  ncclResult_t e = ncclSuccess;
  if (loop)
    loop_group_start();
  else if ((e = rccl().GroupStart()) != ncclSuccess)
    return nccl_fail(e, "ncclGroupStart");
  int rc = GPMDM_OK;
  for (int i = 0; i < n && rc == GPMDM_OK; ++i) {
    gpmdm_pf* pf = pfs[i];
    rc = states ? gather_rows(pf, pf->xs_send, pf->xs_recv, pf->xs_stage, pf->m->d + 1)
                : gather_rows(pf, pf->xl_send, pf->xl_recv, pf->xl_stage, 1);
  }
  if (loop) {
    const int r = loop_group_end();
    if (rc == GPMDM_OK) rc = r;
  } else {
    e = rccl().GroupEnd();
  }
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
int flush_rows(gpmdm_pf* pf, hipStream_t s) {
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

}  // namespace gpmdm::capi

extern "C" {

int gpmdm_pf_propagate_multi(gpmdm_pf_t* pfs, int n, const double* zh, const double* normals,
                             void* const* streams) {
  CHECK(pfs && zh && streams && n >= 1, "null argument");
  CHECK(pfs[0], "null handle");
  if (!pfs[0]->comm_loop) RCCL_OR_FAIL();
  for (int i = 0; i < n; ++i) {
    gpmdm_pf* pf = pfs[i];
    CHECK(pf, "null handle");
    CHECK(pf->comm, "gpmdm_pf_propagate_multi needs every filter's communicator (gpmdm_pf_set_comm)");
    CHECK(pf->comm_loop == pfs[0]->comm_loop, "gpmdm_pf_propagate_multi: every filter's communicator of one kind");
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
  ncclComm_t comm = (ncclComm_t)rccl_comm;
  int n = 0, r = 0, dev = -1;
  LoopComm* lc = as_loop(rccl_comm);
  if (lc) {
    n = lc->g->n;
    r = lc->rank;
    dev = lc->g->dev[(size_t)r];
  } else {
    RCCL_OR_FAIL();
    ncclResult_t e = rccl().CommCount(comm, &n);
    if (e != ncclSuccess) return nccl_fail(e, "ncclCommCount");
    e = rccl().CommUserRank(comm, &r);
    if (e != ncclSuccess) return nccl_fail(e, "ncclCommUserRank");
    e = rccl().CommCuDevice(comm, &dev);
    if (e != ncclSuccess) return nccl_fail(e, "ncclCommCuDevice");
  }
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
  pf->comm_loop = lc != nullptr;
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

int gpmdm_comm_init_loopback(int n, const int* devices, void** comms) {
  CHECK(n >= 1 && devices && comms, "bad argument");
  int cur = 0;
  HIPCHK(hipGetDevice(&cur));
  auto* g = new LoopGroup();
  g->n = n;
  g->dev.assign(devices, devices + n);
  g->ready.assign((size_t)n, nullptr);
  g->done.assign((size_t)n, nullptr);
  g->slot.assign((size_t)n, LoopGroup::Slot{});
  g->refs = n;
  for (int k = 0; k < n; ++k) {
    if (hipSetDevice(devices[k]) != hipSuccess ||
        hipEventCreateWithFlags(&g->ready[(size_t)k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g->done[(size_t)k], hipEventDisableTiming) != hipSuccess) {
      g->refs = 1;
      loop_unref(g);
      (void)hipSetDevice(cur);
      return fail(GPMDM_E_HIP, "loopback communicator: device / events");
    }
  }
  (void)hipSetDevice(cur);
  std::lock_guard<std::mutex> lk(g_loop_mu);
  for (int k = 0; k < n; ++k) {
    auto* c = new LoopComm{g, k};
    g_loop_live.push_back(c);
    comms[k] = c;
  }
  return GPMDM_OK;
}

int gpmdm_comm_destroy(void* comm) {
  if (!comm) return GPMDM_OK;
  if (LoopComm* lc = as_loop(comm)) {
    {
      std::lock_guard<std::mutex> lk(g_loop_mu);
      g_loop_live.erase(std::find(g_loop_live.begin(), g_loop_live.end(), lc));
    }
    loop_unref(lc->g);
    delete lc;
    return GPMDM_OK;
  }
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

int gpmdm_pf_unpack_part(gpmdm_pf_t pf, const double* recv, int part, void* stream) {
  CHECK(pf && recv, "null argument");
  CHECK(part >= GPMDM_PACK_ALL && part <= GPMDM_PACK_LL, "part must be GPMDM_PACK_*");
  HIPCHK(hipSetDevice(pf->m->device));
  return unpack_part(pf, recv, part, (hipStream_t)stream);
}

}  // extern "C"
