// C ABI, multi-rank exchange: pack / unpack of the {class, state} and {ll}
// rows, the library-driven exchange over an RCCL communicator (gpmdm_pf_set_comm,
// gpmdm_comm_*), the staged calls propagate_dynamics / weigh, and rows read in place by the
// resample (replaces the single-process hand-over of gpmdm_pf.py:194-213).
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

int gpmdm_pf_unpack_part(gpmdm_pf_t pf, const double* recv, int part, void* stream) {
  CHECK(pf && recv, "null argument");
  CHECK(part >= GPMDM_PACK_ALL && part <= GPMDM_PACK_LL, "part must be GPMDM_PACK_*");
  HIPCHK(hipSetDevice(pf->m->device));
  return unpack_part(pf, recv, part, (hipStream_t)stream);
}

}  // extern "C"
