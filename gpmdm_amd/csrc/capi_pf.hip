// C ABI, filter and bank lifecycle: create / destroy, init / import / export of the
// particle state (gpmdm_pf.py:78-115), settings (de-duplication, tile images, shard order,
// model rebind, timing), health counters and predict().  The banks are filters with F > 1
// (gpmdm_bank_create): every entry point here serves both.
#include "capi_internal.h"

namespace gpmdm::capi {

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
  ALLOC(obs_tab, 16);
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
    if (halloc(&pf->zpin[k], (size_t)(F * D), hipHostMallocMapped | hipHostMallocCoherent) != GPMDM_OK ||
        hipEventCreateWithFlags(&pf->zev[k], hipEventDisableTiming) != hipSuccess ||
        hipHostGetDevicePointer(&zv, pf->zpin[k], 0) != hipSuccess) {
      delete pf;
      return fail(GPMDM_E_NOMEM, "pinned observation buffer");
    }
    pf->zdev[k] = (const double*)zv;
  }
  if (halloc(&pf->rpin, (size_t)(F * (C + d + 1)), 0) != GPMDM_OK) {
    delete pf;
    return fail(GPMDM_E_NOMEM, "pinned read-out buffer");
  }
  if (sizeof(double) * F * (C + d + 1) <= 32768) {
    void* rv = nullptr;
    if (halloc(&pf->ro_pin, (size_t)(F * (C + d + 1)), hipHostMallocMapped | hipHostMallocCoherent) != GPMDM_OK ||
        hipHostGetDevicePointer(&rv, pf->ro_pin, 0) != hipSuccess) {
      delete pf;
      return fail(GPMDM_E_NOMEM, "mapped read-out buffer");
    }
    pf->ro_dev = (double*)rv;
    void* sv = nullptr;
    if (halloc(&pf->seq_pin, (size_t)(F), hipHostMallocMapped | hipHostMallocCoherent) != GPMDM_OK ||
        hipHostGetDevicePointer(&sv, pf->seq_pin, 0) != hipSuccess) {
      delete pf;
      return fail(GPMDM_E_NOMEM, "mapped read-out number");
    }
    for (long long f = 0; f < F; ++f) pf->seq_pin[f] = 0;
    pf->seq_dev = (long long*)sv;
  }
  {
    void* rv = nullptr;
    if (halloc(&pf->rows_pin, 1, hipHostMallocMapped | hipHostMallocCoherent) != GPMDM_OK ||
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
      if (halloc(&pf->rep_pin[k], (size_t)(n[k]), fl) != GPMDM_OK ||
          hipEventCreateWithFlags(&pf->rep_ev[k], hipEventDisableTiming) != hipSuccess ||
          hipHostGetDevicePointer(&dv, pf->rep_pin[k], 0) != hipSuccess) {
        delete pf;
        return fail(GPMDM_E_NOMEM, "pinned replay-draw buffer");
      }
      pf->rep_dev[k] = (const double*)dv;
    }
    void* cv = nullptr;
    if (halloc(&pf->cnt_pin, (size_t)(kMaxClasses), fl) != GPMDM_OK ||
        hipHostGetDevicePointer(&cv, pf->cnt_pin, 0) != hipSuccess) {
      delete pf;
      return fail(GPMDM_E_NOMEM, "pinned class-count buffer");
    }
    pf->cnt_dev = (int*)cv;
    void* qv = nullptr;
    if (halloc(&pf->cseq_pin, 1, fl) != GPMDM_OK ||
        hipHostGetDevicePointer(&qv, pf->cseq_pin, 0) != hipSuccess) {
      delete pf;
      return fail(GPMDM_E_NOMEM, "mapped class-count number");
    }
    *pf->cseq_pin = 0;
    pf->cseq_dev = (long long*)qv;
    if (F == 1 && n_ranks == 1 && P <= kHostCountsMaxP) {
      void* lv = nullptr;
      if (halloc(&pf->cls_pin, (size_t)(P), fl) != GPMDM_OK ||
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
  hipStream_t life = life_stream(m->device);   // (the lifecycle stream: no null-stream ordering)
  if (!life || hipMemcpyAsync(pf->obs_tab, tab, sizeof(tab), hipMemcpyHostToDevice, life) != hipSuccess ||
      hipMemcpyAsync(pf->T, T, sizeof(double) * C * C, hipMemcpyHostToDevice, life) != hipSuccess ||
      hipMemsetAsync(pf->health, 0, sizeof(unsigned) * kHealthN, life) != hipSuccess ||
      hipMemsetAsync(pf->small, 0, sizeof(int) * 512, life) != hipSuccess || hipStreamSynchronize(life) != hipSuccess) {
    delete pf;
    return fail(GPMDM_E_HIP, "upload of particle-filter tables failed");
  }
  m->add_user(pf);
  *out = pf;
  return GPMDM_OK;
}

ResampleArgs resample_args(gpmdm_pf* pf) {
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
  ra.local = pf->local;
  ra.blockoff = pf->blockoffw;
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

NormArgs norm_args(gpmdm_pf* pf) {
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
  if (pf->ll_pending) {
    na.obs = pf->oa_pending;
    na.obs_pending = 1;
  }
  if (pf->bmax_ready) na.bmax = pf->bmax;
  return na;
}

int flush_ll(gpmdm_pf* pf, hipStream_t s) {
  if (!pf->ll_pending) return GPMDM_OK;
  launch_obs_finish(pf->oa_pending, s);
  pf->ll_pending = false;
  HIPCHK(hipGetLastError());
  return GPMDM_OK;
}

// Undo a pre-switch before a call that reads or rewrites the switch's tables or needs the
// filter between frames: the caller's stream (or, with none, the host) waits for it, and
// the next gpmdm_pf_switch launches the switch again (same draws: the same tables).
int drop_preswitch(gpmdm_pf* pf, hipStream_t s, bool host_wait) {
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

// Wait for everything this filter has launched, and nothing else (DESIGN.md §1 "Lifecycle
// waits"): its pending pre-switch, its last read-out -- every stage of a frame precedes the
// read-out on the frame's stream, which publishes a sequence number in mapped memory (or
// records ro_ev) -- and its own side streams (replay uploads, the exchange's collectives).
// Calls between frames that launch work (export, health, predict, dyn_rows) wait for it
// themselves.  A filter stopped inside a frame (switched or propagated, not yet resampled)
// has no such marker: then, and only then, the device is synchronised.
int quiesce(gpmdm_pf* pf) {
  HIPCHK(hipSetDevice(pf->m->device));
  TRY(drop_preswitch(pf, nullptr, true));
  if (pf->switched || pf->propagated || pf->dyn_done) {
    HIPCHK(hipDeviceSynchronize());
  } else if (pf->seq_pin && pf->ro_seq.load() > 0) {
    HIPCHK(pf->wait_readout(pf->ro_seq.load()));
  } else if (pf->ro_ev_ok) {
    HIPCHK(hipEventSynchronize(pf->ro_ev));
  }
  if (pf->up_stream) HIPCHK(hipStreamSynchronize(pf->up_stream));
  if (pf->cstream) HIPCHK(hipStreamSynchronize(pf->cstream));
  return GPMDM_OK;
}

}  // namespace gpmdm::capi

extern "C" {

int gpmdm_pf_create(gpmdm_model_t m, const double* T, int64_t P, int rng_mode, uint64_t seed,
                    int resample_mode, int n_ranks, int rank, gpmdm_pf_t* out) {
  return pf_create(m, T, 1, P, rng_mode, seed, resample_mode, n_ranks, rank, out);
}

int gpmdm_bank_create(gpmdm_model_t m, const double* T, int64_t n_filters, int64_t P, uint64_t seed,
                      int resample_mode, gpmdm_pf_t* out) {
  return pf_create(m, T, n_filters, P, GPMDM_RNG_PHILOX, seed, resample_mode, 1, 0, out);
}

int gpmdm_pf_shape(gpmdm_pf_t pf, int64_t* n_filters, int64_t* P) {
  CHECK(pf, "null handle");
  if (n_filters) *n_filters = pf->F;
  if (P) *P = pf->Pf;
  return GPMDM_OK;
}

int gpmdm_pf_destroy(gpmdm_pf_t pf) {
  if (!pf) return GPMDM_OK;
  const int rc = quiesce(pf);   // the filter's own launches only: its buffers are then released
  delete pf;                    // in the lifecycle stream's order (memory.hip)
  return rc;
}

int gpmdm_pf_init(gpmdm_pf_t pf, const double* states, const int64_t* classes) {
  CHECK(pf && states && classes, "null argument");
  gpmdm_model* m = pf->m;
  HIPCHK(hipSetDevice(m->device));
  const long long P = pf->P;
  std::vector<int> c32(P);
  for (long long i = 0; i < P; ++i) {
    CHECK(classes[i] >= 0 && classes[i] < m->C, "class id out of range");
    c32[i] = (int)classes[i];
  }
  TRY(quiesce(pf));                    // the filter's own frames, not the device
  pf->bmax_ready = false;
  // the uploads and the read-out of the initial state on the lifecycle stream (memory.hip)
  hipStream_t ls = life_stream(m->device);
  CHECK(ls, "the library's lifecycle stream");
  std::vector<int> r32(P);
  for (long long i = 0; i < P; ++i) r32[i] = (int)(i % pf->Pf);   // no shared ancestors yet
  const std::vector<unsigned long long> neg(pf->F, 0x000fffffffffffffull);   // ord_enc(-inf)
  HIPCHK(hipMemcpyAsync(pf->X, states, sizeof(double) * P * m->d, hipMemcpyHostToDevice, ls));
  HIPCHK(hipMemcpyAsync(pf->cls, c32.data(), sizeof(int) * P, hipMemcpyHostToDevice, ls));
  HIPCHK(hipMemcpyAsync(pf->ridx, r32.data(), sizeof(int) * P, hipMemcpyHostToDevice, ls));
  HIPCHK(hipMemsetAsync(pf->ll, 0, sizeof(double) * P, ls));
  HIPCHK(hipMemcpyAsync(pf->gmax, neg.data(), sizeof(unsigned long long) * pf->F, hipMemcpyHostToDevice, ls));
  if (pf->cls_pin) {
    std::memcpy(pf->cls_pin, c32.data(), sizeof(int) * P);
    pf->cls_host_ok = true;
    pf->cls_ev_pending = false;
  }
  // read-outs of the initial state: ll = log_w = 0, w = 1/P (gpmdm_pf.py:102-104)
  ResampleArgs ra = resample_args(pf);
  ra.identity = 1;
  ra.cls_src = pf->cls;
  ra.X_src = pf->X;
  launch_normalise_resample(norm_args(pf), ra, ls);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(pf->ro_ev, ls));
  HIPCHK(hipStreamSynchronize(ls));
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
  TRY(quiesce(pf));                    // the filter's own frames, not the device
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
  hipStream_t ls = life_stream(m->device);   // uploads and read-outs on the lifecycle stream
  CHECK(ls, "the library's lifecycle stream");
  HIPCHK(hipMemcpyAsync(pf->X, states, sizeof(double) * P * m->d, hipMemcpyHostToDevice, ls));
  HIPCHK(hipMemcpyAsync(pf->cls, c32.data(), sizeof(int) * P, hipMemcpyHostToDevice, ls));
  HIPCHK(hipMemcpyAsync(pf->ridx, r32.data(), sizeof(int) * P, hipMemcpyHostToDevice, ls));
  HIPCHK(hipMemcpyAsync(pf->ll, ll, sizeof(double) * P, hipMemcpyHostToDevice, ls));
  HIPCHK(hipMemcpyAsync(pf->e, w, sizeof(double) * P, hipMemcpyHostToDevice, ls));
  HIPCHK(hipMemcpyAsync(pf->total, ones.data(), sizeof(double) * F, hipMemcpyHostToDevice, ls));
  HIPCHK(hipMemcpyAsync(pf->gmax, gm.data(), sizeof(unsigned long long) * F, hipMemcpyHostToDevice, ls));
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
  launch_resample(ra, ls);
  HIPCHK(hipGetLastError());
  // the next frame's shards: the identity order (the exporter's uniforms are not part of the
  // state; the ownership order changes which rank evaluates a particle, never its values)
  pf->own_valid = false;
  pf->rows_st = pf->rows_ll = nullptr;
  HIPCHK(hipEventRecord(pf->ro_ev, ls));
  HIPCHK(hipStreamSynchronize(ls));
  pf->ro_ev_ok = true;
  if (pf->seq_pin) pf->ro_seq = pf->seq_min();   // (synchronised: nothing to wait for)
  pf->initialised = true;
  pf->switched = pf->propagated = pf->dyn_done = pf->gemm_ahead = false;
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
  // the copies in the caller's stream order, one wait at the end (not the null stream's)
  const long long P = pf->P;
  std::vector<int> tc(classes ? P : 0), tr(ridx ? P : 0);
  std::vector<double> l(P);
  std::vector<unsigned long long> gm(pf->F);
  std::vector<double> S(pf->F);
  if (states) HIPCHK(hipMemcpyAsync(states, pf->X, sizeof(double) * P * m->d, hipMemcpyDeviceToHost, s));
  if (classes) HIPCHK(hipMemcpyAsync(tc.data(), pf->cls, sizeof(int) * P, hipMemcpyDeviceToHost, s));
  if (ridx) HIPCHK(hipMemcpyAsync(tr.data(), pf->ridx, sizeof(int) * P, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(l.data(), pf->ll, sizeof(double) * P, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(gm.data(), pf->gmax, sizeof(unsigned long long) * pf->F, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(S.data(), pf->total, sizeof(double) * pf->F, hipMemcpyDeviceToHost, s));
  if (w) HIPCHK(hipMemcpyAsync(w, pf->e, sizeof(double) * P, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  for (long long i = 0; i < (classes ? P : 0); ++i) classes[i] = tc[i];
  for (long long i = 0; i < (ridx ? P : 0); ++i) ridx[i] = tr[i];
  if (ll) std::memcpy(ll, l.data(), sizeof(double) * P);
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
  if (rc) {
    dfree(qdyn);
    dfree(qobs);
    dfree(sobs);
    return rc;
  }
  // the filter's own launches in flight may still read the old buffers and obs_tab: wait for
  // them (not for the device), then release the old buffers in the lifecycle stream's order
  TRY(quiesce(pf));
  const int tab[5] = {(int)pf->lo, (int)pf->hi, 0, 0, (int)cdiv(pf->nloc, og.pt())};
  hipStream_t ls = life_stream(m->device);
  if (!ls || hipMemcpyAsync(pf->obs_tab, tab, sizeof(tab), hipMemcpyHostToDevice, ls) != hipSuccess ||
      hipStreamSynchronize(ls) != hipSuccess) {
    dfree(qdyn);
    dfree(qobs);
    dfree(sobs);
    return fail(GPMDM_E_HIP, "upload of the observation tile table");
  }
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
  old->remove_user(pf);
  m->add_user(pf);
  pf->m = m;
  model_release(old);
  return GPMDM_OK;
}

int gpmdm_pf_set_obs_cutoff(gpmdm_pf_t pf, int mode) {
  CHECK(pf, "null handle");
  CHECK(mode >= 0 && mode <= 3, "mode: 0 off, 1 on, 2 on with skip statistics, 3 auto");
  if (pf->dyn_done || pf->propagated) return fail(GPMDM_E_STATE, "set_obs_cutoff between propagate and resample");
  gpmdm_model* m = pf->m;
  HIPCHK(hipSetDevice(m->device));
  if (mode && !m->has_cutoff()) return fail(GPMDM_E_STATE, "the model has no cutoff image (gpmdm_model_set_obs_cutoff)");
  if (mode && !pf->own && pf->rng_mode == GPMDM_RNG_PHILOX && pf->F == 1 && uniform_order_supported(pf->P)) {
    // the ownership order for single-rank filters (order_wanted): resampling-ancestor ranges
    // of particles evaluated together, so the cutoff's particle tiles are compact
    pf->own_tmp_bytes = std::max<size_t>(uniform_order_temp_bytes(pf->P), 1);
    if (dalloc(&pf->own, (size_t)pf->P) || dalloc(&pf->own_inv, (size_t)pf->P) || dalloc(&pf->own_next, (size_t)pf->P) ||
        dalloc(&pf->inv_next, (size_t)pf->P) || dalloc(&pf->own_tmp, pf->own_tmp_bytes)) {
      dfree(pf->own);
      dfree(pf->own_inv);
      dfree(pf->own_next);
      dfree(pf->inv_next);
      dfree(pf->own_tmp);
      return fail(GPMDM_E_NOMEM, "ownership order buffers");
    }
  }
  if (!mode && pf->n_ranks == 1) pf->own_valid = false;   // (the order is the cutoff's only)
  if (mode == 2 && !pf->sp_stats) {
    TRY(dalloc(&pf->sp_stats, 2));
    HIPCHK(hipMemset(pf->sp_stats, 0, 2 * sizeof(unsigned long long)));
  }
  if ((mode == 1 || mode == 3) && !pf->cut_auto_dev) {
    void* hv = nullptr;
    TRY(dalloc(&pf->cut_auto_dev, 2));
    HIPCHK(hipMemset(pf->cut_auto_dev, 0, 2 * sizeof(unsigned long long)));
    TRY(halloc(&pf->cut_auto_host, 2, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer(&hv, pf->cut_auto_host, 0));
    pf->cut_auto_hdev = (unsigned long long*)hv;
  }
  pf->obs_cutoff = mode != 0;
  pf->sp_stats_on = mode == 2;
  pf->cut_auto = mode == 3;
  pf->cut_auto_pending = false;        // (a fresh measurement: the next frame probes)
  pf->cut_auto_frac = -1.0;
  return GPMDM_OK;
}

int gpmdm_pf_obs_cutoff_auto(gpmdm_pf_t pf, int* last_cut, double* fraction) {
  CHECK(pf, "null handle");
  if (pf->cut_auto_pending) {          // the last cutoff frame's counters (as the next frame reads them)
    HIPCHK(pf->wait_readout(pf->cut_auto_seq));
    const unsigned long long run = __atomic_load_n(pf->cut_auto_host + 0, __ATOMIC_ACQUIRE);
    const unsigned long long dense = __atomic_load_n(pf->cut_auto_host + 1, __ATOMIC_ACQUIRE);
    pf->cut_auto_frac = dense ? (double)run / (double)dense : 0.0;
    pf->cut_auto_pending = false;
  }
  if (last_cut) *last_cut = pf->cut_frame ? 1 : 0;
  if (fraction) *fraction = pf->cut_auto_frac;
  return GPMDM_OK;
}

int gpmdm_pf_set_obs_cutoff_split(gpmdm_pf_t pf, int policy) {
  CHECK(pf, "null handle");
  CHECK(policy == GPMDM_CUT_SPLIT_AUTO || policy == GPMDM_CUT_SPLIT_NONE || policy == GPMDM_CUT_SPLIT_ALL ||
            policy == GPMDM_CUT_SPLIT_TAIL || policy == GPMDM_CUT_SPLIT_CHUNKS,
        "policy: GPMDM_CUT_SPLIT_AUTO, _NONE, _ALL, _TAIL or _CHUNKS");
  if (pf->dyn_done || pf->propagated) return fail(GPMDM_E_STATE, "set_obs_cutoff_split between propagate and resample");
  pf->cut_split_policy = policy;
  return GPMDM_OK;
}

int gpmdm_pf_obs_cutoff_stats(gpmdm_pf_t pf, int64_t* run, int64_t* dense, int reset, void* stream) {
  CHECK(pf && run && dense, "null argument");
  *run = *dense = 0;
  if (!pf->sp_stats) return GPMDM_OK;
  HIPCHK(hipSetDevice(pf->m->device));
  hipStream_t s = (hipStream_t)stream;
  unsigned long long h[2];
  HIPCHK(hipMemcpyAsync(h, pf->sp_stats, sizeof(h), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  *run = (int64_t)h[0];
  *dense = (int64_t)h[1];
  if (reset) HIPCHK(hipMemsetAsync(pf->sp_stats, 0, sizeof(h), s));
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
