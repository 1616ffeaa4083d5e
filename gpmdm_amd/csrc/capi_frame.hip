// C ABI, the per-frame launch sequence (gpmdm_pf.py:117-262): Markov switch, dynamics GP,
// observation GP + likelihood, normalise / resample / read-outs, and the host read of the
// published read-outs.
#include "capi_internal.h"

namespace gpmdm::capi {

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
int do_switch(gpmdm_pf* pf, const double* E, int64_t* class_counts, hipStream_t s, bool order_ahead,                      bool counts_ahead, bool e_uploaded) {
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
int propagate_dynamics(gpmdm_pf* pf, const double* normals, hipStream_t s, bool zstage) {
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
// Particle tiles of the cutoff launch that run as two workgroups each
// (gpmdm_pf_set_obs_cutoff_split).  AUTO, from the measured policies (DESIGN.md §3 "The grid's
// tail"): every tile when the launch is at most two rounds of the resident slots or its last
// round is at most an eighth full (and the partials fit in max_all_bytes), none at whole
// rounds, otherwise the last round's tiles.
static int cut_split_tiles(const gpmdm_pf* pf, int tiles, int slots, size_t all_bytes) {
  constexpr size_t kMaxAllBytes = size_t(2) << 30;
  const int rem = slots > 0 ? tiles % slots : 0;
  switch (pf->cut_split_policy) {
    case GPMDM_CUT_SPLIT_NONE: return 0;
    case GPMDM_CUT_SPLIT_ALL: return tiles;
    case GPMDM_CUT_SPLIT_TAIL: return slots <= 0 || tiles <= slots ? tiles : rem;
    default: break;
  }
  if (slots <= 0) return 0;
  const bool all_fits = all_bytes <= kMaxAllBytes;
  if (tiles <= 2 * slots) return all_fits ? tiles : std::min(tiles, rem ? rem : tiles);
  if (rem == 0) return 0;
  if (rem <= slots / 8 && all_fits) return tiles;
  return rem;
}

int weigh(gpmdm_pf* pf, const double* zh, hipStream_t s) {
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
    // the opt-in kernel-value cutoff: its own kernel over the cutoff image (obs_cutoff.h),
    // one q and one S partial per particle
    bool cut = pf->obs_cutoff && m->has_cutoff();
    // AUTO (gpmdm_pf::cut_auto): the cutoff while the reach it last measured is below the
    // break-even, a cutoff frame at least every kCutAutoProbe frames to measure it again
    // (mode 1 measures its reach the same way, for the split policy's chunk grid)
    bool auto_frame = false;
    if (cut && pf->cut_measure_active() && !small_resample_ok(norm_args(pf), resample_args(pf))) {
      if (pf->cut_auto_pending) {      // the last cutoff frame's counters, published with its read-out
        HIPCHK(pf->wait_readout(pf->cut_auto_seq));
        const unsigned long long run = __atomic_load_n(pf->cut_auto_host + 0, __ATOMIC_ACQUIRE);
        const unsigned long long dense = __atomic_load_n(pf->cut_auto_host + 1, __ATOMIC_ACQUIRE);
        pf->cut_auto_frac = dense ? (double)run / (double)dense : 0.0;
        pf->cut_auto_pending = false;
      }
      if (pf->cut_auto) {
        const bool probe = pf->cut_auto_frac < 0.0 || (long long)pf->frame - pf->cut_auto_probe >= gpmdm_pf::kCutAutoProbe;
        cut = probe || pf->cut_auto_frac <= gpmdm_pf::kCutAutoMaxRun;
        if (cut) pf->cut_auto_probe = pf->frame;
      }
      auto_frame = cut;
    }
    pf->cut_frame = cut;
    pf->cut_frame_auto = auto_frame;
    const GpImage& oi = *pf->obs_img;
    // Particle order of the tiles: positions [lo, hi) of the ownership order -- or, for a
    // cutoff filter whose switch grouped exactly this rank's particles (one rank, or a
    // multi-rank Philox filter: its slice at grouped positions [0, nloc)), the switch's class
    // grouping (stable within a class in the ownership order, i.e. by resampling ancestor): a
    // tile then holds particles propagated from one (ancestor, class) mean where it can, so
    // its bounding sphere -- and the K-steps it reaches -- are small.  Any order gives the
    // same values (the flush is per value).
    const bool grouped = cut && (pf->n_ranks == 1 || pf->rng_mode == GPMDM_RNG_PHILOX);
    const int* obs_order = grouped ? pf->perm : pf->own_order();
    const long long obs_lo = grouped ? 0 : pf->lo;   // first position of this rank's particles
    bool cut_tail = false;
    long long cut_o0 = 0, cut_ld = 0;
    if (cut) {
      const auto& ci = m->obs_cut;
      CutoffParams cp{};
      cp.X = pf->X_prop;
      cp.perm = obs_order;
      cp.pos_begin = (int)obs_lo;
      cp.pos_end = (int)(obs_lo + nl);
      for (int j = 0; j < d; ++j) cp.ls[j] = m->y_ls[j];
      cp.Xrec = ci.Xrec;
      cp.Bt = ci.Bt;
      cp.toff = ci.toff;
      cp.ksph = ci.sph;
      cp.n_rows = ci.n_rows;
      cp.n_m = ci.n_m;
      cp.T_R = ci.T_R;
      cp.T_M = ci.T_M;
      cp.cut2 = m->cut2;
      cp.t_cut = m->t_cut;
      cp.q = pf->qobs;
      cp.S = pf->sobs;
      cp.z = zsrc;
      cp.lam2 = m->y_lam2_dev;
      cp.Pf = pf->Pf;
      cp.sp_stats = auto_frame ? pf->cut_auto_dev : (pf->sp_stats_on ? pf->sp_stats : nullptr);
      // the grid's tail: equal workgroups run in whole rounds of the resident slots, so the
      // tiles past the last full round are split in two workgroups each (chunks [0, c*) and
      // [c*, nc); bitwise the whole tile's sums, k_obs_ll chains the second part on).  Below
      // one round every tile is split.
      const int PT = cutoff_tile_particles(d), TPC = cutoff_tile_list_chunk();
      const int tiles = (int)cdiv(nl, PT);
      const int slots = cutoff_slots(d);
      // list entries a second part can hold (all but the first chunk's, at least one)
      const long long entries = (long long)ci.T_R + ci.T_M - 1;
      // the chunk grid by request, or under AUTO when the filter's last measured reach is high
      // (every tile's list then spans several chunks: measured 4-7 % faster at reaches 0.68-0.91,
      // 2 % slower at 0.07-0.23, where most chunk workgroups find no chunk)
      const bool grid = (pf->cut_split_policy == GPMDM_CUT_SPLIT_CHUNKS ||
                         (pf->cut_split_policy == GPMDM_CUT_SPLIT_AUTO && pf->cut_auto_frac >= gpmdm_pf::kCutChunksMin)) &&
                        ci.T_R + ci.T_M > TPC;
      int n_split = grid ? tiles : cut_split_tiles(pf, tiles, slots, (size_t)entries * tiles * PT * sizeof(double));
      if (ci.T_R + ci.T_M <= TPC) n_split = 0;   // one chunk: nothing to split
      if (n_split > 0) TRY(pf->ensure_cut_split((size_t)entries * n_split * PT, n_split, s));
      cp.n_whole = tiles - n_split;
      cp.n_split = n_split;
      cp.chunk_grid = grid ? 1 : 0;
      cp.n_chunk_max = (int)cdiv(ci.T_R + ci.T_M, TPC);
      cp.part = pf->cut_part;
      cp.ld_part = (long long)n_split * PT;
      cp.split = pf->cut_split;
      if (!launch_obs_cutoff(cp, d, s)) return fail(GPMDM_E_INVALID, "cutoff launch shape");
      cut_tail = n_split > 0;
      cut_o0 = (long long)cp.n_whole * PT;
      cut_ld = cp.ld_part;
    } else {
      TileParams tp{};
      const int* tab = pf->obs_tab;
      tp.seg[0] = oi.seg();
      tp.n_seg = 1;
      tp.geo = pf->obs_geo;
      tp.tiles_ub = (int)cdiv(nl, tp.geo.pt());
      tp.n_j_max = oi.n_j;
      tp.seg_pos_begin = tab + 0;
      tp.seg_pos_end = tab + 1;
      tp.seg_out_base = tab + 2;
      tp.seg_tile_start = tab + 3;
      tp.perm = obs_order;
      tp.X = pf->X_prop;
      fill_tile_common(tp, m, false);
      tp.qpart = pf->qobs;
      tp.ld_q = nl;
      tp.spart = pf->sobs;
      tp.z = zsrc;
      tp.lam2 = m->y_lam2_dev;
      tp.Pf = pf->Pf;
      launch_gp_tile(tp, d, false, s);
    }
    pf->mark_end(s, GPMDM_STAGE_OBS_GEMM, t0);
    pf->mark_begin(s, GPMDM_STAGE_OBS_FINISH, t0);
    ObsFinishArgs oa{};
    oa.n_out = nl;
    oa.n_parts = cut ? 1 : oi.n_parts();
    oa.D = D;
    oa.qpart = pf->qobs;
    oa.ld_q = nl;
    oa.spart = pf->sobs;
    oa.jm0 = cut ? 0 : oi.jm0();         // first part with mean columns
    oa.n_j = cut ? 1 : oi.n_pblocks();
    oa.sum_log_il2 = m->sum_log_il2;
    oa.z = zsrc;
    oa.Pf = pf->Pf;
    oa.il2 = m->y_il2_dev;
    oa.ll_const = (double)((float)(0.5 * D) * (float)1.8378770351409912);
    oa.ll = pf->ll;
    oa.ll_offset = obs_lo;
    oa.own = obs_order;
    if (cut_tail) {
      oa.cut_part = pf->cut_part;
      oa.cut_ld = cut_ld;
      oa.cut_split = pf->cut_split;
      oa.cut_o0 = cut_o0;
      oa.cut_pt = cutoff_tile_particles(d);
      oa.cut_tpc = cutoff_tile_list_chunk();
      oa.cut_tm = m->obs_cut.T_M;
    }
    oa.health = pf->health;
    pf->ll_pending = false;
    pf->bmax_ready = false;
    if (pf->n_ranks == 1 && !oa.own && oa.ll_offset == 0 && small_resample_ok(norm_args(pf), resample_args(pf))) {
      pf->oa_pending = oa;             // computed by the resampling launch (or flush_ll)
      pf->ll_pending = true;
    } else {
      // single filter (one rank): the maxima for k_norm_exp_scan, in any particle order (the
      // maximum over the blocks' maxima does not depend on which particles a block holds)
      if (pf->bmax && oa.ll_offset == 0) {
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

}  // namespace gpmdm::capi

extern "C" {

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
  const bool auto_stats = pf->cut_frame_auto && !small && pf->seq_pin;
  if (auto_stats) {                    // this frame's cutoff counters travel with the read-out
    ra.cut_stats = pf->cut_auto_dev;
    ra.cut_stats_host = pf->cut_auto_hdev;
  }
  pf->cut_frame_auto = false;
  launch_normalise_resample(na, ra, s);
  if (auto_stats) {
    pf->cut_auto_pending = true;
    pf->cut_auto_seq = ra.seq;
  }
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

}  // extern "C"
