// C ABI, models: gpmdm_model_create / destroy (device images of the observation GP and the
// per-class dynamics GPs, host_image.h) and the predictive maps gpmdm_predict_obs / dyn
// (map_x_to_y, gpmdm.py:923-963; map_x_dynamics_for_class, gpmdm.py:1032-1068); the
// thread-local last error.
#include "capi_internal.h"

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

namespace gpmdm::capi {

// host -> device on the current device's lifecycle stream (memory.hip): not ordered behind the
// legacy null stream's users
int h2d(void* dst, const void* src, size_t bytes) {
  hipStream_t ls = life_stream_current();
  CHECK(ls, "the library's lifecycle stream");
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ls));
  HIPCHK(hipStreamSynchronize(ls));
  return GPMDM_OK;
}

template <typename T>
int upload(T** dst, const std::vector<T>& v) {
  TRY(dalloc(dst, v.size()));
  return h2d(*dst, v.data(), v.size() * sizeof(T));
}

// Wait for the last frame of every filter built on the model (not for the device): the
// caller guarantees none of them is inside a frame or stepping on another thread.
int quiesce_users(gpmdm_model* m) {
  std::vector<gpmdm_pf*> us;
  {
    std::lock_guard<std::mutex> lk(m->life_mu);
    us = m->users;
  }
  for (gpmdm_pf* pf : us) TRY(quiesce(pf));
  HIPCHK(hipSetDevice(m->device));
  return GPMDM_OK;
}

int build_image(GpImage& g, int n_rows, int d, int n_m, const double* X, const double* ls,
                const double* lin_c2, const double* R, const double* M, TileGeo geo) {
  ImagePacker pk(n_rows, d, n_m, X, ls, lin_c2, R, M, geo);
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
    TRY(h2d(g.Bf + off, buf.data(), buf.size() * sizeof(double)));
    off += (long long)buf.size();
  }
  return GPMDM_OK;
}

// The host half of a cutoff image, whichever side packs it: tau (host_image.h
// obs_cutoff_tau, from M = K^-1 Y and the data's scale), the spatial order of the training
// rows, the K-step spheres, the row records in that order and the tile offsets.
int cutoff_plan(gpmdm_model* m, double sigma2, const double* M, const double* y_absmax, CutoffPlan& pl) {
  CHECK(sigma2 > 0.0 && std::isfinite(sigma2), "sigma2 must be positive (the observation noise variance)");
  CHECK(ksteps((int)m->N) <= kMaxCutoffKs, "the cutoff image holds at most 65536 training rows");
  CHECK(m->d <= 16, "the cutoff image is built for latent dimensions d <= 16");
  const int N = (int)m->N, d = m->d;
  pl.tau = obs_cutoff_tau(N, sigma2, M, m->D, y_absmax);
  CHECK(pl.tau > 0.0 && std::isfinite(pl.tau), "no usable cutoff for this model");
  pl.perm = spatial_order(m->X.data(), m->y_ls.data(), N, d);
  CutoffPacker pk(N, d, m->D, m->X.data(), m->y_ls.data(), nullptr, nullptr, pl.perm.data());
  pl.toff = pk.offsets();
  pl.T_R = pk.T_R;
  pl.T_M = pk.T_M;
  // the kernel addresses the image with 32-bit byte offsets (one buffer resource)
  CHECK(pl.toff.back() * 8 < (1LL << 32), "the cutoff image exceeds 4 GiB (about 32k training rows)");
  kstep_spheres(m->X.data(), m->y_ls.data(), pl.perm.data(), N, d, pl.sph);
  pk.records(pl.rec);
  return GPMDM_OK;
}

// Replace the model's cutoff image: wait for the filters built on it (their own last frames),
// release the old image, upload the plan's tables and let `fill` write the image Bt (device,
// toff.back() doubles; toff_dev: the tile offsets on the device).
int cutoff_install(gpmdm_model* m, const CutoffPlan& pl, const std::function<int(double*, const long long*)>& fill) {
  TRY(quiesce_users(m));              // the filters' own launches may still read the old image
  m->release_cutoff();
  auto& ci = m->obs_cut;
  int rc = upload(&ci.sph, pl.sph);
  if (!rc) rc = upload(&ci.Xrec, pl.rec);
  if (!rc) rc = upload(&ci.toff, pl.toff);
  if (!rc) rc = dalloc(&ci.Bt, (size_t)pl.toff.back());
  if (!rc) rc = fill(ci.Bt, ci.toff);
  if (rc) {
    m->release_cutoff();
    return rc;
  }
  ci.n_rows = (int)m->N;
  ci.n_m = m->D;
  ci.T_R = pl.T_R;
  ci.T_M = pl.T_M;
  m->cut_tau = pl.tau;
  m->cut2 = -std::log(pl.tau) * (1.0 + 1e-12) + 1e-6;   // margin over both tests' rounding
  m->t_cut = std::log(pl.tau) * kLog2eX64;
  return GPMDM_OK;
}

const GpImage& obs_pick(const gpmdm_model* m, long long P, long long n, TileGeo& geo) {
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

// ------------------------------------------------------------------------------------
void fill_tile_common(TileParams& tp, const gpmdm_model* m, bool dyn) {
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

}  // namespace gpmdm::capi

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
  if (h2d(m->y_il2_dev, m->y_il2.data(), m->D * sizeof(double)) != GPMDM_OK) {
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
    if (h2d(m->y_lam2_dev, lam2.data(), m->D * sizeof(double)) != GPMDM_OK) {
      delete m;
      return fail(GPMDM_E_HIP, "upload lambda^2");
    }
  }
  *out = m;
  return GPMDM_OK;
}

// The observation GP's opt-in kernel-value cutoff (DESIGN.md §3 "Kernel-value cutoff"):
// the K^-1 image in the symmetric block form over a spatial order of the training rows,
// tile-major (host_image.h CutoffPacker), the per-K-step bounding spheres and tau.
// K_inv = NULL removes it.  (gpmdm_model_build_obs_cutoff, cutoff_image.hip, builds the same
// image on the device from the model's own factor.)
int gpmdm_model_set_obs_cutoff(gpmdm_model_t m, const double* K_inv, const double* beta, double sigma2,
                               const double* y_absmax) {
  CHECK(m, "null model");
  HIPCHK(hipSetDevice(m->device));
  if (!K_inv) {
    TRY(quiesce_users(m));            // the filters' own launches may still read the image
    m->release_cutoff();
    return GPMDM_OK;
  }
  CHECK(beta && y_absmax, "null argument");
  CutoffPlan pl;
  TRY(cutoff_plan(m, sigma2, beta, y_absmax, pl));
  const int N = (int)m->N;
  CutoffPacker pk(N, m->d, m->D, m->X.data(), m->y_ls.data(), K_inv, beta, pl.perm.data());
  // packed and uploaded a group of tiles at a time (the host never holds the whole image)
  return cutoff_install(m, pl, [&](double* Bt, const long long*) -> int {
    const std::vector<long long>& toff = pl.toff;
    std::vector<double> buf;
    for (int t0 = 0; t0 < pk.tiles();) {
      int t1 = t0 + 1;
      while (t1 < pk.tiles() && toff[(size_t)t1 + 1] - toff[(size_t)t0] <= (1LL << 22)) ++t1;
      buf.assign((size_t)(toff[(size_t)t1] - toff[(size_t)t0]), 0.0);
      for (int t = t0; t < t1; ++t) pk.pack_tile(t, buf.data() + (toff[(size_t)t] - toff[(size_t)t0]));
      if (h2d(Bt + toff[(size_t)t0], buf.data(), buf.size() * sizeof(double)) != GPMDM_OK)
        return fail(GPMDM_E_HIP, "upload of the cutoff image");
      t0 = t1;
    }
    return GPMDM_OK;
  });
}

int gpmdm_model_obs_cutoff_image(gpmdm_model_t m, int64_t* n, double* out) {
  CHECK(m && n, "null argument");
  HIPCHK(hipSetDevice(m->device));
  if (!m->has_cutoff()) {
    *n = 0;
    return GPMDM_OK;
  }
  long long cnt = 0;
  HIPCHK(hipMemcpy(&cnt, m->obs_cut.toff + (m->obs_cut.T_R + m->obs_cut.T_M), sizeof(long long), hipMemcpyDeviceToHost));
  *n = cnt;
  if (out) HIPCHK(hipMemcpy(out, m->obs_cut.Bt, sizeof(double) * cnt, hipMemcpyDeviceToHost));
  return GPMDM_OK;
}

int gpmdm_model_obs_cutoff(gpmdm_model_t m, double* tau) {
  CHECK(m && tau, "null argument");
  *tau = m->has_cutoff() ? m->cut_tau : 0.0;
  return GPMDM_OK;
}

int gpmdm_model_destroy(gpmdm_model_t m) {
  model_release(m);   // freed once the last filter built on it is gone
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
  TRY(finish_scratch(q, s));
  HIPCHK(m->note_use(s));   // the model's release is ordered after this map (lifecycle waits)
  return GPMDM_OK;
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
  TRY(finish_scratch(q, s));
  HIPCHK(m->note_use(s));   // the model's release is ordered after this map (lifecycle waits)
  return GPMDM_OK;
}

}  // extern "C"
