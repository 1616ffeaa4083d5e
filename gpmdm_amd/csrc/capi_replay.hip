// C ABI, replay-draw staging: the pinned draw buffers (gpmdm_pf_draw_buffers / draws_free),
// normals staged ahead of the propagate (gpmdm_pf_stage_normals) and the pre-switch
// (gpmdm_pf_preswitch) -- the host side of drawing torch's streams in the reference's order
// (gpmdm_pf.py:137-213) without stalling the device.
#include "capi_internal.h"

namespace gpmdm::capi {

}  // namespace gpmdm::capi

extern "C" {

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

}  // extern "C"
