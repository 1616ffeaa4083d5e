/*
 * gpmdm_hip.h -- C ABI of libgpmdm_hip.so, the MI355X (gfx950) engine for the GPMDM
 * particle-filter inference step.
 *
 * The reference (Priyanshu4/gpmdm) is pure Python: its "boundary" is the class API of
 * gpmdm/gpmdm_pf.py (GPMDM_PF) and the two predictive maps of gpmdm/gpmdm.py it calls.
 * There is no FFI in the reference; each entry point below names the reference call it
 * replaces (file:line under /root/reference).  The Python mirror of the reference API
 * (gpmdm_amd.GPMDM / gpmdm_amd.GPMDM_PF) binds these through ctypes; INTEGRATION.md
 * shows the binding.
 *
 * Conventions
 *   - every function returns int: 0 = ok, < 0 = error (see GPMDM_E_*); the message of
 *     the last error on the calling thread is gpmdm_last_error();
 *   - all floating point is IEEE fp64, row-major, contiguous; class ids are int64 at the
 *     boundary (int32 on the device);
 *   - "host" pointers are ordinary CPU memory; "device" pointers are HIP device memory
 *     owned by the caller (e.g. torch tensors' data_ptr());
 *   - host input arrays are read before the call returns (the library stages them in its
 *     own pinned buffers), so the caller may reuse or free them at once; host output
 *     arrays are complete when the call returns (the call synchronises the stream);
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream).  A handle keeps
 *     no stream of its own: launches go to the stream given to each call;
 *   - a handle is not thread-safe; distinct handles are independent.
 */
#ifndef GPMDM_HIP_H
#define GPMDM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPMDM_OK 0
#define GPMDM_E_INVALID (-1)   /* bad argument / shape (reference raises ValueError) */
#define GPMDM_E_HIP (-2)       /* HIP runtime failure */
#define GPMDM_E_NOMEM (-3)     /* device allocation failed */
#define GPMDM_E_STATE (-4)     /* call out of order (e.g. step before init) */

#define GPMDM_RNG_REPLAY 0     /* draws supplied by the caller (torch-order replay) */
#define GPMDM_RNG_PHILOX 1     /* draws generated on the device (Philox4x32-10) */

#define GPMDM_RESAMPLE_MULTINOMIAL 0  /* torch.multinomial(w, P, True): inverse CDF (reference) */
#define GPMDM_RESAMPLE_SYSTEMATIC 1   /* systematic resampling: one uniform per step, slot s takes
                                         the first i with cum_i >= (s + u0) / P; computed by a
                                         scan over the slots (run starts + max-scan), no search */

typedef struct gpmdm_model* gpmdm_model_t;
typedef struct gpmdm_pf* gpmdm_pf_t;

/*
 * Model descriptor: everything the per-frame path reads, precomputed on the host the
 * way gpmdm.py:1284-1305 (_precompute_kernel_inverses) does, restricted to class blocks.
 * The library copies every array to the device; the caller may free them on return.
 *
 *   obs_R      N x N   upper-triangular U_y^-1 with K_y = U_y^T U_y, so K_y^-1 = R R^T
 *                      (gpmdm.py:1286-1289)
 *   obs_beta   N x D   K_y^-1 Y  (the mean weights of map_x_to_y, gpmdm.py:957)
 *   dyn_R[c]   Nc x Nc upper-triangular U_c^-1 of the class-c block of K_x (gpmdm.py:1299-1305)
 *   dyn_alpha[c] Nc x d  A_c Xout_c  (mean weights of map_x_dynamics_for_class, gpmdm.py:1064)
 */
/* GP-tile workgroup shapes (particles x columns of K* B per workgroup).  The default runs
 * the observation GP as 32x512 (d <= 12) or 64x512 (d > 12) and the dynamics GPs as
 * 16x256; an explicit 64x256 or 64x512 applies to both. */
enum {
  GPMDM_TILE_DEFAULT = 0,
  GPMDM_TILE_64x256 = 1,
  GPMDM_TILE_64x512 = 2,
  GPMDM_TILE_32x512 = 3
};

typedef struct gpmdm_model_desc {
  int64_t N;                     /* training latents (rows of X, Y) */
  int32_t D;                     /* observation dimension */
  int32_t d;                     /* latent dimension (<= 32) */
  int32_t C;                     /* classes */
  int32_t tile_shape;            /* GPMDM_TILE_*: GP-tile workgroup shape (0 = default) */
  const double* X;               /* N x d latents (particle initialisation is host-side) */
  const double* obs_R;           /* N x N */
  const double* obs_beta;        /* N x D */
  const double* y_lengthscales;  /* d  : exp(y_log_lengthscales) */
  const double* y_inv_lambda2;   /* D  : exp(y_log_lambdas)^-2 */
  const int64_t* Nc;             /* C  : dynamics rows per class */
  const double* const* Xin;      /* C pointers, Nc x d : dynamics inputs of class c */
  const double* const* dyn_R;    /* C pointers, Nc x Nc */
  const double* const* dyn_alpha;/* C pointers, Nc x d */
  const double* x_lengthscales;  /* d   : exp(x_log_lengthscales) */
  const double* x_lin_coeff2;    /* d+1 : exp(x_log_lin_coeff)^2 (bias last) */
  const double* x_inv_lambda2;   /* d   : exp(x_log_lambdas)^-2 */
} gpmdm_model_desc;

/* Upload a model (replaces the device-side state GPMDM holds after GPMDM.load /
 * init_X + _precompute_kernel_inverses, gpmdm.py:762-777, 1349-1414). */
int gpmdm_model_create(const gpmdm_model_desc* desc, int device, gpmdm_model_t* out);
int gpmdm_model_destroy(gpmdm_model_t model);

/* GPMDM.map_x_to_y(Xstar, flg_noise=False)  (gpmdm.py:923-963).
 * Xs_dev: n x d; mu_dev, var_dev: n x D (device, caller-owned). */
int gpmdm_predict_obs(gpmdm_model_t model, const double* Xs_dev, int64_t n,
                      double* mu_dev, double* var_dev, void* stream);

/* GPMDM.map_x_dynamics_for_class(Xstar, c, flg_noise=False)  (gpmdm.py:1032-1068).
 * Xs_dev: n x d; mu_dev, var_dev: n x d (device, caller-owned). */
int gpmdm_predict_dyn(gpmdm_model_t model, int c, const double* Xs_dev, int64_t n,
                      double* mu_dev, double* var_dev, void* stream);

/* GPMDM_PF(gpmdm, markov_switching_model, num_particles)  (gpmdm_pf.py:47-85).
 * T: C x C host.  Ranks own the contiguous particle range
 * [rank*P/n_ranks, (rank+1)*P/n_ranks); particle state is replicated on every rank.
 * The per-frame exchange is done either by the library over an RCCL communicator
 * (gpmdm_pf_set_comm; then gpmdm_pf_propagate / gpmdm_pf_step exchange by themselves) or
 * by the caller with the staged calls (gpmdm_pf_pack / gpmdm_pf_unpack). */
int gpmdm_pf_create(gpmdm_model_t model, const double* T, int64_t P, int rng_mode,
                    uint64_t seed, int resample_mode, int n_ranks, int rank,
                    gpmdm_pf_t* out);
int gpmdm_pf_destroy(gpmdm_pf_t pf);

/* Filter bank: n_filters independent filters of P particles each sharing one model (the
 * 39 trials test_gpmdm_pf.ipynb runs one after another).  Device
 * (philox) draws, one rank.  Filter f draws exactly what a single filter created with
 * seed + f draws, so its results are bit-identical to that filter's.  The handle works
 * with every gpmdm_pf_* call below, with per-filter arrays stacked filter-major:
 * states/classes (F*P) in init/export, z (F x D) in propagate, F x C / F x d / F in read.
 * gpmdm_pf_shape reports (F, P) of any handle (F = 1 for gpmdm_pf_create). */
int gpmdm_bank_create(gpmdm_model_t model, const double* T, int64_t n_filters, int64_t P,
                      uint64_t seed, int resample_mode, gpmdm_pf_t* out);
int gpmdm_pf_shape(gpmdm_pf_t pf, int64_t* n_filters, int64_t* P);

/* _init_particles / reset()  (gpmdm_pf.py:87-115, 264-265): states P x d, classes P
 * (host).  Clears weights to 1/P and log-likelihoods to 0 as the reference does. */
int gpmdm_pf_init(gpmdm_pf_t pf, const double* states, const int64_t* classes);

/* Restore a filter state exported by gpmdm_pf_export (checkpoint / resume):
 * the reference filter's state _particle_states, _particle_classes, _log_likelihoods,
 * _log_weights, _weights (gpmdm_pf.py:78-82, 100-104), all host.  states P x d, classes P,
 * ll P, log_w P, w P (all required); ridx P (the last resample's ancestor indices within each
 * filter, or NULL: none shared); frame >= 0 sets the Philox frame counter (< 0 keeps it).
 * log_w must be ll - max(ll) per filter, computed as gpmdm_pf_export computes it (exact
 * comparison; GPMDM_E_INVALID otherwise).  The read-outs right after the import equal the
 * exporter's (posterior, mean, likelihood sum, bit for bit), and a filter of the same
 * configuration and seed continues the exporter's trajectory bit for bit.  A replay
 * filter's draws come from the caller's generator: saving its state is the caller's part.
 * Drops a pending pre-switch; not between switch and resample. */
int gpmdm_pf_import(gpmdm_pf_t pf, const double* states, const int64_t* classes, const double* ll,
                    const double* log_w, const double* w, const int64_t* ridx, int64_t frame);

/* Replay filters: the library's own pinned staging buffers of the three draw streams
 * (exp draws P x C, normals P x d, uniforms P), so a host can draw straight into them.
 * Passing these very pointers to gpmdm_pf_switch / gpmdm_pf_propagate / gpmdm_pf_resample
 * skips the copy into staging.  A buffer may be written only when gpmdm_pf_draws_free
 * (which = 0, 1, 2) has returned: it waits until the launches that read the buffer's last
 * contents have run (a pending replay pre-switch included).  It may be called from another
 * thread than the one stepping the filter (a host drawing ahead) when the buffer is copied
 * to the device (a buffer of more than 32 KB); for smaller, in-place buffers call it
 * from the stepping thread (it reads the pre-switch's bookkeeping). */
int gpmdm_pf_draw_buffers(gpmdm_pf_t pf, double** exp_draws, double** normals, double** uniforms);
int gpmdm_pf_draws_free(gpmdm_pf_t pf, int which);

/* _propogate_markov_switching  (gpmdm_pf.py:137-151).  exp_draws: P x C host (replay)
 * or NULL (philox).  class_counts: C host, or NULL; when given, the post-switch class
 * counts are returned (the replay caller needs them to draw the per-class normals of the
 * next stage): a single replay filter of <= 1024 particles counts them on the host from
 * exp_draws and the classes its last resample left in mapped memory (no stream wait; the
 * device's counts are checked at the next switch), others copy them back synchronously.
 * Philox filters: gpmdm_pf_resample already launched the next frame's switch behind its
 * read-out (its draws need no host input), and this call then only consumes it (the
 * caller's stream waits on it if it is another stream); the call order is still required.
 * A replay filter consumes a pending gpmdm_pf_preswitch when exp_draws is the pointer the
 * pre-switch was given (its counts come from mapped memory once the switch kernels are
 * done, not after the dynamics tiles behind them); another pointer drops it and switches. */
int gpmdm_pf_switch(gpmdm_pf_t pf, const double* exp_draws, int64_t* class_counts,
                    void* stream);

/* The next frame's switch launched now, between frames -- behind the last read-out, while
 * the host is still busy -- instead of in gpmdm_pf_switch.  Replay filters: exp_draws is the
 * next frame's P x C Exp(1) draws (a host draws them ahead: they depend on no device
 * result); the switch, its class counts (into mapped memory) and the dynamics-GP tiles are
 * launched on `stream`, and the next gpmdm_pf_switch with the same exp_draws pointer
 * consumes them.  The caller promises that the array's contents do not change in between;
 * if they do (its generator moved), it calls gpmdm_pf_preswitch again, which drops the
 * earlier pre-switch.  Philox filters: what gpmdm_pf_resample already does (no-op if
 * pending).  Any call that drops a pre-switch (import, predict, set_*) drops this one: the
 * next gpmdm_pf_switch then switches from scratch.  Not inside a step. */
int gpmdm_pf_preswitch(gpmdm_pf_t pf, const double* exp_draws, void* stream);

/* Replay filters: copy values [begin, end) of the next propagate's normals ((sum_c P_c) x d,
 * flattened) to the device now, on `stream` (the propagate must run on the same stream).
 * The next gpmdm_pf_propagate(_dynamics) handed the same `normals` pointer copies nothing if
 * the ranges staged since the last propagate cover every value, else all of them.  A host
 * that knows part of the normals early (the first class's, drawn ahead) stages that part
 * behind the read-out and the rest once drawn; values changed after staging must be staged
 * again.  Small filters (<= 32 KB of normals, read in place) ignore it. */
int gpmdm_pf_stage_normals(gpmdm_pf_t pf, const double* normals, int64_t begin, int64_t end, void* stream);

/* _propogate_dynamics + _update_weights' likelihoods for this rank's particles
 * (gpmdm_pf.py:153-192).  z: D host.  normals: (sum_c P_c) x d host in the reference's
 * per-class order (replay) or NULL (philox).  A single-shard filter of <= 1024 particles
 * per filter leaves the last step of the likelihoods (the per-particle finish) to the
 * next gpmdm_pf_resample launch; gpmdm_pf_export, gpmdm_pf_pack(_part) and
 * gpmdm_pf_health run it first if it is still pending, so every reader sees the same ll.
 * The host arrays (draws, z) are copied before the call returns; small ones are read by
 * the kernels from the library's mapped pinned buffers instead of a copy launch. */
int gpmdm_pf_propagate(gpmdm_pf_t pf, const double* z, const double* normals, void* stream);

/* gpmdm_pf_propagate in two halves, so a multi-rank caller can exchange the new states
 * while the observation GP runs: propagate_dynamics = _propogate_dynamics
 * (gpmdm_pf.py:153-168; normals as for gpmdm_pf_propagate), weigh = _update_weights'
 * likelihoods (gpmdm_pf.py:170-192).  switch -> propagate_dynamics -> weigh -> resample. */
int gpmdm_pf_propagate_dynamics(gpmdm_pf_t pf, const double* normals, void* stream);
int gpmdm_pf_weigh(gpmdm_pf_t pf, const double* z, void* stream);

/* Multi-rank exchange: pack this rank's rows [lo, hi) as (hi-lo) x (d+2) doubles
 * {ll, class, state[d]}; unpack all P rows after an all-gather.  The _part forms move
 * column subsets: GPMDM_PACK_STATES = {class, state[d]} (d+1 wide; valid after
 * propagate_dynamics), GPMDM_PACK_LL = {ll} (1 wide; valid after weigh).
 * Unpacking hands the gathered rows to the filter, which reads them in place during the
 * next gpmdm_pf_resample (its gathers touch only the resampled ancestors' rows; the ll
 * column is read once, with the normaliser's maximum): recv_dev must stay allocated and
 * unmodified until that resample's kernels have run -- stream order on the resample's stream
 * suffices (the next frame's all-gather into the same buffer, enqueued after it, is safe). */
enum { GPMDM_PACK_ALL = 0, GPMDM_PACK_STATES = 1, GPMDM_PACK_LL = 2 };
int gpmdm_pf_exchange_width(gpmdm_pf_t pf, int64_t* width, int64_t* lo, int64_t* hi);
int gpmdm_pf_pack(gpmdm_pf_t pf, double* send_dev, void* stream);
int gpmdm_pf_unpack(gpmdm_pf_t pf, const double* recv_dev, void* stream);
int gpmdm_pf_pack_part(gpmdm_pf_t pf, double* send_dev, int part, void* stream);
int gpmdm_pf_unpack_part(gpmdm_pf_t pf, const double* recv_dev, int part, void* stream);

/* Library-driven exchange over RCCL (SURVEY.md §8(b)'s rccl_comm; it replaces the
 * reference's single-process hand-over from _update_weights to _resample,
 * gpmdm_pf.py:194-213).  rccl_comm: an ncclComm_t of n_ranks ranks in which this process is
 * `rank`, on the model's device (from gpmdm_comm_init or the caller's own
 * ncclCommInitRank); the caller keeps ownership and destroys it after the filter.  While
 * set, gpmdm_pf_propagate (and gpmdm_pf_step) all-gather every rank's new {class, state}
 * rows on a library-owned stream while the observation GP runs on the caller's stream, then
 * the {ll} column; the caller's stream waits for both gathers (events, no host wait) and
 * every rank holds the full replicated filter before gpmdm_pf_resample.  NULL detaches.
 * Also valid with n_ranks = 1 (the exchange then moves this rank's rows only).
 * flags: 0, or GPMDM_COMM_PAD_ROWS -- gather one padding row per rank more than needed,
 * through the uneven-shard path (staging buffer + copy-down; diagnostics and tests).
 * Not between switch and resample; not for filter banks (they shard filters). */
#define GPMDM_COMM_PAD_ROWS 1
#define GPMDM_COMM_ID_BYTES 128   /* sizeof(ncclUniqueId) */
int gpmdm_pf_set_comm(gpmdm_pf_t pf, void* rccl_comm, int flags);

/* RCCL communicator helpers for native hosts that do not link RCCL themselves: rank 0
 * creates a unique id (GPMDM_COMM_ID_BYTES bytes) and hands it to every rank out of band;
 * each rank calls gpmdm_comm_init on its device (ncclCommInitRank: collective over the
 * ranks); gpmdm_comm_destroy after the filters using it are destroyed. */
int gpmdm_comm_unique_id(void* id);
int gpmdm_comm_init(int n_ranks, int rank, const void* id, int device, void** comm);
int gpmdm_comm_destroy(void* comm);

/* One process driving several devices (GPMDM_PF(devices=[...])): gpmdm_comm_init_all makes
 * the n communicators of devices[0..n-1] at once (ncclCommInitAll), comms[i] for rank i.
 * gpmdm_pf_propagate_multi is gpmdm_pf_propagate for the n filters pfs[i] (rank i of n,
 * each with comms[i] set by gpmdm_pf_set_comm, each switched) on streams[i]: every stage
 * runs for every rank and each stage's all-gathers are grouped (ncclGroupStart/End), as a
 * single thread that drives several ranks must.  z and the replay normals are the same
 * host arrays for every rank (the filter is replicated).  RCCL is resolved at run time
 * (librccl.so.1) by these and the calls above; GPMDM_E_HIP when it is missing. */
int gpmdm_comm_init_all(int n, const int* devices, void** comms);

/* TEST ONLY: n in-process loopback communicators, comms[i] = rank i of n on devices[i]
 * (devices may repeat: R ranks on one GPU, which RCCL refuses).  They stand in for RCCL
 * communicators everywhere above (gpmdm_pf_set_comm, gpmdm_pf_propagate_multi,
 * gpmdm_comm_destroy): each all-gather is R x R stream-ordered device copies made when the
 * last rank joins, with RCCL's completion semantics (no rank's stream passes the collective
 * before every rank's rows have landed).  Ranks joined by one thread inside
 * gpmdm_pf_propagate_multi are grouped; ranks on threads of their own block on the host in
 * each collective until all have joined (an error after 120 s).  Not a transport for
 * production: every byte goes through this process's device copies. */
int gpmdm_comm_init_loopback(int n, const int* devices, void** comms);
int gpmdm_pf_propagate_multi(gpmdm_pf_t* pfs, int n, const double* z, const double* normals,
                             void* const* streams);

/* _update_weights' normalisation + _resample + the read-outs  (gpmdm_pf.py:194-262,
 * 302-312).  uniforms: P host (replay, multinomial), 1 host (replay, systematic) or NULL.
 * Philox filters then launch the next frame's switch on the same stream (see
 * gpmdm_pf_switch); gpmdm_pf_predict, gpmdm_pf_init and the gpmdm_pf_set_* calls drop it,
 * and the next gpmdm_pf_switch launches it again (the same draws, the same result).  The
 * stream must stay valid until that next switch or drop (a call that waits for the
 * pre-switch from another stream or the host records its event on this stream then). */
int gpmdm_pf_resample(gpmdm_pf_t pf, const double* uniforms, void* stream);

/* update(z) in one call  (gpmdm_pf.py:117-135): switch + propagate + resample.
 * One rank, or several with a communicator (gpmdm_pf_set_comm); replay draws must all be
 * given (use the staged calls when the per-class normal counts are not known in advance). */
int gpmdm_pf_step(gpmdm_pf_t pf, const double* z, const double* exp_draws,
                  const double* normals, const double* uniforms, void* stream);

/* class_probabilities() / current_state_mean() / log_likelihood()
 * (gpmdm_pf.py:224-262, 215-222).  Waits for the last read-out -- the read-out kernels write
 * it to mapped host memory and then publish a sequence number there, which this call waits
 * on (GPMDM_RO_EVENT=1: an event recorded after the read-out), so not for a pre-launched
 * switch behind it -- or synchronises `stream` when the read-outs need a copy (banks of more
 * than ~800 filters); any pointer may be NULL. */
int gpmdm_pf_read(gpmdm_pf_t pf, double* posterior, double* mean, double* lik, void* stream);

/* Export the full particle state to host (any pointer may be NULL): states P x d,
 * classes P, ll P, log_w P, w P, resample indices P (of the last resample). */
int gpmdm_pf_export(gpmdm_pf_t pf, double* states, int64_t* classes, double* ll,
                    double* log_w, double* w, int64_t* resample_idx, void* stream);

/* Per-stage device time (HIP events on the launch stream).  enable=1 starts recording,
 * 0 stops.  gpmdm_pf_stage_times synchronises and returns, per stage, the summed
 * milliseconds and the number of launches since the last call (then resets). */
#define GPMDM_STAGE_SWITCH 0
#define GPMDM_STAGE_DYN_GEMM 1
#define GPMDM_STAGE_DYN_FINISH 2
#define GPMDM_STAGE_OBS_GEMM 3
#define GPMDM_STAGE_OBS_FINISH 4
#define GPMDM_STAGE_RESAMPLE 5
#define GPMDM_N_STAGES 6
int gpmdm_pf_enable_timing(gpmdm_pf_t pf, int enable);
/* Which stages record events while timing is on: bit (1 << GPMDM_STAGE_*) per stage,
 * default all.  Each recorded stage adds two event records to the stream. */
int gpmdm_pf_timing_stages(gpmdm_pf_t pf, unsigned mask);
int gpmdm_pf_stage_times(gpmdm_pf_t pf, double* ms, int64_t* launches);

/* Ancestor de-duplication of the dynamics GP (default on).  After a resample, offspring of
 * one ancestor carry bit-identical states; the dynamics GP (gpmdm.py:1032-1068) of a
 * (state, class) pair is evaluated once per distinct (ancestor, new class) key of the
 * rank's slice and shared by its offspring.  Results are bitwise identical either way
 * (per-particle arithmetic does not depend on tile membership); enable=0 evaluates every
 * particle, as the reference does.  Must not be toggled between switch and propagate.
 * gpmdm_pf_dyn_rows synchronises `stream` and returns the rows the last dynamics pass
 * evaluated (distinct keys with de-duplication, the slice size without). */
int gpmdm_pf_set_dedup(gpmdm_pf_t pf, int enable);
int gpmdm_pf_dyn_rows(gpmdm_pf_t pf, int64_t* rows, void* stream);

/* Tile shape of the dynamics-GP pass.  AUTO (default): narrow 16x256 tiles for the few
 * de-duplicated rows (short K loops), the observation GP's wide shape when every particle
 * is evaluated (dedup off: a throughput problem).  NARROW / WIDE force one.  For d <= 12 the
 * two are bitwise identical (the 32x512 wide tile reduces each 256-column half in the 16x256
 * order), and AUTO may run a de-duplicated pass on the wide image when a rank's last read
 * frame had many rows; above d = 12 the 64x512 wide shape differs in floating-point
 * summation order (the de-duplication tests pin one shape).  Not between switch and
 * propagate. */
#define GPMDM_DYN_TILES_AUTO 0
#define GPMDM_DYN_TILES_NARROW 1
#define GPMDM_DYN_TILES_WIDE 2
int gpmdm_pf_set_dyn_tiles(gpmdm_pf_t pf, int mode);

/* Ancestor-ordered shards (multi-rank philox filters; default on).  After each resample the
 * particles are put in a stable order of their resampling uniform's bucket floor(256 u) (the
 * inverse-CDF search is monotone in u, so a bucket descends from a contiguous ancestor range;
 * identical on every rank; systematic resampling: the identity order, already ancestor-
 * ordered) and rank r evaluates positions [lo, hi) of that order instead of particles
 * [lo, hi), so its slice covers a contiguous ancestor range and de-duplication keeps ~1/R of
 * the distinct (ancestor, class) keys.  Pack/unpack rows follow the same order, so the all-gathered
 * filter is bitwise the same either way.  No effect on one rank, replay draws or without
 * de-duplication.  Every rank must make the same call, outside switch..resample. */
int gpmdm_pf_set_shard_order(gpmdm_pf_t pf, int enable);

/* Frames (resamples) this handle has done: the Philox counter of the next step's draws
 * (rng_mode GPMDM_RNG_PHILOX; oracle/philox.py restates the draws). */
int gpmdm_pf_frame(gpmdm_pf_t pf, int64_t* frame);

/* Rebind a filter to another model of the same (C, d, D) on the same device -- the
 * reference filter reads its GPMDM's current state on every call (gpmdm_pf.py:164, 183),
 * so a retrained / re-initialised model (GPMDM.set_latents, train_adam) must reach the
 * filter.  Models are reference counted: a filter keeps the model it was built on (or
 * last rebound to) alive, so gpmdm_model_destroy never leaves a filter dangling.  Not
 * between switch and resample. */
int gpmdm_pf_set_model(gpmdm_pf_t pf, gpmdm_model_t model);

/* Observation-GP kernel-value cutoff (opt-in; DESIGN.md §3 "Kernel-value cutoff").  The
 * observation GP of map_x_to_y / _update_weights (gpmdm.py:923-963, gpmdm_pf.py:170-192) with
 * every kernel value k_i = exp(-|x* - X_i|^2 / l^2) below tau replaced by exactly 0, tau the
 * largest cutoff whose effect provably stays below half an ulp of the smallest possible
 * 1 - k^T K_y^-1 k and below half an ulp of each output dimension's largest training
 * observation in the means; the kernel then skips the 16-row K-steps a particle tile cannot
 * reach.  gpmdm_model_set_obs_cutoff builds the model's cutoff image from
 *   K_inv     N x N row-major, K_y^-1 -- the reference's Ky_inv = U^-1 U^-T (gpmdm.py:1286-1290)
 *   beta      N x D row-major, K_y^-1 Y (the mean weights, gpmdm.py:955-957)
 *   sigma2    the noise variance on K_y's diagonal (exp(y_log_sigma_n)^2 + sigma_n_num_Y^2)
 *   y_absmax  D values, max_i |Y_ij|
 * (K_inv = NULL removes it); gpmdm_model_obs_cutoff returns tau (0: none).  The call waits
 * for the last frame of every filter built on the model, not for the device: none of them
 * may be inside a frame or stepping on another thread meanwhile.  A filter uses it
 * after gpmdm_pf_set_obs_cutoff(pf, 1) (2: also count the MFMA groups run against the dense
 * kernel's, read and optionally reset by gpmdm_pf_obs_cutoff_stats; 0: the dense kernel).
 * Results are the dense filter's to rounding (not bit for bit), and do not depend on the
 * tiling or the shard count.  Limits: d <= 16 and an image below 4 GiB (about 32k training
 * rows); GPMDM_E_INVALID otherwise. */
int gpmdm_model_set_obs_cutoff(gpmdm_model_t model, const double* K_inv, const double* beta, double sigma2,
                               const double* y_absmax);
/* The same image built on the model's device from the model's own observation factor: R and
 * K_y^-1 Y are read back out of the device image, K_y^-1 = R R^T is formed by rocBLAS dsyrk
 * and the image is packed by a device kernel (only tau, the spatial order and the K-step
 * spheres are computed on the host, from X and the column sums of K_y^-1 Y).  Byte-equal to
 * gpmdm_model_set_obs_cutoff's image for the same K_y^-1.  kinv_out (N x N) and m_out (N x D)
 * are optional host copies of the K_y^-1 and K_y^-1 Y it packed (tests).  Like
 * gpmdm_model_set_obs_cutoff: no filter on the model may be inside a frame or stepping on
 * another thread during the call (the filters' last frames are waited for, not the device). */
int gpmdm_model_build_obs_cutoff(gpmdm_model_t model, double sigma2, const double* y_absmax, double* kinv_out,
                                 double* m_out);
/* The cutoff image's doubles (*n = their count; out = NULL: the count only).  Tests. */
int gpmdm_model_obs_cutoff_image(gpmdm_model_t model, int64_t* n, double* out);
int gpmdm_model_obs_cutoff(gpmdm_model_t model, double* tau);
int gpmdm_pf_set_obs_cutoff(gpmdm_pf_t pf, int mode);
/* mode 3 = AUTO: per frame the cutoff kernel while the fraction of the dense MFMA work it ran
 * on its last frame is at most 0.75 (its break-even against the dense kernel), else the
 * dense kernel, with a cutoff frame at least every 8 frames to measure again.  The counts
 * travel with the frame's read-out, so the choice is a function of the filter's own
 * trajectory (deterministic).  Single-rank filters and banks whose read-outs are mapped (up
 * to ~800 filters) with more than 1024 particles per filter; others run mode 1 (a rank-local
 * choice would make a particle's result depend on its rank).  Mode 1 filters of that kind
 * count the same way (for the split policy below).  gpmdm_pf_obs_cutoff_auto: did the last
 * frame run the cutoff, and the last measured fraction (< 0: none yet). */
int gpmdm_pf_obs_cutoff_auto(gpmdm_pf_t pf, int* last_cut, double* fraction);
int gpmdm_pf_obs_cutoff_stats(gpmdm_pf_t pf, int64_t* run, int64_t* dense, int reset, void* stream);
/* Scheduling of the cutoff kernel's particle tiles (results are identical under every
 * policy): a split tile runs as two workgroups.  GPMDM_CUT_SPLIT_AUTO (default): the
 * _CHUNKS grid below when the filter's last measured fraction (modes 1 and 3, above) is at
 * least 0.5; otherwise every tile when the launch is at most two rounds of resident workgroups or its last round holds at
 * most an eighth of a round, none at whole rounds, otherwise the tiles of the last round
 * (measured, DESIGN.md §3 "The grid's tail"); _NONE, _ALL, _TAIL (the last round's tiles);
 * _CHUNKS: every 32-tile chunk of every tile's list its own workgroup, the chunks at the
 * lists' ends first (the dense kernel's heavy-first column blocks, for clouds that reach most
 * K-steps).  Between frames only. */
#define GPMDM_CUT_SPLIT_AUTO 0
#define GPMDM_CUT_SPLIT_NONE 1
#define GPMDM_CUT_SPLIT_ALL 2
#define GPMDM_CUT_SPLIT_TAIL 3
#define GPMDM_CUT_SPLIT_CHUNKS 4
int gpmdm_pf_set_obs_cutoff_split(gpmdm_pf_t pf, int policy);

/* Failure detection.  The filter keeps the reference's arithmetic: a
 * non-positive predictive variance gives NaN log-likelihoods / states as it does in
 * gpmdm_pf.py:167-168, 188-192.  Each event is counted on the device (per particle and
 * step) and read here: counts[0] observation-GP variance <= 0, [1] non-finite
 * log-likelihood, [2] dynamics-GP variance <= 0, [3] non-finite propagated state.
 * Synchronises `stream`; reset != 0 zeroes the counters afterwards. */
#define GPMDM_HEALTH_N 4
int gpmdm_pf_health(gpmdm_pf_t pf, int64_t* counts, int reset, void* stream);

/* GPMDM_PF.predict() (BASELINE.json north_star): the one-step dynamics-GP prediction of
 * the latent mean, (1/P) sum_p mu_{c_p}(x_p) with mu_c = map_x_dynamics_for_class's mean
 * (gpmdm.py:1032-1068) over the current particles and classes.  No state change, no draws.
 * mean: F x d host (F = 1 for a single filter).  Synchronises `stream`. */
int gpmdm_pf_predict(gpmdm_pf_t pf, double* mean, void* stream);

/* Device-side GP factor: the recipe of _precompute_kernel_inverses
 * (gpmdm.py:1284-1305) for one GP block -- the observation GP, or one class block of the
 * dynamics GP (the reference's full masked matrix has exact zeros off the class blocks):
 *   K = exp(-|x_i/l - x_j/l|^2) + diag_a I + diag_b I [+ [x_i,1] diag(lin_c2) [x_j,1]^T] + diag_c I
 *   U = chol_upper(K) (rocSOLVER potrf), R = U^-1 (trtri), M = R R^T B (two rocBLAS trmm).
 * X: n x d, lengthscales: d, lin_c2: d+1 (dynamics) or NULL (observations), B: n x k (k may
 * be 0); outputs R (n x n, strictly-lower part zero) and M (n x k).  All host, row-major.
 * The observation GP uses diag_a = sigma_n^2, diag_b = sigma_num^2, diag_c = 0
 * (gpmdm.py:381-406); a dynamics block adds the linear kernel and diag_c = 1e-6
 * (gpmdm.py:408-434, 1299-1305).  A K that is not positive definite is GPMDM_E_INVALID
 * (the reference ignores cholesky_ex's info and continues with garbage). */
int gpmdm_gp_factor(int device, const double* X, int64_t n, int32_t d, const double* lengthscales,
                    const double* lin_c2, double diag_a, double diag_b, double diag_c,
                    const double* B, int64_t k, double* R, double* M);

/* In-place inverse of a symmetric positive-definite n x n matrix on the device (the
 * training loss's K^-1 and log|K|, gpmdm.py:576-584 / 612-619; gpmdm_amd/training.py):
 * rocSOLVER potrf + potri on the caller's buffer A (device, row-major = column-major for a
 * symmetric matrix, leading dimension n), symmetrised; *logdet (host) = 2 sum log diag of
 * the Cholesky factor.  Runs on `stream` (NULL: default) and returns after it completes.
 * A matrix that is not positive definite is GPMDM_E_INVALID and *logdet is NaN. */
int gpmdm_spd_inverse(int device, double* A_dev, int64_t n, double* logdet, void* stream);

/* Replay-mode host helper (no GPU): positions along torch's CPU generator stream, so the
 * reference's per-frame draws (gpmdm_pf.py:137-213: exponential_, normal_, the multinomial's
 * uniforms, all from torch's global generator) can run as parallel chunks of torch's own
 * samplers, each on a private generator set to the state the serial draw would have reached
 * at that chunk -- bit for bit the serial streams.  `state` is torch.Generator.get_state()'s
 * byte image (CPUGeneratorImplState, GPMDM_TORCH_GEN_STATE_BYTES bytes; MT19937,
 * ATen/core/MT19937RNGEngine.h).  A walk covers n_draws random64 draws (two MT outputs each)
 * from `state`; gpmdm_rng_walk_state writes the state after `draws` of them, with the
 * normal-sample cache bytes of `cache_from` (NULL: the start state's). */
#define GPMDM_TORCH_GEN_STATE_BYTES 5056
typedef struct gpmdm_rng_walk* gpmdm_rng_walk_t;
int gpmdm_rng_walk_create(const uint8_t* state, int64_t n_draws, gpmdm_rng_walk_t* out);
/* restart a walk at another state (its buffer is reused when large enough) */
int gpmdm_rng_walk_reset(gpmdm_rng_walk_t walk, const uint8_t* state, int64_t n_draws);
int gpmdm_rng_walk_state(gpmdm_rng_walk_t walk, int64_t draws, const uint8_t* cache_from, uint8_t* out_state);
/* the states at n offsets draws[0..n), written one after the other (n x 5056 bytes) */
int gpmdm_rng_walk_states(gpmdm_rng_walk_t walk, int64_t n, const int64_t* draws, const uint8_t* cache_from,
                          uint8_t* out_states);
int gpmdm_rng_walk_destroy(gpmdm_rng_walk_t walk);

/* Message of the last failed call on this thread ("" if none). */
const char* gpmdm_last_error(void);

/* Library version string. */
const char* gpmdm_version(void);

#ifdef __cplusplus
}
#endif

#endif /* GPMDM_HIP_H */
