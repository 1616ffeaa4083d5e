/*
 * A native host for the particle filter through the C ABI alone (include/gpmdm_hip.h):
 * no Python, no torch.  It does what a notebook does with the reference
 * (GPMDM.load -> GPMDM_PF(...) -> update/class_probabilities/current_state_mean per frame,
 * gpmdm_pf.py:47-262) starting from the model's raw training data:
 *
 *   1. the kernel inverses on the device: gpmdm_gp_factor for the observation GP and for
 *      each class block of the dynamics GP (gpmdm.py:1284-1305);
 *   2. gpmdm_model_create from those factors;
 *   3. gpmdm_pf_create (Philox draws), gpmdm_pf_init with the given initial particles;
 *   4. per frame gpmdm_pf_step + gpmdm_pf_read.
 *
 *   pf_main <input.bin> <output.bin> [--ranks R --rank r --id FILE] [--device k]
 *
 * --ranks: one process per GPU shards the particles (rank r evaluates
 * [rP/R, (r+1)P/R)) and the library exchanges the rows over RCCL itself
 * (gpmdm_pf_set_comm): rank 0 writes an RCCL unique id (gpmdm_comm_unique_id) to FILE,
 * the other ranks read it, every rank joins the communicator (gpmdm_comm_init) on its
 * device.  Every rank then holds the full filter; rank r writes <output.bin>.r (R > 1).
 * --ranks 1 runs the same exchange on one rank.
 *
 * input.bin (little-endian; written by tests/test_gpu_c_host.py):
 *   int64  N, D, d, C, P, F, seed, resample
 *   int64  Nc[C]                                      dynamics pairs per class
 *   double X[N*d], Y[N*D]                             training latents and observations
 *   double Xin[sum Nc * d], Xout[sum Nc * d]          class-major dynamics pairs
 *   double y_ls[d], y_inv_lambda2[D], x_ls[d], x_lin_c2[d+1], x_inv_lambda2[d]
 *   double sy2, num_y2, sx2, num_x2                   noise variances (gpmdm.py:381-434)
 *   double T[C*C], states[P*d]
 *   int64  classes[P]
 *   double Z[F*D]                                     one observation per frame
 * output.bin: per frame double post[C], mean[d], lik.
 * Exit status 0 on success; a failing call prints gpmdm_last_error() and exits 1.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "gpmdm_hip.h"

#define CALL(x)                                                                         \
  do {                                                                                  \
    int rc_ = (x);                                                                      \
    if (rc_ != GPMDM_OK) {                                                              \
      fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, gpmdm_last_error());             \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

static FILE* in;

static void* take(size_t n, size_t size) {
  void* p = malloc(n * size > 0 ? n * size : 1);
  if (!p || fread(p, size, n, in) != n) {
    fprintf(stderr, "short input\n");
    exit(1);
  }
  return p;
}

/* rank 0 publishes the RCCL unique id through `path` (write + rename: readers never see
 * a partial file); the other ranks wait for it (at most ~120 s) */
static void share_id(const char* path, int rank, unsigned char* id) {
  if (rank == 0) {
    CALL(gpmdm_comm_unique_id(id));
    char tmp[4096];
    snprintf(tmp, sizeof tmp, "%s.tmp", path);
    FILE* f = fopen(tmp, "wb");
    if (!f || fwrite(id, 1, GPMDM_COMM_ID_BYTES, f) != GPMDM_COMM_ID_BYTES || fclose(f) != 0 || rename(tmp, path) != 0) {
      perror(path);
      exit(1);
    }
    return;
  }
  for (int i = 0; i < 1200; ++i) {
    FILE* f = fopen(path, "rb");
    if (f) {
      const size_t n = fread(id, 1, GPMDM_COMM_ID_BYTES, f);
      fclose(f);
      if (n == GPMDM_COMM_ID_BYTES) return;
    }
    struct timespec ts = {0, 100000000};
    nanosleep(&ts, NULL);
  }
  fprintf(stderr, "rank %d: no unique id at %s\n", rank, path);
  exit(1);
}

int main(int argc, char** argv) {
  int ranks = 0, rank = 0, device = 0;
  const char* id_path = NULL;
  for (int i = 3; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "--ranks")) ranks = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--rank")) rank = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--device")) device = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--id")) id_path = argv[i + 1];
    else argc = 0;
  }
  if (argc < 3 || (argc - 3) % 2 || (ranks > 0 && (!id_path || rank < 0 || rank >= ranks))) {
    fprintf(stderr, "usage: %s <input.bin> <output.bin> [--ranks R --rank r --id FILE] [--device k]\n", argv[0]);
    return 2;
  }
  in = fopen(argv[1], "rb");
  if (!in) {
    perror(argv[1]);
    return 1;
  }
  int64_t* h = take(8, sizeof(int64_t));
  const int64_t N = h[0], D = h[1], d = h[2], C = h[3], P = h[4], F = h[5];
  const uint64_t seed = (uint64_t)h[6];
  const int resample = (int)h[7];
  int64_t* Nc = take((size_t)C, sizeof(int64_t));
  int64_t nx = 0;
  for (int64_t c = 0; c < C; ++c) nx += Nc[c];
  double* X = take((size_t)(N * d), sizeof(double));
  double* Y = take((size_t)(N * D), sizeof(double));
  double* Xin = take((size_t)(nx * d), sizeof(double));
  double* Xout = take((size_t)(nx * d), sizeof(double));
  double* y_ls = take((size_t)d, sizeof(double));
  double* y_il2 = take((size_t)D, sizeof(double));
  double* x_ls = take((size_t)d, sizeof(double));
  double* x_c2 = take((size_t)(d + 1), sizeof(double));
  double* x_il2 = take((size_t)d, sizeof(double));
  double* noise = take(4, sizeof(double));
  double* T = take((size_t)(C * C), sizeof(double));
  double* states = take((size_t)(P * d), sizeof(double));
  int64_t* classes = take((size_t)P, sizeof(int64_t));
  double* Z = take((size_t)(F * D), sizeof(double));
  fclose(in);

  /* 1. kernel inverses on the device */
  double* Ry = malloc(sizeof(double) * N * N);
  double* beta = malloc(sizeof(double) * N * D);
  CALL(gpmdm_gp_factor(device, X, N, (int32_t)d, y_ls, NULL, noise[0], noise[1], 0.0, Y, D, Ry, beta));
  const double** xin = malloc(sizeof(double*) * C);
  const double** dyn_R = malloc(sizeof(double*) * C);
  const double** dyn_alpha = malloc(sizeof(double*) * C);
  int64_t off = 0;
  for (int64_t c = 0; c < C; ++c) {
    double* R = malloc(sizeof(double) * Nc[c] * Nc[c]);
    double* A = malloc(sizeof(double) * Nc[c] * d);
    CALL(gpmdm_gp_factor(device, Xin + off * d, Nc[c], (int32_t)d, x_ls, x_c2, noise[2], noise[3], 1e-6,
                         Xout + off * d, d, R, A));
    xin[c] = Xin + off * d;
    dyn_R[c] = R;
    dyn_alpha[c] = A;
    off += Nc[c];
  }

  /* 2. the device model */
  gpmdm_model_desc desc = {0};
  desc.N = N;
  desc.D = (int32_t)D;
  desc.d = (int32_t)d;
  desc.C = (int32_t)C;
  desc.tile_shape = GPMDM_TILE_DEFAULT;
  desc.X = X;
  desc.obs_R = Ry;
  desc.obs_beta = beta;
  desc.y_lengthscales = y_ls;
  desc.y_inv_lambda2 = y_il2;
  desc.Nc = Nc;
  desc.Xin = xin;
  desc.dyn_R = dyn_R;
  desc.dyn_alpha = dyn_alpha;
  desc.x_lengthscales = x_ls;
  desc.x_lin_coeff2 = x_c2;
  desc.x_inv_lambda2 = x_il2;
  gpmdm_model_t model;
  CALL(gpmdm_model_create(&desc, device, &model));

  /* 3. the filter (with --ranks: this rank's shard, the library's exchange over RCCL) */
  gpmdm_pf_t pf;
  void* comm = NULL;
  CALL(gpmdm_pf_create(model, T, P, GPMDM_RNG_PHILOX, seed, resample, ranks > 0 ? ranks : 1, rank, &pf));
  if (ranks > 0) {
    unsigned char id[GPMDM_COMM_ID_BYTES];
    share_id(id_path, rank, id);
    CALL(gpmdm_comm_init(ranks, rank, id, device, &comm));
    CALL(gpmdm_pf_set_comm(pf, comm, 0));
  }
  CALL(gpmdm_pf_init(pf, states, classes));

  /* 4. the frame loop */
  char out_path[4096];
  if (ranks > 1) snprintf(out_path, sizeof out_path, "%s.%d", argv[2], rank);
  else snprintf(out_path, sizeof out_path, "%s", argv[2]);
  FILE* out = fopen(out_path, "wb");
  if (!out) {
    perror(out_path);
    return 1;
  }
  double* post = malloc(sizeof(double) * C);
  double* mean = malloc(sizeof(double) * d);
  double lik;
  for (int64_t f = 0; f < F; ++f) {
    CALL(gpmdm_pf_step(pf, Z + f * D, NULL, NULL, NULL, NULL));
    CALL(gpmdm_pf_read(pf, post, mean, &lik, NULL));
    fwrite(post, sizeof(double), (size_t)C, out);
    fwrite(mean, sizeof(double), (size_t)d, out);
    fwrite(&lik, sizeof(double), 1, out);
  }
  fclose(out);
  CALL(gpmdm_pf_destroy(pf));
  CALL(gpmdm_comm_destroy(comm));
  CALL(gpmdm_model_destroy(model));
  printf("pf_main: %lld frames, P=%lld, N=%lld, D=%lld, d=%lld, C=%lld, ranks=%d\n", (long long)F, (long long)P,
         (long long)N, (long long)D, (long long)d, (long long)C, ranks > 0 ? ranks : 1);
  return 0;
}
