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
 *   pf_main <input.bin> <output.bin>
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
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s <input.bin> <output.bin>\n", argv[0]);
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
  CALL(gpmdm_gp_factor(0, X, N, (int32_t)d, y_ls, NULL, noise[0], noise[1], 0.0, Y, D, Ry, beta));
  const double** xin = malloc(sizeof(double*) * C);
  const double** dyn_R = malloc(sizeof(double*) * C);
  const double** dyn_alpha = malloc(sizeof(double*) * C);
  int64_t off = 0;
  for (int64_t c = 0; c < C; ++c) {
    double* R = malloc(sizeof(double) * Nc[c] * Nc[c]);
    double* A = malloc(sizeof(double) * Nc[c] * d);
    CALL(gpmdm_gp_factor(0, Xin + off * d, Nc[c], (int32_t)d, x_ls, x_c2, noise[2], noise[3], 1e-6,
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
  CALL(gpmdm_model_create(&desc, 0, &model));

  /* 3. the filter */
  gpmdm_pf_t pf;
  CALL(gpmdm_pf_create(model, T, P, GPMDM_RNG_PHILOX, seed, resample, 1, 0, &pf));
  CALL(gpmdm_pf_init(pf, states, classes));

  /* 4. the frame loop */
  FILE* out = fopen(argv[2], "wb");
  if (!out) {
    perror(argv[2]);
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
  CALL(gpmdm_model_destroy(model));
  printf("pf_main: %lld frames, P=%lld, N=%lld, D=%lld, d=%lld, C=%lld\n", (long long)F, (long long)P,
         (long long)N, (long long)D, (long long)d, (long long)C);
  return 0;
}
