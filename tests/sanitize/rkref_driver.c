/* TEST INFRASTRUCTURE: drives the C restatement (oracle/rk_ref.c) under AddressSanitizer
 * and UndefinedBehaviorSanitizer, and under MemorySanitizer (uninitialised reads; clang,
 * build/rkref_msan): every method (RK4, DOPRI5, auto,
 * Rosenbrock, BDF — the lockstep group and the per-lane pass of the MH kernels' lane mode,
 * at S = 4 and S = 8), the register path (two_i, chain8) and the wide path (chain20: private-memory
 * Rosenbrock, one walker per group), ragged walker counts, stiff / NaN / negative
 * walkers (a small step budget, so the eviction path runs), the batched MH with Philox and replay draws and a linked '<state>0'
 * parameter.  Any sanitizer report aborts the run (-fno-sanitize-recover). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int ref_integrate(int model, int S, int P, int T, const double* times, int n_obs, const int32_t* tidx,
                  const uint64_t* mask, const double* O, const double* two_s2, const double* lin, int method,
                  int substeps, double rtol, double atol, int max_steps, int64_t W, const double* y0,
                  const double* theta, double* traj, double* chi, double* ssres, int32_t* status, int split,
                  int lane_steps);
int ref_mh(int model, int S, int P, int T, const double* times, int n_obs, const int32_t* tidx, const uint64_t* mask,
           const double* O, const double* two_s2, const double* lin, int method, int substeps, double rtol,
           double atol, int max_steps, double sstot, int pnum, int64_t W, int64_t walker_offset, int nits, int burnin,
           int rng_mode, uint64_t seed, double step_sd, const uint8_t* walk, const int32_t* init_param,
           const double* dz, const double* uu, double* theta, double* y0, double* samples, double* final_stats,
           int32_t* status, int split);

static uint64_t lcg = 88172645463325252ull;
static double unif(void) {
  lcg ^= lcg << 13; lcg ^= lcg >> 7; lcg ^= lcg << 17;
  return (double)(lcg >> 11) * (1.0 / 9007199254740992.0);
}
static double gauss(void) { return sqrt(-2.0 * log(unif() + 1e-300)) * cos(6.283185307179586 * unif()); }

enum { T = 60, NOBS = 8 };
static double times[T];
static int32_t tidx[NOBS] = {0, 8, 15, 15, 30, 44, 52, 59};
static double O[NOBS], two_s2[NOBS], lin[NOBS];

static void run_case(int model, int S, int P, int64_t W, int method, int with_traj, int split) {
  const double base[6] = {7.475e-9, 1.069e-7, 19.73, 1.934, 2.799, 10981000.0};
  uint64_t mask[NOBS];
  for (int k = 0; k < NOBS; ++k) mask[k] = (k % 2) ? (1ull << (S - 1)) : ((1ull << (S - 1)) - 1ull);
  double* y0 = calloc((size_t)S * W, sizeof(double));
  double* th = malloc(sizeof(double) * P * W);
  for (int64_t w = 0; w < W; ++w) {
    y0[0 * W + w] = 5236900.0;
    y0[(int64_t)(S - 1) * W + w] = 10981000.0;
    for (int j = 0; j < P; ++j) th[(int64_t)j * W + w] = base[j] * exp(0.05 * gauss());
  }
  if (W > 9) {
    th[4 * W + 5] = 1e5;          /* stiff lane */
    th[4 * W + W - 1] = 1e9;      /* very stiff, last (ragged) lane */
    th[1 * W + 7] = NAN;          /* non-finite rate */
    y0[0 * W + 9] = -1.0;         /* negative start */
  }
  double* traj = with_traj ? malloc(sizeof(double) * T * S * W) : NULL;
  double* chi = malloc(sizeof(double) * W);
  double* ss = malloc(sizeof(double) * W);
  int32_t* st = malloc(sizeof(int32_t) * W);
  int rc = ref_integrate(model, S, P, T, times, NOBS, tidx, mask, O, two_s2, lin, method, 2, 1.49012e-8, 1.49012e-8,
                         60, W, y0, th, traj, chi, ss, st, split,
                         /* without a trajectory: the MH kernels' per-lane DOPRI5 (lane.cuh) */
                         !with_traj && split <= 1 && S <= 8 && (method == 1 || method == 2 || method == 4));
  if (rc) { fprintf(stderr, "ref_integrate rc=%d (model %d S %d method %d)\n", rc, model, S, method); exit(1); }
  /* Metropolis-Hastings: Philox, then replay with a linked initial state (P + 1) */
  const int nits = 9, burnin = 3, kept = nits - 1 - burnin;
  for (int mode = 1; mode >= 0; --mode) {
    const int PP = mode ? P : P + 1;
    double* thm = malloc(sizeof(double) * PP * W);
    /* fresh, non-stiff draws: the stiff lanes are the integrate cases' business */
    for (int j = 0; j < PP; ++j)
      for (int64_t w = 0; w < W; ++w) thm[(int64_t)j * W + w] = base[j] * exp(0.05 * gauss());
    double* ym = malloc(sizeof(double) * S * W);
    memcpy(ym, y0, sizeof(double) * S * W);
    for (int64_t w = 0; w < W; ++w) ym[w] = 5236900.0;
    uint8_t walk[8];
    for (int j = 0; j < PP; ++j) walk[j] = (j != 2);
    int32_t ip[64];
    for (int s = 0; s < S; ++s) ip[s] = -1;
    if (!mode) ip[S - 1] = P;  /* V <- V0 */
    double* dz = mode ? NULL : malloc(sizeof(double) * (nits - 1) * PP * W);
    double* uu = mode ? NULL : malloc(sizeof(double) * (nits - 1) * W);
    if (!mode) {
      for (int64_t k = 0; k < (int64_t)(nits - 1) * PP * W; ++k) dz[k] = 0.05 * gauss();
      for (int64_t k = 0; k < (int64_t)(nits - 1) * W; ++k) uu[k] = unif();
    }
    double* samples = malloc(sizeof(double) * kept * (PP + 5) * W);
    double* fin = malloc(sizeof(double) * 4 * W);
    int32_t* mst = calloc((size_t)W, sizeof(int32_t));
    rc = ref_mh(model, S, PP, T, times, NOBS, tidx, mask, O, two_s2, lin, method, 2, 1.49012e-8, 1.49012e-8, 60,
                1.0, PP, W, 17, nits, burnin, mode, 42, 0.05, walk, ip, dz, uu, thm, ym, samples, fin, mst,
                split);
    if (rc) { fprintf(stderr, "ref_mh rc=%d (model %d method %d mode %d)\n", rc, model, method, mode); exit(1); }
    free(thm); free(ym); free(dz); free(uu); free(samples); free(fin); free(mst);
  }
  free(y0); free(th); free(traj); free(chi); free(ss); free(st);
  printf("case model=%d S=%d W=%lld method=%d ok\n", model, S, (long long)W, method);
}

int main(void) {
  for (int i = 0; i < T; ++i) times[i] = 3.0 * i / (T - 1);
  for (int k = 0; k < NOBS; ++k) {
    O[k] = 15.0 + 0.3 * k;
    two_s2[k] = 2.0 * 0.1 * 0.1;
    lin[k] = exp(O[k]);
  }
  for (int method = 0; method < 5; ++method) {
    run_case(2, 4, 5, method == 3 ? 12 : 70, method, 1, 0);  /* two_i: ragged groups (Rosenbrock: one) */
    run_case(2, 4, 5, method == 3 ? 3 : 70, method, 0, 0);   /* chi only: the MH kernels' lane mode */
  }
  for (int method = 2; method <= 4; method += 2) {          /* chain8 'auto' / 'bdf': S = 8 */
    run_case(3, 8, 5, 70, method, 1, 0);    /* lockstep groups (trajectory) */
    run_case(3, 8, 5, 70, method, 0, 0);    /* lane mode (per-lane BDF) */
  }
  run_case(3, 20, 5, 66, 1, 1, 0);          /* chain20 DOPRI5 */
  run_case(3, 20, 5, 66, 1, 1, 2);          /* chain20 DOPRI5, split over 2 lanes (32-walker groups) */
  run_case(3, 32, 5, 40, 1, 0, 4);          /* chain32 DOPRI5, split over 4 lanes */
  run_case(3, 20, 5, 66, 2, 1, 0);          /* chain20 auto: the wide (one walker per group) redo */
  run_case(3, 10, 5, 12, 3, 0, 0);          /* chain10 Rosenbrock, private-memory matrices */
  puts("SANITIZE OK");
  return 0;
}
