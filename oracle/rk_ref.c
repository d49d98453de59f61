/*
 * rk_ref.c — TEST INFRASTRUCTURE ONLY: scalar C restatement of the engine's
 * integration algorithms, used by tests/ to check the HIP kernels against the
 * *same* algorithm (the scipy path in cpu_ref.py checks them against the
 * reference's algorithm).  Never linked into the product.
 *
 * What is restated (written independently of odelib_amd/csrc):
 *   - the demo RHS (Demo_InfectionStates.ipynb:60-128) and the chain model
 *     (SURVEY App. C), each a*b - c*d evaluated as fma(a, b, -(c*d));
 *   - fixed-step classical RK4 in the operation order of DESIGN.md §3.1
 *     (compiled with -ffp-contract=off: bitwise equal to the kernel);
 *   - DOPRI5 with the wavefront rule: walkers 64g..64g+63 share one step size,
 *     the step error is the max over those lanes of the per-lane max norm
 *     (DESIGN.md §3.2); for the split kernel (split.cuh, K lanes per walker) groups of
 *     64/K walkers, each walker's norm reduced over its lanes' states in a lane tree;
 *   - the fused likelihood: chi = Σ finite (O − log C)²/(2S²) (stats.py:41),
 *     ssres = Σ non-NaN (C − exp O)² (stats.py:52);
 *   - the batched Metropolis–Hastings step (Samplers.py:104-153) with replay or
 *     Philox4x32-10 draws;
 *   - the stiff methods: DOPRI5 with Hairer's stiffness test and
 *     eviction ('auto'), and the stiffly accurate Rosenbrock method RODAS (Hairer &
 *     Wanner II §VI.4) with the Jacobian from forward-mode dual numbers through the model
 *     RHS, LU with threshold partial pivoting and the method's continuous extension onto
 *     the grid, for 64-lane groups sharing one step size.
 */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define LANES 64
/* study knobs for the 'auto' hand-over (tools/demo_gate_study.py; the defaults are the
   kernels'): NSW_RESUME = ode_kernels.cuh kBdfSwitchSteps; GATE_ALL = 1 runs the stiffness
   test by steps since the start rather than since the last grid point */
#ifndef NSW_RESUME
#define NSW_RESUME 300.0
#endif
#ifndef GATE_ALL
#define GATE_ALL 0
#endif
#ifndef BDF_SWITCH_LONG
#define BDF_SWITCH_LONG 1500.0
#endif
#ifndef BDF_THR_LONG2
#define BDF_THR_LONG2 0.25
#endif
#define MAXS 64
#define MAXP 80

enum { M_ZERO_I = 0, M_ONE_I = 1, M_TWO_I = 2, M_CHAIN = 3 };
enum { ST_NONFINITE = 1, ST_NEGATIVE = 2, ST_MAXSTEP = 4, ST_STIFF = 8 };
enum { METHOD_RK4 = 0, METHOD_DOPRI5 = 1, METHOD_AUTO = 2, METHOD_ROSENBROCK = 3, METHOD_BDF = 4 };

typedef struct {
  int model, S, P, T;
  const double* times;
  int n_obs;
  const int32_t* obs_tidx; /* sorted ascending */
  const uint64_t* obs_mask;
  const double* obs_O;
  const double* obs_two_s2;
  const double* obs_lin;
  int method, substeps, max_steps;
  double rtol, atol;
  int wave_redo; /* batched integrate of S > 8: stiff walkers redone one per group
                    (odelib_amd/csrc/stiff_wave.cuh: one wave per walker, own step size) */
  double newton_tol; /* BDF: Newton convergence tolerance (from rtol, as scipy's BDF) */
  int split;     /* DOPRI5 with a walker over `split` lanes (odelib_amd/csrc/split.cuh): groups of
                    64/split walkers share a step size; a walker's error norm is the argmax over
                    each lane's states, combined in a tree of lanes (lower lane kept on ties) */
  int lane_steps; /* DOPRI5 / 'auto' / 'bdf' without a trajectory, S <= 8 (odelib_amd/csrc/lane.cuh, the
                     MH kernels): every walker takes its own DOPRI5 step sizes, i.e. the lockstep
                     algorithm on a group of one, and method 'bdf' BDF steps and orders per
                     walker.  (The BDF pass of 'auto' is a group of one per walker in every
                     mode, odelib_amd/csrc/bdf.cuh; the integrate kernels' method 'bdf' is the
                     64-lane lockstep group, bdf_wave.cuh.) */
} Prob;

static void rhs(const Prob* pb, const double* y, double t, const double* ps, double* dy) {
  (void)t;
  const int N = pb->S;
  switch (pb->model) {
    case M_ZERO_I: {
      double mu = ps[0], phi = ps[1], beta = ps[2];
      double S = y[0], V = y[1];
      double inf = phi * S * V;
      dy[0] = fma(mu, S, -inf);
      dy[1] = fma(beta, inf, -inf);
      break;
    }
    case M_ONE_I: {
      double mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3];
      double S = y[0], I1 = y[1], V = y[2];
      double inf = phi * S * V;
      dy[0] = fma(mu, S, -inf);
      dy[1] = fma(-lam, I1, inf);
      dy[2] = fma(beta * lam, I1, -inf);
      break;
    }
    case M_TWO_I: {
      double mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3], tau = ps[4];
      double S = y[0], I1 = y[1], I2 = y[2], V = y[3];
      double inf = phi * S * V;
      dy[0] = fma(mu, S, -inf);
      dy[1] = fma(-tau, I1, inf);
      dy[2] = fma(tau, I1, -(lam * I2));
      dy[3] = fma(beta * lam, I2, -inf);
      break;
    }
    default: { /* chain N */
      double mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3], tau = ps[4];
      double S = y[0], V = y[N - 1];
      double inf = phi * S * V;
      dy[0] = fma(mu, S, -inf);
      dy[1] = fma(-tau, y[1], inf);
      for (int k = 2; k <= N - 3; ++k) dy[k] = fma(tau, y[k - 1], -(tau * y[k]));
      dy[N - 2] = fma(tau, y[N - 3], -(lam * y[N - 2]));
      dy[N - 1] = fma(beta * lam, y[N - 2], -inf);
    }
  }
}

typedef struct {
  double chi, ssres;
  double ymin; /* min over emitted states (NaN ignored) */
  int nonfinite;
  int nvalid, status;
} Acc;

static void acc_init(Acc* a) {
  memset(a, 0, sizeof(Acc));
  a->ymin = INFINITY;
}

/* status bits: NONFINITE if any emitted state was NaN/inf, NEGATIVE if the minimum
   emitted state (NaN ignored, -inf counts) was < 0; MAXSTEP from DOPRI5 */
static int finish(const Acc* a) {
  int st = a->status;
  if (a->nonfinite) st |= ST_NONFINITE;
  if (a->ymin < 0.0) st |= ST_NEGATIVE;
  return st;
}

static void check_finite(int S, const double* y, Acc* a) {
  for (int s = 0; s < S; ++s)
    if (!isfinite(y[s])) a->nonfinite = 1;
}

/* output of one walker at grid index i */
static void emit(const Prob* pb, int i, const double* y, double* traj, int64_t W, int64_t w, int* k, Acc* a) {
  const int S = pb->S;
  if (traj)
    for (int s = 0; s < S; ++s) traj[((int64_t)i * S + s) * W + w] = y[s];
  for (int s = 0; s < S; ++s)
    if (!isnan(y[s]) && y[s] < a->ymin) a->ymin = y[s];
  /* finiteness is checked at observation points and at the final state */
  if (*k < pb->n_obs && pb->obs_tidx[*k] == i) check_finite(S, y, a);
  while (*k < pb->n_obs && pb->obs_tidx[*k] == i) {
    double c = 0.0;
    for (int s = 0; s < S; ++s)
      if ((pb->obs_mask[*k] >> s) & 1ull) c = c + y[s];
    double d = pb->obs_O[*k] - log(c);
    double term = (d * d) / pb->obs_two_s2[*k];
    if (isfinite(term)) { a->chi += term; a->nvalid += 1; }
    double r = c - pb->obs_lin[*k];
    double r2 = r * r;
    if (!isnan(r2)) a->ssres += r2;
    ++*k;
  }
}

static int needs_emit(const Prob* pb, int traj, int i, int k) {
  return traj || (k < pb->n_obs && pb->obs_tidx[k] == i);
}

/* ---- fixed-step RK4, one walker advanced over one output interval ---- */
static void rk4_interval(const Prob* pb, double* y, const double* p, double t, double t1) {
  const int S = pb->S;
  double k[MAXS], acc[MAXS], yt[MAXS];
  const int n = pb->substeps;
  double h = (t1 - t) / (double)n;
  for (int j = 0; j < n; ++j) {
    double ts = t + (double)j * h;
    double hh = 0.5 * h, h6 = h / 6.0;
    rhs(pb, y, ts, p, k);
    for (int s = 0; s < S; ++s) { acc[s] = k[s]; yt[s] = fma(hh, k[s], y[s]); }
    rhs(pb, yt, ts + hh, p, k);
    for (int s = 0; s < S; ++s) { acc[s] = fma(2.0, k[s], acc[s]); yt[s] = fma(hh, k[s], y[s]); }
    rhs(pb, yt, ts + hh, p, k);
    for (int s = 0; s < S; ++s) { acc[s] = fma(2.0, k[s], acc[s]); yt[s] = fma(h, k[s], y[s]); }
    rhs(pb, yt, ts + h, p, k);
    for (int s = 0; s < S; ++s) { acc[s] = acc[s] + k[s]; y[s] = fma(h6, acc[s], y[s]); }
  }
}

/* ---- DOPRI5 over one 64-lane group in lockstep ---- */
static const double c2 = 1.0 / 5, c3 = 3.0 / 10, c4 = 4.0 / 5, c5 = 8.0 / 9;
static const double a21 = 1.0 / 5, a31 = 3.0 / 40, a32 = 9.0 / 40, a41 = 44.0 / 45, a42 = -56.0 / 15,
                    a43 = 32.0 / 9, a51 = 19372.0 / 6561, a52 = -25360.0 / 2187, a53 = 64448.0 / 6561,
                    a54 = -212.0 / 729, a61 = 9017.0 / 3168, a62 = -355.0 / 33, a63 = 46732.0 / 5247,
                    a64 = 49.0 / 176, a65 = -5103.0 / 18656, a71 = 35.0 / 384, a73 = 500.0 / 1113,
                    a74 = 125.0 / 192, a75 = -2187.0 / 6784, a76 = 11.0 / 84;
static const double e1 = 71.0 / 57600, e3 = -71.0 / 16695, e4 = 71.0 / 1920, e5 = -17253.0 / 339200,
                    e6 = 22.0 / 525, e7 = -1.0 / 40;
static const double d1 = -12715105075.0 / 11282082432.0, d3 = 87487479700.0 / 32700410799.0,
                    d4 = -10690763975.0 / 1880347072.0, d5 = 701980252875.0 / 199316789632.0,
                    d6 = -1453857185.0 / 822651844.0, d7 = 69997945.0 / 29380423.0;

typedef struct {
  double y[MAXS], k1[MAXS], k2[MAXS], k3[MAXS], k4[MAXS], k5[MAXS], k6[MAXS], k7[MAXS], yt[MAXS], yn[MAXS];
  double el;
  int dead, active;
  int64_t w;
  Acc a;
  int kobs;
  int n_stiff, n_nonstiff; /* auto: consecutive stiff / non-stiff accepted steps */
  int part;                /* rosenbrock: lane takes part in the stiff integration */
  double y0c[MAXS];        /* auto: initial state, for the restart; S <= 8: the hand-over state */
  double t_ev;             /* auto, S <= 8: time of the hand-over to BDF */
  int i_ev, k_ev;          /* ... and the next grid / observation index there */
  int handed;              /* auto, S <= 8: the DOPRI5 pass handed this lane to BDF */
} Lane;

/* x^(-1/5), same operations as ode_kernels.cuh inv_fifth_root (bit-identical) */
static double inv_fifth_root(double x) {
  int e;
  const double m = frexp(x, &e);
  int q = e / 5, r = e % 5;
  if (r < 0) { r += 5; q -= 1; }
  double y = fma(fma(0.2395, m, -0.6505), m, 1.4123);
  for (int it = 0; it < 2; ++it) {
    const double y2 = y * y;
    const double y5 = (y2 * y2) * y;
    y = (y * fma(-m, y5, 6.0)) * 0.2;
  }
  const double c = r == 0 ? 1.0 : r == 1 ? 0.8705505632961241 : r == 2 ? 0.757858283255199
                 : r == 3 ? 0.6597539553864471 : 0.5743491774985174;
  return ldexp(c * y, -q);
}

double ref_inv_fifth_root(double x) { return inv_fifth_root(x); }

/* DOPRI5 step statistics over all groups since the last reset (analysis only:
   tools/dopri5_steps.py) -- accepted and rejected lockstep steps, groups integrated */
static long long g_dp_stats[3], g_ros_stats[2];
void ref_dopri5_stats(long long* out, int reset) {
  for (int j = 0; j < 3; ++j) {
    out[j] = g_dp_stats[j];
    if (reset) g_dp_stats[j] = 0;
  }
}
/* Rosenbrock lockstep steps (accepted + rejected) and groups since the last reset (analysis only) */
void ref_rosenbrock_stats(long long* out, int reset) {
  for (int j = 0; j < 2; ++j) {
    out[j] = g_ros_stats[j];
    if (reset) g_ros_stats[j] = 0;
  }
}

static double grp_max(Lane* L, int n, int use_dead_zero) {
  double m = 0.0;
  (void)use_dead_zero;
  for (int l = 0; l < n; ++l) m = fmax(m, L[l].el);
  return m;
}

/* lanes: up to 64; y in L[l].y; p[l*MAXP ...].  auto: Hairer's stiffness test on every
   accepted step; 15 stiff steps in a row evict the lane (as the step budget does) */
static void dopri5_group(const Prob* pb, Lane* L, int nl, const double* p, double* traj, int64_t W, int autom) {
  const int S = pb->S;
  const double t0 = pb->times[0], tend = pb->times[pb->T - 1];
  const double rtol = pb->rtol, atol = pb->atol;
  /* auto with S <= 8 (ode_kernels.cuh kBdfMaxS): evicted lanes are handed to BDF at the
     eviction point (no NaN poisoning, no further output from this pass) */
  const int resume = autom && S <= 8;
  for (int l = 0; l < nl; ++l) {
    L[l].dead = !L[l].active;
    L[l].handed = 0;
    L[l].kobs = 0;
    L[l].n_stiff = L[l].n_nonstiff = 0;
    emit(pb, 0, L[l].y, L[l].active ? traj : NULL, W, L[l].w, &L[l].kobs, &L[l].a);
    rhs(pb, L[l].y, t0, p + l * MAXP, L[l].k1);
  }
  double t = t0;
  /* HINIT per lane, group minimum */
  double h = INFINITY;
  for (int l = 0; l < nl; ++l) {
    Lane* q = &L[l];
    double d0 = 0.0, d1v = 0.0;
    for (int s = 0; s < S; ++s) {
      double sk = atol + rtol * fabs(q->y[s]);
      d0 = fmax(d0, fabs(q->y[s]) / sk);
      d1v = fmax(d1v, fabs(q->k1[s]) / sk);
    }
    double h0 = (d0 <= 1e-5 || d1v <= 1e-5) ? 1e-6 : 0.01 * (d0 / d1v);
    h0 = fmin(h0, tend - t0);
    for (int s = 0; s < S; ++s) q->yt[s] = fma(h0, q->k1[s], q->y[s]);
    rhs(pb, q->yt, t + h0, p + l * MAXP, q->k2);
    double d2 = 0.0;
    for (int s = 0; s < S; ++s) {
      double sk = atol + rtol * fabs(q->y[s]);
      d2 = fmax(d2, fabs(q->k2[s] - q->k1[s]) / sk);
    }
    d2 = d2 / h0;
    double dm = fmax(d1v, d2);
    double h1 = (dm <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : inv_fifth_root(dm / 0.01);
    double hl = fmin(100.0 * h0, h1);
    if (q->dead || !isfinite(hl) || !(hl > 0.0)) hl = tend - t0;
    h = fmin(h, hl);
  }
  h = fmin(h, tend - t0);
  const double span = tend - t0;
  const double hmin = 1e-14 * fmax(fabs(tend), fabs(t0)) + 1e-300;
  int i = 1, nst = 0, last_rej = 0, nst_all = 0;
  long long n_acc = 0, n_rej = 0;
  while (i < pb->T) {
    int last = 0;
    if (t + h >= tend) { h = tend - t; last = 1; }
    /* h-scaled tableau, one fma chain per stage and state */
    const double b21 = h * a21;
    const double b31 = h * a31, b32 = h * a32;
    const double b41 = h * a41, b42 = h * a42, b43 = h * a43;
    const double b51 = h * a51, b52 = h * a52, b53 = h * a53, b54 = h * a54;
    const double b61 = h * a61, b62 = h * a62, b63 = h * a63, b64 = h * a64, b65 = h * a65;
    const double b71 = h * a71, b73 = h * a73, b74 = h * a74, b75 = h * a75, b76 = h * a76;
    const double g1 = h * e1, g3 = h * e3, g4 = h * e4, g5 = h * e5, g6 = h * e6, g7 = h * e7;
    for (int l = 0; l < nl; ++l) {
      Lane* q = &L[l];
      const double* pl = p + l * MAXP;
      for (int s = 0; s < S; ++s) q->yt[s] = fma(b21, q->k1[s], q->y[s]);
      rhs(pb, q->yt, t + c2 * h, pl, q->k2);
      for (int s = 0; s < S; ++s) q->yt[s] = fma(b32, q->k2[s], fma(b31, q->k1[s], q->y[s]));
      rhs(pb, q->yt, t + c3 * h, pl, q->k3);
      for (int s = 0; s < S; ++s) q->yt[s] = fma(b43, q->k3[s], fma(b42, q->k2[s], fma(b41, q->k1[s], q->y[s])));
      rhs(pb, q->yt, t + c4 * h, pl, q->k4);
      for (int s = 0; s < S; ++s)
        q->yt[s] = fma(b54, q->k4[s], fma(b53, q->k3[s], fma(b52, q->k2[s], fma(b51, q->k1[s], q->y[s]))));
      rhs(pb, q->yt, t + c5 * h, pl, q->k5);
      for (int s = 0; s < S; ++s)
        q->yt[s] = fma(b65, q->k5[s], fma(b64, q->k4[s], fma(b63, q->k3[s], fma(b62, q->k2[s], fma(b61, q->k1[s], q->y[s])))));
      rhs(pb, q->yt, t + h, pl, q->k6);
      for (int s = 0; s < S; ++s)
        q->yn[s] = fma(b76, q->k6[s], fma(b75, q->k5[s], fma(b74, q->k4[s], fma(b73, q->k3[s], fma(b71, q->k1[s], q->y[s])))));
      rhs(pb, q->yn, t + h, pl, q->k7);
      /* argmax of |e|/sk by exact cross-multiplication, then one division; a split walker
         takes the argmax per lane (states [r*m, r*m+m)), then the lane tree */
      const int K = pb->split > 1 ? pb->split : 1, m = S / K;
      double pnum[4], pden[4], nfe = 0.0;
      for (int r = 0; r < K; ++r) {
        double num = 0.0, den = 1.0, nfr = 0.0;
        for (int j = 0; j < m; ++j) {
          const int s = r * m + j;
          double e = fma(g7, q->k7[s], fma(g6, q->k6[s], fma(g5, q->k5[s], fma(g4, q->k4[s], fma(g3, q->k3[s], g1 * q->k1[s])))));
          double ae = fabs(e);
          double sk = fma(rtol, fmax(fabs(q->y[s]), fabs(q->yn[s])), atol);
          nfr = fma(ae, 0.0, nfr);
          if (j == 0 || ae * den > num * sk) { num = ae; den = sk; }
        }
        pnum[r] = num;
        pden[r] = den;
        nfe = nfe + nfr;
      }
      for (int d = 1; d < K; d <<= 1)
        for (int r = 0; r < K; r += 2 * d) /* lanes r (lower) and r + d (upper) */
          if (pnum[r + d] * pden[r] > pnum[r] * pden[r + d]) { pnum[r] = pnum[r + d]; pden[r] = pden[r + d]; }
      double el = pnum[0] / pden[0];
      if (!isfinite(el) || isnan(nfe)) el = 1e30;
      if (q->dead) el = 0.0;
      q->el = el;
    }
    double err = grp_max(L, nl, 1);
    ++nst;
    ++nst_all;
    if (err <= 1.0) {
      /* cost gate (ode_kernels.cuh kStiffSwitchSteps / kStiffSwitchStepsSlow): tested only
         while the shared step is below (tend - t)/N */
      const double nsw = resume ? NSW_RESUME : (S <= 8 || pb->wave_redo) ? 4000.0 : 40000.0;
      const int ntest = resume ? 2 : 3; /* ode_kernels.cuh kBdfTestSteps / kStiffTestSteps */
      /* (h|lambda|)^2 above which a tested step counts as stiff: resume (S <= 8) 2.5^2 at the
         stability limit, or 0.5^2 while finishing at this step would take over 1500 more steps
         (accuracy-limited on a fast component, where BDF takes far fewer); otherwise 3.25^2 */
      const double thr2 = !resume ? 10.5625 : ((tend - t) > BDF_SWITCH_LONG * h) ? BDF_THR_LONG2 : 6.25;
      if (autom && (resume && GATE_ALL ? nst_all : nst) >= ntest && (tend - t) > nsw * h) { /* ode_kernels.cuh kBdfSwitchSteps */
        for (int l = 0; l < nl; ++l) {
          Lane* q = &L[l];
          /* components weighted by 1/(atol + rtol·max(|y|,|ynew|)), the error scale */
          double stnum = 0.0, stden = 0.0;
          for (int s = 0; s < S; ++s) {
            double r = 1.0 / fma(rtol, fmax(fabs(q->y[s]), fabs(q->yn[s])), atol);
            double dk = (q->k7[s] - q->k6[s]) * r, dy = (q->yn[s] - q->yt[s]) * r;
            stnum = fma(dk, dk, stnum);
            stden = fma(dy, dy, stden);
          }
          if (stden > 0.0 && (h * h) * stnum > thr2 * stden) {
            q->n_nonstiff = 0;
            ++q->n_stiff;
          } else if (++q->n_nonstiff >= 6) {
            q->n_stiff = 0;
          }
          if (!q->dead && q->n_stiff >= 15) {
            q->dead = 1;
            if (resume) { /* hand over at the start of this step: (t, y), next grid index i */
              q->handed = 1;
              memcpy(q->y0c, q->y, sizeof(double) * S);
              q->t_ev = t;
              q->i_ev = i;
              q->k_ev = q->kobs;
            }
            for (int s = 0; s < S; ++s) q->yn[s] = q->k7[s] = NAN;
          }
        }
      }
      if (resume) { /* every lane handed over (or idle): nothing left for this pass */
        int alive = 0;
        for (int l = 0; l < nl; ++l) alive |= !L[l].dead;
        if (!alive) break;
      }
      double tn = last ? tend : t + h;
      const double rh = 1.0 / h;
      const double hd1 = h * d1, hd3 = h * d3, hd4 = h * d4, hd5 = h * d5, hd6 = h * d6, hd7 = h * d7;
      while (i < pb->T && pb->times[i] <= tn) {
        for (int l = 0; l < nl; ++l) {
          Lane* q = &L[l];
          if (q->handed || !needs_emit(pb, traj != NULL, i, q->kobs)) continue;
          double yo[MAXS];
          double ti = pb->times[i];
          if (ti == tn) {
            for (int s = 0; s < S; ++s) yo[s] = q->yn[s];
          } else {
            double th = (ti - t) * rh, th1 = 1.0 - th;
            for (int s = 0; s < S; ++s) {
              double ydf = q->yn[s] - q->y[s];
              double bsp = fma(h, q->k1[s], -ydf);
              double r4 = fma(-h, q->k7[s], ydf) - bsp;
              double r5 = fma(hd7, q->k7[s], fma(hd6, q->k6[s], fma(hd5, q->k5[s], fma(hd4, q->k4[s], fma(hd3, q->k3[s], hd1 * q->k1[s])))));
              yo[s] = fma(th, fma(th1, fma(th, fma(th1, r5, r4), bsp), ydf), q->y[s]);
            }
          }
          if (q->dead)
            for (int s = 0; s < S; ++s) yo[s] = NAN;
          emit(pb, i, yo, q->active ? traj : NULL, W, q->w, &q->kobs, &q->a);
        }
        ++i;
        nst = 0;
      }
      for (int l = 0; l < nl; ++l) {
        memcpy(L[l].y, L[l].yn, sizeof(double) * S);
        memcpy(L[l].k1, L[l].k7, sizeof(double) * S);
      }
      t = tn;
      double fac = (err > 0.0) ? 0.9 * inv_fifth_root(err) : 10.0;
      fac = fmin(10.0, fmax(0.2, fac));
      if (last_rej) fac = fmin(fac, 1.0);
      h = h * fac;
      last_rej = 0;
      ++n_acc;
    } else {
      h = h * fmax(0.2, 0.9 * inv_fifth_root(err));
      last_rej = 1;
      ++n_rej;
    }
    if (i < pb->T && (nst >= pb->max_steps || h < hmin)) {  /* not after the last grid point */
      for (int l = 0; l < nl; ++l)
        if (!L[l].dead && L[l].el >= 0.5 * err) {
          L[l].dead = 1;
          if (resume) { /* handed to BDF at the current state */
            L[l].handed = 1;
            memcpy(L[l].y0c, L[l].y, sizeof(double) * S);
            L[l].t_ev = t;
            L[l].i_ev = i;
            L[l].k_ev = L[l].kobs;
            continue;
          }
          L[l].a.status |= ST_MAXSTEP;
          for (int s = 0; s < S; ++s) L[l].y[s] = L[l].k1[s] = NAN; /* evicted: NaN from here on */
        }
      nst = pb->max_steps / 2;
      int alive = 0;
      for (int l = 0; l < nl; ++l) alive |= !L[l].dead;
      if (!alive) {
        double yo[MAXS];
        for (int s = 0; s < S; ++s) yo[s] = NAN;
        for (; i < pb->T; ++i)
          for (int l = 0; l < nl; ++l)
            if (!L[l].handed && needs_emit(pb, traj != NULL, i, L[l].kobs))
              emit(pb, i, yo, L[l].active ? traj : NULL, W, L[l].w, &L[l].kobs, &L[l].a);
        break;
      }
      if (h < hmin) h = fmin(1e-3 * span, tend - t);
    }
  }
  for (int l = 0; l < nl; ++l) {
    if (L[l].handed) continue; /* its output and status come from the BDF pass */
    if (L[l].dead && L[l].active) L[l].a.status |= ST_MAXSTEP;
    check_finite(S, L[l].y, &L[l].a);
  }
#pragma omp atomic
  g_dp_stats[0] += n_acc;
#pragma omp atomic
  g_dp_stats[1] += n_rej;
#pragma omp atomic
  g_dp_stats[2] += 1;
}


/* ---- stiff methods ---- */

/* forward-mode dual number: value + n tangents (n = S + 1: the states, then t) */
typedef struct {
  double v;
  double d[MAXS + 1];
} Dl;

static Dl dl_c(double x, int n) {
  Dl r;
  r.v = x;
  for (int i = 0; i < n; ++i) r.d[i] = 0.0;
  return r;
}
static Dl dl_neg(Dl a, int n) {
  Dl r;
  r.v = -a.v;
  for (int i = 0; i < n; ++i) r.d[i] = -a.d[i];
  return r;
}
static Dl dl_mul(Dl a, Dl b, int n) {
  Dl r;
  r.v = a.v * b.v;
  for (int i = 0; i < n; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i];
  return r;
}
static Dl dl_fma(Dl a, Dl b, Dl c, int n) {
  Dl r;
  r.v = fma(a.v, b.v, c.v);
  for (int i = 0; i < n; ++i) r.d[i] = (a.d[i] * b.v + a.v * b.d[i]) + c.d[i];
  return r;
}

/* the built-in right-hand sides over dual numbers, operation for operation as rhs() */
static void dual_rhs(const Prob* pb, const Dl* y, const Dl* ps, Dl* dy, int n) {
  const int N = pb->S;
  switch (pb->model) {
    case M_ZERO_I: {
      Dl mu = ps[0], phi = ps[1], beta = ps[2];
      Dl Sv = y[0], V = y[1];
      Dl inf = dl_mul(dl_mul(phi, Sv, n), V, n);
      dy[0] = dl_fma(mu, Sv, dl_neg(inf, n), n);
      dy[1] = dl_fma(beta, inf, dl_neg(inf, n), n);
      break;
    }
    case M_ONE_I: {
      Dl mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3];
      Dl Sv = y[0], I1 = y[1], V = y[2];
      Dl inf = dl_mul(dl_mul(phi, Sv, n), V, n);
      dy[0] = dl_fma(mu, Sv, dl_neg(inf, n), n);
      dy[1] = dl_fma(dl_neg(lam, n), I1, inf, n);
      dy[2] = dl_fma(dl_mul(beta, lam, n), I1, dl_neg(inf, n), n);
      break;
    }
    case M_TWO_I: {
      Dl mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3], tau = ps[4];
      Dl Sv = y[0], I1 = y[1], I2 = y[2], V = y[3];
      Dl inf = dl_mul(dl_mul(phi, Sv, n), V, n);
      dy[0] = dl_fma(mu, Sv, dl_neg(inf, n), n);
      dy[1] = dl_fma(dl_neg(tau, n), I1, inf, n);
      dy[2] = dl_fma(tau, I1, dl_neg(dl_mul(lam, I2, n), n), n);
      dy[3] = dl_fma(dl_mul(beta, lam, n), I2, dl_neg(inf, n), n);
      break;
    }
    default: {
      Dl mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3], tau = ps[4];
      Dl Sv = y[0], V = y[N - 1];
      Dl inf = dl_mul(dl_mul(phi, Sv, n), V, n);
      dy[0] = dl_fma(mu, Sv, dl_neg(inf, n), n);
      dy[1] = dl_fma(dl_neg(tau, n), y[1], inf, n);
      for (int k = 2; k <= N - 3; ++k) dy[k] = dl_fma(tau, y[k - 1], dl_neg(dl_mul(tau, y[k], n), n), n);
      dy[N - 2] = dl_fma(tau, y[N - 3], dl_neg(dl_mul(lam, y[N - 2], n), n), n);
      dy[N - 1] = dl_fma(dl_mul(beta, lam, n), y[N - 2], dl_neg(inf, n), n);
    }
  }
}

/* f, J = df/dy (row s = df_s) and df/dt at (t, y) */
static void jac_eval(const Prob* pb, const double* y, double t, const double* p, double* f, double* J, double* ft) {
  const int S = pb->S, n = S + 1;
  Dl yd[MAXS], pd[MAXP], fd[MAXS];
  for (int s = 0; s < S; ++s) { yd[s] = dl_c(y[s], n); yd[s].d[s] = 1.0; }
  Dl td = dl_c(t, n);
  td.d[S] = 1.0;
  (void)td; /* the built-in models are autonomous: t enters no product */
  for (int j = 0; j < MAXP; ++j) pd[j] = dl_c(p[j], n);
  dual_rhs(pb, yd, pd, fd, n);
  for (int s = 0; s < S; ++s) {
    f[s] = fd[s].v;
    for (int j = 0; j < S; ++j) J[s * S + j] = fd[s].d[j];
    ft[s] = fd[s].d[S];
  }
}

/* RODAS (Hairer & Wanner II §VI.4): stiffly accurate Rosenbrock 4(3), 6 stages, L-stable
   embedded estimate, order-3 continuous extension (stiff.cuh namespace ros) */
static const double r_inv_gam = 4.0, r_a21 = 1.544, r_a31 = 0.9466785280815826, r_a32 = 0.2557011698983284,
                    r_a41 = 3.314825187068521, r_a42 = 2.896124015972201, r_a43 = 0.9986419139977817,
                    r_a51 = 1.221224509226641, r_a52 = 6.019134481288629, r_a53 = 12.53708332932087,
                    r_a54 = -0.687886036105895;
static const double r_c21 = -5.6688, r_c31 = -2.430093356833875, r_c32 = -0.2063599157091915,
                    r_c41 = -0.1073529058151375, r_c42 = -9.594562251023355, r_c43 = -20.47028614809616,
                    r_c51 = 7.496443313967647, r_c52 = -10.24680431464352, r_c53 = -33.99990352819905,
                    r_c54 = 11.7089089320616, r_c61 = 8.083246795921522, r_c62 = -7.981132988064893,
                    r_c63 = -31.52159432874371, r_c64 = 16.31930543123136, r_c65 = -6.058818238834054;
static const double r_c2x = 0.386, r_c3x = 0.21, r_c4x = 0.63;
static const double r_d1 = 0.25, r_d2 = -0.1043, r_d3 = 0.1035, r_d4 = -0.03620000000000023;
static const double r_h21 = 10.12623508344586, r_h22 = -7.487995877610167, r_h23 = -34.80091861555747,
                    r_h24 = -7.992771707568823, r_h25 = 1.025137723295662, r_h31 = -0.6762803392801253,
                    r_h32 = 6.087714651680015, r_h33 = 16.43084320892478, r_h34 = 24.76722511418386,
                    r_h35 = -6.594389125716872;

/* x^(-1/4), same operations as stiff.cuh inv_fourth_root (bit-identical) */
static double inv_fourth_root(double x) {
  int e;
  const double m = frexp(x, &e);
  int q = e / 4, r = e % 4;
  if (r < 0) { r += 4; q -= 1; }
  double y = fma(fma(0.3171, m, -0.8457), m, 1.5304);
  for (int it = 0; it < 3; ++it) {
    const double y2 = y * y;
    y = (y * fma(-m, y2 * y2, 5.0)) * 0.25;
  }
  const double c = r == 0 ? 1.0 : r == 1 ? 0.8408964152537145 : r == 2 ? 0.7071067811865476 : 0.5946035575013605;
  return ldexp(c * y, -q);
}

double ref_inv_fourth_root(double x) { return inv_fourth_root(x); }

/* LU with threshold partial pivoting (stiff.cuh lu_factor): column k is pivoted only when
   |a_kk| < 0.1 x max_{i>k} |a_ik|, then on the first maximum; a is S x S row-major */
static void lu_factor(int S, double* a, int* piv, double* dinv) {
  for (int k = 0; k < S; ++k) {
    int pk = k;
    if (k + 1 < S) {
      double colmax = 0.0;
      for (int i = k + 1; i < S; ++i) colmax = fmax(colmax, fabs(a[i * S + k]));
      if (fabs(a[k * S + k]) < 0.1 * colmax) {
        double best = fabs(a[k * S + k]);
        for (int i = k + 1; i < S; ++i) {
          double v = fabs(a[i * S + k]);
          if (v > best) { best = v; pk = i; }
        }
      }
    }
    piv[k] = pk;
    if (pk != k)
      for (int j = 0; j < S; ++j) { double tmp = a[k * S + j]; a[k * S + j] = a[pk * S + j]; a[pk * S + j] = tmp; }
    const double inv = 1.0 / a[k * S + k];
    dinv[k] = inv;
    for (int i = k + 1; i < S; ++i) {
      const double l = a[i * S + k] * inv;
      a[i * S + k] = l;
      for (int j = k + 1; j < S; ++j) a[i * S + j] = fma(-l, a[k * S + j], a[i * S + j]);
    }
  }
}

static void lu_solve(int S, const double* a, const int* piv, const double* dinv, double* b) {
  for (int k = 0; k < S; ++k)
    if (piv[k] != k) { double tmp = b[k]; b[k] = b[piv[k]]; b[piv[k]] = tmp; }
  for (int k = 0; k < S; ++k)
    for (int i = k + 1; i < S; ++i) b[i] = fma(-a[i * S + k], b[k], b[i]);
  for (int k = S - 1; k >= 0; --k) {
    double x = b[k];
    for (int j = k + 1; j < S; ++j) x = fma(-a[k * S + j], b[j], x);
    b[k] = x * dinv[k];
  }
}

typedef struct {
  double f0[MAXS], J[MAXS * MAXS], ft[MAXS], y1[MAXS], q3[MAXS], q4[MAXS];
} RosLane;

/* Rosenbrock (RODAS) over a 64-lane group: lanes with part set integrate from their
   L[l].y, the others sit out (no emit, no vote on the step size).  Grid points inside a
   step from the continuous extension, a grid point on the step's end = the new state. */
static void rodas_group(const Prob* pb, Lane* L, int nl, const double* p, double* traj, int64_t W) {
  static __thread RosLane R[LANES];
  const int S = pb->S;
  const double t0 = pb->times[0], tend = pb->times[pb->T - 1];
  const double rtol = pb->rtol, atol = pb->atol;
  const int tr = traj != NULL;
  double t = t0;
  for (int l = 0; l < nl; ++l) {
    Lane* q = &L[l];
    q->dead = !q->part;
    q->kobs = 0;
    if (q->part) emit(pb, 0, q->y, q->active ? traj : NULL, W, q->w, &q->kobs, &q->a);
    if (q->part) jac_eval(pb, q->y, t, p + l * MAXP, R[l].f0, R[l].J, R[l].ft);
  }
  double h = INFINITY;
  for (int l = 0; l < nl; ++l) {
    Lane* q = &L[l];
    if (q->dead) { h = fmin(h, tend - t0); continue; } /* sits out: votes the whole span */
    double d0 = 0.0, d1v = 0.0;
    for (int s = 0; s < S; ++s) {
      double sk = atol + rtol * fabs(q->y[s]);
      d0 = fmax(d0, fabs(q->y[s]) / sk);
      d1v = fmax(d1v, fabs(R[l].f0[s]) / sk);
    }
    double h0 = (d0 <= 1e-5 || d1v <= 1e-5) ? 1e-6 : 0.01 * (d0 / d1v);
    h0 = fmin(h0, tend - t0);
    double yt[MAXS], f1[MAXS];
    for (int s = 0; s < S; ++s) yt[s] = fma(h0, R[l].f0[s], q->y[s]);
    rhs(pb, yt, t + h0, p + l * MAXP, f1);
    double d2 = 0.0;
    for (int s = 0; s < S; ++s) {
      double sk = atol + rtol * fabs(q->y[s]);
      d2 = fmax(d2, fabs(f1[s] - R[l].f0[s]) / sk);
    }
    d2 = d2 / h0;
    double dm = fmax(d1v, d2);
    double h1 = (dm <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : inv_fourth_root(dm / 0.01);
    double hl = fmin(100.0 * h0, h1);
    if (q->dead || !isfinite(hl) || !(hl > 0.0)) hl = tend - t0;
    h = fmin(h, hl);
  }
  h = fmin(h, tend - t0);
  const double span = tend - t0;
  const double hmin = 1e-14 * fmax(fabs(tend), fabs(t0)) + 1e-300;
  const int budget = 8 * pb->max_steps; /* stiff.cuh kRosBudget */
  int i = 1, nst = 0, last_rej = 0;
  long long n_ros = 0;
  while (i < pb->T) {
    ++n_ros;
    int last = 0;
    if (t + h >= tend) { h = tend - t; last = 1; }
    const double rh = 1.0 / h, gh = rh * r_inv_gam;
    const double c21h = r_c21 * rh, c31h = r_c31 * rh, c32h = r_c32 * rh, c41h = r_c41 * rh, c42h = r_c42 * rh,
                 c43h = r_c43 * rh, c51h = r_c51 * rh, c52h = r_c52 * rh, c53h = r_c53 * rh, c54h = r_c54 * rh,
                 c61h = r_c61 * rh, c62h = r_c62 * rh, c63h = r_c63 * rh, c64h = r_c64 * rh, c65h = r_c65 * rh;
    const double hd1 = h * r_d1, hd2 = h * r_d2, hd3 = h * r_d3, hd4 = h * r_d4;
    for (int l = 0; l < nl; ++l) {
      Lane* q = &L[l];
      RosLane* rl = &R[l];
      const double* pl = p + l * MAXP;
      if (q->dead) { q->el = 0.0; continue; } /* bystanders and evicted lanes: no vote (the
                                                  kernel computes them and discards the result) */
      double lu[MAXS * MAXS], dinv[MAXS];
      int piv[MAXS];
      for (int r = 0; r < S; ++r)
        for (int c = 0; c < S; ++c) lu[r * S + c] = (r == c) ? gh - rl->J[r * S + c] : -rl->J[r * S + c];
      lu_factor(S, lu, piv, dinv);
      double k1[MAXS], k2[MAXS], k3[MAXS], k4[MAXS], k5[MAXS], k6[MAXS], yt[MAXS], fv[MAXS];
      const double* y = q->y;
      for (int s = 0; s < S; ++s) k1[s] = fma(hd1, rl->ft[s], rl->f0[s]);
      lu_solve(S, lu, piv, dinv, k1);
      for (int s = 0; s < S; ++s) yt[s] = fma(r_a21, k1[s], y[s]);
      rhs(pb, yt, t + r_c2x * h, pl, fv);
      for (int s = 0; s < S; ++s) k2[s] = fma(hd2, rl->ft[s], fma(c21h, k1[s], fv[s]));
      lu_solve(S, lu, piv, dinv, k2);
      for (int s = 0; s < S; ++s) yt[s] = fma(r_a32, k2[s], fma(r_a31, k1[s], y[s]));
      rhs(pb, yt, t + r_c3x * h, pl, fv);
      for (int s = 0; s < S; ++s) k3[s] = fma(hd3, rl->ft[s], fma(c32h, k2[s], fma(c31h, k1[s], fv[s])));
      lu_solve(S, lu, piv, dinv, k3);
      for (int s = 0; s < S; ++s) yt[s] = fma(r_a43, k3[s], fma(r_a42, k2[s], fma(r_a41, k1[s], y[s])));
      rhs(pb, yt, t + r_c4x * h, pl, fv);
      for (int s = 0; s < S; ++s)
        k4[s] = fma(hd4, rl->ft[s], fma(c43h, k3[s], fma(c42h, k2[s], fma(c41h, k1[s], fv[s]))));
      lu_solve(S, lu, piv, dinv, k4);
      for (int s = 0; s < S; ++s)
        yt[s] = fma(r_a54, k4[s], fma(r_a53, k3[s], fma(r_a52, k2[s], fma(r_a51, k1[s], y[s]))));
      rhs(pb, yt, t + h, pl, fv);
      for (int s = 0; s < S; ++s)
        k5[s] = fma(c54h, k4[s], fma(c53h, k3[s], fma(c52h, k2[s], fma(c51h, k1[s], fv[s]))));
      lu_solve(S, lu, piv, dinv, k5);
      for (int s = 0; s < S; ++s) yt[s] = yt[s] + k5[s];
      rhs(pb, yt, t + h, pl, fv);
      for (int s = 0; s < S; ++s)
        k6[s] = fma(c65h, k5[s], fma(c64h, k4[s], fma(c63h, k3[s], fma(c62h, k2[s], fma(c61h, k1[s], fv[s])))));
      lu_solve(S, lu, piv, dinv, k6);
      double num = 0.0, den = 1.0, nfe = 0.0;
      for (int s = 0; s < S; ++s) {
        rl->y1[s] = yt[s] + k6[s];
        double ae = fabs(k6[s]);
        double sk = fma(rtol, fmax(fabs(y[s]), fabs(rl->y1[s])), atol);
        nfe = fma(ae, 0.0, nfe);
        nfe = fma(rl->y1[s], 0.0, nfe);
        if (s == 0 || ae * den > num * sk) { num = ae; den = sk; }
        rl->q3[s] = fma(r_h25, k5[s], fma(r_h24, k4[s], fma(r_h23, k3[s], fma(r_h22, k2[s], r_h21 * k1[s]))));
        rl->q4[s] = fma(r_h35, k5[s], fma(r_h34, k4[s], fma(r_h33, k3[s], fma(r_h32, k2[s], r_h31 * k1[s]))));
      }
      double el = num / den;
      if (!isfinite(el) || isnan(nfe)) el = 1e30;
      q->el = el;
    }
    double err = grp_max(L, nl, 1);
    ++nst;
    if (err <= 1.0) {
      const double tn = last ? tend : t + h;
      while (i < pb->T && pb->times[i] < tn) {
        const double th = (pb->times[i] - t) * rh, th1 = 1.0 - th;
        for (int l = 0; l < nl; ++l) {
          Lane* q = &L[l];
          if (!q->part || !needs_emit(pb, tr, i, q->kobs)) continue;
          double yo[MAXS];
          for (int s = 0; s < S; ++s) yo[s] = fma(th, fma(th1, fma(th, R[l].q4[s], R[l].q3[s]), R[l].y1[s]), th1 * q->y[s]);
          emit(pb, i, yo, q->active ? traj : NULL, W, q->w, &q->kobs, &q->a);
        }
        ++i;
        nst = 0;
      }
      for (int l = 0; l < nl; ++l)
        if (L[l].part && !L[l].dead) memcpy(L[l].y, R[l].y1, sizeof(double) * S); /* evicted: stays NaN */
      t = tn;
      if (i < pb->T && pb->times[i] == tn) {
        for (int l = 0; l < nl; ++l)
          if (L[l].part && needs_emit(pb, tr, i, L[l].kobs))
            emit(pb, i, L[l].y, L[l].active ? traj : NULL, W, L[l].w, &L[l].kobs, &L[l].a);
        ++i;
        nst = 0;
      }
      if (i < pb->T)
        for (int l = 0; l < nl; ++l)
          if (!L[l].dead) jac_eval(pb, L[l].y, t, p + l * MAXP, R[l].f0, R[l].J, R[l].ft);
      double fac = (err > 0.0) ? 0.9 * inv_fourth_root(err) : 6.0;
      fac = fmin(6.0, fmax(0.2, fac));
      if (last_rej) fac = fmin(fac, 1.0);
      h = h * fac;
      last_rej = 0;
    } else {
      h = h * fmax(0.2, 0.9 * inv_fourth_root(err));
      last_rej = 1;
    }
    if (i < pb->T && (nst >= budget || h < hmin)) {  /* not after the last grid point */
      for (int l = 0; l < nl; ++l)
        if (!L[l].dead && L[l].el >= 0.5 * err) {
          L[l].dead = 1;
          L[l].a.status |= ST_MAXSTEP;
          for (int s = 0; s < S; ++s) L[l].y[s] = NAN;
        }
      nst = budget / 2;
      int alive = 0;
      for (int l = 0; l < nl; ++l) alive |= !L[l].dead;
      if (!alive) {
        double yo[MAXS];
        for (int s = 0; s < S; ++s) yo[s] = NAN;
        for (; i < pb->T; ++i)
          for (int l = 0; l < nl; ++l)
            if (L[l].part && needs_emit(pb, tr, i, L[l].kobs))
              emit(pb, i, yo, L[l].active ? traj : NULL, W, L[l].w, &L[l].kobs, &L[l].a);
        break;
      }
      if (h < hmin) h = fmin(1e-3 * span, tend - t);
    }
  }
  for (int l = 0; l < nl; ++l)
    if (L[l].part) check_finite(S, L[l].y, &L[l].a);
#pragma omp atomic
  g_ros_stats[0] += n_ros;
#pragma omp atomic
  g_ros_stats[1] += 1;
}


/* ---- BDF: variable order 1..5 in the fixed-leading-coefficient backward-difference form of
   scipy's BDF solver (Shampine & Reichelt's NDF family with kappa = 0 at orders 1..5 replaced
   by scipy's kappa table), for lanes with their OWN time and a shared step size and order
   (bdf.cuh).  Max norm (as LSODA), modified Newton: the LU factors of I - c J are kept across
   steps and rebuilt from a fresh Jacobian -- at the current state when the step size or the
   order changed, at the predictor when Newton fails on factors from an earlier step.  Steps may end past t_end; grid points come from the
   backward-difference interpolant.  'auto' with S <= 8 hands a lane here at its DOPRI5
   eviction point; method 'bdf' starts every lane at t0. ---- */
#define BDF_MAXQ 5
#define BDF_NEWTON_MAXITER 4
#define BDF_BUDGET 8 /* steps per output interval, in units of max_steps */
static const double bdf_gamma[6] = {0.0, 1.0, 1.5, 1.8333333333333333, 2.083333333333333, 2.283333333333333};
static const double bdf_inv_alpha[6] = {0.0, 0.8438818565400843, 0.6, 0.5039772202296456, 0.4608737397983678,
                                        0.43795620437956206};
static const double bdf_ec[6] = {1.0, 0.315, 0.16666666666666666, 0.09911666666666669, 0.11354166666666668,
                                 0.16666666666666666};
static const double bdf_safety[5] = {0.0, 0.8999999999999999, 0.8099999999999999, 0.7363636363636363,
                                     0.6749999999999999};
static const double bdf_inv_i[6] = {0.0, 1.0, 0.5, 0.3333333333333333, 0.25, 0.2};

static double bdf_newton_tol(double rtol) { return fmax(10.0 * 2.220446049250313e-16 / rtol, fmin(0.03, sqrt(rtol))); }

/* x^(-1/q), q = 1..6, for the step-size factors: frexp/ldexp and IEEE mul/fma only (bit-identical
   to bdf.cuh inv_root); x <= 0 (a zero error norm) -> +inf, x = +inf -> 0 */
static const double ir_s[7] = {0.0, -2.0, -0.8284271247461903, -0.5198420997897464, -0.37841423000544205,
                               -0.2973967099940702, -0.24492409661874603};
static const double ir_i[7] = {0.0, 3.0, 1.8284271247461903, 1.5198420997897464, 1.378414230005442,
                               1.2973967099940702, 1.244924096618746};
static const double ir_rq[7] = {0.0, 1.0, 0.5, 0.3333333333333333, 0.25, 0.2, 0.16666666666666666};
static const double ir_c[7][6] = {
    {1.0, 0, 0, 0, 0, 0},
    {1.0, 0, 0, 0, 0, 0},
    {1.0, 0.7071067811865476, 0, 0, 0, 0},
    {1.0, 0.7937005259840998, 0.6299605249474366, 0, 0, 0},
    {1.0, 0.8408964152537145, 0.7071067811865476, 0.5946035575013605, 0, 0},
    {1.0, 0.8705505632961241, 0.757858283255199, 0.6597539553864471, 0.5743491774985174, 0},
    {1.0, 0.8908987181403393, 0.7937005259840998, 0.7071067811865476, 0.6299605249474366, 0.5612310241546865}};
static double inv_root(double x, int q) {
  if (!(x > 0.0)) return INFINITY;
  if (isinf(x)) return 0.0;
  int e;
  const double m = frexp(x, &e);
  int Q = e / q, r = e % q;
  if (r < 0) { r += q; Q -= 1; }
  double y = fma(ir_s[q], m, ir_i[q]);
  for (int it = 0; it < 6; ++it) {
    double yq = y;
    for (int j = 1; j < q; ++j) yq = yq * y;
    y = (y * fma(-m, yq, (double)(q + 1))) * ir_rq[q];
  }
  return ldexp(ir_c[q][r] * y, -Q);
}
double ref_inv_root(double x, int q) { return inv_root(x, q); }

typedef struct {
  double t, D[BDF_MAXQ + 3][MAXS], lu[MAXS * MAXS], dinv[MAXS];
  int piv[MAXS];
  double yp[MAXS], psi[MAXS], rs[MAXS], d[MAXS], yn[MAXS];
  double dold, el;
  int i, conv, fail, nst, live;
} BdfLane;

/* scipy's change_D for a step-size change by `factor` at order q (D[0..q] <- (R U)^T D), in
   two stages: E = R(q, factor)^T D, then D = U^T E with U[m][j] = (-1)^m C(j, m) exact
   (bdf.cuh change_D) */
static const double bdf_U[6][6] = {{1, 1, 1, 1, 1, 1},    {0, -1, -2, -3, -4, -5}, {0, 0, 1, 3, 6, 10},
                                   {0, 0, 0, -1, -4, -10}, {0, 0, 0, 0, 1, 5},      {0, 0, 0, 0, 0, -1}};
static void bdf_change_D(BdfLane* B, int nl, int order, double factor, int S) {
  double r[6][6]; /* r[m][i] = R[i][m] */
  for (int m = 1; m <= order; ++m) {
    double v = 1.0;
    for (int i = 1; i <= order; ++i) {
      v = v * (((double)(i - 1) - factor * (double)m) * bdf_inv_i[i]);
      r[m][i] = v;
    }
  }
  for (int l = 0; l < nl; ++l) {
    if (!B[l].live) continue;
    for (int s = 0; s < S; ++s) {
      double E[6];
      E[0] = B[l].D[0][s];
      for (int m = 1; m <= order; ++m) {
        double e = B[l].D[0][s];
        for (int i = 1; i <= order; ++i) e = fma(r[m][i], B[l].D[i][s], e);
        E[m] = e;
      }
      for (int j = 0; j <= order; ++j) {
        double acc = E[0];
        for (int m = 1; m <= j; ++m) acc = fma(bdf_U[m][j], E[m], acc);
        B[l].D[j][s] = acc;
      }
    }
  }
}

/* per-lane max norm of c*v against atol + rtol|y| (argmax by cross-multiplication, one
   division; non-finite -> 1e30) */
static double bdf_norm(int S, double c, const double* v, const double* y, double rtol, double atol) {
  double num = 0.0, den = 1.0, nfe = 0.0;
  for (int s = 0; s < S; ++s) {
    const double ae = fabs(c * v[s]);
    const double sk = fma(rtol, fabs(y[s]), atol);
    nfe = fma(ae, 0.0, nfe);
    if (s == 0 || ae * den > num * sk) { num = ae; den = sk; }
  }
  double el = num / den;
  if (!isfinite(el) || isnan(nfe)) el = 1e30;
  return el;
}

/* LU factors of I - c J(t, y) */
static void bdf_factor(const Prob* pb, BdfLane* b, double c, const double* y, double t, const double* p) {
  const int S = pb->S;
  double f[MAXS], ft[MAXS];
  jac_eval(pb, y, t, p, f, b->lu, ft);
  for (int r = 0; r < S; ++r)
    for (int cc = 0; cc < S; ++cc) {
      const double a = c * b->lu[r * S + cc];
      b->lu[r * S + cc] = (r == cc) ? 1.0 - a : -a;
    }
  lu_factor(S, b->lu, b->piv, b->dinv);
}

static long long g_bdf_stats[3]; /* steps (accepted + rejected), Jacobians, groups */
/* per-phase counts (tools: where a BDF step's time goes): accepted, rejected on the error,
   rejected on Newton, Newton iterations, order/step selections, grid points emitted */
static long long g_bdf_detail[6];
void ref_bdf_detail(long long* out, int reset) {
  for (int j = 0; j < 6; ++j) {
    out[j] = g_bdf_detail[j];
    if (reset) g_bdf_detail[j] = 0;
  }
}
void ref_bdf_stats(long long* out, int reset) {
  for (int j = 0; j < 3; ++j) {
    out[j] = g_bdf_stats[j];
    if (reset) g_bdf_stats[j] = 0;
  }
}

/* lanes with `part` set start at (t_ev, y0c, grid index i_ev, observation index k_ev) with
   their accumulators as they are */
static void bdf_group(const Prob* pb, Lane* L, int nl, const double* p, double* traj, int64_t W) {
  static __thread BdfLane B[LANES];
  const int S = pb->S;
  const double tend = pb->times[pb->T - 1], t0 = pb->times[0];
  const double rtol = pb->rtol, atol = pb->atol, ntol = pb->newton_tol;
  const int tr = traj != NULL;
  const int budget = BDF_BUDGET * pb->max_steps;
  long long n_steps = 0, n_jac = 0;
  double h = INFINITY;
  for (int l = 0; l < nl; ++l) {
    BdfLane* b = &B[l];
    Lane* q = &L[l];
    b->live = q->part;
    if (!b->live) continue;
    const double* pl = p + l * MAXP;
    b->t = q->t_ev;
    b->i = q->i_ev;
    q->kobs = q->k_ev;
    b->nst = 0;
    const double* y = q->y0c;
    double f[MAXS];
    rhs(pb, y, b->t, pl, f);
    /* initial step: HINIT for order 1 (max norm), minimum over the lanes */
    double d0 = 0.0, d1v = 0.0;
    for (int s = 0; s < S; ++s) {
      const double sk = atol + rtol * fabs(y[s]);
      d0 = fmax(d0, fabs(y[s]) / sk);
      d1v = fmax(d1v, fabs(f[s]) / sk);
    }
    const double rest = tend - b->t;
    double h0 = (d0 <= 1e-5 || d1v <= 1e-5) ? 1e-6 : 0.01 * (d0 / d1v);
    h0 = fmin(h0, rest);
    double yt[MAXS], f1[MAXS];
    for (int s = 0; s < S; ++s) yt[s] = fma(h0, f[s], y[s]);
    rhs(pb, yt, b->t + h0, pl, f1);
    double d2 = 0.0;
    for (int s = 0; s < S; ++s) {
      const double sk = atol + rtol * fabs(y[s]);
      d2 = fmax(d2, fabs(f1[s] - f[s]) / sk);
    }
    d2 = d2 / h0;
    const double dm = fmax(d1v, d2);
    const double h1 = (dm <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : inv_root(dm / 0.01, 2);
    double hl = fmin(100.0 * h0, h1);
    if (!isfinite(hl) || !(hl > 0.0)) hl = rest;
    h = fmin(h, hl);
    for (int j = 0; j < BDF_MAXQ + 3; ++j)
      for (int s = 0; s < S; ++s) b->D[j][s] = 0.0;
    for (int s = 0; s < S; ++s) { b->D[0][s] = y[s]; b->D[1][s] = f[s]; }
  }
  for (int l = 0; l < nl; ++l)
    if (B[l].live)
      for (int s = 0; s < S; ++s) B[l].D[1][s] = B[l].D[1][s] * h;
  const double hmin = 1e-14 * fmax(fabs(tend), fabs(t0)) + 1e-300;
  int order = 1, neq = 0, lu_ok = 0, fresh = 0;
  for (;;) {
    int any = 0;
    for (int l = 0; l < nl; ++l) any |= B[l].live;
    if (!any) break;
    ++n_steps;
    const double c = h * bdf_inv_alpha[order];
    for (int l = 0; l < nl; ++l) {
      BdfLane* b = &B[l];
      if (!b->live) continue;
      for (int s = 0; s < S; ++s) {
        double yp = b->D[0][s], ps = 0.0;
        for (int j = 1; j <= order; ++j) {
          yp = yp + b->D[j][s];
          ps = fma(bdf_gamma[j], b->D[j][s], ps);
        }
        b->yp[s] = yp;
        b->psi[s] = ps * bdf_inv_alpha[order];
        b->rs[s] = 1.0 / fma(rtol, fabs(yp), atol);
      }
    }
    int bad = 0, niter = 0;
    if (!lu_ok) { /* factors for this step size and order, Jacobian at the current state */
      for (int l = 0; l < nl; ++l)
        if (B[l].live) bdf_factor(pb, &B[l], c, B[l].D[0] /* row 0 = the state */, B[l].t, p + l * MAXP);
      ++n_jac;
      lu_ok = 1;
      fresh = 1;
    }
    for (;;) {
      for (int l = 0; l < nl; ++l) {
        BdfLane* b = &B[l];
        if (!b->live) continue;
        memcpy(b->yn, b->yp, sizeof(double) * S);
        for (int s = 0; s < S; ++s) b->d[s] = 0.0;
        b->conv = b->fail = 0;
        b->dold = 0.0;
      }
      niter = 0;
      for (int k = 0; k < BDF_NEWTON_MAXITER; ++k) {
        int act = 0;
        for (int l = 0; l < nl; ++l) act |= B[l].live && !B[l].conv && !B[l].fail;
        if (!act) break;
        niter = k + 1;
        for (int l = 0; l < nl; ++l) {
          BdfLane* b = &B[l];
          if (!b->live || b->conv || b->fail) continue;
          double f[MAXS], dy[MAXS], nf = 0.0;
          rhs(pb, b->yn, b->t + h, p + l * MAXP, f);
          for (int s = 0; s < S; ++s) {
            nf = fma(f[s], 0.0, nf);
            dy[s] = (c * f[s] - b->psi[s]) - b->d[s];
          }
          if (isnan(nf)) { b->fail = 1; continue; }
          lu_solve(S, b->lu, b->piv, b->dinv, dy);
          double dn = 0.0;
          for (int s = 0; s < S; ++s) dn = fmax(dn, fabs(dy[s]) * b->rs[s]);
          double rate = 0.0;
          if (k > 0) {
            rate = dn / b->dold;
            const double pw = (k == 1) ? (rate * rate) * rate : (k == 2) ? rate * rate : rate;
            if (!(rate < 1.0) || pw * dn > ntol * (1.0 - rate)) { b->fail = 1; continue; }
          }
          for (int s = 0; s < S; ++s) {
            b->yn[s] = b->yn[s] + dy[s];
            b->d[s] = b->d[s] + dy[s];
          }
          if (dn == 0.0 || (k > 0 && rate * dn < ntol * (1.0 - rate))) b->conv = 1;
          b->dold = dn;
        }
      }
      bad = 0;
      for (int l = 0; l < nl; ++l) bad |= B[l].live && !B[l].conv;
#pragma omp atomic
      g_bdf_detail[3] += niter;
      if (!bad || fresh) break;
      for (int l = 0; l < nl; ++l)
        if (B[l].live) bdf_factor(pb, &B[l], c, B[l].yp, B[l].t + h, p + l * MAXP);
      ++n_jac;
      fresh = 1;
    }
    if (bad) {
#pragma omp atomic
      g_bdf_detail[2] += 1;
      h = h * 0.5;
      bdf_change_D(B, nl, order, 0.5, S);
      neq = 0;
      lu_ok = 0;
    } else {
      const double safety = bdf_safety[niter];
      double en = 0.0;
      for (int l = 0; l < nl; ++l) {
        BdfLane* b = &B[l];
        if (!b->live) continue;
        b->el = bdf_norm(S, bdf_ec[order], b->d, b->yn, rtol, atol);
        en = fmax(en, b->el);
      }
      if (en > 1.0) {
#pragma omp atomic
        g_bdf_detail[1] += 1;
        const double factor = fmax(0.2, safety * inv_root(en, order + 1));
        h = h * factor;
        bdf_change_D(B, nl, order, factor, S);
        neq = 0;
      } else {
        /* accepted: differences, grid points, lanes that reach t_end leave */
        if (getenv("RKREF_BDF_TRACE") && B[0].live) fprintf(stderr, "ACC Q=%d t=%.17g h=%.17g niter=%d\n", order, B[0].t, h, niter);
        ++neq;
        fresh = 0;
#pragma omp atomic
        g_bdf_detail[0] += 1;
        double em = 0.0, ep = 0.0;
        int voters = 0;
        for (int l = 0; l < nl; ++l) {
          BdfLane* b = &B[l];
          Lane* q = &L[l];
          if (!b->live) continue;
          const double tn = b->t + h;
          for (int s = 0; s < S; ++s) {
            b->D[order + 2][s] = b->d[s] - b->D[order + 1][s];
            b->D[order + 1][s] = b->d[s];
          }
          for (int j = order; j >= 0; --j)
            for (int s = 0; s < S; ++s) b->D[j][s] = b->D[j][s] + b->D[j + 1][s];
          ++b->nst;
          double yo[MAXS], rden[BDF_MAXQ + 1];
          for (int j = 1; j <= order; ++j) rden[j] = 1.0 / ((double)j * h);
          if (getenv("RKREF_BDF_TRACE_D") && l == 0) {
            fprintf(stderr, "STEPD q=%d tn=%a h=%a i=%d\n", order, tn, h, b->i);
            for (int j = 0; j <= order; ++j) {
              fprintf(stderr, "STEPD D%d", j);
              for (int s = 0; s < S; ++s) fprintf(stderr, " %a", b->D[j][s]);
              fprintf(stderr, "\n");
            }
          }
          while (b->i < pb->T && pb->times[b->i] <= tn) {
            const double ti = pb->times[b->i];
            double prod = 1.0;
            for (int s = 0; s < S; ++s) yo[s] = b->D[0][s];
            for (int j = 1; j <= order; ++j) {
              const double x = (ti - (tn - (double)(j - 1) * h)) * rden[j];
              prod = prod * x;
              for (int s = 0; s < S; ++s) yo[s] = fma(b->D[j][s], prod, yo[s]);
            }
            if (getenv("RKREF_BDF_TRACE") && l == 0) {
              fprintf(stderr, "EMIT i=%d y1=%.17g\n", b->i, yo[1]);
              if (getenv("RKREF_BDF_TRACE_D")) {
                fprintf(stderr, "EMITD q=%d ti=%a tn=%a h=%a t=%a\n", order, ti, tn, h, b->t);
                for (int j = 0; j <= order + 2; ++j) {
                  fprintf(stderr, "EMITD D%d", j);
                  for (int s = 0; s < S; ++s) fprintf(stderr, " %a", b->D[j][s]);
                  fprintf(stderr, "\n");
                }
              }
            }
            if (needs_emit(pb, tr, b->i, q->kobs)) emit(pb, b->i, yo, q->active ? traj : NULL, W, q->w, &q->kobs, &q->a);
#pragma omp atomic
            g_bdf_detail[5] += 1;
            ++b->i;
            b->nst = 0;
          }
          b->t = tn;
          if (b->i >= pb->T) { /* done: the final state is the last grid point's */
            memcpy(q->y, yo, sizeof(double) * S);
            b->live = 0;
            continue;
          }
          if (neq >= order + 1) {
            if (l == 0) {
#pragma omp atomic
              g_bdf_detail[4] += 1;
            }
            ++voters;
            if (order > 1) em = fmax(em, bdf_norm(S, bdf_ec[order - 1], b->D[order], b->yn, rtol, atol));
            if (order < BDF_MAXQ) ep = fmax(ep, bdf_norm(S, bdf_ec[order + 1], b->D[order + 2], b->yn, rtol, atol));
          }
        }
        if (neq >= order + 1 && voters) {
          const double fm = (order > 1) ? inv_root(em, order) : 0.0;
          const double fe = inv_root(en, order + 1);
          const double fp = (order < BDF_MAXQ) ? inv_root(ep, order + 2) : 0.0;
          int dq = 0;
          double fmx = fm;
          if (fe > fmx) { fmx = fe; dq = 1; }
          if (fp > fmx) { fmx = fp; dq = 2; }
          order += dq - 1;
          const double factor = fmin(10.0, safety * fmx);
          h = h * factor;
          bdf_change_D(B, nl, order, factor, S);
          neq = 0;
          lu_ok = 0;
        }
      }
    }
    /* budget: a lane that needs more than `budget` steps inside one output interval, or a
       step below hmin, is abandoned (MAXSTEP, NaN for the rest of its grid) */
    for (int l = 0; l < nl; ++l) {
      BdfLane* b = &B[l];
      Lane* q = &L[l];
      if (!b->live || (b->nst < budget && !(h < hmin))) continue;
      b->live = 0;
      q->a.status |= ST_MAXSTEP;
      double yo[MAXS];
      for (int s = 0; s < S; ++s) yo[s] = NAN;
      for (; b->i < pb->T; ++b->i)
        if (needs_emit(pb, tr, b->i, q->kobs)) emit(pb, b->i, yo, q->active ? traj : NULL, W, q->w, &q->kobs, &q->a);
      memcpy(q->y, yo, sizeof(double) * S);
    }
  }
  for (int l = 0; l < nl; ++l)
    if (L[l].part) check_finite(S, L[l].y, &L[l].a);
#pragma omp atomic
  g_bdf_stats[0] += n_steps;
#pragma omp atomic
  g_bdf_stats[1] += n_jac;
#pragma omp atomic
  g_bdf_stats[2] += 1;
}

/* 'auto': DOPRI5 with the stiffness test; S <= 8: the lanes it evicts continue from the
   eviction point with BDF; wider models: evicted walkers again from t0 by RODAS */
static void auto_group(const Prob* pb, Lane* L, int nl, const double* p, double* traj, int64_t W) {
  const int S = pb->S;
  if (S <= 8) {
    if (pb->lane_steps)
      for (int l = 0; l < nl; ++l) dopri5_group(pb, L + l, 1, p + l * MAXP, traj, W, 1);
    else
      dopri5_group(pb, L, nl, p, traj, W, 1);
    int any = 0;
    for (int l = 0; l < nl; ++l) {
      L[l].part = L[l].handed && L[l].active;
      any |= L[l].part;
      if (L[l].part) L[l].a.status |= ST_STIFF;
    }
    /* every handed lane on its own: the device's BDF pass (bdf.cuh integrate_bdf_lane) gives each lane
       its own step size and order, in every kernel */
    if (any)
      for (int l = 0; l < nl; ++l)
        if (L[l].part) bdf_group(pb, L + l, 1, p + l * MAXP, traj, W);
    return;
  }
  for (int l = 0; l < nl; ++l) memcpy(L[l].y0c, L[l].y, sizeof(double) * S);
  dopri5_group(pb, L, nl, p, traj, W, 1);
  int any = 0;
  for (int l = 0; l < nl; ++l) {
    L[l].part = L[l].dead && L[l].active;
    any |= L[l].part;
  }
  if (!any) return;
  for (int l = 0; l < nl; ++l)
    if (L[l].part) {
      memcpy(L[l].y, L[l].y0c, sizeof(double) * S);
      acc_init(&L[l].a);
      L[l].a.status = ST_STIFF;
    }
  if (pb->wave_redo) {
    for (int l = 0; l < nl; ++l)
      if (L[l].part) rodas_group(pb, L + l, 1, p + l * MAXP, traj, W);
  } else {
    rodas_group(pb, L, nl, p, traj, W);
  }
}

static Prob make_prob(int model, int S, int P, int T, const double* times, int n_obs, const int32_t* tidx,
                      const uint64_t* mask, const double* O, const double* two_s2, const double* lin, int method,
                      int substeps, double rtol, double atol, int max_steps) {
  Prob pb = {model, S, P, T, times, n_obs, tidx, mask, O, two_s2, lin, method, substeps, max_steps, rtol, atol, 0, 0, 0, 0};
  pb.newton_tol = bdf_newton_tol(rtol);
  return pb;
}

/* Integrate walkers [g*64, g*64+64) of a batch; y0/theta/outputs are [..][W]. */
/* walkers per lockstep group: 64, or 64/split for the split DOPRI5 kernel */
static int group_size(const Prob* pb) { return pb->split > 1 ? LANES / pb->split : LANES; }

static void integrate_group(const Prob* pb, int64_t W, int64_t g, const double* y0, const double* theta,
                            double* traj, Acc* out_acc /*[64]*/) {
  static __thread Lane L[LANES];
  static __thread double p[LANES * MAXP];
  const int S = pb->S, P = pb->P;
  const int G = group_size(pb);
  for (int l = 0; l < G; ++l) {
    int64_t gw = g * G + l;
    int active = gw < W;
    int64_t w = active ? gw : W - 1;
    L[l].active = active;
    L[l].w = w;
    acc_init(&L[l].a);
    for (int s = 0; s < S; ++s) L[l].y[s] = y0[(int64_t)s * W + w];
    for (int j = 0; j < MAXP; ++j) p[l * MAXP + j] = (j < P) ? theta[(int64_t)j * W + w] : 0.0;
  }
  if (pb->method == 0) {
    /* interval-major over the group, so each trajectory row is written as runs of
       consecutive walkers (per-walker arithmetic unchanged) */
    for (int l = 0; l < LANES; ++l)
      if (L[l].active) { L[l].kobs = 0; emit(pb, 0, L[l].y, traj, W, L[l].w, &L[l].kobs, &L[l].a); }
    for (int i = 1; i < pb->T; ++i) {
      const double t = pb->times[i - 1], t1 = pb->times[i];
      for (int l = 0; l < LANES; ++l) {
        if (!L[l].active) continue;
        rk4_interval(pb, L[l].y, p + l * MAXP, t, t1);
        if (needs_emit(pb, traj != NULL, i, L[l].kobs)) emit(pb, i, L[l].y, traj, W, L[l].w, &L[l].kobs, &L[l].a);
      }
    }
    for (int l = 0; l < LANES; ++l)
      if (L[l].active) check_finite(pb->S, L[l].y, &L[l].a);
  } else if (pb->method == METHOD_DOPRI5) {
    if (pb->lane_steps)
      for (int l = 0; l < G; ++l) dopri5_group(pb, L + l, 1, p + l * MAXP, traj, W, 0);
    else
      dopri5_group(pb, L, G, p, traj, W, 0);
  } else if (pb->method == METHOD_AUTO) {
    auto_group(pb, L, LANES, p, traj, W);
  } else if (pb->method == METHOD_BDF) {
    for (int l = 0; l < LANES; ++l) {
      Lane* q = &L[l];
      q->part = q->active;
      q->kobs = 0;
      if (q->active) emit(pb, 0, q->y, traj, W, q->w, &q->kobs, &q->a);
      memcpy(q->y0c, q->y, sizeof(double) * pb->S);
      q->t_ev = pb->times[0];
      q->i_ev = 1;
      q->k_ev = q->kobs;
    }
    if (pb->lane_steps) { /* the MH kernels: a group of one per walker (bdf.cuh) */
      for (int l = 0; l < LANES; ++l)
        if (L[l].part) bdf_group(pb, L + l, 1, p + l * MAXP, traj, W);
    } else { /* the integrate kernels: the 64-lane wave in lockstep (bdf_wave.cuh) */
      bdf_group(pb, L, LANES, p, traj, W);
    }
  } else {
    for (int l = 0; l < LANES; ++l) L[l].part = L[l].active;
    if (pb->wave_redo) {
      for (int l = 0; l < LANES; ++l)
        if (L[l].part) rodas_group(pb, L + l, 1, p + l * MAXP, traj, W);
    } else {
      rodas_group(pb, L, LANES, p, traj, W);
    }
  }
  for (int l = 0; l < G; ++l) out_acc[l] = L[l].a;
}

int ref_integrate(int model, int S, int P, int T, const double* times, int n_obs, const int32_t* tidx,
                  const uint64_t* mask, const double* O, const double* two_s2, const double* lin, int method,
                  int substeps, double rtol, double atol, int max_steps, int64_t W, const double* y0,
                  const double* theta, double* traj, double* chi, double* ssres, int32_t* status, int split,
                  int lane_steps) {
  if (S > MAXS || P > MAXP || W <= 0) return -1;
  if (split > 1 && (method != METHOD_DOPRI5 || split > 4 || S % split)) return -1;
  if (lane_steps && (traj || split > 1 || S > 8 || (method != METHOD_DOPRI5 && method != METHOD_AUTO &&
                                                      method != METHOD_BDF)))
    return -1;
  Prob pb = make_prob(model, S, P, T, times, n_obs, tidx, mask, O, two_s2, lin, method, substeps, rtol, atol, max_steps);
  pb.wave_redo = S > 8; /* ode_kernels.cuh kStiffRegS */
  pb.split = split;
  pb.lane_steps = lane_steps;
  const int G = group_size(&pb);
  const int64_t ngroups = (W + G - 1) / G;
  /* groups are independent: OpenMP over groups gives the same bits as the serial loop */
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t g = 0; g < ngroups; ++g) {
    Acc acc[LANES];
    integrate_group(&pb, W, g, y0, theta, traj, acc);
    for (int l = 0; l < G; ++l) {
      int64_t w = g * G + l;
      if (w >= W) break;
      if (chi) chi[w] = acc[l].nvalid ? acc[l].chi : NAN;
      if (ssres) ssres[w] = acc[l].ssres;
      if (status) status[w] = finish(&acc[l]);
    }
  }
  return 0;
}

/* ---- Philox4x32-10 (Salmon et al. SC'11; Random123 constants) ---- */
void ref_philox4x32_10(const uint32_t* ctr_in, const uint32_t* key_in, uint32_t* out) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2v = ctr_in[2], c3v = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2v;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3v ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2v = n2; c3v = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2v; out[3] = c3v;
}

static double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

/* proposal draws of walker gid at iteration it: z[0..npar) normals, *u uniform */
void ref_philox_draws(uint64_t seed, uint64_t gid, int it, int npar, double* z, double* u) {
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t r[4];
  for (int j = 0; j < npar; j += 2) {
    uint32_t ctr[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)it, (uint32_t)(j >> 1)};
    ref_philox4x32_10(ctr, key, r);
    double u1 = 1.0 - u53(r[0], r[1]);
    double u2 = u53(r[2], r[3]);
    double rad = sqrt(-2.0 * log(u1));
    double ang = 6.283185307179586 * u2;
    z[j] = rad * cos(ang);
    if (j + 1 < npar) z[j + 1] = rad * sin(ang);
  }
  uint32_t ctr[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)it, 0x80000000u};
  ref_philox4x32_10(ctr, key, r);
  *u = u53(r[0], r[1]);
}

/* ---- batched MH (Samplers.py:104-153), groups of 64 walkers in lockstep ---- */
int ref_mh(int model, int S, int P, int T, const double* times, int n_obs, const int32_t* tidx, const uint64_t* mask,
           const double* O, const double* two_s2, const double* lin, int method, int substeps, double rtol,
           double atol, int max_steps, double sstot, int pnum, int64_t W, int64_t walker_offset, int nits, int burnin,
           int rng_mode, uint64_t seed, double step_sd, const uint8_t* walk, const int32_t* init_param,
           const double* dz, const double* uu, double* theta /*[P][W] io*/, double* y0 /*[S][W] io*/,
           double* samples /*[kept][P+5][W]*/, double* final_stats /*[4][W]*/, int32_t* status /*[W]*/, int split) {
  if (S > MAXS || P > MAXP || W <= 0) return -1;
  if (split > 1 && (method != METHOD_DOPRI5 || split > 4 || S % split)) return -1;
  Prob pb = make_prob(model, S, P, T, times, n_obs, tidx, mask, O, two_s2, lin, method, substeps, rtol, atol, max_steps);
  pb.split = split; /* the split MH kernel (split.cuh k_mh_split): 64/split walkers per step size */
  /* the one-lane MH kernels step every chain on its own (ode_kernels.cuh kLaneSteps) */
  pb.lane_steps = split <= 1 && S <= 8 && (method == METHOD_DOPRI5 || method == METHOD_AUTO || method == METHOD_BDF);
  const int G = group_size(&pb);
  int any_walk = 0;
  for (int j = 0; j < P; ++j) any_walk |= walk[j] != 0;
  const int PS = P + 5;
  double* th_new = (double*)malloc(sizeof(double) * P * W);
  double* y_new = (double*)malloc(sizeof(double) * S * W);
  double* cur = (double*)malloc(sizeof(double) * 4 * W);
  double* u_it = (double*)malloc(sizeof(double) * W);
  Acc acc[LANES];
  /* a-priori fit */
  for (int64_t g = 0; g * G < W; ++g) {
    integrate_group(&pb, W, g, y0, theta, NULL, acc);
    for (int l = 0; l < G && g * G + l < W; ++l) {
      int64_t w = g * G + l;
      double c = acc[l].nvalid ? acc[l].chi : NAN;
      cur[w] = c;
      cur[W + w] = 1.0 - acc[l].ssres / sstot;
      cur[2 * W + w] = -2.0 * (-c) + 2.0 * (double)pnum;
      cur[3 * W + w] = 0.0;
      status[w] = finish(&acc[l]);
    }
  }
  for (int it = 1; it < nits; ++it) {
    /* proposals */
    for (int64_t w = 0; w < W; ++w) {
      double z[MAXP + 1];
      double u;
      if (rng_mode == 0) {
        for (int j = 0; j < P; ++j) z[j] = dz[((int64_t)(it - 1) * P + j) * W + w];
        u = uu[(int64_t)(it - 1) * W + w];
      } else {
        ref_philox_draws(seed, (uint64_t)(walker_offset + w), it, P + S, z, &u);
        for (int j = 0; j < P; ++j) z[j] = step_sd * z[j];
      }
      u_it[w] = u;
      for (int j = 0; j < P; ++j) {
        double v = theta[(int64_t)j * W + w];
        th_new[(int64_t)j * W + w] = walk[j] ? exp(log(v) + z[j]) : v;
      }
      for (int s = 0; s < S; ++s) {
        int pi = init_param[s];
        y_new[(int64_t)s * W + w] = (any_walk && pi >= 0) ? th_new[(int64_t)pi * W + w] : y0[(int64_t)s * W + w];
      }
    }
    for (int64_t g = 0; g * G < W; ++g) {
      integrate_group(&pb, W, g, y_new, th_new, NULL, acc);
      for (int l = 0; l < G && g * G + l < W; ++l) {
        int64_t w = g * G + l;
        double chin = acc[l].nvalid ? acc[l].chi : NAN;
        double lr = exp(cur[w] - chin);
        double accp = exp(log(lr));
        if (accp > u_it[w]) {
          cur[w] = chin;
          cur[W + w] = 1.0 - acc[l].ssres / sstot;
          cur[2 * W + w] = -2.0 * (-chin) + 2.0 * (double)pnum;
          cur[3 * W + w] += 1.0;
          for (int j = 0; j < P; ++j) theta[(int64_t)j * W + w] = th_new[(int64_t)j * W + w];
          for (int s = 0; s < S; ++s) y0[(int64_t)s * W + w] = y_new[(int64_t)s * W + w];
          status[w] = finish(&acc[l]);
        } else {
          for (int s = 0; s < S; ++s) {
            int pi = init_param[s];
            if (any_walk && pi >= 0) y0[(int64_t)s * W + w] = theta[(int64_t)pi * W + w];
          }
        }
        if (it > burnin) {
          double* row = samples + (int64_t)(it - burnin - 1) * PS * W + w;
          for (int j = 0; j < P; ++j) row[(int64_t)j * W] = theta[(int64_t)j * W + w];
          row[(int64_t)P * W] = cur[w];
          row[(int64_t)(P + 1) * W] = cur[W + w];
          row[(int64_t)(P + 2) * W] = cur[2 * W + w];
          row[(int64_t)(P + 3) * W] = (double)it;
          row[(int64_t)(P + 4) * W] = cur[3 * W + w] / (double)it;
        }
      }
    }
  }
  if (final_stats) memcpy(final_stats, cur, sizeof(double) * 4 * W);
  free(th_new); free(y_new); free(cur); free(u_it);
  return 0;
}
