// bdf_wave.cuh — the wave-lockstep BDF pass of the integrate kernels' method 'bdf' (every
// walker BDF from t0, k_integrate with and without a trajectory, S <= 8): the algorithm of
// bdf.cuh with the lanes of a wave sharing h and q (wave-max norms), so every vector
// operation is uniform.  Lanes carry their own time; steps may end past t_end (LSODA
// itask = 1); grid points come from the backward-difference interpolant.
//
// Why two passes.  The per-lane pass (bdf.cuh) gives every walker its own step sizes and
// orders — what the MH chains need (a chain's bits independent of its wave-mates) and the
// cheaper form for the few lanes 'auto' hands over.  With EVERY lane of a wave in BDF, though,
// lanes at independent phases make each loop trip pay for the union of their work (some lane
// refactors on nearly every trip, Newton runs to the slowest lane's count, two or three order
// cases run): 65 536 demo walkers with trajectories 10.6 ms per-lane against 2.95 ms
// lockstep (profiles/NOTES.md, round 5).  The trajectory kernels' DOPRI5 is lockstep for the
// same reason, so their 'bdf' is too; the C restatement groups lanes the same way
// (oracle/rk_ref.c bdf_group over a 64-lane group).
#pragma once

namespace oe {
namespace bdf {
constexpr int kRows = kMaxQ + 3;  // D[0..q+2]
// scipy's BDF tables: gamma_q = Σ_{j<=q} 1/j, alpha_q = (1 − kappa_q)·gamma_q (1/alpha here),
// error constants kappa_q·gamma_q + 1/(q+1), Newton-count safety 0.9·(2·4+1)/(2·4+n)
__device__ const double kGamma[6] = {0.0, 1.0, 1.5, 1.8333333333333333, 2.083333333333333, 2.283333333333333};
__device__ const double kInvAlpha[6] = {0.0, 0.8438818565400843, 0.6, 0.5039772202296456, 0.4608737397983678,
                                        0.43795620437956206};
__device__ const double kEc[6] = {1.0, 0.315, 0.16666666666666666, 0.09911666666666669, 0.11354166666666668,
                                  0.16666666666666666};
__device__ const double kSafety[5] = {0.0, 0.8999999999999999, 0.8099999999999999, 0.7363636363636363,
                                      0.6749999999999999};
__device__ const double kInvI[6] = {0.0, 1.0, 0.5, 0.3333333333333333, 0.25, 0.2};
// U of scipy's change_D (R(q, 1)): U[m][j] = (−1)^m·C(j, m), exact integers
__device__ const double kU[6][6] = {{1, 1, 1, 1, 1, 1},    {0, -1, -2, -3, -4, -5}, {0, 0, 1, 3, 6, 10},
                                    {0, 0, 0, -1, -4, -10}, {0, 0, 0, 0, 1, 5},      {0, 0, 0, 0, 0, -1}};
// scipy's change_D for a step-size change by `factor` at order q, in two stages:
// E = R(q, factor)^T D, then D = U^T E (the same product as (RU)^T D, U exact).  The R
// coefficients r[m][i] = R[i][m] once (wave-uniform), then state by state, so only one
// state's E is live.
template <int S>
__device__ __forceinline__ void change_D(double (&D)[kRows][S], int q, double factor) {
  const cptr<double> U = kconst(&kU[0][0]), inv_i = kconst(kInvI);
  double r[kMaxQ + 1][kMaxQ + 1];
#pragma unroll
  for (int m = 1; m <= kMaxQ; ++m) {
    if (m > q) break;
    double v = 1.0;
#pragma unroll
    for (int i = 1; i <= kMaxQ; ++i) {
      if (i > q) break;
      v = v * (((double)(i - 1) - factor * (double)m) * inv_i[i]);
      r[m][i] = v;
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    double E[kMaxQ + 1];
    E[0] = D[0][s];
#pragma unroll
    for (int m = 1; m <= kMaxQ; ++m) {
      if (m > q) break;
      double e = D[0][s];
#pragma unroll
      for (int i = 1; i <= kMaxQ; ++i) {
        if (i > q) break;
        e = fma(r[m][i], D[i][s], e);
      }
      E[m] = e;
    }
#pragma unroll
    for (int j = 0; j <= kMaxQ; ++j) {
      if (j > q) break;
      double acc = E[0];
#pragma unroll
      for (int m = 1; m <= kMaxQ; ++m) {
        if (m > j) break;
        acc = fma(U[m * 6 + j], E[m], acc);
      }
      D[j][s] = acc;
    }
  }
}

// row `j` (wave-uniform, runtime) of D without indexing the register array
template <int S>
__device__ __forceinline__ void row(const double (&D)[kRows][S], int j, double (&out)[S]) {
#pragma unroll
  for (int s = 0; s < S; ++s) out[s] = 0.0;
#pragma unroll
  for (int r = 0; r < kRows; ++r)
    if (r == j) {
#pragma unroll
      for (int s = 0; s < S; ++s) out[s] = D[r][s];
    }
}
}  // namespace bdf

// the observations at grid index i (the lane's next observed one): fused chi / R² terms, and
// the next observed index
template <int S>
__device__ __forceinline__ void observe_lane(const DevProblem& pb, int i, const double (&y)[S], int& k, int& nxt,
                                             Acc& a) {
  const Obs* obs = pb.obs;
  check_finite(y, a);
  while (k < pb.n_obs && obs[k].tidx == i) {
    const uint64_t mask = obs[k].mask;
    const double O = obs[k].O, two_s2 = obs[k].two_s2, O_lin = obs[k].O_lin;
    double c = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s)
      if ((mask >> s) & 1ull) c = c + y[s];
    const double d = O - oe_log(c);
    const double term = (d * d) / two_s2;
    if (__builtin_isfinite(term)) { a.chi += term; a.nvalid += 1; }
    const double r = c - O_lin;
    const double r2 = r * r;
    if (!__builtin_isnan(r2)) a.ssres += r2;
    ++k;
  }
  nxt = (k < pb.n_obs) ? obs[k].tidx : 0x7fffffff;
}

// Output of one lane at its own grid index i (trajectory row store + minimum + observations):
// per-lane addresses, so plain stores/loads instead of the uniform buffer descriptors.
// Without a trajectory only observed grid points are emitted (as the DOPRI5 pass does).
// `nxt` is the lane's next observed grid index, carried in a register: an unobserved row does
// no load.  The row stores come last: on gfx950 a vector load's wait also waits for every
// store issued before it, so a load after the stores (the old obs[k] test) held each row
// until its stores had completed (C2-stiffmix `auto`: ~2.3 us per BDF row).
template <int S, bool TRAJ, bool NT>
__device__ __forceinline__ void emit_lane(const DevProblem& pb, int i, const double (&y)[S], double* traj, int64_t W,
                                          int64_t w, bool active, int& k, int& nxt, Acc& a) {
  const bool observed = i == nxt;
  if (!TRAJ && !observed) return;
  track_min<S>(y, a);
  if (observed) observe_lane<S>(pb, i, y, k, nxt, a);
  if constexpr (TRAJ) {
    if (active) {
      double* row = traj + (int64_t)i * S * W + w;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if constexpr (NT) __builtin_nontemporal_store(y[s], row + (int64_t)s * W);
        else row[(int64_t)s * W] = y[s];
      }
    }
  }
}

// The per-lane state of the BDF pass and the wave-shared controls.
template <int S>
struct BdfState {
  double D[bdf::kRows][S];  // backward differences (scipy's D)
  double lu[S][S], dinv[S]; // LU of I − c·J (J evaluated when the factors are built)
  int piv[S];
  double t;                 // this lane's time
  double ti;                // times[i] (times[T] is the +inf sentinel), loaded ahead
  int i, k, nst;            // next grid index, next observation, steps since the last grid point
  int nxt;                  // grid index of observation k (INT_MAX past the last)
  bool live;
  // wave-uniform
  double h;
  int order, neq;
  bool lu_ok, fresh, any_swap;  // factors valid; built in this step (from this step's Jacobian)
};

// LU factors of I − c·J(t, y) for the lanes taking part
template <class M, int PMAX>
__device__ __forceinline__ void bdf_factor(BdfState<M::S>& st, double c, const double (&y)[M::S], double t,
                                           const double (&p)[PMAX]) {
  constexpr int S = M::S;
  double f[S], ft[S];
  jac_eval<M, PMAX>(y, t, p, f, st.lu, ft);
#pragma unroll
  for (int r = 0; r < S; ++r)
#pragma unroll
    for (int q = 0; q < S; ++q) {
      const double av = c * st.lu[r][q];
      st.lu[r][q] = (r == q) ? 1.0 - av : -av;
    }
  st.any_swap = ros::lu_factor<S>(st.lu, st.piv, st.dinv);
}

// What an accepted step hands to the (order-generic) output and order selection.
struct BdfAccepted {
  double h, en, safety;  // the step size used, the wave error norm, the Newton-count safety
  double em_l, ep_l;     // this lane's norms at orders q − 1 and q + 1 (select steps)
  bool select;           // wave-uniform: order and step selection after this step
};

// One step attempt at order Q (compile-time, so the difference rows are fixed registers and
// the loops over them are straight-line code).  Returns false on a rejected attempt (h and D
// already rescaled for the retry); on acceptance the lanes' differences are updated and the
// grid output and order selection follow in bdf_output / bdf_select (order-generic: written
// once rather than once per order).
template <class M, int PMAX, int Q>
__device__ __forceinline__ bool bdf_attempt(const DevProblem& pb, BdfState<M::S>& st, const double (&p)[PMAX],
                                            BdfAccepted& acc) {
  using namespace bdf;
  constexpr int S = M::S;
  const double rtol = pb.rtol, atol = pb.atol, ntol = pb.newton_tol;
  const cptr<double> gam = kconst(kGamma);
  const double ialpha = kconst(kInvAlpha)[Q];
  const double h = st.h;
  const double c = h * ialpha;
  double yp[S], psi[S], rs[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    double v = st.D[0][s], ps = 0.0;
#pragma unroll
    for (int j = 1; j <= Q; ++j) {
      v = v + st.D[j][s];
      ps = fma(gam[j], st.D[j][s], ps);
    }
    yp[s] = v;
    psi[s] = ps * ialpha;
    rs[s] = 1.0 / fma(rtol, fabs(v), atol);
  }
  double yn[S], d[S];
  bool bad = false;
  int niter = 0;
  if (!st.lu_ok) {  // factors for this step size and order, Jacobian at the current state
    double y0[S];
#pragma unroll
    for (int s = 0; s < S; ++s) y0[s] = st.D[0][s];
    bdf_factor<M, PMAX>(st, c, y0, st.t, p);
    st.lu_ok = true;
    st.fresh = true;
  }
  for (;;) {  // Newton; once more on factors from this step's predictor if it fails on older ones
#pragma unroll
    for (int s = 0; s < S; ++s) { yn[s] = yp[s]; d[s] = 0.0; }
    bool conv = false, fail = false;
    double dold = 0.0;
    niter = 0;
    for (int kk = 0; kk < kNewtonMaxIter; ++kk) {
      const bool act = st.live && !conv && !fail;
      if (__ballot(act) == 0ull) break;
      niter = kk + 1;
      if (act) {
        double f[S], dy[S], nf = 0.0;
        M::rhs(yn, st.t + h, p, f);
#pragma unroll
        for (int s = 0; s < S; ++s) {
          nf = fma(f[s], 0.0, nf);
          dy[s] = (c * f[s] - psi[s]) - d[s];
        }
        if (__builtin_isnan(nf)) {
          fail = true;
        } else {
          ros::lu_solve<S>(st.lu, st.piv, st.dinv, st.any_swap, dy);
          double dn = 0.0;
#pragma unroll
          for (int s = 0; s < S; ++s) dn = fmax(dn, fabs(dy[s]) * rs[s]);
          double rate = 0.0;
          bool ok = true;
          if (kk > 0) {
            rate = dn / dold;
            const double pw = (kk == 1) ? (rate * rate) * rate : (kk == 2) ? rate * rate : rate;
            if (!(rate < 1.0) || pw * dn > ntol * (1.0 - rate)) { fail = true; ok = false; }
          }
          if (ok) {
#pragma unroll
            for (int s = 0; s < S; ++s) {
              yn[s] = yn[s] + dy[s];
              d[s] = d[s] + dy[s];
            }
            if (dn == 0.0 || (kk > 0 && rate * dn < ntol * (1.0 - rate))) conv = true;
            dold = dn;
          }
        }
      }
    }
    bad = __ballot(st.live && !conv) != 0ull;
    if (!bad || st.fresh) break;
    bdf_factor<M, PMAX>(st, c, yp, st.t + h, p);
    st.fresh = true;
  }
  if (bad) {
    st.h = h * 0.5;
    change_D<S>(st.D, Q, 0.5);
    st.neq = 0;
    st.lu_ok = false;
    return false;
  }
  const double safety = kconst(kSafety)[niter];
  const cptr<double> ec = kconst(kEc);
  const double el = st.live ? norm_max<S>(ec[Q], d, yn, rtol, atol) : 0.0;
  const double en = wave_max(el);
  if (en > 1.0) {
    const double factor = fmax(0.2, safety * inv_root(en, Q + 1));
    st.h = h * factor;
    change_D<S>(st.D, Q, factor);
    st.neq = 0;
    return false;
  }
#ifdef OE_BDF_TRACE
  if (st.live && blockIdx.x == 0 && threadIdx.x == 0) printf("ACC Q=%d t=%.17g h=%.17g niter=%d\n", Q, st.t, h, niter);
#endif
  ++st.neq;
  st.fresh = false;
  acc.h = h;
  acc.en = en;
  acc.safety = safety;
  acc.select = st.neq >= Q + 1;
  acc.em_l = 0.0;
  acc.ep_l = 0.0;
  if (st.live) {  // the differences of the accepted step
#pragma unroll
    for (int s = 0; s < S; ++s) {
      st.D[Q + 2][s] = d[s] - st.D[Q + 1][s];
      st.D[Q + 1][s] = d[s];
    }
#pragma unroll
    for (int j = Q; j >= 0; --j)
#pragma unroll
      for (int s = 0; s < S; ++s) st.D[j][s] = st.D[j][s] + st.D[j + 1][s];
    if (acc.select) {  // the candidates' norms (used by the lanes still running after the output)
      if constexpr (Q > 1) acc.em_l = norm_max<S>(ec[Q - 1], st.D[Q], yn, rtol, atol);
      if constexpr (Q < kMaxQ) acc.ep_l = norm_max<S>(ec[Q + 1], st.D[Q + 2], yn, rtol, atol);
    }
  }
  return true;
}

// The grid points of an accepted step of order q (wave-uniform, runtime) from the
// backward-difference interpolant; a lane past its last grid point leaves (y = that row).
template <int S, bool TRAJ, bool NT>
__device__ __forceinline__ void bdf_output(const DevProblem& pb, BdfState<S>& st, int q, double h, double (&y)[S],
                                           double* traj, int64_t W, int64_t w, bool active, Acc& a) {
  using namespace bdf;
  if (!st.live) return;
  const double tn = st.t + h;
  ++st.nst;
  double yo[S];
  const double* times = pb.times;
  double rden[kMaxQ + 1];  // 1/(j·h): one division per order per step, not per grid point
#pragma unroll
  for (int j = 1; j <= kMaxQ; ++j) {
    if (j > q) break;
    rden[j] = 1.0 / ((double)j * h);
  }
  while (st.ti <= tn) {  // (st.i < T: times[T] is +inf)
    const double ti = st.ti;
    const int i = st.i;
    st.i = i + 1;
    const double tnext = times[st.i];  // in flight while this row is formed and stored
    if (TRAJ || i == st.nxt || i == pb.T - 1) {  // without a trajectory: observed rows, the final state
      double prod = 1.0;
#pragma unroll
      for (int s = 0; s < S; ++s) yo[s] = st.D[0][s];
#pragma unroll
      for (int j = 1; j <= kMaxQ; ++j) {
        if (j > q) break;
        const double x = (ti - (tn - (double)(j - 1) * h)) * rden[j];
        prod = prod * x;
#pragma unroll
        for (int s = 0; s < S; ++s) yo[s] = fma(st.D[j][s], prod, yo[s]);
      }
#ifdef OE_BDF_TRACE
      if (blockIdx.x == 0 && threadIdx.x == 0) printf("EMIT i=%d y1=%.17g\n", i, yo[1]);
#endif
      emit_lane<S, TRAJ, NT>(pb, i, yo, traj, W, w, active, st.k, st.nxt, a);
    }
    st.ti = tnext;
    st.nst = 0;
  }
  st.t = tn;
  if (st.i >= pb.T) {
#pragma unroll
    for (int s = 0; s < S; ++s) y[s] = yo[s];
    st.live = false;
  }
}

// Order and step-size selection after an accepted select step of order q (scipy's rule:
// the largest of the three factors, capped at 10), voted by the lanes still running.
template <int S>
__device__ __forceinline__ void bdf_select(BdfState<S>& st, int q, const BdfAccepted& acc) {
  using namespace bdf;
  const bool voter = st.live;
  if (__ballot(voter) == 0ull) return;
  const double em = wave_max(voter ? acc.em_l : 0.0), ep = wave_max(voter ? acc.ep_l : 0.0);
  const double fm = (q > 1) ? inv_root(em, q) : 0.0;
  const double fe = inv_root(acc.en, q + 1);
  const double fp = (q < kMaxQ) ? inv_root(ep, q + 2) : 0.0;
  int dq = 0;
  double fmx = fm;
  if (fe > fmx) { fmx = fe; dq = 1; }
  if (fp > fmx) { fmx = fp; dq = 2; }
  const int nq = q + dq - 1;
  const double factor = fmin(10.0, acc.safety * fmx);
  st.h = acc.h * factor;
  change_D<S>(st.D, nq, factor);
  st.order = nq;
  st.neq = 0;
  st.lu_ok = false;
}

// The same selection with the order a template parameter (constant divisions in the roots,
// unrolled loops, change_D at a constant order; the same operations): 11 % faster on 65 536
// walkers with trajectories (2.63 vs 2.95 ms).  In r04 a build of it failed the chain8 'bdf'
// parity test deterministically while every other stiff case stayed bitwise (profiles/NOTES.md
// r04n); rebuilt in r05 it is bitwise on every stiff test (NOTES.md round 5), so it is the
// default again; OE_BDF_WAVE_SELECT_TEMPLATED=0 builds the order-generic selection.
#ifndef OE_BDF_WAVE_SELECT_TEMPLATED
#define OE_BDF_WAVE_SELECT_TEMPLATED 1
#endif
template <int S, int Q>
__device__ __forceinline__ void bdf_select_q(BdfState<S>& st, const BdfAccepted& acc) {
  using namespace bdf;
  const bool voter = st.live;
  if (__ballot(voter) == 0ull) return;
  const double em = wave_max(voter ? acc.em_l : 0.0), ep = wave_max(voter ? acc.ep_l : 0.0);
  double fm = 0.0, fp = 0.0;
  if constexpr (Q > 1) fm = bdfl::inv_root<Q>(em);
  const double fe = bdfl::inv_root<Q + 1>(acc.en);
  if constexpr (Q < kMaxQ) fp = bdfl::inv_root<Q + 2>(ep);
  int dq = 0;
  double fmx = fm;
  if (fe > fmx) { fmx = fe; dq = 1; }
  if (fp > fmx) { fmx = fp; dq = 2; }
  const double factor = fmin(10.0, acc.safety * fmx);
  st.h = acc.h * factor;
  if (dq == 0) {
    if constexpr (Q > 1) change_D<S>(st.D, Q - 1, factor);
  } else if (dq == 1) {
    change_D<S>(st.D, Q, factor);
  } else {
    if constexpr (Q < kMaxQ) change_D<S>(st.D, Q + 1, factor);
  }
  st.order = Q + dq - 1;
  st.neq = 0;
  st.lu_ok = false;
}

// BDF integration of the lanes with `part` set from their own (t, y, grid index i,
// observation index k) with their accumulators as they are; the others sit out (no vote,
// no output).  y is the final state (the last grid point's) on return.
template <class M, int PMAX, bool TRAJ, bool NT>
__device__ __forceinline__ void integrate_bdf(const DevProblem& pb, double (&y)[M::S], double t, int i, int k,
                                              const double (&p)[PMAX], double* traj, int64_t W, int64_t w,
                                              bool active, bool part, Acc& a) {
  using namespace bdf;
  constexpr int S = M::S;
  const cptr<double> ctimes = kconst(pb.times);
  const double tend = ctimes[pb.T - 1], t0 = ctimes[0];
  const double rtol = pb.rtol, atol = pb.atol;
  const int budget = kBudget * pb.max_steps;
  BdfState<S> st;
  st.live = part;
  st.t = t;
  st.i = i;
  st.k = k;
  st.ti = pb.times[i];
  st.nxt = (k < pb.n_obs) ? pb.obs[k].tidx : 0x7fffffff;
  st.nst = 0;
  {
    double f[S];
    M::rhs(y, t, p, f);
    // initial step: HINIT for order 1 (max norm), wave minimum over the lanes taking part
    double d0 = 0.0, d1v = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double sk = atol + rtol * fabs(y[s]);
      d0 = fmax(d0, fabs(y[s]) / sk);
      d1v = fmax(d1v, fabs(f[s]) / sk);
    }
    const double rest = tend - t;
    double h0 = (d0 <= 1e-5 || d1v <= 1e-5) ? 1e-6 : 0.01 * (d0 / d1v);
    h0 = fmin(h0, rest);
    double yt[S], f1[S];
#pragma unroll
    for (int s = 0; s < S; ++s) yt[s] = fma(h0, f[s], y[s]);
    M::rhs(yt, t + h0, p, f1);
    double d2 = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double sk = atol + rtol * fabs(y[s]);
      d2 = fmax(d2, fabs(f1[s] - f[s]) / sk);
    }
    d2 = d2 / h0;
    const double dm = fmax(d1v, d2);
    const double h1 = (dm <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : inv_root(dm / 0.01, 2);
    double hl = fmin(100.0 * h0, h1);
    if (!__builtin_isfinite(hl) || !(hl > 0.0)) hl = rest;
    if (!st.live) hl = __builtin_inf();
    st.h = wave_min(hl);
#pragma unroll
    for (int j = 0; j < kRows; ++j)
#pragma unroll
      for (int s = 0; s < S; ++s) st.D[j][s] = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) { st.D[0][s] = y[s]; st.D[1][s] = f[s] * st.h; }
  }
  const double hmin = 1e-14 * fmax(fabs(tend), fabs(t0)) + 1e-300;
  st.order = 1;
  st.neq = 0;
  st.lu_ok = false;
  st.fresh = false;
  st.any_swap = false;
  while (__ballot(st.live) != 0ull) {
    const int q = st.order;  // wave-uniform
    BdfAccepted acc;
    bool ok;
    switch (q) {
      case 1: ok = bdf_attempt<M, PMAX, 1>(pb, st, p, acc); break;
      case 2: ok = bdf_attempt<M, PMAX, 2>(pb, st, p, acc); break;
      case 3: ok = bdf_attempt<M, PMAX, 3>(pb, st, p, acc); break;
      case 4: ok = bdf_attempt<M, PMAX, 4>(pb, st, p, acc); break;
      default: ok = bdf_attempt<M, PMAX, 5>(pb, st, p, acc); break;
    }
    if (ok) {
      bdf_output<S, TRAJ, NT>(pb, st, q, acc.h, y, traj, W, w, active, a);
#if OE_BDF_WAVE_SELECT_TEMPLATED
      if (acc.select) {
        switch (q) {
          case 1: bdf_select_q<S, 1>(st, acc); break;
          case 2: bdf_select_q<S, 2>(st, acc); break;
          case 3: bdf_select_q<S, 3>(st, acc); break;
          case 4: bdf_select_q<S, 4>(st, acc); break;
          default: bdf_select_q<S, 5>(st, acc); break;
        }
      }
#else
      if (acc.select) bdf_select<S>(st, q, acc);
#endif
    }
    // budget: a lane that needs more than `budget` steps inside one output interval, or a
    // step below hmin, is abandoned (MAXSTEP, NaN for the rest of its grid)
    if (st.live && (st.nst >= budget || st.h < hmin)) {
      st.live = false;
      a.status |= ST_MAXSTEP;
      double yo[S];
#pragma unroll
      for (int s = 0; s < S; ++s) yo[s] = __builtin_nan("");
      for (; st.i < pb.T; ++st.i) emit_lane<S, TRAJ, NT>(pb, st.i, yo, traj, W, w, active, st.k, st.nxt, a);
#pragma unroll
      for (int s = 0; s < S; ++s) y[s] = yo[s];
    }
  }
  if (part) check_finite(y, a);
}

}  // namespace oe
