// stiff_wave.cuh — the stiff redo of models wider than the register path (S > kStiffRegS)
// with ONE WAVE PER WALKER: lane r holds row r of the RODAS iteration matrix (then of its
// LU factors) and element r of every state vector, so a 20-state walker's 400-entry
// matrix is 20 doubles per lane in registers instead of 3.2 KB of private memory per lane
// (integrate_rosenbrock_big, ~17-20x slower than the register path per stiff walker:
// its per-wave working set lives in L2).
//
//   * vector updates (stage sums, error terms, dense output) are one lane-parallel
//     instruction each; the right-hand side is evaluated on the wave-uniform state
//     (gathered with v_readlane) and each lane keeps its own component;
//   * the Jacobian: lane j evaluates the model's RHS on one-tangent dual numbers seeded
//     at y_j (lane S at t), i.e. column j, and an LDS transpose hands row r to lane r —
//     every entry bitwise the (S+1)-tangent evaluation's;
//   * LU (right-looking, threshold partial pivoting exactly as ros::lu_factor): row k is
//     broadcast by v_readlane and the lanes below it eliminate in parallel; the pivot
//     search scans the gathered column in the register path's order;
//   * triangular solves: forward substitution lane-parallel (each b_i receives its
//     updates in k order, as the sequential loop), backward substitution as the
//     sequential row dot products (ascending j) on broadcast finalised values.
// The arithmetic is ros:: operation for operation; only the step size is the walker's
// own (no wave-shared h: one walker per wave).  The C restatement (oracle/rk_ref.c)
// redoes S > 8 walkers one per group to match.
#pragma once

namespace oe {

__device__ __forceinline__ double lane_bcast(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

template <int S>
__device__ __forceinline__ void gather_vec(double v, double (&u)[S]) {
#pragma unroll
  for (int s = 0; s < S; ++s) u[s] = lane_bcast(v, s);
}

// u[ln] for this lane's index ln (0 for ln >= S)
template <int S>
__device__ __forceinline__ double lane_pick(const double (&u)[S], int ln) {
  double v = 0.0;
#pragma unroll
  for (int s = 0; s < S; ++s) v = (s == ln) ? u[s] : v;
  return v;
}

namespace ros {

// LU of the row-distributed matrix a (lane r: row r) with ros::lu_factor's pivoting rule
template <int S>
__device__ __forceinline__ bool lu_factor_wave(double (&a)[S], int (&piv)[S], double (&dinv)[S], int ln) {
  bool any_swap = false;
#pragma unroll
  for (int k = 0; k < S; ++k) {
    piv[k] = k;
    if (k + 1 < S) {
      double col[S];
#pragma unroll
      for (int i = k; i < S; ++i) col[i] = lane_bcast(a[k], i);
      double colmax = 0.0;
#pragma unroll
      for (int i = k + 1; i < S; ++i) colmax = fmax(colmax, fabs(col[i]));
      const bool need = fabs(col[k]) < kPivotThreshold * colmax;
      if (need) {  // wave-uniform
        any_swap = true;
        int pk = k;
        double best = fabs(col[k]);
#pragma unroll
        for (int i = k + 1; i < S; ++i) {
          const double v = fabs(col[i]);
          if (v > best) { best = v; pk = i; }
        }
        piv[k] = pk;
        if (pk != k) {
#pragma unroll
          for (int c = 0; c < S; ++c) {
            const double rk = lane_bcast(a[c], k), rp = lane_bcast(a[c], pk);
            a[c] = (ln == k) ? rp : (ln == pk) ? rk : a[c];
          }
        }
      }
    }
    const double akk = lane_bcast(a[k], k);
    const double inv = 1.0 / akk;
    dinv[k] = inv;
    double rowk[S];
#pragma unroll
    for (int c = k + 1; c < S; ++c) rowk[c] = lane_bcast(a[c], k);
    if (ln > k && ln < S) {
      const double l = a[k] * inv;
      a[k] = l;
#pragma unroll
      for (int c = k + 1; c < S; ++c) a[c] = fma(-l, rowk[c], a[c]);
    }
  }
  return any_swap;
}

// solve (LU) x = P b for the lane-distributed b (lane i: b_i), in place
template <int S>
__device__ __forceinline__ void lu_solve_wave(const double (&a)[S], const int (&piv)[S], const double (&dinv)[S],
                                              bool any_swap, double& b, int ln) {
  if (any_swap) {
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const int pk = piv[k];
      if (pk != k) {
        const double bk = lane_bcast(b, k), bp = lane_bcast(b, pk);
        b = (ln == k) ? bp : (ln == pk) ? bk : b;
      }
    }
  }
#pragma unroll
  for (int k = 0; k + 1 < S; ++k) {
    const double bk = lane_bcast(b, k);
    if (ln > k) b = fma(-a[k], bk, b);
  }
  double xf[S];
#pragma unroll
  for (int k = S - 1; k >= 0; --k) {
    double x = b;  // lane k's row; the other lanes' results are discarded
#pragma unroll
    for (int j = k + 1; j < S; ++j) x = fma(-a[j], xf[j], x);
    xf[k] = lane_bcast(x * dinv[k], k);
  }
  b = lane_pick(xf, ln);
}
}  // namespace ros

// right-hand side of the lane-distributed state x at time t: this lane's component
template <class M, int PMAX>
__device__ __forceinline__ double rhs_wave(double x, double t, const double (&p)[PMAX], int ln) {
  constexpr int S = M::S;
  double xu[S], fu[S];
  gather_vec<S>(x, xu);
  M::rhs(xu, t, p, fu);
  return lane_pick(fu, ln);
}

// f, this lane's Jacobian row and ∂f/∂t component at the lane-distributed y
template <class M, int PMAX>
__device__ __forceinline__ void jac_wave(double y, double t, const double (&p)[PMAX], int ln, double* lds,
                                         double& f, double (&Jrow)[M::S], double& ft) {
  constexpr int S = M::S;
  using D = Dual<1>;
  double yu[S];
  gather_vec<S>(y, yu);
  D yd[S], pd[PMAX], fd[S];
#pragma unroll
  for (int s = 0; s < S; ++s) { yd[s] = D(yu[s]); yd[s].d[0] = (s == ln) ? 1.0 : 0.0; }
  D td(t);
  td.d[0] = (ln == S) ? 1.0 : 0.0;
#pragma unroll
  for (int q = 0; q < PMAX; ++q) pd[q] = D(p[q]);
  M::rhs(yd, td, pd, fd);
  // lane j <= S holds column j (∂f/∂y_j, or ∂f/∂t for j = S): transpose through LDS
  if (ln <= S) {
#pragma unroll
    for (int r = 0; r < S; ++r) lds[r * (S + 1) + ln] = fd[r].d[0];
  }
  __syncthreads();
  if (ln < S) {
#pragma unroll
    for (int c = 0; c < S; ++c) Jrow[c] = lds[ln * (S + 1) + c];
    ft = lds[ln * (S + 1) + S];
  }
  __syncthreads();
  double fu[S];
#pragma unroll
  for (int s = 0; s < S; ++s) fu[s] = fd[s].v;
  f = lane_pick(fu, ln);
}

// one trajectory row / observation step for the lane-distributed state yo (grid index i)
template <int S, bool TRAJ, bool NT>
__device__ __forceinline__ void emit_wave(const DevProblem& pb, int i, double yo, double* traj, int64_t W, int64_t w,
                                          int ln, int& k, Acc& a) {
  if constexpr (TRAJ) {
    if (ln < S) traj[((int64_t)i * S + ln) * W + w] = yo;
  }
  double yu[S];
  gather_vec<S>(yo, yu);
  track_min<S>(yu, a);
  observe<S>(pb, i, yu, k, a);
}

// RODAS integration of walker w by the whole wave (every lane runs it; the accumulator
// is wave-uniform).  y: this lane's initial state component.
template <class M, int PMAX, bool TRAJ, bool NT>
__device__ __forceinline__ void rosenbrock_walker_wave(const DevProblem& pb, double y, const double (&p)[PMAX],
                                                       double* traj, int64_t W, int64_t w, int ln, double* lds,
                                                       Acc& a) {
  using namespace ros;
  constexpr int S = M::S;
  const cptr<double> times = kconst(pb.times);
  const double t0 = times[0], tend = times[pb.T - 1];
  const double rtol = pb.rtol, atol = pb.atol;
  bool dead = false;
  int k = 0;
  emit_wave<S, TRAJ, NT>(pb, 0, y, traj, W, w, ln, k, a);
  double t = t0;
  double f0 = 0.0, ft = 0.0, J[S];
#pragma unroll
  for (int c = 0; c < S; ++c) J[c] = 0.0;
  jac_wave<M, PMAX>(y, t, p, ln, lds, f0, J, ft);

  double h;
  {
    double yu[S], fu[S];
    gather_vec<S>(y, yu);
    gather_vec<S>(f0, fu);
    double d0 = 0.0, d1v = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double sk = atol + rtol * fabs(yu[s]);
      d0 = fmax(d0, fabs(yu[s]) / sk);
      d1v = fmax(d1v, fabs(fu[s]) / sk);
    }
    double h0 = (d0 <= 1e-5 || d1v <= 1e-5) ? 1e-6 : 0.01 * (d0 / d1v);
    h0 = fmin(h0, tend - t0);
    const double f1 = rhs_wave<M, PMAX>(fma(h0, f0, y), t + h0, p, ln);
    double f1u[S];
    gather_vec<S>(f1, f1u);
    double d2 = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double sk = atol + rtol * fabs(yu[s]);
      d2 = fmax(d2, fabs(f1u[s] - fu[s]) / sk);
    }
    d2 = d2 / h0;
    const double dm = fmax(d1v, d2);
    const double h1 = (dm <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : inv_fourth_root(dm / 0.01);
    double hl = fmin(100.0 * h0, h1);
    if (!__builtin_isfinite(hl) || !(hl > 0.0)) hl = tend - t0;
    h = fmin(hl, tend - t0);
  }
  const double hmin = 1e-14 * fmax(fabs(tend), fabs(t0)) + 1e-300;
  const int budget = kRosBudget * pb.max_steps;
  int i = 1, nst = 0;
  bool last_rej = false;
  while (i < pb.T) {
    bool last = false;
    if (t + h >= tend) { h = tend - t; last = true; }
    const double rh = 1.0 / h;
    const double gh = rh * inv_gam;
    const double c21h = c21 * rh, c31h = c31 * rh, c32h = c32 * rh, c41h = c41 * rh, c42h = c42 * rh,
                 c43h = c43 * rh, c51h = c51 * rh, c52h = c52 * rh, c53h = c53 * rh, c54h = c54 * rh,
                 c61h = c61 * rh, c62h = c62 * rh, c63h = c63 * rh, c64h = c64 * rh, c65h = c65 * rh;
    const double hd1 = h * d1, hd2 = h * d2, hd3 = h * d3, hd4 = h * d4;
    double lu[S], dinv[S];
    int piv[S];
#pragma unroll
    for (int c = 0; c < S; ++c) lu[c] = (c == ln) ? gh - J[c] : -J[c];
    const bool any_swap = lu_factor_wave<S>(lu, piv, dinv, ln);
    double k1 = fma(hd1, ft, f0);
    lu_solve_wave<S>(lu, piv, dinv, any_swap, k1, ln);
    double yt = fma(a21, k1, y);
    double fv = rhs_wave<M, PMAX>(yt, t + c2x * h, p, ln);
    double k2 = fma(hd2, ft, fma(c21h, k1, fv));
    lu_solve_wave<S>(lu, piv, dinv, any_swap, k2, ln);
    yt = fma(a32, k2, fma(a31, k1, y));
    fv = rhs_wave<M, PMAX>(yt, t + c3x * h, p, ln);
    double k3 = fma(hd3, ft, fma(c32h, k2, fma(c31h, k1, fv)));
    lu_solve_wave<S>(lu, piv, dinv, any_swap, k3, ln);
    yt = fma(a43, k3, fma(a42, k2, fma(a41, k1, y)));
    fv = rhs_wave<M, PMAX>(yt, t + c4x * h, p, ln);
    double k4 = fma(hd4, ft, fma(c43h, k3, fma(c42h, k2, fma(c41h, k1, fv))));
    lu_solve_wave<S>(lu, piv, dinv, any_swap, k4, ln);
    yt = fma(a54, k4, fma(a53, k3, fma(a52, k2, fma(a51, k1, y))));
    fv = rhs_wave<M, PMAX>(yt, t + h, p, ln);
    double k5 = fma(c54h, k4, fma(c53h, k3, fma(c52h, k2, fma(c51h, k1, fv))));
    lu_solve_wave<S>(lu, piv, dinv, any_swap, k5, ln);
    yt = yt + k5;  // the embedded solution
    fv = rhs_wave<M, PMAX>(yt, t + h, p, ln);
    double k6 = fma(c65h, k5, fma(c64h, k4, fma(c63h, k3, fma(c62h, k2, fma(c61h, k1, fv)))));
    lu_solve_wave<S>(lu, piv, dinv, any_swap, k6, ln);
    const double y1 = yt + k6;
    // error norm: the register path's sequential argmax over the gathered components
    double aeu[S], sku[S], y1u[S];
    gather_vec<S>(fabs(k6), aeu);
    gather_vec<S>(fma(rtol, max_abs_raw(y, y1), atol), sku);
    gather_vec<S>(y1, y1u);
    double num = 0.0, den = 1.0, nfe = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      nfe = fma(aeu[s], 0.0, nfe);
      nfe = fma(y1u[s], 0.0, nfe);
      if (s == 0 || aeu[s] * den > num * sku[s]) { num = aeu[s]; den = sku[s]; }
    }
    double el = num / den;
    if (!__builtin_isfinite(el) || __builtin_isnan(nfe)) el = 1e30;
    if (dead) el = 0.0;
    const double err = el;
    ++nst;
    if (err <= 1.0) {
      const double tn = last ? tend : t + h;
      if (i < pb.T && times[i] < tn) {  // a grid point inside the step
        const double q3 = fma(h25, k5, fma(h24, k4, fma(h23, k3, fma(h22, k2, h21 * k1))));
        const double q4 = fma(h35, k5, fma(h34, k4, fma(h33, k3, fma(h32, k2, h31 * k1))));
        while (i < pb.T && times[i] < tn) {
          if (grid_needs_emit<S, TRAJ>(pb, i, k)) {
            const double th = (times[i] - t) * rh;
            const double th1 = 1.0 - th;
            const double yo = fma(th, fma(th1, fma(th, q4, q3), y1), th1 * y);
            emit_wave<S, TRAJ, NT>(pb, i, yo, traj, W, w, ln, k, a);
          }
          ++i;
          nst = 0;
        }
      }
      y = y1;
      t = tn;
      if (i < pb.T && times[i] == tn) {  // a grid point on the step's end
        if (grid_needs_emit<S, TRAJ>(pb, i, k)) emit_wave<S, TRAJ, NT>(pb, i, y, traj, W, w, ln, k, a);
        ++i;
        nst = 0;
      }
      if (i < pb.T) jac_wave<M, PMAX>(y, t, p, ln, lds, f0, J, ft);
      double fac = (err > 0.0) ? safe * inv_fourth_root(err) : facmax;
      fac = fmin(facmax, fmax(facmin, fac));
      if (last_rej) fac = fmin(fac, 1.0);
      h = h * fac;
      last_rej = false;
    } else {
      h = h * fmax(facmin, safe * inv_fourth_root(err));
      last_rej = true;
    }
    if (i < pb.T && (nst >= budget || h < hmin)) {  // (not after the last grid point)
      // the walker pins its own step: evicted (status MAXSTEP, NaN output from here on)
      dead = true;
      a.status |= ST_MAXSTEP;
      y = __builtin_nan("");
      for (; i < pb.T; ++i)
        if (grid_needs_emit<S, TRAJ>(pb, i, k)) emit_wave<S, TRAJ, NT>(pb, i, y, traj, W, w, ln, k, a);
      break;
    }
  }
  double yu[S];
  gather_vec<S>(y, yu);
  check_finite(yu, a);
}

// ---------------------------------------------------------------------------------
// Kernel: the stiff walkers of an 'auto' pass (status bit ST_STIFF set by the DOPRI5
// kernel) or every walker ('rosenbrock'), one 64-thread workgroup per walker, in a
// grid-stride loop over the walker ids (count read on the device: no host round trip;
// every wave reaches the loop's end).
// ---------------------------------------------------------------------------------
struct StiffWaveArgs {
  const double* y0;     // [S][W]
  const double* theta;  // [P][W]
  double* traj;         // [T][S][W] or null
  double* chi;          // [W] or null
  double* ssres;        // [W] or null
  int32_t* status;      // [W] (required: carries the ST_STIFF marks of the 'auto' pass)
  const int32_t* list;  // walker ids to redo (null: every walker, count = W)
  const int32_t* count; // number of ids in list (device)
  int64_t W;
};

template <class M, bool TRAJ, bool NT>
__global__ void __launch_bounds__(64) k_stiff_wave(const DevProblem pb, const StiffWaveArgs sa) {
  constexpr int S = M::S;
  constexpr int PMAX = kPmax<M>;
  static_assert(S < 64, "one lane per state (and one for the time tangent)");
  __shared__ double lds[S * (S + 1)];
  const int ln = threadIdx.x & 63;
  const int64_t n = sa.list ? (int64_t)*kconst(sa.count) : sa.W;
  for (int64_t j = blockIdx.x; j < n; j += gridDim.x) {
    const int64_t w = sa.list ? (int64_t)sa.list[j] : j;
    const int64_t W = sa.W;
    double p[PMAX];
#pragma unroll
    for (int q = 0; q < PMAX; ++q) p[q] = (q < pb.P) ? sa.theta[(int64_t)q * W + w] : 0.0;
    const double y = (ln < S) ? sa.y0[(int64_t)ln * W + w] : 0.0;
    Acc a = acc_init();
    a.status = sa.list ? ST_STIFF : 0;
    rosenbrock_walker_wave<M, PMAX, TRAJ, NT>(pb, y, p, sa.traj, W, w, ln, lds, a);
    if (ln == 0) {
      if (sa.chi) sa.chi[w] = a.nvalid ? a.chi : __builtin_nan("");
      if (sa.ssres) sa.ssres[w] = a.ssres;
      sa.status[w] = finish(a);
    }
  }
}

}  // namespace oe
