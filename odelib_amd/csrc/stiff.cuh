// stiff.cuh — the stiff half of odeint's LSODA (Framework.py:656) on the device.
//
// LSODA integrates with Adams methods and switches to BDF when it detects stiffness.
// Here the non-stiff integrator is the wave-lockstep DOPRI5 (ode_kernels.cuh); the
// stiff integrator is the stiffly accurate Rosenbrock method RODAS of order 4 with an
// L-stable embedded order-3 error estimate and an order-3 continuous extension (Hairer &
// Wanner, Solving ODEs II, §VI.4; γ = 0.25, 6 stages, 5 RHS evaluations per step).  The method
// 'auto' (OE_METHOD_AUTO) runs DOPRI5 with Hairer's per-lane stiffness test
// (h·|λ| ≥ 3.25 on 15 accepted steps in a row) and evicts stiff lanes — and lanes over
// the step budget — from the wave; those walkers are then integrated again from t0 by
// the Rosenbrock method, still one lane per walker and one step size per wave.
//
//   * Jacobian: exact, by forward-mode dual numbers through the model's own templated
//     RHS (built-in models and hipRTC user models alike): J = ∂f/∂y and ∂f/∂t in one
//     evaluation with S + 1 tangents, value part bitwise equal to the plain RHS.
//   * Linear algebra: (1/(γh) I − J) is factored per lane in registers (LU with threshold
//     partial pivoting; row swaps by selects, so nothing is indexed by a per-lane value,
//     skipped by a wave none of whose lanes needs them).
//   * Output: the method's own continuous extension (from the stage increments, valid on
//     stiff components, unlike Hermite interpolation from f) for grid times inside a
//     step; a grid time on a step's end takes the new state.
//   * Step control: max-norm error as DOPRI5, fac = 0.9·err^(−1/4) in [0.2, 6], wave
//     maximum over the participating lanes; eviction as DOPRI5, with a step budget of
//     kRosBudget × max_steps per output interval.
// Everything is IEEE add/mul/fma/div plus frexp/ldexp, restated operation for operation
// in oracle/rk_ref.c, so the kernel is bitwise testable.
#pragma once

namespace oe {

// ---- forward-mode dual numbers (value + N tangents) ---------------------------------
// Hidden friends only: found by argument-dependent lookup when a Dual is involved, so
// they never shadow the double overloads of fma/exp/... used everywhere else.
// Mixed operations promote the double to a Dual with zero tangents and apply the same
// formula (the oracle does the same, so the tangent bits agree).
template <int N>
struct Dual {
  double v;
  double d[N];
  __host__ __device__ Dual() {}
  __host__ __device__ Dual(double x) : v(x) {  // implicit: constants in model code
#pragma unroll
    for (int i = 0; i < N; ++i) d[i] = 0.0;
  }
#define OE_D_LOOP _Pragma("unroll") for (int i = 0; i < N; ++i)
  friend __host__ __device__ inline Dual operator-(const Dual& a) {
    Dual r; r.v = -a.v;
    OE_D_LOOP r.d[i] = -a.d[i];
    return r;
  }
  friend __host__ __device__ inline Dual operator+(const Dual& a, const Dual& b) {
    Dual r; r.v = a.v + b.v;
    OE_D_LOOP r.d[i] = a.d[i] + b.d[i];
    return r;
  }
  friend __host__ __device__ inline Dual operator-(const Dual& a, const Dual& b) {
    Dual r; r.v = a.v - b.v;
    OE_D_LOOP r.d[i] = a.d[i] - b.d[i];
    return r;
  }
  friend __host__ __device__ inline Dual operator*(const Dual& a, const Dual& b) {
    Dual r; r.v = a.v * b.v;
    OE_D_LOOP r.d[i] = a.d[i] * b.v + a.v * b.d[i];
    return r;
  }
  friend __host__ __device__ inline Dual operator/(const Dual& a, const Dual& b) {
    Dual r; r.v = a.v / b.v;
    OE_D_LOOP r.d[i] = (a.d[i] - r.v * b.d[i]) / b.v;
    return r;
  }
  friend __host__ __device__ inline Dual fma(const Dual& a, const Dual& b, const Dual& c) {
    Dual r; r.v = ::fma(a.v, b.v, c.v);
    OE_D_LOOP r.d[i] = (a.d[i] * b.v + a.v * b.d[i]) + c.d[i];
    return r;
  }
#define OE_D_MIXED2(OP)                                                                            \
  friend __host__ __device__ inline Dual OP(const Dual& a, double b) { return OP(a, Dual(b)); }    \
  friend __host__ __device__ inline Dual OP(double a, const Dual& b) { return OP(Dual(a), b); }
  OE_D_MIXED2(operator+)
  OE_D_MIXED2(operator-)
  OE_D_MIXED2(operator*)
  OE_D_MIXED2(operator/)
  friend __host__ __device__ inline Dual fma(double a, const Dual& b, const Dual& c) { return fma(Dual(a), b, c); }
  friend __host__ __device__ inline Dual fma(const Dual& a, double b, const Dual& c) { return fma(a, Dual(b), c); }
  friend __host__ __device__ inline Dual fma(const Dual& a, const Dual& b, double c) { return fma(a, b, Dual(c)); }
  friend __host__ __device__ inline Dual fma(double a, double b, const Dual& c) { return fma(Dual(a), Dual(b), c); }
  friend __host__ __device__ inline Dual fma(double a, const Dual& b, double c) { return fma(Dual(a), b, Dual(c)); }
  friend __host__ __device__ inline Dual fma(const Dual& a, double b, double c) { return fma(a, Dual(b), Dual(c)); }
  __host__ __device__ Dual& operator+=(const Dual& b) { return *this = *this + b; }
  __host__ __device__ Dual& operator-=(const Dual& b) { return *this = *this - b; }
  __host__ __device__ Dual& operator*=(const Dual& b) { return *this = *this * b; }
  __host__ __device__ Dual& operator/=(const Dual& b) { return *this = *this / b; }
  // comparisons act on values (branches of user code)
#define OE_D_CMP(OP)                                                                                    \
  friend __host__ __device__ inline bool operator OP(const Dual& a, const Dual& b) { return a.v OP b.v; } \
  friend __host__ __device__ inline bool operator OP(const Dual& a, double b) { return a.v OP b; }        \
  friend __host__ __device__ inline bool operator OP(double a, const Dual& b) { return a OP b.v; }
  OE_D_CMP(<)
  OE_D_CMP(<=)
  OE_D_CMP(>)
  OE_D_CMP(>=)
  OE_D_CMP(==)
  OE_D_CMP(!=)
  // elementary functions: value, then tangent = f'(a.v) * a.d
  friend __host__ __device__ inline Dual chain_(const Dual& a, double fv, double dfv) {
    Dual r; r.v = fv;
    OE_D_LOOP r.d[i] = dfv * a.d[i];
    return r;
  }
  friend __host__ __device__ inline Dual exp(const Dual& a) { const double e = ::exp(a.v); return chain_(a, e, e); }
  friend __host__ __device__ inline Dual exp2(const Dual& a) {
    const double e = ::exp2(a.v);
    return chain_(a, e, e * 0.6931471805599453);
  }
  friend __host__ __device__ inline Dual expm1(const Dual& a) { return chain_(a, ::expm1(a.v), ::exp(a.v)); }
  friend __host__ __device__ inline Dual log(const Dual& a) { return chain_(a, ::log(a.v), 1.0 / a.v); }
  friend __host__ __device__ inline Dual log2(const Dual& a) { return chain_(a, ::log2(a.v), 1.0 / (a.v * 0.6931471805599453)); }
  friend __host__ __device__ inline Dual log10(const Dual& a) { return chain_(a, ::log10(a.v), 1.0 / (a.v * 2.302585092994046)); }
  friend __host__ __device__ inline Dual log1p(const Dual& a) { return chain_(a, ::log1p(a.v), 1.0 / (1.0 + a.v)); }
  friend __host__ __device__ inline Dual sqrt(const Dual& a) { const double s = ::sqrt(a.v); return chain_(a, s, 0.5 / s); }
  friend __host__ __device__ inline Dual sin(const Dual& a) { return chain_(a, ::sin(a.v), ::cos(a.v)); }
  friend __host__ __device__ inline Dual cos(const Dual& a) { return chain_(a, ::cos(a.v), -::sin(a.v)); }
  friend __host__ __device__ inline Dual tan(const Dual& a) {
    const double c = ::cos(a.v);
    return chain_(a, ::tan(a.v), 1.0 / (c * c));
  }
  friend __host__ __device__ inline Dual sinh(const Dual& a) { return chain_(a, ::sinh(a.v), ::cosh(a.v)); }
  friend __host__ __device__ inline Dual cosh(const Dual& a) { return chain_(a, ::cosh(a.v), ::sinh(a.v)); }
  friend __host__ __device__ inline Dual tanh(const Dual& a) {
    const double th = ::tanh(a.v);
    return chain_(a, th, 1.0 - th * th);
  }
  friend __host__ __device__ inline Dual atan(const Dual& a) { return chain_(a, ::atan(a.v), 1.0 / (1.0 + a.v * a.v)); }
  friend __host__ __device__ inline Dual fabs(const Dual& a) { return chain_(a, ::fabs(a.v), a.v < 0.0 ? -1.0 : 1.0); }
  friend __host__ __device__ inline Dual pow(const Dual& a, double b) {
    // constant exponent: d = b * a^(b-1) * da (finite for a <= 0 and integral b)
    return chain_(a, ::pow(a.v, b), b == 0.0 ? 0.0 : b * ::pow(a.v, b - 1.0));
  }
  // The exponent's tangent term a^b·log(a)·db is added only where db != 0: in jac_eval the
  // parameters are duals with zero tangents, and a base of 0 or below (a state starting at
  // 0 raised to a parameter power, y**p) has log(a) = -inf or NaN, so the product with a
  // zero tangent would be NaN and poison the whole Jacobian row.
  friend __host__ __device__ inline Dual pow(double a, const Dual& b) {
    Dual r; r.v = ::pow(a, b.v);
    const double dv = r.v * ::log(a);
    OE_D_LOOP r.d[i] = b.d[i] != 0.0 ? dv * b.d[i] : 0.0;
    return r;
  }
  friend __host__ __device__ inline Dual pow(const Dual& a, const Dual& b) {
    Dual r; r.v = ::pow(a.v, b.v);
    const double la = ::log(a.v), da = b.v * ::pow(a.v, b.v - 1.0);
    OE_D_LOOP r.d[i] = b.d[i] != 0.0 ? da * a.d[i] + (r.v * la) * b.d[i] : da * a.d[i];
    return r;
  }
  friend __host__ __device__ inline Dual fmax(const Dual& a, const Dual& b) { return (b.v > a.v || a.v != a.v) ? b : a; }
  friend __host__ __device__ inline Dual fmin(const Dual& a, const Dual& b) { return (b.v < a.v || a.v != a.v) ? b : a; }
  OE_D_MIXED2(fmax)
  OE_D_MIXED2(fmin)
#undef OE_D_MIXED2
#undef OE_D_CMP
#undef OE_D_LOOP
};

// f, ∂f/∂y (row s = ∂f_s) and ∂f/∂t at (t, y) in one dual evaluation of the model's RHS.
template <class M, int PMAX>
__device__ __forceinline__ void jac_eval(const double (&y)[M::S], double t, const double (&p)[PMAX],
                                         double (&f)[M::S], double (&J)[M::S][M::S], double (&ft)[M::S]) {
  constexpr int S = M::S;
  using D = Dual<S + 1>;
  D yd[S], pd[PMAX], fd[S];
#pragma unroll
  for (int s = 0; s < S; ++s) { yd[s] = D(y[s]); yd[s].d[s] = 1.0; }
  D td(t);
  td.d[S] = 1.0;
#pragma unroll
  for (int j = 0; j < PMAX; ++j) pd[j] = D(p[j]);
  M::rhs(yd, td, pd, fd);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    f[s] = fd[s].v;
#pragma unroll
    for (int j = 0; j < S; ++j) J[s][j] = fd[s].d[j];
    ft[s] = fd[s].d[S];
  }
}

// ---- RODAS (Hairer & Wanner II, §VI.4): Rosenbrock 4(3), 6 stages, stiffly accurate ----
// Both the solution and the embedded order-3 solution are L-stable, so the error
// estimate (the last stage increment k6) stays small on stiff components that sit on
// their slow manifold.  An order-4 method whose embedded estimate is not L-stable (the
// 4-stage ROS4 family used before) reads the O(ε) manifold offset of a fast component as
// error and takes ~8x the steps at odeint's tolerances (two_i with τ = 1e5: 14 200 steps
// vs 1 640).  Stages 5 and 6 are evaluated at t + h; the continuous
// extension (order 3) gives the grid points inside a step, so steps need not end on them.
namespace ros {
constexpr double gam = 0.25;
constexpr double inv_gam = 4.0;
constexpr double a21 = 1.544, a31 = 0.9466785280815826, a32 = 0.2557011698983284, a41 = 3.314825187068521,
                 a42 = 2.896124015972201, a43 = 0.9986419139977817, a51 = 1.221224509226641,
                 a52 = 6.019134481288629, a53 = 12.53708332932087, a54 = -0.687886036105895;
constexpr double c21 = -5.6688, c31 = -2.430093356833875, c32 = -0.2063599157091915, c41 = -0.1073529058151375,
                 c42 = -9.594562251023355, c43 = -20.47028614809616, c51 = 7.496443313967647,
                 c52 = -10.24680431464352, c53 = -33.99990352819905, c54 = 11.7089089320616,
                 c61 = 8.083246795921522, c62 = -7.981132988064893, c63 = -31.52159432874371,
                 c64 = 16.31930543123136, c65 = -6.058818238834054;
constexpr double c2x = 0.386, c3x = 0.21, c4x = 0.63;                      // stage times (α_i)
constexpr double d1 = 0.25, d2 = -0.1043, d3 = 0.1035, d4 = -0.03620000000000023;  // ∂f/∂t weights (γ_i)
constexpr double h21 = 10.12623508344586, h22 = -7.487995877610167, h23 = -34.80091861555747,
                 h24 = -7.992771707568823, h25 = 1.025137723295662;         // dense output
constexpr double h31 = -0.6762803392801253, h32 = 6.087714651680015, h33 = 16.43084320892478,
                 h34 = 24.76722511418386, h35 = -6.594389125716872;
constexpr double safe = 0.9, facmin = 0.2, facmax = 6.0;
constexpr int kRosBudget = 8;  // step budget per output interval, in units of max_steps

// x^(-1/4) for finite x > 0 from frexp/ldexp and IEEE mul/fma only (bit-identical in
// oracle/rk_ref.c): x = m·2^e, e = 4q + r; m^(-1/4) on [0.5, 1) from a quadratic start
// (2e-3) and three Newton steps y <- y·(5 − m·y^4)/4 (1e-5, 3e-10, 2e-16).
__device__ __forceinline__ double inv_fourth_root(double x) {
  int e;
  const double m = frexp(x, &e);
  int q = e / 4, r = e % 4;
  if (r < 0) { r += 4; q -= 1; }
  double y = fma(fma(0.3171, m, -0.8457), m, 1.5304);
#pragma unroll
  for (int it = 0; it < 3; ++it) {
    const double y2 = y * y;
    y = (y * fma(-m, y2 * y2, 5.0)) * 0.25;
  }
  constexpr double kC[4] = {1.0, 0.8408964152537145, 0.7071067811865476, 0.5946035575013605};
  return ldexp(dp::select_r(r, kC) * y, -q);
}

// LU with threshold partial pivoting: column k is pivoted only when |a_kk| < 0.1 x the
// largest |a_ik| below it, and then on the first maximum (full-row interchanges by
// selects).  (1/(γh))·I − J is nearly always diagonally dominant enough, so a wave skips
// the interchange work of a column (and the solves skip theirs) unless one of its lanes
// needs it: the selects cost ~40 % of a Rosenbrock step when done unconditionally.
constexpr double kPivotThreshold = 0.1;

template <int S>
__device__ __forceinline__ bool lu_factor(double (&a)[S][S], int (&piv)[S], double (&dinv)[S]) {
  bool any_swap = false;  // wave-uniform: some lane interchanged rows
#pragma unroll
  for (int k = 0; k < S; ++k) {
    piv[k] = k;
    if (k + 1 < S) {
      double colmax = 0.0;
#pragma unroll
      for (int i = k + 1; i < S; ++i) colmax = fmax(colmax, fabs(a[i][k]));
      const bool need = fabs(a[k][k]) < kPivotThreshold * colmax;
      if (__ballot(need) != 0ull) {
        any_swap = true;
        int pk = k;
        double best = fabs(a[k][k]);
#pragma unroll
        for (int i = k + 1; i < S; ++i) {
          const double v = fabs(a[i][k]);
          if (v > best) { best = v; pk = i; }
        }
        if (!need) pk = k;
        piv[k] = pk;
#pragma unroll
        for (int i = k + 1; i < S; ++i) {
          const bool sw = pk == i;
#pragma unroll
          for (int j = 0; j < S; ++j) {
            const double ak = a[k][j], ai = a[i][j];
            a[k][j] = sw ? ai : ak;
            a[i][j] = sw ? ak : ai;
          }
        }
      }
    }
    const double inv = 1.0 / a[k][k];
    dinv[k] = inv;
#pragma unroll
    for (int i = k + 1; i < S; ++i) {
      const double l = a[i][k] * inv;
      a[i][k] = l;
#pragma unroll
      for (int j = k + 1; j < S; ++j) a[i][j] = fma(-l, a[k][j], a[i][j]);
    }
  }
  return any_swap;
}

// solve (LU) x = P b in place: all interchanges (skipped when no lane of the wave made
// one), then L (unit) forward, U backward
template <int S>
__device__ __forceinline__ void lu_solve(const double (&a)[S][S], const int (&piv)[S], const double (&dinv)[S],
                                         bool any_swap, double (&b)[S]) {
  if (any_swap) {
#pragma unroll
    for (int k = 0; k < S; ++k) {
#pragma unroll
      for (int i = k + 1; i < S; ++i) {
        const bool sw = piv[k] == i;
        const double bk = b[k], bi = b[i];
        b[k] = sw ? bi : bk;
        b[i] = sw ? bk : bi;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < S; ++k)
#pragma unroll
    for (int i = k + 1; i < S; ++i) b[i] = fma(-a[i][k], b[k], b[i]);
#pragma unroll
  for (int k = S - 1; k >= 0; --k) {
    double x = b[k];
#pragma unroll
    for (int j = k + 1; j < S; ++j) x = fma(-a[k][j], b[j], x);
    b[k] = x * dinv[k];
  }
}
}  // namespace ros

// Rosenbrock (RODAS) integration of the lanes with `part` set (the others sit out: they
// neither steer the step size nor emit).  Wave-lockstep: one step size per wave; grid
// points inside a step come from the continuous extension, a grid point on the step's
// end is the new state itself.  y is the initial state on entry, the final on return.
template <class M, int PMAX, bool TRAJ, bool NT>
__device__ __forceinline__ void integrate_rosenbrock(const DevProblem& pb, double (&y)[M::S],
                                                     const double (&p)[PMAX], double* traj, int64_t W,
                                                     uint32_t off, bool active, bool part, Acc& a) {
  using namespace ros;
  constexpr int S = M::S;
  const cptr<double> times = kconst(pb.times);
  const double t0 = times[0], tend = times[pb.T - 1];
  const double rtol = pb.rtol, atol = pb.atol;
  const bool emit_ok = active && part;
  bool dead = !part;
  int k = 0;
  if (part) emit<S, TRAJ, NT>(pb, 0, y, traj, W, off, emit_ok, k, a);
  double t = t0;
  double f0[S], J[S][S], ft[S];
  jac_eval<M, PMAX>(y, t, p, f0, J, ft);

  // initial step: Hairer's HINIT for order 4 (max norm), wave minimum
  double h;
  {
    double d0 = 0.0, d1v = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double sk = atol + rtol * fabs(y[s]);
      d0 = fmax(d0, fabs(y[s]) / sk);
      d1v = fmax(d1v, fabs(f0[s]) / sk);
    }
    double h0 = (d0 <= 1e-5 || d1v <= 1e-5) ? 1e-6 : 0.01 * (d0 / d1v);
    h0 = fmin(h0, tend - t0);
    double yt[S], f1[S];
#pragma unroll
    for (int s = 0; s < S; ++s) yt[s] = fma(h0, f0[s], y[s]);
    M::rhs(yt, t + h0, p, f1);
    double d2 = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double sk = atol + rtol * fabs(y[s]);
      d2 = fmax(d2, fabs(f1[s] - f0[s]) / sk);
    }
    d2 = d2 / h0;
    const double dm = fmax(d1v, d2);
    const double h1 = (dm <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : inv_fourth_root(dm / 0.01);
    double hl = fmin(100.0 * h0, h1);
    if (dead || !__builtin_isfinite(hl) || !(hl > 0.0)) hl = tend - t0;
    h = wave_min(hl);
    h = fmin(h, tend - t0);
  }
  const double span = tend - t0;
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
    double lu[S][S], dinv[S];
    int piv[S];
#pragma unroll
    for (int r = 0; r < S; ++r)
#pragma unroll
      for (int c = 0; c < S; ++c) lu[r][c] = (r == c) ? gh - J[r][c] : -J[r][c];
    const bool any_swap = lu_factor<S>(lu, piv, dinv);
    double k1[S], k2[S], k3[S], k4[S], k5[S], k6[S], yt[S], fv[S];
#pragma unroll
    for (int s = 0; s < S; ++s) k1[s] = fma(hd1, ft[s], f0[s]);
    lu_solve<S>(lu, piv, dinv, any_swap, k1);
#pragma unroll
    for (int s = 0; s < S; ++s) yt[s] = fma(a21, k1[s], y[s]);
    M::rhs(yt, t + c2x * h, p, fv);
#pragma unroll
    for (int s = 0; s < S; ++s) k2[s] = fma(hd2, ft[s], fma(c21h, k1[s], fv[s]));
    lu_solve<S>(lu, piv, dinv, any_swap, k2);
#pragma unroll
    for (int s = 0; s < S; ++s) yt[s] = fma(a32, k2[s], fma(a31, k1[s], y[s]));
    M::rhs(yt, t + c3x * h, p, fv);
#pragma unroll
    for (int s = 0; s < S; ++s) k3[s] = fma(hd3, ft[s], fma(c32h, k2[s], fma(c31h, k1[s], fv[s])));
    lu_solve<S>(lu, piv, dinv, any_swap, k3);
#pragma unroll
    for (int s = 0; s < S; ++s) yt[s] = fma(a43, k3[s], fma(a42, k2[s], fma(a41, k1[s], y[s])));
    M::rhs(yt, t + c4x * h, p, fv);
#pragma unroll
    for (int s = 0; s < S; ++s) k4[s] = fma(hd4, ft[s], fma(c43h, k3[s], fma(c42h, k2[s], fma(c41h, k1[s], fv[s]))));
    lu_solve<S>(lu, piv, dinv, any_swap, k4);
#pragma unroll
    for (int s = 0; s < S; ++s) yt[s] = fma(a54, k4[s], fma(a53, k3[s], fma(a52, k2[s], fma(a51, k1[s], y[s]))));
    M::rhs(yt, t + h, p, fv);
#pragma unroll
    for (int s = 0; s < S; ++s) k5[s] = fma(c54h, k4[s], fma(c53h, k3[s], fma(c52h, k2[s], fma(c51h, k1[s], fv[s]))));
    lu_solve<S>(lu, piv, dinv, any_swap, k5);
#pragma unroll
    for (int s = 0; s < S; ++s) yt[s] = yt[s] + k5[s];  // the embedded solution
    M::rhs(yt, t + h, p, fv);
#pragma unroll
    for (int s = 0; s < S; ++s)
      k6[s] = fma(c65h, k5[s], fma(c64h, k4[s], fma(c63h, k3[s], fma(c62h, k2[s], fma(c61h, k1[s], fv[s])))));
    lu_solve<S>(lu, piv, dinv, any_swap, k6);
    double y1[S];
    double num = 0.0, den = 1.0, nfe = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      y1[s] = yt[s] + k6[s];
      const double ae = fabs(k6[s]);  // solution minus embedded solution
      const double sk = fma(rtol, max_abs_raw(y[s], y1[s]), atol);
      nfe = fma(ae, 0.0, nfe);
      nfe = fma(y1[s], 0.0, nfe);
      if (s == 0 || ae * den > num * sk) { num = ae; den = sk; }
    }
    double el = num / den;
    if (!__builtin_isfinite(el) || __builtin_isnan(nfe)) el = 1e30;
    if (dead) el = 0.0;
    const double err = wave_max(el);
    ++nst;
    if (err <= 1.0) {
      const double tn = last ? tend : t + h;
      if (i < pb.T && times[i] < tn) {  // wave-uniform: a grid point inside the step
        double q3[S], q4[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
          q3[s] = fma(h25, k5[s], fma(h24, k4[s], fma(h23, k3[s], fma(h22, k2[s], h21 * k1[s]))));
          q4[s] = fma(h35, k5[s], fma(h34, k4[s], fma(h33, k3[s], fma(h32, k2[s], h31 * k1[s]))));
        }
        while (i < pb.T && times[i] < tn) {
          if (part && grid_needs_emit<S, TRAJ>(pb, i, k)) {
            const double th = (times[i] - t) * rh;
            const double th1 = 1.0 - th;
            double yo[S];
#pragma unroll
            for (int s = 0; s < S; ++s) yo[s] = fma(th, fma(th1, fma(th, q4[s], q3[s]), y1[s]), th1 * y[s]);
            emit<S, TRAJ, NT>(pb, i, yo, traj, W, off, emit_ok, k, a);
          }
          ++i;
          nst = 0;
        }
      }
#pragma unroll
      for (int s = 0; s < S; ++s) y[s] = part ? y1[s] : y[s];  // bystanders keep their state
      t = tn;
      if (i < pb.T && times[i] == tn) {  // a grid point on the step's end
        if (part && grid_needs_emit<S, TRAJ>(pb, i, k)) emit<S, TRAJ, NT>(pb, i, y, traj, W, off, emit_ok, k, a);
        ++i;
        nst = 0;
      }
      if (i < pb.T) jac_eval<M, PMAX>(y, t, p, f0, J, ft);
      double fac = (err > 0.0) ? safe * inv_fourth_root(err) : facmax;
      fac = fmin(facmax, fmax(facmin, fac));
      if (last_rej) fac = fmin(fac, 1.0);
      h = h * fac;
      last_rej = false;
    } else {
      h = h * fmax(facmin, safe * inv_fourth_root(err));
      last_rej = true;
    }
    // ---- budget: evict the walkers that pin the wave's step (as DOPRI5) ----
    if (i < pb.T && (nst >= budget || h < hmin)) {  // (not after the last grid point)
      if (!dead && el >= 0.5 * err) {
        dead = true;
        a.status |= ST_MAXSTEP;
#pragma unroll
        for (int s = 0; s < S; ++s) y[s] = __builtin_nan("");
      }
      nst = budget / 2;
      if (__ballot(!dead) == 0ull) {
        double yo[S];
#pragma unroll
        for (int s = 0; s < S; ++s) yo[s] = __builtin_nan("");
        for (; i < pb.T; ++i)
          if (part && grid_needs_emit<S, TRAJ>(pb, i, k)) emit<S, TRAJ, NT>(pb, i, yo, traj, W, off, emit_ok, k, a);
        break;
      }
      if (h < hmin) h = fmin(1e-3 * span, tend - t);
    }
  }
  if (part) check_finite(y, a);
}


// ---- S > kStiffRegS: the same RODAS integration with its matrices in private memory ----
// (1/(γh))·I − J at S = 20 is 400 doubles per lane, and J another 400: beyond the VGPR
// file, so the wide models keep J, the LU factors and the stage vectors in private
// (scratch) memory, indexed at run time in non-unrolled loops — the rare stiff walkers of
// a wide model pay memory traffic instead of every kernel paying registers.  The
// arithmetic is the register version's, operation for operation (the row interchanges
// move rows instead of selecting, the same data movement), so the C restatement covers
// both.  The Jacobian is taken column by column with one-tangent dual numbers: each
// tangent of Dual<S+1> is computed by the same operations whatever the other tangents
// hold, so every entry is bitwise the one the (S+1)-tangent evaluation gives.
template <class M, int PMAX>
__device__ __forceinline__ void jac_eval_cols(const double (&y)[M::S], double t, const double (&p)[PMAX],
                                              double (&f)[M::S], double (&J)[M::S * M::S], double (&ft)[M::S]) {
  constexpr int S = M::S;
  using D = Dual<1>;
#pragma unroll 1
  for (int j = 0; j <= S; ++j) {
    D yd[S], pd[PMAX], fd[S];
#pragma unroll
    for (int s = 0; s < S; ++s) { yd[s] = D(y[s]); yd[s].d[0] = (s == j) ? 1.0 : 0.0; }
    D td(t);
    td.d[0] = (j == S) ? 1.0 : 0.0;
#pragma unroll
    for (int q = 0; q < PMAX; ++q) pd[q] = D(p[q]);
    M::rhs(yd, td, pd, fd);
    if (j < S) {
#pragma unroll
      for (int s = 0; s < S; ++s) J[s * S + j] = fd[s].d[0];
    } else {
#pragma unroll
      for (int s = 0; s < S; ++s) { ft[s] = fd[s].d[0]; f[s] = fd[s].v; }
    }
  }
}

namespace ros {
template <int S>
__device__ __forceinline__ bool lu_factor_big(double (&a)[S * S], int (&piv)[S], double (&dinv)[S]) {
  bool any_swap = false;
#pragma unroll 1
  for (int k = 0; k < S; ++k) {
    piv[k] = k;
    if (k + 1 < S) {
      double colmax = 0.0;
#pragma unroll 1
      for (int i = k + 1; i < S; ++i) colmax = fmax(colmax, fabs(a[i * S + k]));
      const bool need = fabs(a[k * S + k]) < kPivotThreshold * colmax;
      if (__ballot(need) != 0ull) {
        any_swap = true;
        int pk = k;
        double best = fabs(a[k * S + k]);
#pragma unroll 1
        for (int i = k + 1; i < S; ++i) {
          const double v = fabs(a[i * S + k]);
          if (v > best) { best = v; pk = i; }
        }
        if (!need) pk = k;
        piv[k] = pk;
        if (pk != k) {
#pragma unroll 1
          for (int j = 0; j < S; ++j) {
            const double ak = a[k * S + j];
            a[k * S + j] = a[pk * S + j];
            a[pk * S + j] = ak;
          }
        }
      }
    }
    const double inv = 1.0 / a[k * S + k];
    dinv[k] = inv;
#pragma unroll 1
    for (int i = k + 1; i < S; ++i) {
      const double l = a[i * S + k] * inv;
      a[i * S + k] = l;
#pragma unroll 1
      for (int j = k + 1; j < S; ++j) a[i * S + j] = fma(-l, a[k * S + j], a[i * S + j]);
    }
  }
  return any_swap;
}

template <int S>
__device__ __forceinline__ void lu_solve_big(const double (&a)[S * S], const int (&piv)[S], const double (&dinv)[S],
                                             bool any_swap, double (&b)[S]) {
  if (any_swap) {
#pragma unroll 1
    for (int k = 0; k < S; ++k) {
      const int pk = piv[k];
      if (pk != k) {
        const double bk = b[k];
        b[k] = b[pk];
        b[pk] = bk;
      }
    }
  }
#pragma unroll 1
  for (int k = 0; k < S; ++k) {
    const double bk = b[k];
#pragma unroll 1
    for (int i = k + 1; i < S; ++i) b[i] = fma(-a[i * S + k], bk, b[i]);
  }
#pragma unroll 1
  for (int k = S - 1; k >= 0; --k) {
    double x = b[k];
#pragma unroll 1
    for (int j = k + 1; j < S; ++j) x = fma(-a[k * S + j], b[j], x);
    b[k] = x * dinv[k];
  }
}
}  // namespace ros

// Called on copies of the caller's state, parameters and accumulators: the run-time
// indexed arrays live in private memory, the caller's own stay in registers.  (Out of
// line it measured slower in MH: chain10 'auto' 2.44 vs 2.09 ms per iteration at 262 144
// walkers; profiles/r02zh_*.)
template <class M, int PMAX, bool TRAJ, bool NT>
__device__ __forceinline__ void integrate_rosenbrock_big(const DevProblem& pb, double (&y)[M::S], const double (&p)[PMAX],
                                                      double* traj, int64_t W, uint32_t off, bool active, bool part,
                                                      Acc& a) {
  using namespace ros;
  constexpr int S = M::S;
  const cptr<double> times = kconst(pb.times);
  const double t0 = times[0], tend = times[pb.T - 1];
  const double rtol = pb.rtol, atol = pb.atol;
  const bool emit_ok = active && part;
  bool dead = !part;
  int k = 0;
  if (part) emit<S, TRAJ, NT>(pb, 0, y, traj, W, off, emit_ok, k, a);
  double t = t0;
  double f0[S], J[S * S], ft[S];
  jac_eval_cols<M, PMAX>(y, t, p, f0, J, ft);

  double h;
  {
    double d0 = 0.0, d1v = 0.0;
#pragma unroll 1
    for (int s = 0; s < S; ++s) {
      const double sk = atol + rtol * fabs(y[s]);
      d0 = fmax(d0, fabs(y[s]) / sk);
      d1v = fmax(d1v, fabs(f0[s]) / sk);
    }
    double h0 = (d0 <= 1e-5 || d1v <= 1e-5) ? 1e-6 : 0.01 * (d0 / d1v);
    h0 = fmin(h0, tend - t0);
    double yt[S], f1[S];
#pragma unroll 1
    for (int s = 0; s < S; ++s) yt[s] = fma(h0, f0[s], y[s]);
    M::rhs(yt, t + h0, p, f1);
    double d2 = 0.0;
#pragma unroll 1
    for (int s = 0; s < S; ++s) {
      const double sk = atol + rtol * fabs(y[s]);
      d2 = fmax(d2, fabs(f1[s] - f0[s]) / sk);
    }
    d2 = d2 / h0;
    const double dm = fmax(d1v, d2);
    const double h1 = (dm <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : inv_fourth_root(dm / 0.01);
    double hl = fmin(100.0 * h0, h1);
    if (dead || !__builtin_isfinite(hl) || !(hl > 0.0)) hl = tend - t0;
    h = wave_min(hl);
    h = fmin(h, tend - t0);
  }
  const double span = tend - t0;
  const double hmin = 1e-14 * fmax(fabs(tend), fabs(t0)) + 1e-300;
  const int budget = kRosBudget * pb.max_steps;
  int i = 1, nst = 0;
  bool last_rej = false;
  double lu[S * S], dinv[S];
  int piv[S];
  double k1[S], k2[S], k3[S], k4[S], k5[S], k6[S], yt[S], fv[S], y1[S];
  while (i < pb.T) {
    bool last = false;
    if (t + h >= tend) { h = tend - t; last = true; }
    const double rh = 1.0 / h;
    const double gh = rh * inv_gam;
    const double c21h = c21 * rh, c31h = c31 * rh, c32h = c32 * rh, c41h = c41 * rh, c42h = c42 * rh,
                 c43h = c43 * rh, c51h = c51 * rh, c52h = c52 * rh, c53h = c53 * rh, c54h = c54 * rh,
                 c61h = c61 * rh, c62h = c62 * rh, c63h = c63 * rh, c64h = c64 * rh, c65h = c65 * rh;
    const double hd1 = h * d1, hd2 = h * d2, hd3 = h * d3, hd4 = h * d4;
#pragma unroll 1
    for (int r = 0; r < S; ++r)
#pragma unroll 1
      for (int c = 0; c < S; ++c) lu[r * S + c] = (r == c) ? gh - J[r * S + c] : -J[r * S + c];
    const bool any_swap = lu_factor_big<S>(lu, piv, dinv);
#pragma unroll 1
    for (int s = 0; s < S; ++s) k1[s] = fma(hd1, ft[s], f0[s]);
    lu_solve_big<S>(lu, piv, dinv, any_swap, k1);
#pragma unroll 1
    for (int s = 0; s < S; ++s) yt[s] = fma(a21, k1[s], y[s]);
    M::rhs(yt, t + c2x * h, p, fv);
#pragma unroll 1
    for (int s = 0; s < S; ++s) k2[s] = fma(hd2, ft[s], fma(c21h, k1[s], fv[s]));
    lu_solve_big<S>(lu, piv, dinv, any_swap, k2);
#pragma unroll 1
    for (int s = 0; s < S; ++s) yt[s] = fma(a32, k2[s], fma(a31, k1[s], y[s]));
    M::rhs(yt, t + c3x * h, p, fv);
#pragma unroll 1
    for (int s = 0; s < S; ++s) k3[s] = fma(hd3, ft[s], fma(c32h, k2[s], fma(c31h, k1[s], fv[s])));
    lu_solve_big<S>(lu, piv, dinv, any_swap, k3);
#pragma unroll 1
    for (int s = 0; s < S; ++s) yt[s] = fma(a43, k3[s], fma(a42, k2[s], fma(a41, k1[s], y[s])));
    M::rhs(yt, t + c4x * h, p, fv);
#pragma unroll 1
    for (int s = 0; s < S; ++s) k4[s] = fma(hd4, ft[s], fma(c43h, k3[s], fma(c42h, k2[s], fma(c41h, k1[s], fv[s]))));
    lu_solve_big<S>(lu, piv, dinv, any_swap, k4);
#pragma unroll 1
    for (int s = 0; s < S; ++s) yt[s] = fma(a54, k4[s], fma(a53, k3[s], fma(a52, k2[s], fma(a51, k1[s], y[s]))));
    M::rhs(yt, t + h, p, fv);
#pragma unroll 1
    for (int s = 0; s < S; ++s) k5[s] = fma(c54h, k4[s], fma(c53h, k3[s], fma(c52h, k2[s], fma(c51h, k1[s], fv[s]))));
    lu_solve_big<S>(lu, piv, dinv, any_swap, k5);
#pragma unroll 1
    for (int s = 0; s < S; ++s) yt[s] = yt[s] + k5[s];  // the embedded solution
    M::rhs(yt, t + h, p, fv);
#pragma unroll 1
    for (int s = 0; s < S; ++s)
      k6[s] = fma(c65h, k5[s], fma(c64h, k4[s], fma(c63h, k3[s], fma(c62h, k2[s], fma(c61h, k1[s], fv[s])))));
    lu_solve_big<S>(lu, piv, dinv, any_swap, k6);
    double num = 0.0, den = 1.0, nfe = 0.0;
#pragma unroll 1
    for (int s = 0; s < S; ++s) {
      y1[s] = yt[s] + k6[s];
      const double ae = fabs(k6[s]);
      const double sk = fma(rtol, max_abs_raw(y[s], y1[s]), atol);
      nfe = fma(ae, 0.0, nfe);
      nfe = fma(y1[s], 0.0, nfe);
      if (s == 0 || ae * den > num * sk) { num = ae; den = sk; }
    }
    double el = num / den;
    if (!__builtin_isfinite(el) || __builtin_isnan(nfe)) el = 1e30;
    if (dead) el = 0.0;
    const double err = wave_max(el);
    ++nst;
    if (err <= 1.0) {
      const double tn = last ? tend : t + h;
      if (i < pb.T && times[i] < tn) {  // wave-uniform: a grid point inside the step
        // q3, q4 of the continuous extension, kept in k2 and k3 (not needed any more)
#pragma unroll 1
        for (int s = 0; s < S; ++s) {
          const double q3 = fma(h25, k5[s], fma(h24, k4[s], fma(h23, k3[s], fma(h22, k2[s], h21 * k1[s]))));
          const double q4 = fma(h35, k5[s], fma(h34, k4[s], fma(h33, k3[s], fma(h32, k2[s], h31 * k1[s]))));
          k2[s] = q3;
          k3[s] = q4;
        }
        while (i < pb.T && times[i] < tn) {
          if (part && grid_needs_emit<S, TRAJ>(pb, i, k)) {
            const double th = (times[i] - t) * rh;
            const double th1 = 1.0 - th;
            double yo[S];
#pragma unroll 1
            for (int s = 0; s < S; ++s) yo[s] = fma(th, fma(th1, fma(th, k3[s], k2[s]), y1[s]), th1 * y[s]);
            emit<S, TRAJ, NT>(pb, i, yo, traj, W, off, emit_ok, k, a);
          }
          ++i;
          nst = 0;
        }
      }
#pragma unroll 1
      for (int s = 0; s < S; ++s) y[s] = part ? y1[s] : y[s];  // bystanders keep their state
      t = tn;
      if (i < pb.T && times[i] == tn) {  // a grid point on the step's end
        if (part && grid_needs_emit<S, TRAJ>(pb, i, k)) emit<S, TRAJ, NT>(pb, i, y, traj, W, off, emit_ok, k, a);
        ++i;
        nst = 0;
      }
      if (i < pb.T) jac_eval_cols<M, PMAX>(y, t, p, f0, J, ft);
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
      if (!dead && el >= 0.5 * err) {
        dead = true;
        a.status |= ST_MAXSTEP;
#pragma unroll 1
        for (int s = 0; s < S; ++s) y[s] = __builtin_nan("");
      }
      nst = budget / 2;
      if (__ballot(!dead) == 0ull) {
        double yo[S];
#pragma unroll 1
        for (int s = 0; s < S; ++s) yo[s] = __builtin_nan("");
        for (; i < pb.T; ++i)
          if (part && grid_needs_emit<S, TRAJ>(pb, i, k)) emit<S, TRAJ, NT>(pb, i, yo, traj, W, off, emit_ok, k, a);
        break;
      }
      if (h < hmin) h = fmin(1e-3 * span, tend - t);
    }
  }
  if (part) check_finite(y, a);
}

// Rosenbrock integration of the `part` lanes: registers for S <= kStiffRegS, private
// memory above (on copies, see integrate_rosenbrock_big).
template <class M, int PMAX, bool TRAJ, bool NT>
__device__ __forceinline__ void rosenbrock_lanes(const DevProblem& pb, double (&y)[M::S], const double (&p)[PMAX],
                                                 double* traj, int64_t W, uint32_t off, bool active, bool part,
                                                 Acc& a) {
  constexpr int S = M::S;
  if constexpr (S <= kStiffRegS) {
    integrate_rosenbrock<M, PMAX, TRAJ, NT>(pb, y, p, traj, W, off, active, part, a);
  } else {
    double yc[S], pc[PMAX];
#pragma unroll
    for (int s = 0; s < S; ++s) yc[s] = y[s];
#pragma unroll
    for (int q = 0; q < PMAX; ++q) pc[q] = p[q];
    Acc ac = a;
    integrate_rosenbrock_big<M, PMAX, TRAJ, NT>(pb, yc, pc, traj, W, off, active, part, ac);
#pragma unroll
    for (int s = 0; s < S; ++s) y[s] = yc[s];
    a = ac;
  }
}

}  // namespace oe
