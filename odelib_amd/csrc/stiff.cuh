// stiff.cuh — the stiff half of odeint's LSODA (Framework.py:656) on the device.
//
// LSODA integrates with Adams methods and switches to BDF when it detects stiffness.
// Here the non-stiff integrator is the wave-lockstep DOPRI5 (ode_kernels.cuh); the
// stiff integrator is an L-stable Rosenbrock method of order 4 with an embedded order-3
// error estimate (Hairer & Wanner, Solving ODEs II, §IV.7, the 4-stage ROS4 family in the
// Kaps–Rentrop form with γ = 0.57282, three RHS evaluations per step).  The method
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
//   * Output: steps end on every grid time (no interpolation; stiff components make
//     Hermite interpolation from f useless), so each row is a step endpoint.
//   * Step control: max-norm error as DOPRI5, fac = 0.9·err^(−1/4) in [0.2, 6], wave
//     maximum over the participating lanes; eviction as DOPRI5, with a step budget of
//     kRosBudget × max_steps per output interval (an order-4 method takes several times
//     LSODA's BDF steps through a stiff transient at odeint's tolerances).
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
  friend __host__ __device__ inline Dual pow(double a, const Dual& b) {
    const double v = ::pow(a, b.v);
    return chain_(b, v, v * ::log(a));
  }
  friend __host__ __device__ inline Dual pow(const Dual& a, const Dual& b) {
    Dual r; r.v = ::pow(a.v, b.v);
    const double la = ::log(a.v), da = b.v * ::pow(a.v, b.v - 1.0);
    OE_D_LOOP r.d[i] = da * a.d[i] + (r.v * la) * b.d[i];
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

// ---- ROS4, L-stable parameter set (Hairer & Wanner II, §IV.7), Kaps–Rentrop form ----
namespace ros {
constexpr double gam = 0.57282;
constexpr double a21 = 2.0, a31 = 1.867943637803922, a32 = 0.2344449711399156;
constexpr double c21 = -7.137615036412310, c31 = 2.580708087951457, c32 = 0.6515950076447975,
                 c41 = -2.137148994382534, c42 = -0.3214669691237626, c43 = -0.6949742501781779;
constexpr double m1 = 2.255570073418735, m2 = 0.2870493262186792, m3 = 0.435317943184018, m4 = 1.093502252409163;
constexpr double e1 = -0.2815431932141155, e2 = -0.0727619912493892, e3 = -0.1082196201495311,
                 e4 = -1.093502252409163;
constexpr double a2x = 1.14564, a3x = 0.65521686381559;
constexpr double g1x = 0.57282, g2x = -1.769193891319233, g3x = 0.7592633437920482, g4x = -0.104902108710045;
constexpr double inv_gam = 1.0 / gam;
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
  const double c = r == 0 ? 1.0 : r == 1 ? 0.8408964152537145 : r == 2 ? 0.7071067811865476 : 0.5946035575013605;
  return ldexp(c * y, -q);
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

// Rosenbrock integration of the lanes with `part` set (the others sit out: they neither
// steer the step size nor emit).  Wave-lockstep: one step size per wave, steps end on
// every grid time.  y is the initial state on entry and the final state on return.
template <class M, int PMAX, bool TRAJ, bool NT>
__device__ __forceinline__ void integrate_ros4(const DevProblem& pb, double (&y)[M::S], const double (&p)[PMAX],
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
    const double ti = times[i];
    const double hp = h;
    bool clip = false;
    if (t + h >= ti) { h = ti - t; clip = true; }
    const double rh = 1.0 / h;
    const double gh = rh * inv_gam;
    const double c21h = c21 * rh, c31h = c31 * rh, c32h = c32 * rh, c41h = c41 * rh, c42h = c42 * rh,
                 c43h = c43 * rh;
    const double hg1 = h * g1x, hg2 = h * g2x, hg3 = h * g3x, hg4 = h * g4x;
    double lu[S][S], dinv[S];
    int piv[S];
#pragma unroll
    for (int r = 0; r < S; ++r)
#pragma unroll
      for (int c = 0; c < S; ++c) lu[r][c] = (r == c) ? gh - J[r][c] : -J[r][c];
    const bool any_swap = lu_factor<S>(lu, piv, dinv);
    double g1[S], g2[S], g3[S], g4[S], yt[S], fv[S];
#pragma unroll
    for (int s = 0; s < S; ++s) g1[s] = fma(hg1, ft[s], f0[s]);
    lu_solve<S>(lu, piv, dinv, any_swap, g1);
#pragma unroll
    for (int s = 0; s < S; ++s) yt[s] = fma(a21, g1[s], y[s]);
    M::rhs(yt, t + a2x * h, p, fv);
#pragma unroll
    for (int s = 0; s < S; ++s) g2[s] = fma(hg2, ft[s], fma(c21h, g1[s], fv[s]));
    lu_solve<S>(lu, piv, dinv, any_swap, g2);
#pragma unroll
    for (int s = 0; s < S; ++s) yt[s] = fma(a32, g2[s], fma(a31, g1[s], y[s]));
    M::rhs(yt, t + a3x * h, p, fv);
#pragma unroll
    for (int s = 0; s < S; ++s) g3[s] = fma(hg3, ft[s], fma(c32h, g2[s], fma(c31h, g1[s], fv[s])));
    lu_solve<S>(lu, piv, dinv, any_swap, g3);
#pragma unroll
    for (int s = 0; s < S; ++s) g4[s] = fma(hg4, ft[s], fma(c43h, g3[s], fma(c42h, g2[s], fma(c41h, g1[s], fv[s]))));
    lu_solve<S>(lu, piv, dinv, any_swap, g4);
    double y1[S];
    double num = 0.0, den = 1.0, nfe = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      y1[s] = fma(m4, g4[s], fma(m3, g3[s], fma(m2, g2[s], fma(m1, g1[s], y[s]))));
      const double e = fma(e4, g4[s], fma(e3, g3[s], fma(e2, g2[s], e1 * g1[s])));
      const double ae = fabs(e);
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
      const double tn = clip ? ti : t + h;
#pragma unroll
      for (int s = 0; s < S; ++s) y[s] = part ? y1[s] : y[s];  // bystanders keep their state
      t = tn;
      if (clip) {
        if (part) emit<S, TRAJ, NT>(pb, i, y, traj, W, off, emit_ok, k, a);
        ++i;
        nst = 0;
      }
      if (i < pb.T) jac_eval<M, PMAX>(y, t, p, f0, J, ft);
      double fac = (err > 0.0) ? safe * inv_fourth_root(err) : facmax;
      fac = fmin(facmax, fmax(facmin, fac));
      if (last_rej) fac = fmin(fac, 1.0);
      const double hn = h * fac;
      // a step cut short by the grid does not shrink the planned step
      h = clip ? fmax(hn, hp) : hn;
      last_rej = false;
    } else {
      h = h * fmax(facmin, safe * inv_fourth_root(err));
      last_rej = true;
    }
    // ---- budget: evict the walkers that pin the wave's step (as DOPRI5) ----
    if (nst >= budget || h < hmin) {
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
          if (part) emit<S, TRAJ, NT>(pb, i, yo, traj, W, off, emit_ok, k, a);
        break;
      }
      if (h < hmin) h = fmin(1e-3 * span, tend - t);
    }
  }
  if (part) check_finite(y, a);
}

}  // namespace oe
