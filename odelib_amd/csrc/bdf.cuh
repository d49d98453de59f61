// bdf.cuh — the BDF half of odeint's LSODA (Framework.py:656) on the device: variable-order
// (1..5) backward differentiation formulas in the fixed-leading-coefficient backward-difference
// form of scipy's BDF solver (the NDF scheme of Shampine & Reichelt with scipy's kappa table),
// with the max norm LSODA uses and a modified Newton iteration: the LU factors of I − c·J are
// kept across steps and rebuilt, from a fresh Jacobian, when the step size or the order
// changes or Newton fails on factors from an earlier step.  (Jacobian: scipy's BDF keeps J
// across step-size and order changes and refactors only I − c·J; LSODA re-evaluates J when
// the step size changes by more than 30 % (ccmax 0.3) and every 20 steps.  Here J is taken
// afresh with each new factorisation — no J is kept, S² doubles fewer per lane — which sits
// between the two; parity with the reference is to its tolerance, not its step counts.)
//
// Why BDF and not the Rosenbrock method for the walkers 'auto' hands over:
// LSODA switches to BDF, and on the draws that make the reference's fits expensive the two
// differ by an order of magnitude.  A stiff component sitting on its quasi-steady state
// (two_i's I1 at τ = 1e4: I1 ≈ φ·S·V/τ) drives a one-step Rosenbrock method into order
// reduction — RODAS takes 3 688 steps at odeint's tolerances — while a multistep method's
// error on it is the smooth (q+1)-th difference: 550-650 BDF steps, each ~2.4 RHS
// evaluations and 1/5 of an LU factorisation (scipy's BDF: 546; LSODA: 734).
//
// Everything is IEEE add/mul/fma/div plus frexp/ldexp, restated operation for operation in
// oracle/rk_ref.c (bdf_group on a group of one), so the kernels are bitwise testable.
#pragma once

namespace oe {
namespace bdf {
constexpr int kMaxQ = 5;
constexpr int kNewtonMaxIter = 4;
constexpr int kBudget = 8;  // steps per output interval, in units of max_steps
// x^(-1/q), q = 1..6: a linear start on m ∈ [0.5, 1), six Newton steps, the exponent part
// 2^(−r/q)·2^(−Q) from a table (as inv_fifth_root)
__device__ const double kIrS[7] = {0.0, -2.0, -0.8284271247461903, -0.5198420997897464, -0.37841423000544205,
                                   -0.2973967099940702, -0.24492409661874603};
__device__ const double kIrI[7] = {0.0, 3.0, 1.8284271247461903, 1.5198420997897464, 1.378414230005442,
                                   1.2973967099940702, 1.244924096618746};
__device__ const double kIrRq[7] = {0.0, 1.0, 0.5, 0.3333333333333333, 0.25, 0.2, 0.16666666666666666};
__device__ const double kIrC[7][6] = {
    {1.0, 0, 0, 0, 0, 0},
    {1.0, 0, 0, 0, 0, 0},
    {1.0, 0.7071067811865476, 0, 0, 0, 0},
    {1.0, 0.7937005259840998, 0.6299605249474366, 0, 0, 0},
    {1.0, 0.8408964152537145, 0.7071067811865476, 0.5946035575013605, 0, 0},
    {1.0, 0.8705505632961241, 0.757858283255199, 0.6597539553864471, 0.5743491774985174, 0},
    {1.0, 0.8908987181403393, 0.7937005259840998, 0.7071067811865476, 0.6299605249474366, 0.5612310241546865}};

// x^(-1/q) for the step-size factors (x ≤ 0 → +inf: a zero error norm leaves the factor to
// its clamp; +inf → 0).  q is wave-uniform at every call.
__device__ __forceinline__ double inv_root(double x, int q) {
  if (!(x > 0.0)) return __builtin_inf();
  if (__builtin_isinf(x)) return 0.0;
  int e;
  const double m = frexp(x, &e);
  int Q = e / q, r = e % q;
  if (r < 0) { r += q; Q -= 1; }
  const cptr<double> s = kconst(kIrS), ic = kconst(kIrI), rq = kconst(kIrRq);
  double y = fma(s[q], m, ic[q]);
  const double q1 = (double)(q + 1), rqq = rq[q];
  for (int it = 0; it < 6; ++it) {
    double yq = y;
    for (int j = 1; j < q; ++j) yq = yq * y;
    y = (y * fma(-m, yq, q1)) * rqq;
  }
  return ldexp(kconst(&kIrC[0][0])[q * 6 + r] * y, -Q);
}

// per-lane max norm of |c·v| against atol + rtol·|y| (argmax by cross-multiplication, one
// division; non-finite → 1e30)
template <int S>
__device__ __forceinline__ double norm_max(double c, const double (&v)[S], const double (&y)[S], double rtol,
                                           double atol) {
  double num = 0.0, den = 1.0, nfe = 0.0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const double ae = fabs(c * v[s]);
    const double sk = fma(rtol, fabs(y[s]), atol);
    nfe = fma(ae, 0.0, nfe);
    if (s == 0 || ae * den > num * sk) { num = ae; den = sk; }
  }
  double el = num / den;
  if (!__builtin_isfinite(el) || __builtin_isnan(nfe)) el = 1e30;
  return el;
}
}  // namespace bdf
}  // namespace oe

// ---- The pass: one step size and one order per lane (every kernel with S <= 8) ----------
// In the reference every walker is integrated by its own odeint call (Framework.py:656, one
// chain per process at :779-780), so nothing a walker computes depends on the others.  (Until
// round 4 the lanes handed to BDF shared h and q over the wave, which made an MH chain's
// bits depend on which proposals shared its wave: the speculation depth, the rank count.)
// Every decision is the lane's own — HINIT without a wave minimum, the error norm without a
// wave maximum, its own Newton outcome, order selection and budget — so a lane's result is
// bdf_group of oracle/rk_ref.c on a group of one, operation for operation.  Against the
// shared-step pass it also costs 20-30 % less per step on a lone stiff lane
// (tools/bdf_cost.py, profiles/NOTES.md round 5).
//
// Layout of a step (one attempt per live lane per loop trip, lanes diverge freely):
//   A  predictor (order-dependent: a switch on the lane's q, each case straight-line code
//      for a compile-time order, so lanes at one order run it once);
//   B  factors of I − c·J if needed and the modified Newton iteration (order-independent:
//      every live lane together, whatever its order);
//   C  the error test, the difference update, the grid points and the order selection
//      (again a switch on q).
// A Newton failure on factors from an earlier step retries the same attempt on the next
// trip with factors at the predictor (the predictor is recomputed from unchanged inputs:
// the same bits), as scipy's BDF and the group restatement do within one attempt.
//
// Registers (the MH kernels sit at one wave per SIMD): the Jacobian is taken column by
// column with one-tangent dual numbers straight into the LU array (an S + 1-tangent
// evaluation, stiff.cuh jac_eval, holds S² + S·(S + 2) doubles at once), the difference table
// holds rows 0..q+1 plus the order-up row, i.e. kMaxQ + 2 rows (row kMaxQ + 2 is never read),
// in LDS (below), and grid times come through a 4-entry window.
//
// Observations are deferred: at an observed grid point the lane only forms each record's
// sum C (and tracks the minimum and finiteness), storing C to a per-lane column of the
// launch's scratch (DevProblem::obs_c, [n_obs][lanes]); after the pass the wave adds the
// chi / R² terms of every lane's records in record order, in uniform control flow — the
// same terms in the same order as an immediate evaluation, and the out-of-line log is
// never called under a partial EXEC mask.

namespace oe {
namespace bdfl {
constexpr int kMaxQ = bdf::kMaxQ;
constexpr int kRows = kMaxQ + 2;  // D[0..kMaxQ+1]; D[q+2] only while q < kMaxQ
constexpr int kWin = 4;           // grid-time window (times[] carries kGridWin + 1 >= kWin sentinels)
static_assert(kWin <= kGridWin + 1, "grid window past the sentinels");

// bdf.cuh's tables as compile-time functions: with a template order they fold to immediates
__device__ __forceinline__ constexpr double gam(int j) {
  return j == 1 ? 1.0 : j == 2 ? 1.5 : j == 3 ? 1.8333333333333333 : j == 4 ? 2.083333333333333 : 2.283333333333333;
}
__device__ __forceinline__ constexpr double ialpha(int q) {
  return q == 1 ? 0.8438818565400843 : q == 2 ? 0.6 : q == 3 ? 0.5039772202296456 : q == 4 ? 0.4608737397983678
                                                                                             : 0.43795620437956206;
}
__device__ __forceinline__ constexpr double ec(int q) {
  return q == 0 ? 1.0 : q == 1 ? 0.315 : q == 2 ? 0.16666666666666666 : q == 3 ? 0.09911666666666669
         : q == 4 ? 0.11354166666666668 : 0.16666666666666666;
}
__device__ __forceinline__ constexpr double inv_i(int i) {
  return i == 1 ? 1.0 : i == 2 ? 0.5 : i == 3 ? 0.3333333333333333 : i == 4 ? 0.25 : 0.2;
}
// U[m][j] = (−1)^m·C(j, m)
__device__ __forceinline__ constexpr double U(int m, int j) {
  double c = 1.0;
  for (int k = 0; k < m; ++k) c = c * (double)(j - k) / (double)(k + 1);
  return (m & 1) ? -c : c;
}
// x^(-1/q) start and scale tables (bdf.cuh kIrS / kIrI / kIrRq / kIrC)
__device__ __forceinline__ constexpr double ir_s(int q) {
  return q == 1 ? -2.0 : q == 2 ? -0.8284271247461903 : q == 3 ? -0.5198420997897464 : q == 4 ? -0.37841423000544205
         : q == 5 ? -0.2973967099940702 : -0.24492409661874603;
}
__device__ __forceinline__ constexpr double ir_i(int q) {
  return q == 1 ? 3.0 : q == 2 ? 1.8284271247461903 : q == 3 ? 1.5198420997897464 : q == 4 ? 1.378414230005442
         : q == 5 ? 1.2973967099940702 : 1.244924096618746;
}
__device__ __forceinline__ constexpr double ir_rq(int q) {
  return q == 1 ? 1.0 : q == 2 ? 0.5 : q == 3 ? 0.3333333333333333 : q == 4 ? 0.25 : q == 5 ? 0.2 : 0.16666666666666666;
}
template <int Q>
__device__ __forceinline__ double ir_c(int r) {
  static_assert(Q >= 1 && Q <= 6, "order");
  if constexpr (Q == 1) return 1.0;
  if constexpr (Q == 2) {
    constexpr double c[2] = {1.0, 0.7071067811865476};
    return dp::select_r(r, c);
  }
  if constexpr (Q == 3) {
    constexpr double c[3] = {1.0, 0.7937005259840998, 0.6299605249474366};
    return dp::select_r(r, c);
  }
  if constexpr (Q == 4) {
    constexpr double c[4] = {1.0, 0.8408964152537145, 0.7071067811865476, 0.5946035575013605};
    return dp::select_r(r, c);
  }
  if constexpr (Q == 5) {
    constexpr double c[5] = {1.0, 0.8705505632961241, 0.757858283255199, 0.6597539553864471, 0.5743491774985174};
    return dp::select_r(r, c);
  }
  if constexpr (Q == 6) {
    constexpr double c[6] = {1.0, 0.8908987181403393, 0.7937005259840998, 0.7071067811865476, 0.6299605249474366,
                             0.5612310241546865};
    return dp::select_r(r, c);
  }
}
// bdf::inv_root for a compile-time q: the same operations (constant division, unrolled
// powers), the same bits
template <int Q>
__device__ __forceinline__ double inv_root(double x) {
  if (!(x > 0.0)) return __builtin_inf();
  if (__builtin_isinf(x)) return 0.0;
  int e;
  const double m = frexp(x, &e);
  int E = e / Q, r = e % Q;
  if (r < 0) { r += Q; E -= 1; }
  double y = fma(ir_s(Q), m, ir_i(Q));
  constexpr double q1 = (double)(Q + 1), rqq = ir_rq(Q);
#pragma unroll
  for (int it = 0; it < 6; ++it) {
    double yq = y;
#pragma unroll
    for (int j = 1; j < Q; ++j) yq = yq * y;
    y = (y * fma(-m, yq, q1)) * rqq;
  }
  return ldexp(ir_c<Q>(r) * y, -E);
}
// Newton-count safety 0.9·(2·4 + 1)/(2·4 + n), n = 1..4
__device__ __forceinline__ double safety(int n) {
  return n == 1 ? 0.8999999999999999 : n == 2 ? 0.8099999999999999 : n == 3 ? 0.7363636363636363 : 0.6749999999999999;
}
}  // namespace bdfl

// A lane's difference table lives in LDS, lane-minor ([row·S + s][kMhBlock] doubles, a
// 512-B row per wave access): in registers, an update of the table inside the per-lane
// switch on the order keeps two copies of it live (the new rows of the lanes in one case
// while the next case runs on the old rows) — 28 doubles more at S = 4, which pushed the
// kernel past 256 VGPRs.  In LDS the lanes' stores are masked writes in place.
constexpr int kMhBlock = 256;  // threads per workgroup of every kernel with a BDF pass (capi.hip kBlock)
#ifndef OE_BDF_NEWTON_UNROLL  // 0: the Newton loop kept rolled (measured slower: C2 + 0.1 % stiff 2.68 vs 2.26-2.50 ms)
#define OE_BDF_NEWTON_UNROLL 1
#endif
#ifndef OE_BDF_D_REGS  // measurement builds: the difference table in registers (tools/build_alt.sh)
#define OE_BDF_D_REGS 0
#endif
template <int S, int LD = kMhBlock>
struct DTab {
#if OE_BDF_D_REGS
  double v[bdfl::kRows * S];
  __device__ __forceinline__ double& operator()(int r, int s) { return v[r * S + s]; }
  __device__ __forceinline__ double operator()(int r, int s) const { return v[r * S + s]; }
#else
  double* p;  // this lane's column (LDS: the address space is inferred after inlining)
  __device__ __forceinline__ double& operator()(int r, int s) const { return p[(r * S + s) * LD]; }
#endif
};
// LD = 0: the table in registers (a kernel with the registers to spare: k_bdf_hq after the
// DOPRI5 kernel, one walker per wave — no LDS round trip in the predictor and the update)
template <int S>
struct DTab<S, 0> {
  double v[bdfl::kRows * S];
  __device__ __forceinline__ double& operator()(int r, int s) { return v[r * S + s]; }
  __device__ __forceinline__ double operator()(int r, int s) const { return v[r * S + s]; }
};
// LD: columns of the table = threads of the workgroup (kMhBlock; 64 in k_bdf_hq beside)
template <int S, int LD = kMhBlock>
__device__ __forceinline__ DTab<S, LD> dtab_column() {
#if OE_BDF_D_REGS
  return DTab<S, LD>{};
#else
  if constexpr (LD == 0) {
    return DTab<S, 0>{};
  } else {
    __shared__ double tab[bdfl::kRows * S * LD];
    return DTab<S, LD>{tab + threadIdx.x};
  }
#endif
}

// Measurement builds (tools/build_alt.sh … -DOE_BDF_CLOCKS=1, tools/bdf_phases.py): shader
// cycles (s_memtime) per phase of the per-lane step, summed over a lane's pass and printed
// at its end — for one-walker runs; =2: no printf, the lane's chi / R² outputs carry the
// cycles from its wave's start to the pass and in the pass.  0 in every shipped build.
#ifndef OE_BDF_CLOCKS
#define OE_BDF_CLOCKS 0
#endif
#ifndef OE_LANE_CLOCKS  // the same for a lane's DOPRI5 step (lane.cuh, tools/lane_phases.py)
#define OE_LANE_CLOCKS 0
#endif
enum BdfPhase { kPhPredict, kPhFactor, kPhNewton, kPhErr, kPhDiff, kPhGrid, kPhSelect, kPhFail, kPhN };
struct BdfClk {
#if OE_BDF_CLOCKS || OE_LANE_CLOCKS
  uint64_t c[kPhN], last;
  uint32_t n[kPhN];
  __device__ __forceinline__ void start() {
    for (int j = 0; j < kPhN; ++j) { c[j] = 0; n[j] = 0; }
    last = __builtin_amdgcn_s_memtime();
  }
  __device__ __forceinline__ void mark(int ph) {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    c[ph] += now - last;
    n[ph] += 1;
    last = now;
  }
#else
  __device__ __forceinline__ void start() {}
  __device__ __forceinline__ void mark(int) {}
#endif
};

#if OE_BDF_CLOCKS
// the s_memtime at which each wave of the workgroup entered its kernel (k_integrate, k_mh)
__device__ __forceinline__ uint64_t* bdf_clk_wave_start() {
  __shared__ uint64_t t[16];
  return t;
}
#endif

template <int S, int LD = kMhBlock>
struct BdfLane {
  DTab<S, LD> D;                 // backward differences (scipy's D), in LDS
  double lu[S][S], dinv[S];  // LU of I − c·J
  int piv[S];
  double t, h;               // this lane's time and step size
  double wv[bdfl::kWin];     // times[i .. i + kWin)
  int q, neq, nst;           // order, steps at this h and q, steps since the last grid point
  int i, k, nxt;             // next grid index, next observation record, its grid index
  bool live, lu_ok, fresh, refac, swp;
  BdfClk clk;
};

// scipy's change_D at a compile-time order Q (bdf::change_D's operations)
template <int S, int Q, int LD>
__device__ __forceinline__ void bdfl_change_D(DTab<S, LD>& D, double factor) {
  using namespace bdfl;
  double r[Q + 1][Q + 1];
#pragma unroll
  for (int m = 1; m <= Q; ++m) {
    double v = 1.0;
#pragma unroll
    for (int i = 1; i <= Q; ++i) {
      v = v * (((double)(i - 1) - factor * (double)m) * inv_i(i));
      r[m][i] = v;
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    double E[Q + 1];
    E[0] = D(0, s);
#pragma unroll
    for (int m = 1; m <= Q; ++m) {
      double e = D(0, s);
#pragma unroll
      for (int i = 1; i <= Q; ++i) e = fma(r[m][i], D(i, s), e);
      E[m] = e;
    }
#pragma unroll
    for (int j = 0; j <= Q; ++j) {
      double acc = E[0];
#pragma unroll
      for (int m = 1; m <= j; ++m) acc = fma(U(m, j), E[m], acc);
      D(j, s) = acc;
    }
  }
}

template <int S, int LD>
__device__ __forceinline__ void bdfl_change_D(DTab<S, LD>& D, int q, double factor) {
  switch (q) {
    case 1: bdfl_change_D<S, 1>(D, factor); break;
    case 2: bdfl_change_D<S, 2>(D, factor); break;
    case 3: bdfl_change_D<S, 3>(D, factor); break;
    case 4: bdfl_change_D<S, 4>(D, factor); break;
    default: bdfl_change_D<S, 5>(D, factor); break;
  }
}

// Phase A: predictor y_p = Σ_{j<=Q} D_j, ψ = Σ γ_j D_j / α_Q, c = h / α_Q
template <int S, int Q, int LD>
__device__ __forceinline__ void bdfl_predict(const BdfLane<S, LD>& st, double (&yp)[S], double (&psi)[S], double& c) {
  using namespace bdfl;
  constexpr double ia = ialpha(Q);
  c = st.h * ia;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    double v = st.D(0, s), ps = 0.0;
#pragma unroll
    for (int j = 1; j <= Q; ++j) {
      v = v + st.D(j, s);
      ps = fma(gam(j), st.D(j, s), ps);
    }
    yp[s] = v;
    psi[s] = ps * ia;
  }
}

// LU factors of I − c·J(t, y): J column by column (one-tangent duals; each entry the same
// bits as the S + 1-tangent evaluation), straight into the LU array
template <class M, int PMAX, int LD>
__device__ __forceinline__ void bdfl_factor(BdfLane<M::S, LD>& st, double c, const double (&y)[M::S], double t,
                                            const double (&p)[PMAX]) {
  constexpr int S = M::S;
  using D1 = Dual<1>;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    D1 yd[S], pd[PMAX], fd[S];
#pragma unroll
    for (int s = 0; s < S; ++s) { yd[s] = D1(y[s]); yd[s].d[0] = (s == j) ? 1.0 : 0.0; }
    const D1 td(t);
#pragma unroll
    for (int q = 0; q < PMAX; ++q) pd[q] = D1(p[q]);
    M::rhs(yd, td, pd, fd);
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double av = c * fd[s].d[0];
      st.lu[s][j] = (s == j) ? 1.0 - av : -av;
    }
  }
  st.swp = ros::lu_factor<S>(st.lu, st.piv, st.dinv);
}

// the launch's deferred-observation scratch: record k of lane `col` at obs_c[k·ld + col]
struct ObsCol {
  double* c;
  int64_t ld, col;
};
// TRAJ: this lane's column of the [T][S][W] trajectory
struct TrajCol {
  double* traj;
  int64_t W, w;
  bool active;
};

// the observations at grid index nxt (the lane's next observed one): finiteness, and each
// record's sum C to the scratch (the chi / R² terms follow after the pass)
template <int S, int LD>
__device__ __forceinline__ void bdfl_observe(const DevProblem& pb, BdfLane<S, LD>& st, const double (&yo)[S], const ObsCol& oc,
                                             Acc& a) {
  check_finite(yo, a);
  const Obs* obs = pb.obs;
  const int i = st.nxt;
  int k = st.k;
  while (k < pb.n_obs && obs[k].tidx == i) {
    const uint64_t mask = obs[k].mask;
    double c = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s)
      if ((mask >> s) & 1ull) c = c + yo[s];
    oc.c[(int64_t)k * oc.ld + oc.col] = c;
    ++k;
  }
  st.k = k;
  st.nxt = (k < pb.n_obs) ? obs[k].tidx : 0x7fffffff;
}

// the backward-difference interpolant of the step just accepted (order Q, ending at tn) at ti
template <int S, int Q, int LD>
__device__ __forceinline__ void bdfl_interp(const BdfLane<S, LD>& st, double tn, double ti, double (&yo)[S]) {
  const double h = st.h;
  double prod = 1.0;
#pragma unroll
  for (int s = 0; s < S; ++s) yo[s] = st.D(0, s);
#pragma unroll
  for (int j = 1; j <= Q; ++j) {
    const double rden = 1.0 / ((double)j * h);
    const double x = (ti - (tn - (double)(j - 1) * h)) * rden;
    prod = prod * x;
#pragma unroll
    for (int s = 0; s < S; ++s) yo[s] = fma(st.D(j, s), prod, yo[s]);
  }
}

// Phase C at order Q: error test; on acceptance the differences, the grid points of
// (t, t + h] and — every Q + 1 equal steps — the order and step selection
template <class M, int Q, bool TRAJ, bool NT, int LD>
__device__ __forceinline__ void bdfl_conclude(const DevProblem& pb, BdfLane<M::S, LD>& st, const double (&yn)[M::S],
                                              const double (&d)[M::S], int niter, double (&y)[M::S], const ObsCol& oc,
                                              const TrajCol& tc, Acc& a) {
  using namespace bdfl;
  constexpr int S = M::S;
  const double rtol = pb.rtol, atol = pb.atol;
  const double sf = safety(niter);
  const double el = bdf::norm_max<S>(ec(Q), d, yn, rtol, atol);
  if (el > 1.0) {  // rejected on the error (the factors are kept, as scipy)
    const double factor = fmax(0.2, sf * inv_root<Q + 1>(el));
    st.h = st.h * factor;
    bdfl_change_D<S, Q>(st.D, factor);
    st.neq = 0;
    st.clk.mark(kPhFail);
    return;
  }
  st.clk.mark(kPhErr);
  ++st.neq;
  st.fresh = false;
  const double tn = st.t + st.h;
  // scipy's update D[q+2] = d − D[q+1], D[q+1] = d, D[j] += D[j+1] (j = q..0), one state at a
  // time with all of its old rows read first: the LDS reads go out together instead of one
  // read-add-write round trip per row (the chain carries the new D[j+1] in a register)
#pragma unroll
  for (int s = 0; s < S; ++s) {
    double od[Q + 2];
#pragma unroll
    for (int j = 0; j <= Q + 1; ++j) od[j] = st.D(j, s);
    if constexpr (Q + 2 < kRows) st.D(Q + 2, s) = d[s] - od[Q + 1];
    st.D(Q + 1, s) = d[s];
    double nx = d[s];
#pragma unroll
    for (int j = Q; j >= 0; --j) {
      nx = od[j] + nx;
      st.D(j, s) = nx;
    }
  }
  ++st.nst;
  st.clk.mark(kPhDiff);
  // grid points in (t, tn]: counted on the window, a window's worth at a time; the rows
  // (TRAJ), the observed points and T − 1 (the final state) from the interpolant
  int i = st.i, c;
  bool crossed = false;
  do {
    c = dp::count_le(st.wv, tn);
    if (c == 0) break;
    crossed = true;
    // the next window goes straight into st.wv, loaded BEFORE this chunk's row stores (on
    // gfx950 a vector load's wait also waits for every store issued ahead of it) and first
    // read by the next step's count: neither the load's latency nor the stores' is waited for
    // here (a window copied in at the end of the chunk waited ~1 000 cycles per step, 18 % of
    // a lone lane's step: tools/bdf_phases.py).  The chunk reads the old window from ow.
    double ow[kWin];
#pragma unroll
    for (int j = 0; j < kWin; ++j) ow[j] = st.wv[j];
#pragma unroll
    for (int j = 0; j < kWin; ++j) st.wv[j] = pb.times[i + c + j];  // (times[T..] are +inf sentinels)
    for (int j = 0; j < c; ++j) {
      const int g = i + j;
      const bool observed = g == st.nxt;
      if (TRAJ || observed || g == pb.T - 1) {
        double yo[S];
        bdfl_interp<S, Q>(st, tn, pick(ow, j), yo);
        if (TRAJ || observed) track_min<S>(yo, a);
        if constexpr (TRAJ) {
          if (tc.active) {
            double* row = tc.traj + (int64_t)g * S * tc.W + tc.w;
#pragma unroll
            for (int s = 0; s < S; ++s) {
              if constexpr (NT) __builtin_nontemporal_store(yo[s], row + (int64_t)s * tc.W);
              else row[(int64_t)s * tc.W] = yo[s];
            }
          }
        }
        if (observed) bdfl_observe<S>(pb, st, yo, oc, a);
        if (g == pb.T - 1) {
#pragma unroll
          for (int s = 0; s < S; ++s) y[s] = yo[s];
        }
      }
    }
    i += c;
  } while (c == kWin);
  if (crossed) {
    st.nst = 0;
    st.i = i;
    if (i >= pb.T) {  // past the last grid point: done (y holds its interpolant)
      st.t = tn;
      st.live = false;
      st.clk.mark(kPhGrid);
      return;
    }
  }
  st.t = tn;
  st.clk.mark(kPhGrid);
  if (st.neq >= Q + 1) {  // order and step selection (scipy's rule, capped at 10)
    double fm = 0.0, fp = 0.0;
    if constexpr (Q > 1) {
      double v[S];
#pragma unroll
      for (int s = 0; s < S; ++s) v[s] = st.D(Q, s);
      fm = inv_root<Q>(bdf::norm_max<S>(ec(Q - 1), v, yn, rtol, atol));
    }
    const double fe = inv_root<Q + 1>(el);
    if constexpr (Q < kMaxQ) {
      double v[S];
#pragma unroll
      for (int s = 0; s < S; ++s) v[s] = st.D(Q + 2, s);
      fp = inv_root<Q + 2>(bdf::norm_max<S>(ec(Q + 1), v, yn, rtol, atol));
    }
    int dq = 0;
    double fmx = fm;
    if (fe > fmx) { fmx = fe; dq = 1; }
    if (fp > fmx) { fmx = fp; dq = 2; }
    const double factor = fmin(10.0, sf * fmx);
    st.h = st.h * factor;
    if (dq == 0) {
      if constexpr (Q > 1) bdfl_change_D<S, Q - 1>(st.D, factor);
    } else if (dq == 1) {
      bdfl_change_D<S, Q>(st.D, factor);
    } else {
      if constexpr (Q < kMaxQ) bdfl_change_D<S, Q + 1>(st.D, factor);
    }
    st.q = Q + dq - 1;
    st.neq = 0;
    st.lu_ok = false;
    st.clk.mark(kPhSelect);
  }
}

// One step attempt of a live lane (called in divergent control flow)
template <class M, int PMAX, bool TRAJ, bool NT, int LD>
__device__ __forceinline__ void bdfl_step(const DevProblem& pb, BdfLane<M::S, LD>& st, const double (&p)[PMAX],
                                          double (&y)[M::S], const ObsCol& oc, const TrajCol& tc, Acc& a) {
  using namespace bdfl;
  constexpr int S = M::S;
  const double rtol = pb.rtol, atol = pb.atol, ntol = pb.newton_tol;
  double yp[S], psi[S], c;
  switch (st.q) {
    case 1: bdfl_predict<S, 1>(st, yp, psi, c); break;
    case 2: bdfl_predict<S, 2>(st, yp, psi, c); break;
    case 3: bdfl_predict<S, 3>(st, yp, psi, c); break;
    case 4: bdfl_predict<S, 4>(st, yp, psi, c); break;
    default: bdfl_predict<S, 5>(st, yp, psi, c); break;
  }
  double rs[S];
#pragma unroll
  for (int s = 0; s < S; ++s) rs[s] = 1.0 / fma(rtol, fabs(yp[s]), atol);
  st.clk.mark(kPhPredict);
  if (!st.lu_ok || st.refac) {  // at the current state (new h or q), or at the predictor (retry)
    double fy[S];
#pragma unroll
    for (int s = 0; s < S; ++s) fy[s] = st.refac ? yp[s] : st.D(0, s);
    bdfl_factor<M, PMAX>(st, c, fy, st.refac ? st.t + st.h : st.t, p);
    st.lu_ok = true;
    st.fresh = true;
    st.refac = false;
    st.clk.mark(kPhFactor);
  }
  // ---- B: modified Newton (every live lane, whatever its order) ----
  const double tn = st.t + st.h;
  double yn[S], d[S];
#pragma unroll
  for (int s = 0; s < S; ++s) { yn[s] = yp[s]; d[s] = 0.0; }
  bool conv = false, fail = false;
  double dold = 0.0;
  int niter = 0;
#if OE_BDF_NEWTON_UNROLL
#pragma unroll
#else
#pragma unroll 1
#endif
  for (int kk = 0; kk < bdf::kNewtonMaxIter; ++kk) {
    const bool act = !conv && !fail;
    if (__ballot(act) == 0ull) break;
    if (act) {
      niter = kk + 1;
      double f[S], dy[S], nf = 0.0;
      M::rhs(yn, tn, p, f);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        nf = fma(f[s], 0.0, nf);
        dy[s] = (c * f[s] - psi[s]) - d[s];
      }
      if (__builtin_isnan(nf)) {
        fail = true;
      } else {
        ros::lu_solve<S>(st.lu, st.piv, st.dinv, st.swp, dy);
        double dn = 0.0;
#pragma unroll
        for (int s = 0; s < S; ++s) dn = fmax(dn, fabs(dy[s]) * rs[s]);
        // scipy's tests rate^n/(1 − rate)·dn > tol (diverging) and rate/(1 − rate)·dn < tol
        // (converged), multiplied through by 1 − rate > 0: one division per iteration, not three
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
  st.clk.mark(kPhNewton);
  if (!conv) {
    if (!st.fresh) {  // failed on older factors: this attempt again, on factors at the predictor
      st.refac = true;
      return;
    }
    st.h = st.h * 0.5;
    bdfl_change_D<S>(st.D, st.q, 0.5);
    st.neq = 0;
    st.lu_ok = false;
    st.clk.mark(kPhFail);
    return;
  }
  // ---- C ----
  switch (st.q) {
    case 1: bdfl_conclude<M, 1, TRAJ, NT>(pb, st, yn, d, niter, y, oc, tc, a); break;
    case 2: bdfl_conclude<M, 2, TRAJ, NT>(pb, st, yn, d, niter, y, oc, tc, a); break;
    case 3: bdfl_conclude<M, 3, TRAJ, NT>(pb, st, yn, d, niter, y, oc, tc, a); break;
    case 4: bdfl_conclude<M, 4, TRAJ, NT>(pb, st, yn, d, niter, y, oc, tc, a); break;
    default: bdfl_conclude<M, 5, TRAJ, NT>(pb, st, yn, d, niter, y, oc, tc, a); break;
  }
}

// BDF integration, one step size and order per lane, of the lanes with `part` set from
// their own (t, y, grid index i, observation record k); y is the final state on return.
// W lanes in the launch, this lane's column w (the trajectory rows, TRAJ, and the scratch of
// deferred observations).
template <class M, int PMAX, bool TRAJ, bool NT, int LD = kMhBlock>
__device__ __forceinline__ void integrate_bdf_lane(const DevProblem& pb, double (&y)[M::S], double t, int i, int k,
                                                   const double (&p)[PMAX], double* traj, int64_t W, int64_t w,
                                                   bool active, bool part, Acc& a) {
  using namespace bdfl;
  constexpr int S = M::S;
  const cptr<double> ctimes = kconst(pb.times);
  const double tend = ctimes[pb.T - 1], t0 = ctimes[0];
  const double rtol = pb.rtol, atol = pb.atol;
  const int budget = bdf::kBudget * pb.max_steps;
  const ObsCol oc{pb.obs_c, W, w};
  const TrajCol tc{traj, W, w, active};
  const int k_first = k;
  BdfLane<S, LD> st;
  st.D = dtab_column<S, LD>();
  st.live = part;
  st.t = t;
  st.i = i;
  st.k = k;
  st.nxt = (k < pb.n_obs) ? pb.obs[k].tidx : 0x7fffffff;
#pragma unroll
  for (int j = 0; j < kWin; ++j) st.wv[j] = pb.times[i + j];
  st.nst = 0;
  {
    double f[S];
    M::rhs(y, t, p, f);
    // initial step: HINIT for order 1 (max norm), this lane's own
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
    const double h1 = (dm <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : bdf::inv_root(dm / 0.01, 2);
    double hl = fmin(100.0 * h0, h1);
    if (!__builtin_isfinite(hl) || !(hl > 0.0)) hl = rest;
    st.h = hl;
#pragma unroll
    for (int j = 0; j < kRows; ++j)
#pragma unroll
      for (int s = 0; s < S; ++s) st.D(j, s) = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) { st.D(0, s) = y[s]; st.D(1, s) = f[s] * st.h; }
  }
  const double hmin = 1e-14 * fmax(fabs(tend), fabs(t0)) + 1e-300;
  st.q = 1;
  st.neq = 0;
  st.lu_ok = false;
  st.fresh = false;
  st.refac = false;
  st.swp = false;
  st.clk.start();
#if OE_BDF_CLOCKS
  const uint64_t t_entry = st.clk.last;
#endif
  while (__ballot(st.live) != 0ull) {
    if (st.live) {
      bdfl_step<M, PMAX, TRAJ, NT>(pb, st, p, y, oc, tc, a);
      // budget: more than `budget` steps inside one output interval, or a step below hmin:
      // abandoned (MAXSTEP; NaN at the later points — their records are not added)
      if (st.live && (st.nst >= budget || st.h < hmin)) {
        st.live = false;
        a.status |= ST_MAXSTEP;
#pragma unroll
        for (int s = 0; s < S; ++s) y[s] = __builtin_nan("");
        if constexpr (TRAJ) {  // NaN rows for the rest of the grid
          if (active)
            for (int g = st.i; g < pb.T; ++g) {
              double* row = traj + (int64_t)g * S * W + w;
#pragma unroll
              for (int s = 0; s < S; ++s) {
                if constexpr (NT) __builtin_nontemporal_store(y[s], row + (int64_t)s * W);
                else row[(int64_t)s * W] = y[s];
              }
            }
        }
      }
    }
  }
  // deferred observations: records [k_first, st.k) of each taking-part lane, in record
  // order, uniform control flow (every lane runs every record; the others drop it)
  const double kmin = wave_min(part ? (double)k_first : __builtin_inf());
  if (kmin < (double)pb.n_obs) {
    const cptr<Obs> obs = kconst(pb.obs);
    for (int kk = (int)kmin; kk < pb.n_obs; ++kk) {
      const bool in = part && kk >= k_first && kk < st.k;
      const double c = in ? oc.c[(int64_t)kk * oc.ld + oc.col] : 1.0;
      const double O = obs[kk].O, two_s2 = obs[kk].two_s2, O_lin = obs[kk].O_lin;
      const double dd = O - oe_log(c);
      const double term = (dd * dd) / two_s2;
      if (in && __builtin_isfinite(term)) { a.chi += term; a.nvalid += 1; }
      const double r = c - O_lin;
      const double r2 = r * r;
      if (in && !__builtin_isnan(r2)) a.ssres += r2;
    }
  }
  if (part) check_finite(y, a);
#if OE_BDF_CLOCKS == 2  // no printf (a hostcall per lane perturbs a many-lane launch): the lane's
                        // chi / R² outputs carry the cycles before the pass and in it
  if (part) {
    a.chi = (double)(t_entry - bdf_clk_wave_start()[threadIdx.x >> 6]);
    a.ssres = (double)(__builtin_amdgcn_s_memtime() - t_entry);
    a.nvalid = 1;
  }
#elif OE_BDF_CLOCKS
  if (part)
    printf("bdf_clocks lane %d since_wave_start %lu bdf_pass %lu predict %lu %u factor %lu %u newton %lu %u "
           "err %lu %u diff %lu %u grid %lu %u select %lu %u fail %lu %u\n",
           (int)w, t_entry - bdf_clk_wave_start()[threadIdx.x >> 6], __builtin_amdgcn_s_memtime() - t_entry,
           st.clk.c[0], st.clk.n[0], st.clk.c[1], st.clk.n[1], st.clk.c[2], st.clk.n[2], st.clk.c[3],
           st.clk.n[3], st.clk.c[4], st.clk.n[4], st.clk.c[5], st.clk.n[5], st.clk.c[6], st.clk.n[6], st.clk.c[7],
           st.clk.n[7]);
#endif
}

}  // namespace oe
