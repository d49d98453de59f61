// models.cuh — built-in right-hand sides, re-declared as device callbacks.
//
// The reference user writes `ODE(y, t, ps) -> np.ndarray` (ODElib/Framework.py:177-180)
// and odeint calls it from Fortran (Framework.py:656).  Here the RHS is a
// `__device__` function of one walker's state held in VGPRs: the same function as the
// demo notebook's Python source (demo/Demo_InfectionStates.ipynb:60-128), evaluated
// with explicit fused multiply-adds (each `a*b - c*d` is fma(a, b, -(c*d)): one
// rounding fewer per term, 6 instead of 10 fp64 operations for two_i).  The library is
// compiled with -ffp-contract=off, so these fma() calls are the ONLY fusions and the
// oracle's C restatement (oracle/rk_ref.c) reproduces every bit.
#pragma once

namespace oe {

// notebook zero_i (Demo_InfectionStates.ipynb:112-128): S, V | mu, phi, beta
struct ZeroI {
  static constexpr int S = 2, P = 3;
  template <class R>
  __host__ __device__ static inline void rhs(const R* y, R /*t*/, const R* ps, R* dy) {
    const R mu = ps[0], phi = ps[1], beta = ps[2];
    const R Sv = y[0], V = y[1];
    const R inf = phi * Sv * V;          // infections phi*S*V
    dy[0] = fma(mu, Sv, -inf);           // mu*S - phi*S*V
    dy[1] = fma(beta, inf, -inf);        // beta*phi*S*V - phi*S*V
  }
};

// notebook one_i (Demo_InfectionStates.ipynb:78-94): S, I1, V | mu, phi, beta, lam
struct OneI {
  static constexpr int S = 3, P = 4;
  template <class R>
  __host__ __device__ static inline void rhs(const R* y, R /*t*/, const R* ps, R* dy) {
    const R mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3];
    const R Sv = y[0], I1 = y[1], V = y[2];
    const R inf = phi * Sv * V;
    dy[0] = fma(mu, Sv, -inf);           // mu*S - phi*S*V
    dy[1] = fma(-lam, I1, inf);          // phi*S*V - lam*I1
    dy[2] = fma(beta * lam, I1, -inf);   // beta*lam*I1 - phi*S*V
  }
};

// notebook two_i (Demo_InfectionStates.ipynb:60-75): S, I1, I2, V | mu, phi, beta, lam, tau
struct TwoI {
  static constexpr int S = 4, P = 5;
  template <class R>
  __host__ __device__ static inline void rhs(const R* y, R /*t*/, const R* ps, R* dy) {
    const R mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3], tau = ps[4];
    const R Sv = y[0], I1 = y[1], I2 = y[2], V = y[3];
    const R inf = phi * Sv * V;
    dy[0] = fma(mu, Sv, -inf);           // mu*S - phi*S*V
    dy[1] = fma(-tau, I1, inf);          // phi*S*V - tau*I1
    dy[2] = fma(tau, I1, -(lam * I2));   // tau*I1 - lam*I2
    dy[3] = fma(beta * lam, I2, -inf);   // beta*lam*I2 - phi*S*V
  }
};

// Synthetic N-state chain: S, I1..I_{N-2}, V | mu, phi, beta, lam, tau.
// N = 4 is exactly two_i.
template <int N>
struct Chain {
  static_assert(N >= 4, "chain model needs N >= 4");
  static constexpr int S = N, P = 5;
  template <class R>
  __host__ __device__ static inline void rhs(const R* y, R /*t*/, const R* ps, R* dy) {
    const R mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3], tau = ps[4];
    const R Sv = y[0], V = y[N - 1];
    const R inf = phi * Sv * V;
    dy[0] = fma(mu, Sv, -inf);                      // mu*S - phi*S*V
    dy[1] = fma(-tau, y[1], inf);                   // phi*S*V - tau*I1
#pragma unroll
    for (int k = 2; k <= N - 3; ++k) dy[k] = fma(tau, y[k - 1], -(tau * y[k]));  // tau*I(k-1) - tau*Ik
    dy[N - 2] = fma(tau, y[N - 3], -(lam * y[N - 2]));  // tau*I(N-3) - lam*I(N-2)
    dy[N - 1] = fma(beta * lam, y[N - 2], -inf);        // beta*lam*I(N-2) - phi*S*V
  }
};

}  // namespace oe
