// models.cuh — built-in right-hand sides, re-declared as device callbacks.
//
// The reference user writes `ODE(y, t, ps) -> np.ndarray` (ODElib/Framework.py:177-180)
// and odeint calls it from Fortran (Framework.py:656).  Here the RHS is a
// `__device__` function of one walker's state held in VGPRs.  Every expression
// keeps the operand order of the demo notebook's Python source
// (demo/Demo_InfectionStates.ipynb:60-128) and the library is compiled with
// -ffp-contract=off, so one RHS evaluation is bit-identical to numpy's scalar
// evaluation of the same Python function.
#pragma once

namespace oe {

// notebook zero_i (Demo_InfectionStates.ipynb:112-128): S, V | mu, phi, beta
struct ZeroI {
  static constexpr int S = 2, P = 3;
  template <class R>
  __host__ __device__ static inline void rhs(const R* y, R /*t*/, const R* ps, R* dy) {
    const R mu = ps[0], phi = ps[1], beta = ps[2];
    const R Sv = y[0], V = y[1];
    dy[0] = mu * Sv - phi * Sv * V;
    dy[1] = beta * phi * Sv * V - phi * Sv * V;
  }
};

// notebook one_i (Demo_InfectionStates.ipynb:78-94): S, I1, V | mu, phi, beta, lam
struct OneI {
  static constexpr int S = 3, P = 4;
  template <class R>
  __host__ __device__ static inline void rhs(const R* y, R /*t*/, const R* ps, R* dy) {
    const R mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3];
    const R Sv = y[0], I1 = y[1], V = y[2];
    dy[0] = mu * Sv - phi * Sv * V;
    dy[1] = phi * Sv * V - lam * I1;
    dy[2] = beta * lam * I1 - phi * Sv * V;
  }
};

// notebook two_i (Demo_InfectionStates.ipynb:60-75): S, I1, I2, V | mu, phi, beta, lam, tau
struct TwoI {
  static constexpr int S = 4, P = 5;
  template <class R>
  __host__ __device__ static inline void rhs(const R* y, R /*t*/, const R* ps, R* dy) {
    const R mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3], tau = ps[4];
    const R Sv = y[0], I1 = y[1], I2 = y[2], V = y[3];
    dy[0] = mu * Sv - phi * Sv * V;
    dy[1] = phi * Sv * V - tau * I1;
    dy[2] = tau * I1 - lam * I2;
    dy[3] = beta * lam * I2 - phi * Sv * V;
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
    dy[0] = mu * Sv - phi * Sv * V;
    dy[1] = phi * Sv * V - tau * y[1];
#pragma unroll
    for (int k = 2; k <= N - 3; ++k) dy[k] = tau * y[k - 1] - tau * y[k];
    dy[N - 2] = tau * y[N - 3] - lam * y[N - 2];
    dy[N - 1] = beta * lam * y[N - 2] - phi * Sv * V;
  }
};

}  // namespace oe
