// ode_kernels.cuh — batched ODE integration + fused likelihood + Metropolis–Hastings
// for MI355X (gfx950).  Header-only templates over a Model (models.cuh).
//
// Execution model:
//   * one lane = one walker; state y[S], parameters θ[P] and RK stages live in VGPRs;
//   * batched HBM layouts are walker-minor: y0/θ are [S|P][W], the trajectory is
//     [T][S][W], so each wave-instruction moves 64 × 8 B = 512 contiguous bytes;
//   * the time grid and the observation records are wave-uniform and are read
//     with scalar loads (SGPR/K$), never per lane;
//   * the likelihood (get_chi, Framework.py:685-697 / stats.py:41) and the R²
//     residual (stats.py:52) are accumulated inside the time loop at the
//     observation grid indices, so MCMC mode writes nothing per time step;
//   * DOPRI5 runs the 64 lanes of a wavefront in lockstep with one shared step
//     size: the per-lane max-norm error is max-reduced across the wave with
//     __shfl_xor, so there is no divergence.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "models.cuh"

namespace oe {

// ---- wave-uniform problem description (device copy made by oe_problem_set) ----
struct Obs {         // one observation, records sorted by grid index
  int32_t tidx;      // grid index (Framework.py:316 first-nearest)
  int32_t pad;
  uint64_t mask;     // states summed into the observed column (Framework.py:659-664)
  double O;          // observed log abundance
  double two_s2;     // 2*(S**2), stats.py:41
  double O_lin;      // exp(O) as numpy computed it (Framework.py:700)
};

// Wave-uniform, read-only tables are read through the constant address space so the
// loads are scalar (s_load → lgkmcnt).  A generic-pointer load would be a vector load
// the compiler must order against the trajectory stores, i.e. an s_waitcnt vmcnt(0)
// that drains every outstanding store each time step.
template <class T>
using cptr = const __attribute__((address_space(4))) T*;
template <class T>
__device__ __forceinline__ cptr<T> kconst(const T* p) {
  return (cptr<T>)(p);
}

struct DevProblem {
  const double* times;  // [T + 1]: the grid, then a +inf sentinel
  const double* rk4;    // [T][4]: h, h/2, h/6, t_i per interval (host-computed); row T-1 repeats row T-2
  const Obs* obs;       // [n_obs]
  int32_t T;
  int32_t n_obs;
  int32_t P;            // runtime parameter count (<= kPmax<Model>)
  int32_t substeps;     // RK4 steps per output interval
  double rtol, atol;
  int32_t max_steps;    // DOPRI5 steps per output interval
  int32_t pnum;         // AIC parameter count
  double sstot;         // R² denominator
  double newton_tol;    // BDF Newton tolerance, max(10·eps/rtol, min(0.03, sqrt(rtol))) (host-computed)
  double* obs_c;        // MH launches: [n_obs][lanes] scratch of the per-lane BDF pass's deferred
                        // observations (bdf.cuh); null elsewhere
};

enum : int32_t { ST_NONFINITE = 1, ST_NEGATIVE = 2, ST_MAXSTEP = 4, ST_STIFF = 8, ST_INTERNAL = 16 };

// integrators (OE_METHOD_*): fixed-step RK4, DOPRI5, DOPRI5 with stiffness detection and
// the Rosenbrock fallback for stiff / over-budget walkers (LSODA-like), Rosenbrock only
enum : int { kRK4 = 0, kDOPRI5 = 1, kAuto = 2, kRosenbrock = 3, kBdf = 4 };
constexpr int kMethods = 5;
constexpr int kStiffRegS = 8;   // up to here the stiff methods factor the S x S matrix in registers,
constexpr int kStiffMaxS = 32;  // above it in private memory (stiff.cuh); wider models: DOPRI5 only
constexpr int kStiffTestSteps = 3;  // auto: stiffness test from the 3rd step within one output interval
// auto: the stiffness test runs (and a lane it flags is handed to the Rosenbrock method)
// only while the wave's step is below (t_end - t)/kStiffSwitchSteps, i.e. while finishing
// at the stability limit would take DOPRI5 more steps than the Rosenbrock redo costs
// (LSODA switches on cost too).  Measured on one wave without trajectory (profiles/r02zu_stiff_onewave.log): DOPRI5
// at the stability limit ~1.1 us per step, the register RODAS redo 3-6.5 ms, so ~4000
// steps; the wide-model in-kernel redo (MH, matrices in private memory) is ~10-20x slower.
constexpr double kStiffSwitchSteps = 4000.0, kStiffSwitchStepsSlow = 40000.0;
// auto with S <= kStiffRegS: an evicted lane continues from its eviction point with BDF
// (bdf.cuh), which costs only the rest of the span, so the hand-over is cheap and taken
// early: the test runs from the 2nd step inside an output interval while finishing would
// take over kBdfSwitchSteps DOPRI5 steps, and a step counts as stiff at h·|λ| > 2.5 (the
// stability-limited crawl sits at 3.0-3.7) or, while over kBdfSwitchLong steps remain, at
// h·|λ| > 0.5 (accuracy-limited on a fast component: two_i τ = 1e3 takes DOPRI5 2 359
// steps at h·|λ| ≈ 0.9, the hand-over 94 + 436 BDF).
constexpr int kBdfTestSteps = 2;
constexpr double kBdfSwitchSteps = 300.0, kBdfSwitchLong = 1500.0;
constexpr double kBdfThr2 = 6.25, kBdfThrLong2 = 0.25;


// per-lane accumulators of the fused likelihood
struct Acc {
  double chi;     // Σ finite (O - log C)^2 / (2 S^2)
  double ssres;   // Σ non-NaN (C - O_lin)^2
  double nf;      // Σ y*0 over emitted states: NaN iff some state was non-finite
  double ymin;    // min over emitted states (fmin ignores NaN)
  int32_t nvalid; // number of finite chi terms
  int32_t status; // MAXSTEP bit set by DOPRI5; the other bits come from finish()
};

__device__ __forceinline__ Acc acc_init() { return Acc{0.0, 0.0, 0.0, __builtin_inf(), 0, 0}; }

// where 'auto' (S <= kStiffRegS) hands a lane to BDF: the state at the start of the step it
// was evicted on (or after the step that exhausted the budget), the next grid and
// observation indices, and the accumulators so far
template <int S>
struct Resume {
  double y[S];
  double t;
  int32_t i, k;
  Acc a;
};

__device__ __forceinline__ int32_t finish(const Acc& a) {
  int32_t st = a.status;
  if (__builtin_isnan(a.nf)) st |= ST_NONFINITE;
  if (a.ymin < 0.0) st |= ST_NEGATIVE;
  return st;
}

// Cross-lane max/min of a double over the 64-lane wave with DPP row operations
// (quad_perm xor1/xor2, row_half_mirror, row_mirror, row_bcast15, row_bcast31), then
// v_readlane of lane 63: ~18 VALU ops and no LDS round trip (ds_bpermute costs a lone
// wave ~60+ cycles per hop).  Result is wave-uniform.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int lo2 = __builtin_amdgcn_update_dpp(lo, lo, CTRL, ROW_MASK, 0xF, false);
  const int hi2 = __builtin_amdgcn_update_dpp(hi, hi, CTRL, ROW_MASK, 0xF, false);
  return __hiloint2double(hi2, lo2);
}
__device__ __forceinline__ double lane63(double v) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), 63);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), 63);
  return __hiloint2double(hi, lo);
}
// Wave maximum of NON-NEGATIVE, non-NaN values (the DOPRI5 error norm): every DPP hop is
// a plain mov_dpp with bound_ctrl and all rows enabled (a lane with no source reads 0,
// neutral for max; a bcast hop that also writes rows 0/2 hands them some in-wave value,
// which never exceeds the true maximum, and lane 63 still sees every row), and the max is
// a raw v_max_f64 — no copy for the DPP `old` operand and no canonicalising max of the
// DPP result: 3 VALU ops per hop instead of 6.  max is exact, so the hop order cannot
// change the result.
template <int CTRL>
__device__ __forceinline__ double dpp0_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double max_raw(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// fmax(|a|, |b|) in one op (the compiler canonicalises one operand first).  Quiet NaN in
// one operand returns the other, as C fmax does; the kernels never make signalling NaNs.
__device__ __forceinline__ double max_abs_raw(double a, double b) {
  double r;
  asm("v_max_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double min_raw(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double wave_max(double v) {
  v = max_raw(v, dpp0_f64<0xB1>(v));   // quad_perm [1,0,3,2]
  v = max_raw(v, dpp0_f64<0x4E>(v));   // quad_perm [2,3,0,1]
  v = max_raw(v, dpp0_f64<0x141>(v));  // row_half_mirror
  v = max_raw(v, dpp0_f64<0x140>(v));  // row_mirror
  v = max_raw(v, dpp0_f64<0x142>(v));  // row_bcast15: row r gets row r-1's maximum
  v = max_raw(v, dpp0_f64<0x143>(v));  // row_bcast31: rows 2, 3 get rows 0-1's maximum
  return lane63(v);
}
__device__ __forceinline__ double wave_min(double v) {
  v = fmin(v, dpp_f64<0xB1>(v));
  v = fmin(v, dpp_f64<0x4E>(v));
  v = fmin(v, dpp_f64<0x141>(v));
  v = fmin(v, dpp_f64<0x140>(v));
  v = fmin(v, dpp_f64<0x142, 0xA>(v));
  v = fmin(v, dpp_f64<0x143, 0xC>(v));
  return lane63(v);
}

template <bool B, class T, class F>
struct pick_type { using type = T; };
template <class T, class F>
struct pick_type<false, T, F> { using type = F; };

// register-array element at a (uniform) runtime index without spilling the array
// to scratch: a compile-time-unrolled select chain
template <int N>
__device__ __forceinline__ double pick(const double (&a)[N], int idx) {
  double v = 0.0;
#pragma unroll
  for (int j = 0; j < N; ++j) v = (j == idx) ? a[j] : v;
  return v;
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Store one trajectory row element through a buffer resource: descriptor (row base,
// row bytes) in SGPRs, lane offset w*8 in one VGPR, state offset s*W*8 in an SGPR —
// no per-store 64-bit VALU address arithmetic.  aux = 2 sets the non-temporal bit.
// Cache-policy bits of the trajectory row stores (gfx950: 1 sc0, 2 nt, 16 sc1).  nt + sc1
// (device scope) measured 1.9 % faster than nt alone on C1 back to back (0.3858 vs 0.3932
// ms, three runs each) and 2.3 % at 131 072 walkers (profiles/r02q_*); sc0+sc1+nt and
// sc0+sc1 within noise of it; plain stores 66 % slower (profiles/r02p_*).
#ifndef OE_NT_AUX
#define OE_NT_AUX 18
#endif
template <bool NT>
__device__ __forceinline__ void st_row(__amdgpu_buffer_rsrc_t rsrc, uint32_t lane_off, uint32_t s_off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rsrc, lane_off, s_off, NT ? OE_NT_AUX : 0);
}

// Out-of-line transcendentals.  Inlined, ocml's f64 log/exp polynomial constants are
// loop-invariant and get hoisted out of the time and MH loops into registers that stay
// live for the whole kernel (~40 doubles in the MH kernel); behind a call they are
// materialised per call (a call per observation / proposal, not per step).  A callee
// starts with s_waitcnt vmcnt(0), which drains the trajectory stores in flight, so the
// RK4 trajectory kernel (67 VGPRs either way) keeps the inline log (observe<S, true>).
#ifndef OE_TRANSC_CALL
#define OE_TRANSC_CALL 1
#endif
#if OE_TRANSC_CALL
__device__ __attribute__((noinline)) double oe_log(double x) { return log(x); }
__device__ __attribute__((noinline)) double oe_exp(double x) { return exp(x); }
#else
__device__ __forceinline__ double oe_log(double x) { return log(x); }
__device__ __forceinline__ double oe_exp(double x) { return exp(x); }
#endif

// NaN-propagating finiteness accumulator: a.nf becomes NaN iff some y[s] is NaN/inf.
template <int S>
__device__ __forceinline__ void check_finite(const double (&y)[S], Acc& a) {
#pragma unroll
  for (int s = 0; s < S; ++s) a.nf = fma(y[s], 0.0, a.nf);
}

// Store grid row i of the trajectory (TRAJ) and track the minimum state.  `off` is
// the lane's byte offset w*8 (32-bit); rows are stored through a per-row buffer
// descriptor (S*W*8 < 2^32, checked on the host): no per-store VALU address math.
template <int S>
__device__ __forceinline__ void track_min(const double (&y)[S], Acc& a) {
  // raw v_min_f64 (fmin's canonicalising copies of both operands doubled the VALU count
  // of the minimum); a quiet NaN operand returns the other, as C fmin does.  Pairwise
  // over the states (min is exact, so the order cannot change the result), then one
  // min into the running value: a shorter dependency chain than a serial fold.
  if constexpr (S == 1) {
    a.ymin = min_raw(a.ymin, y[0]);
  } else {
    double m[(S + 1) / 2];
#pragma unroll
    for (int j = 0; j < S / 2; ++j) m[j] = min_raw(y[2 * j], y[2 * j + 1]);
    if constexpr (S % 2) m[S / 2] = y[S - 1];
    double r = m[0];
#pragma unroll
    for (int j = 1; j < (S + 1) / 2; ++j) r = min_raw(r, m[j]);
    a.ymin = min_raw(a.ymin, r);
  }
}

// Store one trajectory row whose first element is at `row` (= traj + i*S*W).
template <int S, bool TRAJ, bool NT>
__device__ __forceinline__ void store_row_at(double* row, const double (&y)[S], int64_t W, uint32_t off,
                                             bool active, Acc& a) {
  track_min<S>(y, a);  // first: it schedules among the producer's VALU, not after the stores
  if constexpr (TRAJ) {
    if (active) {
      const uint32_t row_bytes = (uint32_t)(S * W * 8);
      const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)row, 0, row_bytes, 0x00020000);
#pragma unroll
      for (int s = 0; s < S; ++s) st_row<NT>(rsrc, off, (uint32_t)(s * W * 8), y[s]);
    }
  }
}

template <int S, bool TRAJ, bool NT>
__device__ __forceinline__ void store_row(int i, const double (&y)[S], double* __restrict__ traj,
                                          int64_t W, uint32_t off, bool active, Acc& a) {
  store_row_at<S, TRAJ, NT>(TRAJ ? traj + (int64_t)i * S * W : nullptr, y, W, off, active, a);
}

// Fold every observation recorded at grid index i into the likelihood (caller knows
// one exists or checks `k`).  Finiteness is checked here and at the final state
// (NaN/inf propagate through the RHS), not at every step.
template <int S, bool INLINE_LOG = false>
__device__ __forceinline__ void observe(const DevProblem& pb, int i, const double (&y)[S], int& k, Acc& a) {
  const cptr<Obs> obs = kconst(pb.obs);
  if (!(k < pb.n_obs && obs[k].tidx == i)) return;
  check_finite(y, a);
  while (k < pb.n_obs && obs[k].tidx == i) {
    const uint64_t mask = obs[k].mask;
    const double O = obs[k].O, two_s2 = obs[k].two_s2, O_lin = obs[k].O_lin;
    double c = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s)
      if ((mask >> s) & 1ull) c = c + y[s];  // increasing state order, as numpy's sum
    // chi term, in the operation order of stats.py:41
    const double d = O - (INLINE_LOG ? log(c) : oe_log(c));
    const double term = (d * d) / two_s2;
    if (__builtin_isfinite(term)) { a.chi += term; a.nvalid += 1; }
    // R² residual (stats.py:52 np.nansum skips NaN only)
    const double r = c - O_lin;
    const double r2 = r * r;
    if (!__builtin_isnan(r2)) a.ssres += r2;
    ++k;
  }
}

// observe() with the next observed grid index carried in a (uniform) register, so a
// grid point without an observation costs a compare instead of a scalar load + wait.
template <int S>
__device__ __forceinline__ void observe_next(const DevProblem& pb, int i, const double (&y)[S], int& k,
                                             int& nxt, Acc& a) {
  if (i != nxt) return;
  observe<S>(pb, i, y, k, a);
  nxt = (k < pb.n_obs) ? kconst(pb.obs)[k].tidx : 0x7fffffff;
}

// Emit grid point i: row store + minimum + observations.
template <int S, bool TRAJ, bool NT, bool INLINE_LOG = false>
__device__ __forceinline__ void emit(const DevProblem& pb, int i, const double (&y)[S],
                                     double* __restrict__ traj, int64_t W, uint32_t off,
                                     bool active, int& k, Acc& a) {
  store_row<S, TRAJ, NT>(i, y, traj, W, off, active, a);
  observe<S, INLINE_LOG>(pb, i, y, k, a);
}

template <int S, bool TRAJ>
__device__ __forceinline__ bool grid_needs_emit(const DevProblem& pb, int i, int k) {
  if constexpr (TRAJ) return true;
  return k < pb.n_obs && kconst(pb.obs)[k].tidx == i;
}

// ---------------------------------------------------------------------------------
// Fixed-step classical RK4; `substeps` steps per output interval.  Operation order
// (restated independently in oracle/rk_ref.c):
//   h = (t_i - t_{i-1})/n; hh = 0.5*h; h6 = h/6 (host table); substep j starts at t_{i-1} + j*h
//   k1 = f(t, y); yt = fma(hh,k1,y); k2 = f(t+hh, yt); yt = fma(hh,k2,y);
//   k3 = f(t+hh, yt); yt = fma(h,k3,y); k4 = f(t+h, yt)
//   acc = fma(2,k2,k1); acc = fma(2,k3,acc); acc = acc + k4; y = fma(h6,acc,y)
// ---------------------------------------------------------------------------------
template <class M, int PMAX>
__device__ __forceinline__ void rk4_step(double (&y)[M::S], double t, double h, double hh, double h6,
                                         const double (&p)[PMAX]) {
  constexpr int S = M::S;
  double k[S], acc[S], yt[S];
  M::rhs(y, t, p, k);
#pragma unroll
  for (int s = 0; s < S; ++s) { acc[s] = k[s]; yt[s] = fma(hh, k[s], y[s]); }
  M::rhs(yt, t + hh, p, k);
#pragma unroll
  for (int s = 0; s < S; ++s) { acc[s] = fma(2.0, k[s], acc[s]); yt[s] = fma(hh, k[s], y[s]); }
  M::rhs(yt, t + hh, p, k);
#pragma unroll
  for (int s = 0; s < S; ++s) { acc[s] = fma(2.0, k[s], acc[s]); yt[s] = fma(h, k[s], y[s]); }
  M::rhs(yt, t + h, p, k);
#pragma unroll
  for (int s = 0; s < S; ++s) { acc[s] = acc[s] + k[s]; y[s] = fma(h6, acc[s], y[s]); }
}

template <class M, int PMAX, bool TRAJ, bool NT>
__device__ __forceinline__ void integrate_rk4(const DevProblem& pb, double (&y)[M::S],
                                              const double (&p)[PMAX], double* traj,
                                              int64_t W, uint32_t off, bool active, Acc& a) {
  constexpr int S = M::S;
  int k = 0;
  emit<S, TRAJ, NT, TRAJ>(pb, 0, y, traj, W, off, active, k, a);
  const int n = pb.substeps;
  const cptr<Obs> obs = kconst(pb.obs);
  // Per-interval constants computed on the host exactly as h = (t_i - t_{i-1}) / n,
  // hh = 0.5*h, h6 = h/6, t_{i-1}; substep j starts at t_{i-1} + j*h.  The NEXT
  // interval's row is loaded while this interval computes: a lone wave otherwise waits
  // out a scalar-cache miss (one 64-B line per two intervals) every other step.  The
  // table has a padding row at the end, so the look-ahead pointer needs no clamp, and
  // the trajectory row pointer advances with the grid index (no per-row multiply: a
  // lone wave issues scalar instructions one per slot, like VALU).
  cptr<double> tab = kconst(pb.rk4);
  double h = tab[0], hh = tab[1], h6 = tab[2], t = tab[3];
  tab += 4;
  double* trow = TRAJ ? traj + (int64_t)S * W : nullptr;
  auto interval = [&]() {
    const double hn = tab[0], hhn = tab[1], h6n = tab[2], tn = tab[3];
    tab += 4;
    for (int j = 0; j < n; ++j) rk4_step<M, PMAX>(y, t + (double)j * h, h, hh, h6, p);
    h = hn; hh = hhn; h6 = h6n; t = tn;
  };
  int i = 1;
  while (i < pb.T) {
    // observation-free segment [i, next): step + row store only (no per-step obs logic)
    const int next = (k < pb.n_obs) ? obs[k].tidx : pb.T;
    for (; i < next; ++i) {
      interval();
      if constexpr (TRAJ) {
        store_row_at<S, TRAJ, NT>(trow, y, W, off, active, a);
        trow += S * W;
      }
    }
    if (i < pb.T) {  // i == next: an observed grid point
      interval();
      if constexpr (TRAJ) {
        store_row_at<S, TRAJ, NT>(trow, y, W, off, active, a);
        trow += S * W;
      }
      observe<S, TRAJ>(pb, i, y, k, a);
      ++i;
    }
  }
  check_finite(y, a);
}

// ---------------------------------------------------------------------------------
// Dormand–Prince 5(4) with FSAL and Hairer's 4th-order dense output; the 64 lanes
// of a wave share one step size (wave max of the per-lane max-norm error
//   err_lane = max_s |e_s| / (atol + rtol*max(|y_s|, |ynew_s|))).
// Walkers that pin the wave's step beyond the budget are evicted (status MAXSTEP,
// NaN output) so the rest of the wave keeps going.
// ---------------------------------------------------------------------------------
namespace dp {
constexpr double c2 = 1.0 / 5, c3 = 3.0 / 10, c4 = 4.0 / 5, c5 = 8.0 / 9;
constexpr double a21 = 1.0 / 5;
constexpr double a31 = 3.0 / 40, a32 = 9.0 / 40;
constexpr double a41 = 44.0 / 45, a42 = -56.0 / 15, a43 = 32.0 / 9;
constexpr double a51 = 19372.0 / 6561, a52 = -25360.0 / 2187, a53 = 64448.0 / 6561,
                 a54 = -212.0 / 729;
constexpr double a61 = 9017.0 / 3168, a62 = -355.0 / 33, a63 = 46732.0 / 5247,
                 a64 = 49.0 / 176, a65 = -5103.0 / 18656;
constexpr double a71 = 35.0 / 384, a73 = 500.0 / 1113, a74 = 125.0 / 192,
                 a75 = -2187.0 / 6784, a76 = 11.0 / 84;
constexpr double e1 = 71.0 / 57600, e3 = -71.0 / 16695, e4 = 71.0 / 1920,
                 e5 = -17253.0 / 339200, e6 = 22.0 / 525, e7 = -1.0 / 40;
constexpr double d1 = -12715105075.0 / 11282082432.0, d3 = 87487479700.0 / 32700410799.0,
                 d4 = -10690763975.0 / 1880347072.0, d5 = 701980252875.0 / 199316789632.0,
                 d6 = -1453857185.0 / 822651844.0, d7 = 69997945.0 / 29380423.0;
constexpr double safe = 0.9, facmin = 0.2, facmax = 10.0;

// The tableau as a table in device memory: trajectory kernels (one wave per SIMD, VGPRs
// to spare) load it once per lane into VGPRs instead of re-materialising each 64-bit
// constant with two s_mov per use and step.
__device__ const double kTab[36] = {a21, a31, a32, a41, a42, a43, a51, a52, a53, a54, a61, a62, a63, a64, a65,
                                    a71, a73, a74, a75, a76, e1, e3, e4, e5, e6, e7, d1, d3, d4, d5, d6, d7,
                                    c2, c3, c4, c5};
constexpr double kTabC[36] = {a21, a31, a32, a41, a42, a43, a51, a52, a53, a54, a61, a62, a63, a64, a65,
                              a71, a73, a74, a75, a76, e1, e3, e4, e5, e6, e7, d1, d3, d4, d5, d6, d7,
                              c2, c3, c4, c5};
struct Tab {
  double v[36];
};
// MIX (with VREG; k_integrate_hq): the stage couplings a_ij in VGPRs, the error, dense-output
// and node coefficients (e, d, c: 16 of 36) as immediates — 32 VGPRs fewer, for the
// co-residency budget of the hand-over queue's DOPRI5 kernel.
template <bool VREG, bool MIX = false, bool PIN = false>
__device__ __forceinline__ Tab load_tab() {
  Tab t;
  if constexpr (VREG) {
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));  // opaque per-lane zero: vector loads, values stay in VGPRs
    const double* p = kTab + z;
#pragma unroll
    for (int j = 0; j < 36; ++j) t.v[j] = (MIX && j >= 20) ? kTabC[j] : p[j];
  } else {
    const double c[36] = {a21, a31, a32, a41, a42, a43, a51, a52, a53, a54, a61, a62, a63, a64, a65,
                          a71, a73, a74, a75, a76, e1, e3, e4, e5, e6, e7, d1, d3, d4, d5, d6, d7,
                          c2, c3, c4, c5};
#pragma unroll
    for (int j = 0; j < 36; ++j) {
      if constexpr (PIN) {
        // SGPR immediates materialised here, at the integration's start (two s_mov inside a
        // volatile asm), instead of hoisted into the kernel's prologue: in the MH kernels they
        // would live across the whole iteration loop (proposal, accept, every call site),
        // where they are spilled to VGPR lanes
        constexpr uint64_t kOne = 1;
        const uint64_t b = __builtin_bit_cast(uint64_t, c[j]);
        uint32_t lo, hi;
        asm volatile("s_mov_b32 %0, %2\n\ts_mov_b32 %1, %3" : "=s"(lo), "=s"(hi)
                     : "i"((uint32_t)(b & 0xffffffffu)), "i"((uint32_t)(b >> 32)));
        (void)kOne;
        t.v[j] = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
      } else {
        t.v[j] = c[j];
      }
    }
  }
  return t;
}

// c[r] for a per-lane r in [0, N), N <= 8, as selects on r's bits.  (A chain of
// r == k ? … ternaries becomes a switch, lowered for a divergent r to compare-and-branch
// blocks with EXEC-mask bookkeeping: ~20 scalar instructions and four branches, which a
// lone wave issues one per slot.)
template <int N>
__device__ __forceinline__ double select_r(int r, const double (&c)[N]) {
  static_assert(N >= 1 && N <= 8, "select_r: at most 8 entries");
  auto at = [&](int k) { return c[k < N ? k : N - 1]; };
  const bool b0 = (r & 1) != 0, b1 = (r & 2) != 0, b2 = (r & 4) != 0;
  const double l0 = b0 ? at(1) : at(0), l1 = b0 ? at(3) : at(2);
  const double l2 = b0 ? at(5) : at(4), l3 = b0 ? at(7) : at(6);
  const double m0 = b1 ? l1 : l0, m1 = b1 ? l3 : l2;
  return b2 ? m1 : m0;
}

// how many of the grid times w[0..N) are <= x, per lane: the running count made opaque after
// each term (an empty asm on its VGPR), so the count is N compare + add-with-carry.  (Summed as
// plain bools, the vectoriser packs the N predicates into a bit mask and the callers'
// c != 0 / c == N tests become bit operations: ~2x the VALU, with hazard nops.)
template <int N>
__device__ __forceinline__ int count_le(const double (&w)[N], double x) {
  int c = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    c += (w[j] <= x) ? 1 : 0;
    asm("" : "+v"(c));
  }
  return c;
}

// x^(-1/5) for finite x > 0 (the step controller's err^(-1/5) and HINIT's
// (0.01/dm)^(1/5)).  Only exact scalings (frexp/ldexp) and IEEE mul/fma, so the host
// restatement (oracle/rk_ref.c inv_fifth_root) reproduces it bit for bit — libm's and
// ocml's pow/exp/log do not agree to the last ulp — and it is ~25 VALU ops instead
// of an exp(log()) pair.  x = m·2^e, e = 5q + r: x^(-1/5) = m^(-1/5)·2^(-r/5)·2^(-q);
// m^(-1/5) on [0.5, 1) from a quadratic start (1.5e-3) and two Newton steps (1.5e-10).
__device__ __forceinline__ double inv_fifth_root(double x) {
  int e;
  const double m = frexp(x, &e);
  int q = e / 5, r = e % 5;
  if (r < 0) { r += 5; q -= 1; }
  double y = fma(fma(0.2395, m, -0.6505), m, 1.4123);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const double y2 = y * y;
    const double y5 = (y2 * y2) * y;
    y = (y * fma(-m, y5, 6.0)) * 0.2;
  }
  constexpr double kC[5] = {1.0, 0.8705505632961241, 0.757858283255199, 0.6597539553864471, 0.5743491774985174};
  return ldexp(select_r(r, kC) * y, -q);
}

// inv_fifth_root of a WAVE-UNIFORM x (the step controller's err): the exponent part
// 2^(-r/5)·2^(-q) comes from one scalar load of kFifthScale[e + kFifthBias] instead of
// the integer division, the 5-way select and the ldexp (~30 scalar instructions, which a
// lone wave issues one per slot like VALU).  kFifthScale[e] = c_r·2^(-q) is exact (a
// power-of-two scaling of a normal number) and c_r·y ∈ (0.5, 1.3), so (c_r·2^(-q))·y is
// the same double as ldexp(c_r·y, -q): bit-identical to inv_fifth_root.
constexpr int kFifthBias = 1088;  // frexp exponents of finite positive doubles: -1073 .. 1024
struct FifthScale {
  double v[2 * kFifthBias];
  constexpr FifthScale() : v() {
    const double c[5] = {1.0, 0.8705505632961241, 0.757858283255199, 0.6597539553864471, 0.5743491774985174};
    for (int j = 0; j < 2 * kFifthBias; ++j) {
      const int e = j - kFifthBias;
      int q = e / 5, r = e % 5;
      if (r < 0) { r += 5; q -= 1; }
      const int be = 1023 - q;  // 2^(-q), a normal double for every e above
      v[j] = (be > 0 && be < 2047) ? c[r] * __builtin_bit_cast(double, (unsigned long long)be << 52) : 0.0;
    }
  }
};
__device__ const FifthScale kFifthScale{};
__device__ __forceinline__ double inv_fifth_root_uniform(double x, cptr<double> scale) {
  int e;
  const double m = frexp(x, &e);
  e = __builtin_amdgcn_readfirstlane(e);
  const double sc = scale[e + kFifthBias];
  double y = fma(fma(0.2395, m, -0.6505), m, 1.4123);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const double y2 = y * y;
    const double y5 = (y2 * y2) * y;
    y = (y * fma(-m, y5, 6.0)) * 0.2;
  }
  return sc * y;
}
}  // namespace dp

// AUTO: Hairer's stiffness test on every accepted step (h·|λ| estimated from the last two
// stages, ≥ 3.25 on 15 accepted steps in a row evicts the lane, as does the step
// budget); returns whether this (active) lane was evicted, i.e. needs the stiff method.
// ---- DOPRI5 trajectory output through store waves (k_integrate_dopri5_piped) ----------
// A compute wave publishes, per accepted step that reaches a grid time, the step's dense-
// output coefficients (y, ydf, bsp, r4, r5, ynew: 6·S doubles per lane) and the uniform
// (t, t_new, 1/h) into its own LDS slot ring; its store wave evaluates the dense output at
// every grid time of the step (the compute wave's own operations, so the same bits), tracks
// the running minimum and writes the rows with NT buffer stores.  The two waves synchronise
// through a produced / consumed counter pair per compute wave — no barrier couples the
// compute waves, whose step sequences differ.  Observed rows are still evaluated by the
// compute wave (the likelihood), every other row never costs it an instruction.
constexpr int kDpPipeFields = 6;  // y, ydf, bsp, r4, r5, ynew
template <int S>
constexpr int dp_pipe_slots() {  // slots per compute wave: 4 compute waves in 150 KiB of LDS
  return (150 * 1024) / (4 * (kDpPipeFields * S * 64 * 8 + 32)) < 8 ? (150 * 1024) / (4 * (kDpPipeFields * S * 64 * 8 + 32)) : 8;
}
template <int S>
struct DpPipe {
  double* ring;            // [R][6·S][64] this wave's slots
  double* uni;             // [R][4]: t, t_new, 1/h
  volatile int* produced;  // slots published by the compute wave
  volatile int* consumed;  // slots released by the store wave
  int lane, R, n, cons_seen;
};

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// wait for a free slot, fill it, publish it
template <int S>
__device__ __forceinline__ void dp_pipe_publish(DpPipe<S>& pp, double t, double tn, double rh, const double (&y)[S],
                                                const double (&ydf)[S], const double (&bsp)[S], const double (&r4)[S],
                                                const double (&r5)[S], const double (&yn)[S]) {
  while (pp.n - pp.cons_seen >= pp.R) {  // ring full: see how far the store wave is
    pp.cons_seen = *pp.consumed;
    if (pp.n - pp.cons_seen >= pp.R) __builtin_amdgcn_s_sleep(1);
  }
  const int slot = pp.n % pp.R;
  double* f = pp.ring + (size_t)slot * kDpPipeFields * S * 64 + pp.lane;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    f[(0 * S + s) * 64] = y[s];
    f[(1 * S + s) * 64] = ydf[s];
    f[(2 * S + s) * 64] = bsp[s];
    f[(3 * S + s) * 64] = r4[s];
    f[(4 * S + s) * 64] = r5[s];
    f[(5 * S + s) * 64] = yn[s];
  }
  if (pp.lane == 0) {
    pp.uni[slot * 4 + 0] = t;
    pp.uni[slot * 4 + 1] = tn;
    pp.uni[slot * 4 + 2] = rh;
  }
  lds_fence();  // the slot's data before the counter
  ++pp.n;
  if (pp.lane == 0) *pp.produced = pp.n;
}

#ifndef OE_LANE_INTEGRATE  // measurement / debug builds: chi-only oe_integrate on the per-lane DOPRI5 too
#define OE_LANE_INTEGRATE 0
#endif
// ---- The hand-over queue of 'auto' (S <= kHandMaxS: k_integrate_hq / k_bdf_hq) ----
// In k_integrate<M, auto> a lane handed to BDF waits for its wave's whole DOPRI5 pass and then
// runs its BDF pass in that wave: the wave's time is its DOPRI5 pass plus its slowest handed
// lane's BDF pass, at the pace of a lane sharing its CU with DOPRI5 waves.  The queue splits
// LSODA's two halves over two kernels: k_integrate_hq (the lockstep DOPRI5 pass without the
// BDF code, ~200 registers) puts a handed walker's state into a device-memory slot at its
// eviction point, and k_bdf_hq (one-wave workgroups, ~310 registers) runs the per-lane BDF
// pass (bdf.cuh) of each slot, one walker per wave.  Small ensembles (<= OE_HQ_MAX_W_PER_CU
// walkers per CU) launch k_bdf_hq beside the DOPRI5 kernel on a second stream (200 + 312 <= 512
// registers per SIMD: the BDF waves sit next to the DOPRI5 waves and start as walkers are
// handed over); larger ones launch it after the DOPRI5 kernel on the same stream, where every
// handed walker gets a SIMD of its own instead of one shared with DOPRI5 waves.  A per-lane
// BDF pass does not depend on the lane or wave running it (profiles/NOTES.md r05o): the same
// bits as the in-wave pass.  Measured against it (NOTES round 6, r06p; ms, 0.1 % / 1 % stiff):
// 1 024 walkers 1.92 -> 1.61 / 2.97 -> 1.79; 4 096: 2.09 -> 1.79 / 3.17 -> 1.80; 16 384: 2.35 ->
// 2.19 / 3.09 -> 2.22; 65 536 (C2): 2.49 -> 2.37 / 2.85 -> 2.87; none stiff: within 0.05 ms
// (after the DOPRI5 kernel the difference table then went to registers: C2 2.33 -> 2.26 / 2.86
// -> 2.77, r06z3).
// Rejected on the way: BDF waves inside the DOPRI5 workgroups (every wave then gets 256
// registers; BDF steps ~1.5x slower), the BDF kernel beside the DOPRI5 kernel for large
// ensembles (each BDF wave shares a SIMD with an issue-bound DOPRI5 wave: C2 + 1 % stiff
// 6.2 ms), slots claimed by CAS (a thousand waves on one counter: claims over 6.7 ms).
// Protocol (device scope): a producer lane reserves slot j (atomic ctl[0]), writes its state
// and publishes ready[j] = epoch with a release store; each producer wave adds one to ctl[2]
// after its pass.  BDF wave g's lane l takes slot g + l·G and waits until it is published or
// every producer wave is done without having reserved it.  Producers never wait on the BDF
// kernel, so any schedule of the two kernels finishes; a BDF wave also leaves, flagging ctl[3],
// past kHandTimeout.
constexpr int kHandMaxS = 4;  // the co-residency budget above (S = 5..8 keep the in-wave pass)
// the built-in models whose 'auto' integrate runs through the queue (always: OE_LANE_INTEGRATE
// measurement builds keep k_integrate's per-lane path instead)
template <class M, int METHOD>
constexpr bool kHandQueue = METHOD == kAuto && M::S <= kHandMaxS && !OE_LANE_INTEGRATE;
#ifndef OE_HQ_MAX_W_PER_CU  // oe_integrate takes the queue up to this many walkers per CU (r06i:
#define OE_HQ_MAX_W_PER_CU 16  // W = 1 024 / 4 096 win 20-40 %, 16 384 mixed, 65 536 loses)
#endif
#ifndef OE_HQ_POLL  // measurement builds: s_sleep(127)s between two polls of the queue
#define OE_HQ_POLL 8
#endif
#ifndef OE_HQ_MIX  // measurement builds: 0 = every tableau coefficient in VGPRs (breaks the budget)
#define OE_HQ_MIX 1
#endif
#ifndef OE_HQ_WAVES  // measurement builds: the most one-wave workgroups of k_bdf_hq
#define OE_HQ_WAVES 4096
#endif
#ifndef OE_HQ_PRIO  // measurement builds: 0 = the BDF waves at the default priority
#define OE_HQ_PRIO 1
#endif
#ifndef OE_HQ_TRACE  // measurement builds: a handed walker's chi / R² outputs carry, in µs from the
#define OE_HQ_TRACE 0  // DOPRI5 kernel's first wave, its BDF wave's start and (claim·1e5 + BDF pass)
#endif
constexpr uint64_t kHandTimeout = 6000000000ull;  // s_memrealtime ticks (100 MHz): 60 s
struct HandQ {
  double* d;        // [(S + 5)][cap]: y[0..S), t, chi, ssres, nf, ymin
  int32_t* n;       // [6][cap]: i, k, nvalid, status, walker, ready
  int32_t* ctl;     // [0] reserved, [1] claimed, [2] producer waves done, [3] timeout, [4] BDF waves
                    // that claimed or left (trace builds: [6..9] two 64-bit clocks)
  int32_t cap;      // slots (>= walkers of the launch)
  int32_t epoch;    // ready[j] == epoch: slot j of this launch is published
  int32_t n_waves;  // producer waves of the launch
};
// Polls are relaxed device-scope loads: an acquire load at agent scope invalidates the XCD's L2
// on every poll, and a few hundred polling waves then cost the DOPRI5 kernel 3x its time
// (r06c).  One acquire fence follows a successful poll (the slot data, the final count).
__device__ __forceinline__ int32_t hq_load(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void hq_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); }
// a producer lane's hand-over: its state at the eviction point (y, t, grid index i, next
// observation record k, accumulators; status gets ST_STIFF as the BDF pass's input)
template <int S>
__device__ __forceinline__ void hand_push(const HandQ& q, const double (&y)[S], double t, int i, int k,
                                          const Acc& a, int64_t w) {
  const int64_t c = q.cap;
  const int j = atomicAdd(q.ctl, 1);
#pragma unroll
  for (int s = 0; s < S; ++s) q.d[s * c + j] = y[s];
  q.d[S * c + j] = t;
  q.d[(S + 1) * c + j] = a.chi;
  q.d[(S + 2) * c + j] = a.ssres;
  q.d[(S + 3) * c + j] = a.nf;
  q.d[(S + 4) * c + j] = a.ymin;
  q.n[j] = i;
  q.n[c + j] = k;
  q.n[2 * c + j] = a.nvalid;
  q.n[3 * c + j] = a.status | ST_STIFF;
  q.n[4 * c + j] = (int32_t)w;
  __hip_atomic_store(q.n + 5 * c + j, q.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// RESUME (auto, S <= kStiffRegS): an evicted lane is handed over to BDF — its state at the
// eviction point goes to *rs and the return value says so — instead of being redone from t0.
// QUEUE (with RESUME, k_integrate_hq): it goes to the hand-over queue *hq instead, and the lane
// stores no more rows (the BDF kernel writes them).
// PIPE (trajectory mode, S <= 8, k_integrate_dopri5_piped): the rows go through *pp to the
// store wave (same values, same minimum), the compute wave only evaluates observed rows.
template <class M, int PMAX, bool TRAJ, bool NT, bool AUTO = false, bool SLOW_REDO = false, bool RESUME = false,
          bool PIPE = false, bool QUEUE = false, bool MIX = false>
__device__ __forceinline__ bool integrate_dopri5(const DevProblem& pb, double (&y)[M::S],
                                                 const double (&p)[PMAX], double* traj,
                                                 int64_t W, uint32_t off, bool active, Acc& a,
                                                 Resume<M::S>* rs = nullptr, DpPipe<M::S>* pp = nullptr,
                                                 const HandQ* hq = nullptr) {
  using namespace dp;
  constexpr int S = M::S;
  static_assert(!PIPE || (TRAJ && S <= 8 && !AUTO), "the piped output is DOPRI5 trajectory mode's, S <= 8");
  static_assert(!QUEUE || RESUME, "the hand-over queue takes the RESUME hand-over");
  int k = 0;
  if constexpr (PIPE) {  // row 0 = the initial state: a slot whose end time is times[0]
    const double t00 = kconst(pb.times)[0];
    dp_pipe_publish<S>(*pp, t00, t00, 0.0, y, y, y, y, y, y);
    observe<S>(pb, 0, y, k, a);
  } else {
    emit<S, TRAJ, NT>(pb, 0, y, traj, W, off, active, k, a);
  }
  const cptr<double> times = kconst(pb.times);
  const double t0 = times[0];
  const double tend = times[pb.T - 1];
  const double rtol = pb.rtol, atol = pb.atol;
  bool dead = !active;  // dead lanes never enter the wave norm
  bool handed = false;  // RESUME: this lane was handed over to BDF
  double t = t0;
  const Tab tb = load_tab<TRAJ && (M::S <= 8), MIX && OE_HQ_MIX>();
  double k1[S], k2[S], k3[S], k4[S], k5[S], k6[S], k7[S], yt[S], yn[S];
  M::rhs(y, t, p, k1);

  // ---- initial step: Hairer's HINIT per lane (max norm), wave minimum ----
  double h;
  {
    double d0 = 0.0, d1v = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double sk = atol + rtol * fabs(y[s]);
      d0 = fmax(d0, fabs(y[s]) / sk);
      d1v = fmax(d1v, fabs(k1[s]) / sk);
    }
    double h0 = (d0 <= 1e-5 || d1v <= 1e-5) ? 1e-6 : 0.01 * (d0 / d1v);
    h0 = fmin(h0, tend - t0);
#pragma unroll
    for (int s = 0; s < S; ++s) yt[s] = fma(h0, k1[s], y[s]);
    M::rhs(yt, t + h0, p, k2);
    double d2 = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double sk = atol + rtol * fabs(y[s]);
      d2 = fmax(d2, fabs(k2[s] - k1[s]) / sk);
    }
    d2 = d2 / h0;
    const double dm = fmax(d1v, d2);
    const double h1 = (dm <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : inv_fifth_root(dm / 0.01);
    double hl = fmin(100.0 * h0, h1);
    if (dead || !__builtin_isfinite(hl) || !(hl > 0.0)) hl = tend - t0;
    h = wave_min(hl);
    h = fmin(h, tend - t0);
  }

  const double span = tend - t0;
  const double hmin = 1e-14 * fmax(fabs(tend), fabs(t0)) + 1e-300;
  // S <= 8: times[i] loaded one grid point ahead, next observed index carried, evicted
  // lanes poisoned with NaN (no per-point select).  S > 8 sits at the register limit,
  // so it keeps the leaner form (same outputs and status bits).
  constexpr bool kLean = S > 8;
  static_assert(!RESUME || (AUTO && !kLean), "the BDF hand-over is the register path's");
  int i = 1;
  double t_i = times[1];
  cptr<double> tnext = times + 2;  // &times[i + 1]
  // row i of the trajectory, advanced with i (no 64-bit multiply per emitted row)
  double* trow = TRAJ ? traj + (int64_t)S * W : nullptr;
  const cptr<double> fifth = kconst(kFifthScale.v);
  int nxt = (k < pb.n_obs) ? kconst(pb.obs)[k].tidx : 0x7fffffff;  // next observed index
  double t_obs = (nxt < pb.T) ? times[nxt] : __builtin_inf();        // and its time
  int nst = 0;  // steps since the last grid point
  bool last_rej = false;
  int n_stiff = 0, n_nonstiff = 0;  // AUTO: consecutive stiff / non-stiff accepted steps
  while (i < pb.T) {
    bool last = false;
    if (t + h >= tend) { h = tend - t; last = true; }
    // h-scaled tableau (wave-uniform), then one fma chain per stage and state
    const double b21 = h * tb.v[0];
    const double b31 = h * tb.v[1], b32 = h * tb.v[2];
    const double b41 = h * tb.v[3], b42 = h * tb.v[4], b43 = h * tb.v[5];
    const double b51 = h * tb.v[6], b52 = h * tb.v[7], b53 = h * tb.v[8], b54 = h * tb.v[9];
    const double b61 = h * tb.v[10], b62 = h * tb.v[11], b63 = h * tb.v[12], b64 = h * tb.v[13], b65 = h * tb.v[14];
    const double b71 = h * tb.v[15], b73 = h * tb.v[16], b74 = h * tb.v[17], b75 = h * tb.v[18], b76 = h * tb.v[19];
#pragma unroll
    for (int s = 0; s < S; ++s) yt[s] = fma(b21, k1[s], y[s]);
    M::rhs(yt, t + tb.v[32] * h, p, k2);
#pragma unroll
    for (int s = 0; s < S; ++s) yt[s] = fma(b32, k2[s], fma(b31, k1[s], y[s]));
    M::rhs(yt, t + tb.v[33] * h, p, k3);
#pragma unroll
    for (int s = 0; s < S; ++s) yt[s] = fma(b43, k3[s], fma(b42, k2[s], fma(b41, k1[s], y[s])));
    M::rhs(yt, t + tb.v[34] * h, p, k4);
#pragma unroll
    for (int s = 0; s < S; ++s)
      yt[s] = fma(b54, k4[s], fma(b53, k3[s], fma(b52, k2[s], fma(b51, k1[s], y[s]))));
    M::rhs(yt, t + tb.v[35] * h, p, k5);
#pragma unroll
    for (int s = 0; s < S; ++s)
      yt[s] = fma(b65, k5[s], fma(b64, k4[s], fma(b63, k3[s], fma(b62, k2[s], fma(b61, k1[s], y[s])))));
    M::rhs(yt, t + h, p, k6);
#pragma unroll
    for (int s = 0; s < S; ++s)
      yn[s] = fma(b76, k6[s], fma(b75, k5[s], fma(b74, k4[s], fma(b73, k3[s], fma(b71, k1[s], y[s])))));
    // AUTO, wide models: the stiffness test's Σ(ynew − y6)² is summed here, on the steps
    // that will test (the same wave-uniform gate, one step ahead of the ++nst below), so
    // the stage-6 input dies before k7 instead of living through the error norm — S more
    // doubles at the kernel's register peak (same values, same order: bit-identical)
    constexpr double kSwitch = RESUME ? kBdfSwitchSteps : SLOW_REDO ? kStiffSwitchStepsSlow : kStiffSwitchSteps;
    constexpr int kTestSteps = RESUME ? kBdfTestSteps : kStiffTestSteps;
    double stden_early = 0.0;
    if constexpr (AUTO && kLean) {
      if (nst + 1 >= kTestSteps && (tend - t) > kSwitch * h) {
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const double r = 1.0 / fma(rtol, max_abs_raw(y[s], yn[s]), atol);
          const double dy = (yn[s] - yt[s]) * r;
          stden_early = fma(dy, dy, stden_early);
        }
      }
    }
    M::rhs(yn, t + h, p, k7);
    // ---- per-lane max-norm error: argmax of |e_s|/sk_s by exact cross-multiplication,
    //      then ONE division; non-finite anywhere -> 1e30 (forces a reject) ----
    const double g1 = h * tb.v[20], g3 = h * tb.v[21], g4 = h * tb.v[22], g5 = h * tb.v[23], g6 = h * tb.v[24],
                 g7 = h * tb.v[25];
    double num = 0.0, den = 1.0, nfe = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double e = fma(g7, k7[s], fma(g6, k6[s], fma(g5, k5[s], fma(g4, k4[s], fma(g3, k3[s], g1 * k1[s])))));
      const double ae = fabs(e);
      const double sk = fma(rtol, max_abs_raw(y[s], yn[s]), atol);
      nfe = fma(ae, 0.0, nfe);
      if (s == 0 || ae * den > num * sk) { num = ae; den = sk; }
    }
    double el = num / den;
    if (!__builtin_isfinite(el) || __builtin_isnan(nfe)) el = 1e30;
    if (dead) el = 0.0;
    const double err = wave_max(el);
    ++nst;

    if (err <= 1.0) {
      // stiffness: h²·Σ(k7−k6)² > 3.25²·Σ(ynew − y6)² (y6 = the stage-6 input), i.e.
      // h·|λ| > 3.25 (Hairer & Wanner I, §II.10); exact products, no square root.  Each
      // component is weighted by 1/(atol + rtol·max(|y|,|ynew|)), the error control's
      // scale: unweighted, the 1e7-sized host/virus compartments swamp a stiff mode in a
      // small compartment (two_i with tau = 1e4 or 3e4 was never flagged and crawled at
      // 11-28 ms per integration, where RODAS takes 6 ms).  Tested
      // only on steps that stay within one output interval for the 3rd time or more (a
      // wave-uniform gate): a stiff lane pins the shared step far below the grid spacing,
      // while a non-stiff wave spans grid points with nearly every step and never pays.
      // The test also runs only while the shared step is below (t_end - t)/kSwitch (the
      // cost gate above), so a mildly stiff wave that DOPRI5 finishes cheaper than the
      // Rosenbrock redo never pays for it.
      if (AUTO && nst >= kTestSteps && (tend - t) > kSwitch * h) {
        double stnum = 0.0, stden = stden_early;
        const double thr2 = !RESUME ? 10.5625 : ((tend - t) > kBdfSwitchLong * h) ? kBdfThrLong2 : kBdfThr2;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const double r = 1.0 / fma(rtol, max_abs_raw(y[s], yn[s]), atol);
          const double dk = (k7[s] - k6[s]) * r;
          stnum = fma(dk, dk, stnum);
          if constexpr (!kLean) {
            const double dy = (yn[s] - yt[s]) * r;
            stden = fma(dy, dy, stden);
          }
        }
        if (stden > 0.0 && (h * h) * stnum > thr2 * stden) {
          n_nonstiff = 0;
          ++n_stiff;
        } else if (++n_nonstiff >= 6) {
          n_stiff = 0;
        }
        if (!dead && n_stiff >= 15) {  // hand the walker to the stiff method
          dead = true;
          if constexpr (QUEUE) {  // at the start of this step, to the BDF kernel
            handed = true;
            hand_push<S>(*hq, y, t, i, k, a, (int64_t)(off >> 3));
          } else if constexpr (RESUME) {  // at the start of this step
            handed = true;
#pragma unroll
            for (int s = 0; s < S; ++s) rs->y[s] = y[s];
            rs->t = t;
            rs->i = i;
            rs->k = k;
            rs->a = a;
          }
#pragma unroll
          for (int s = 0; s < S; ++s) { yn[s] = __builtin_nan(""); k7[s] = __builtin_nan(""); }
        }
      }
      if constexpr (RESUME) {  // every lane handed over (or idle): nothing left for this pass
        if (__ballot(!dead) == 0ull) break;
      }
      const double tn = last ? tend : t + h;
      // Dense output for every grid point in (t, tn] from Hairer's coefficients
      // ydf, bsp, r4, r5.  Trajectory mode: formed eagerly once per accepted step (a grid
      // point nearly always falls in the step, and k2..k6 die before the output loop).
      // Otherwise (observed points only): small S forms them on the first observed point
      // of the step, large S per observed point (lazily kept k's would spill).
      // S <= 8 without trajectory: formed once, eagerly, in the steps that reach the next
      // observed time (the k's then die before the output loop); S > 8 per observed point.
      const bool kEager = TRAJ || (!kLean && t_obs <= tn);
      constexpr bool kHoist = TRAJ || S <= 8;
      const double rh = 1.0 / h;  // one division per step, not per grid point
      double ydf[kHoist ? S : 1], bsp[kHoist ? S : 1], r4[kHoist ? S : 1], r5[kHoist ? S : 1];
      const double hd1 = h * tb.v[26], hd3 = h * tb.v[27], hd4 = h * tb.v[28], hd5 = h * tb.v[29],
                   hd6 = h * tb.v[30], hd7 = h * tb.v[31];
      if (kHoist && kEager) {
#pragma unroll
        for (int s = 0; s < S; ++s) {
          ydf[s] = yn[s] - y[s];
          bsp[s] = fma(h, k1[s], -ydf[s]);
          r4[s] = fma(-h, k7[s], ydf[s]) - bsp[s];
          r5[s] = fma(hd7, k7[s], fma(hd6, k6[s], fma(hd5, k5[s], fma(hd4, k4[s], fma(hd3, k3[s], hd1 * k1[s])))));
        }
      }
      if constexpr (!kLean) {
        // PIPE: a step that reaches a grid time hands its coefficients to the store wave
        if constexpr (PIPE) {
          if (t_i <= tn) dp_pipe_publish<S>(*pp, t, tn, rh, y, ydf, bsp, r4, r5, yn);
        }
        constexpr bool kAll = TRAJ && !PIPE;  // every grid point evaluated here
        // grid points strictly inside the step: dense output (no per-point test for the
        // end point, whose row is the new state itself: handled after the loop, so the
        // dense values go straight to the store registers)
        // (times[T] is a +inf sentinel: the look-ahead load needs no clamp, and t_i < tn
        //  fails once i reaches T)
        while (t_i < tn) {
          const double ti = t_i;
          t_i = *tnext++;  // times[i + 1]: issued now, used next iteration
          if (kAll || i == nxt) {
            const double th = (ti - t) * rh;
            const double th1 = 1.0 - th;
            double yo[S];
#pragma unroll
            for (int s = 0; s < S; ++s)
              yo[s] = fma(th, fma(th1, fma(th, fma(th1, r5[s], r4[s]), bsp[s]), ydf[s]), y[s]);
            // (an evicted lane's state is NaN, so its dense output is NaN already)
            if constexpr (!PIPE) store_row_at<S, TRAJ, NT>(trow, yo, W, off, QUEUE ? active && !handed : active, a);
            if (i == nxt) {
              observe_next<S>(pb, i, yo, k, nxt, a);
              t_obs = times[nxt < pb.T ? nxt : pb.T];
            }
          }
          ++i;
          if constexpr (kAll) trow += S * W;
          nst = 0;
        }
        if (t_i == tn) {  // a grid point on the step's end
          t_i = *tnext++;
          if (kAll || i == nxt) {
            if constexpr (!PIPE) store_row_at<S, TRAJ, NT>(trow, yn, W, off, QUEUE ? active && !handed : active, a);
            if (i == nxt) {
              observe_next<S>(pb, i, yn, k, nxt, a);
              t_obs = times[nxt < pb.T ? nxt : pb.T];
            }
          }
          ++i;
          if constexpr (kAll) trow += S * W;
          nst = 0;
        }
      } else {
        while (i < pb.T && times[i] <= tn) {
          const double ti = times[i];
          if (grid_needs_emit<S, TRAJ>(pb, i, k)) {
            double yo[S];
            if (ti == tn) {
#pragma unroll
              for (int s = 0; s < S; ++s) yo[s] = yn[s];
            } else {
              const double th = (ti - t) * rh;
              const double th1 = 1.0 - th;
              if constexpr (kHoist) {  // coefficients formed above (every emitted point has them)
#pragma unroll
                for (int s = 0; s < S; ++s)
                  yo[s] = fma(th, fma(th1, fma(th, fma(th1, r5[s], r4[s]), bsp[s]), ydf[s]), y[s]);
              } else {
#pragma unroll
                for (int s = 0; s < S; ++s) {
                  const double ydf1 = yn[s] - y[s];
                  const double bsp1 = fma(h, k1[s], -ydf1);
                  const double r41 = fma(-h, k7[s], ydf1) - bsp1;
                  const double r51 = fma(hd7, k7[s], fma(hd6, k6[s], fma(hd5, k5[s], fma(hd4, k4[s], fma(hd3, k3[s], hd1 * k1[s])))));
                  yo[s] = fma(th, fma(th1, fma(th, fma(th1, r51, r41), bsp1), ydf1), y[s]);
                }
              }
            }
            if (dead) {
#pragma unroll
              for (int s = 0; s < S; ++s) yo[s] = __builtin_nan("");
            }
            emit<S, TRAJ, NT>(pb, i, yo, traj, W, off, active, k, a);
          }
          ++i;
          nst = 0;
        }
      }
#pragma unroll
      for (int s = 0; s < S; ++s) { y[s] = yn[s]; k1[s] = k7[s]; }
      t = tn;
      double fac = (err > 0.0) ? safe * inv_fifth_root_uniform(err, fifth) : facmax;
      fac = fmin(facmax, fmax(facmin, fac));
      if (last_rej) fac = fmin(fac, 1.0);
      h = h * fac;
      last_rej = false;
    } else {
      h = h * fmax(facmin, safe * inv_fifth_root_uniform(err, fifth));
      last_rej = true;
    }
    // ---- budget: evict the walkers that pin the wave's step ----
    if (i < pb.T && (nst >= pb.max_steps || h < hmin)) {  // (not after the last grid point)
      if (!dead && el >= 0.5 * err) {
        dead = true;
        if constexpr (QUEUE) {  // handed over at its current state, to the BDF kernel
          handed = true;
          hand_push<S>(*hq, y, t, i, k, a, (int64_t)(off >> 3));
        } else if constexpr (RESUME) {  // handed over at its current state
          handed = true;
#pragma unroll
          for (int s = 0; s < S; ++s) rs->y[s] = y[s];
          rs->t = t;
          rs->i = i;
          rs->k = k;
          rs->a = a;
        } else {
          a.status |= ST_MAXSTEP;
        }
        // poison the lane: every later dense output (and the final state) is NaN
        if constexpr (!kLean) {
#pragma unroll
          for (int s = 0; s < S; ++s) { y[s] = __builtin_nan(""); k1[s] = __builtin_nan(""); }
        }
      }
      nst = pb.max_steps / 2;
      if (__ballot(!dead) == 0ull) {
        // every lane is out: emit NaN rows for the rest of the grid and stop
        double yo[S];
#pragma unroll
        for (int s = 0; s < S; ++s) yo[s] = __builtin_nan("");
        if constexpr (PIPE) {  // one slot of NaN coefficients reaching t = +inf: NaN rows to the end
          dp_pipe_publish<S>(*pp, t, __builtin_inf(), 0.0, yo, yo, yo, yo, yo, yo);
          for (; i < pb.T; ++i) observe<S>(pb, i, yo, k, a);
        } else if constexpr (RESUME) {
          // every lane handed over (or idle): the BDF pass writes their rows
        } else {
          for (; i < pb.T; ++i)
            if (grid_needs_emit<S, TRAJ>(pb, i, k)) emit<S, TRAJ, NT>(pb, i, yo, traj, W, off, active, k, a);
        }
        break;
      }
      if (h < hmin) h = fmin(1e-3 * span, tend - t);
    }
  }
  if (dead && active) a.status |= ST_MAXSTEP;
  check_finite(y, a);
  if (kLean && dead) a.nf = __builtin_nan("");  // as if poisoned: final state non-finite
  if constexpr (RESUME) return handed && active;
  return dead && active;
}

}  // namespace oe
namespace oe {
#ifndef OE_GRID_WIN  // measurement builds (tools/build_alt.sh): the per-lane DOPRI5's grid window
#define OE_GRID_WIN 8
#endif
constexpr int kGridWin = OE_GRID_WIN;  // the time grid buffer carries kGridWin + 1 +inf sentinels (lane.cuh)
}
#include "stiff.cuh"
#include "bdf.cuh"
#include "bdf_wave.cuh"
#include "lane.cuh"
namespace oe {

// WAVE_REDO (batched integrate of models wider than kStiffRegS): 'auto' only marks the
// walkers the DOPRI5 pass evicts (status ST_STIFF); k_stiff_wave redoes them one wave per
// walker (stiff_wave.cuh).  The MH kernel redoes them in place (private-memory path).
// LANE (kernels without a trajectory, S <= 8): DOPRI5 with a step size per lane (lane.cuh)
// instead of one per wave.
template <class M, int METHOD>
constexpr bool kLaneSteps = (METHOD == kDOPRI5 || METHOD == kAuto || METHOD == kBdf) && M::S <= kStiffRegS;

template <class M, int PMAX, int METHOD, bool TRAJ, bool NT, bool WAVE_REDO = false, bool LANE = false>
__device__ __forceinline__ void integrate_walker(const DevProblem& pb, double (&y)[M::S],
                                                 const double (&p)[PMAX], double* traj,
                                                 int64_t W, int64_t w, bool active, Acc& a) {
  static_assert(!LANE || (!TRAJ && kLaneSteps<M, METHOD>), "per-lane steps: no trajectory, DOPRI5/auto/bdf, S <= 8");
  const uint32_t off = (uint32_t)w * 8u;  // byte offset of walker w in a [..][W] row
  if constexpr (METHOD == kRK4) {
    integrate_rk4<M, PMAX, TRAJ, NT>(pb, y, p, traj, W, off, active, a);
  } else if constexpr (LANE && METHOD == kDOPRI5) {
    integrate_dopri5_lane<M, PMAX, false>(pb, y, p, W, off, active, a);
  } else if constexpr (METHOD == kDOPRI5 || M::S > kStiffMaxS) {
    integrate_dopri5<M, PMAX, TRAJ, NT>(pb, y, p, traj, W, off, active, a);
  } else if constexpr (METHOD == kBdf) {  // LSODA's BDF branch for every walker (S <= kStiffRegS)
    static_assert(M::S <= kStiffRegS, "bdf: register path only");
    int k = 0;
    emit<M::S, TRAJ, NT>(pb, 0, y, traj, W, off, active, k, a);
    if constexpr (LANE)  // MH kernels: every chain with its own step sizes and orders (bdf.cuh)
      integrate_bdf_lane<M, PMAX, TRAJ, NT>(pb, y, kconst(pb.times)[0], 1, k, p, traj, W, w, active, active, a);
    else  // integrate kernels: the wave-lockstep pass (bdf_wave.cuh), as their DOPRI5
      integrate_bdf<M, PMAX, TRAJ, NT>(pb, y, kconst(pb.times)[0], 1, k, p, traj, W, w, active, active, a);
  } else if constexpr (METHOD == kAuto && M::S <= kStiffRegS && LANE) {
    // per-lane DOPRI5 whose flagged lanes continue with BDF from their own eviction points
    // (the BDF pass is lane.cuh's tail: it starts from the DOPRI5 pass's live state)
    integrate_dopri5_lane<M, PMAX, true>(pb, y, p, W, off, active, a);
  } else if constexpr (METHOD == kAuto && M::S <= kStiffRegS) {
    // LSODA-like: DOPRI5 with the stiffness test; a lane it evicts (stiff, or over the step
    // budget) continues from the eviction point with BDF (status bit ST_STIFF)
    Resume<M::S> rs;  // defined for every lane (only handed lanes use it)
#pragma unroll
    for (int s = 0; s < M::S; ++s) rs.y[s] = y[s];
    rs.t = 0.0;
    rs.i = pb.T;
    rs.k = 0;
    rs.a = a;
    const bool handed = integrate_dopri5<M, PMAX, TRAJ, NT, true, false, true>(pb, y, p, traj, W, off, active, a, &rs);
    if (__ballot(handed) != 0ull) {  // wave-uniform
      if (handed) {
        a = rs.a;
        a.status |= ST_STIFF;
      }
      integrate_bdf_lane<M, PMAX, TRAJ, NT>(pb, rs.y, rs.t, rs.i, rs.k, p, traj, W, w, active, handed, a);
      if (handed) {
#pragma unroll
        for (int s = 0; s < M::S; ++s) y[s] = rs.y[s];
      }
    }
  } else if constexpr (METHOD == kAuto && WAVE_REDO) {
    if (integrate_dopri5<M, PMAX, TRAJ, NT, true>(pb, y, p, traj, W, off, active, a)) a.status |= ST_STIFF;
  } else if constexpr (METHOD == kAuto) {
    // LSODA-like: DOPRI5 with the stiffness test; walkers it evicts (stiff, or over the
    // step budget) are integrated again from their initial state by the Rosenbrock
    // method, their likelihood accumulated afresh (status bit ST_STIFF)
    constexpr int S = M::S;
    // the initial state for a restart; wide models keep it in private memory rather than
    // in S register pairs live across the whole DOPRI5 pass
    using YI = typename pick_type<(S <= kStiffRegS), double, volatile double>::type;
    YI yi[S];
#pragma unroll
    for (int s = 0; s < S; ++s) yi[s] = y[s];
    const bool redo = integrate_dopri5<M, PMAX, TRAJ, NT, true, (S > kStiffRegS)>(pb, y, p, traj, W, off, active, a);
    if (__ballot(redo) != 0ull) {  // wave-uniform
      if (redo) {
#pragma unroll
        for (int s = 0; s < S; ++s) y[s] = yi[s];
        a = acc_init();
        a.status = ST_STIFF;
      }
      rosenbrock_lanes<M, PMAX, TRAJ, NT>(pb, y, p, traj, W, off, active, redo, a);
    }
  } else {  // kRosenbrock: the Rosenbrock method for every walker
    rosenbrock_lanes<M, PMAX, TRAJ, NT>(pb, y, p, traj, W, off, active, active, a);
  }
}

// ---------------------------------------------------------------------------------
// Kernel 1: batched integrate (+ fused chi / R² residual).
// ---------------------------------------------------------------------------------
struct IntegrateArgs {
  int64_t W;
  const double* y0;     // [S][W]
  const double* theta;  // [P][W]
  double* traj;         // [T][S][W] or null
  double* chi;          // [W] or null
  double* ssres;        // [W] or null
  int32_t* status;      // [W] or null
  int32_t half;         // 1: 32 walkers per wavefront (lanes 32-63 idle), 0: 64
  int32_t xcd_remap;    // 0: walker blocks in blockIdx order; c > 0: the blocks dispatched to
                        //    the 8 XCDs (blockIdx % 8, round-robin) take runs of c consecutive
                        //    walker blocks in turn (xcd_block)
};

// Workgroups are dispatched round-robin over the 8 XCDs (each with its own L2).  Map
// them so the XCDs take runs of c consecutive walker blocks in turn: XCD x's j-th block
// is block (j mod c) of run (j / c) * 8 + x.  With c blocks = 512 walkers every XCD writes
// 4 KiB runs of each state row (pure [T][S][W] row stores, 65 536 walkers: 5.7-5.9 TB/s,
// against 5.4-5.5 for one contiguous walker range per XCD and 4.7-4.9 for blockIdx order,
// the 2 KiB pieces of a 256-walker block interleaved over the XCDs; tools/fill_bench.hip,
// DESIGN.md §6).  Blocks past the last whole round of 8c keep their index: a bijection on
// [0, G) for any G.  c = G/8 (G a multiple of 8) is one contiguous range per XCD.
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t G, int32_t c) {
  const int64_t full = G / (8 * c) * (8 * c);
  if (b >= full) return b;
  const int64_t x = b & 7, j = b >> 3;
  return ((j / c) * 8 + x) * c + j % c;
}

// parameter registers: the model's own P plus up to 4 '<state>0' initial-condition
// parameters (oe_problem_set enforces n_params <= kPmax<M>)
template <class M>
constexpr int kPmax = M::P + (M::S < 4 ? M::S : 4);

// S = 5 Rosenbrock: the RODAS kernel needs 256 VGPRs + 14-22 AGPRs (one wave per SIMD);
// asking for two leaves 32-48 B of scratch and measured (262 144 walkers, profiles/r02o_occ*)
// `rosenbrock` 6.3 vs 8.3 ms (the r02 DOPRI5 + RODAS `auto` kernel: 1.25 vs 1.70 ms without
// trajectory).  The r04 `auto` (DOPRI5 + BDF hand-over) and `bdf` kernels need ~280 registers
// even for S = 4 (the difference table, LU factors and Newton vectors of the BDF pass): at two
// waves per SIMD they spill 250-400 B per lane, so they run at one (VGPRs + AGPRs, no scratch);
// below 65 536 walkers (the MH and speculative-round ensembles) that is one wave per SIMD anyway.
template <class M, int METHOD, bool TRAJ, bool NT>
__global__ void __launch_bounds__(256)
    __attribute__((amdgpu_waves_per_eu((METHOD == kRosenbrock && M::S == 5) ? 2 : 1)))
    k_integrate(const DevProblem pb, const IntegrateArgs ia) {
  constexpr int S = M::S;
  constexpr int PMAX = kPmax<M>;
#if OE_BDF_CLOCKS
  if ((threadIdx.x & 63) == 0) bdf_clk_wave_start()[threadIdx.x >> 6] = __builtin_amdgcn_s_memtime();
#endif
  const int64_t blk = ia.xcd_remap ? xcd_block(blockIdx.x, gridDim.x, ia.xcd_remap) : (int64_t)blockIdx.x;
  int64_t gw = blk * blockDim.x + threadIdx.x;
  bool idle = false;
  if (ia.half) {  // walker = (wave, lane < 32); the upper half-wave idles (DOPRI5: dead lanes)
    const int lane = threadIdx.x & 63;
    gw = (blk * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 32 + (lane & 31);
    idle = lane >= 32;
    if (METHOD == 0 && idle) return;
  }
  const bool active = gw < ia.W && !idle;
  const int64_t w = gw < ia.W ? gw : ia.W - 1;  // tail lanes shadow the last walker, never store
  const int64_t W = ia.W;
  double y[S], p[PMAX];
#pragma unroll
  for (int s = 0; s < S; ++s) y[s] = ia.y0[(int64_t)s * W + w];
#pragma unroll
  for (int j = 0; j < PMAX; ++j) p[j] = (j < pb.P) ? ia.theta[(int64_t)j * W + w] : 0.0;
  Acc a = acc_init();
  integrate_walker<M, PMAX, METHOD, TRAJ, NT, (M::S > kStiffRegS), (OE_LANE_INTEGRATE && !TRAJ && kLaneSteps<M, METHOD>)>(
      pb, y, p, ia.traj, W, w, active, a);
  if (active) {
    if (ia.chi) ia.chi[w] = a.nvalid ? a.chi : __builtin_nan("");
    if (ia.ssres) ia.ssres[w] = a.ssres;
    if (ia.status) ia.status[w] = finish(a);
  }
}

// ---------------------------------------------------------------------------------
// Kernels 1d/1e: 'auto' (S <= kHandMaxS) as two concurrent kernels over the hand-over
// queue (HandQ above).  k_integrate_hq is k_integrate<M, auto>'s lockstep DOPRI5 pass with
// the queue in place of the in-wave BDF pass; k_bdf_hq, launched at the same time on a second
// stream, runs the per-lane BDF pass of each handed walker from its hand-over state.
// Together: k_integrate<M, auto, TRAJ, NT>'s outputs, bit for bit.
// ---------------------------------------------------------------------------------
// MIX: the tableau's e / d / c coefficients as SGPR immediates (load_tab MIX), ~200 registers
// for the co-residency budget when k_bdf_hq runs beside it; without (k_bdf_hq after it) every
// coefficient in VGPRs as k_integrate<M, DOPRI5>: the immediates cost the DOPRI5 step 2 s_mov
// per use (C2: SALU 2.70e7 -> 4.09e7 per dispatch, profiles/r06/pmc).
template <class M, bool TRAJ, bool NT, bool MIX>
__global__ void __launch_bounds__(256) k_integrate_hq(const DevProblem pb, const IntegrateArgs ia, const HandQ hq) {
  constexpr int S = M::S;
  constexpr int PMAX = kPmax<M>;
  static_assert(S <= kHandMaxS, "the hand-over queue's co-residency budget");
#if OE_HQ_TRACE
  if (blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store((uint64_t*)(hq.ctl + 6), __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
#endif
  const int64_t blk = ia.xcd_remap ? xcd_block(blockIdx.x, gridDim.x, ia.xcd_remap) : (int64_t)blockIdx.x;
  const int64_t gw = blk * blockDim.x + threadIdx.x;
  const bool active = gw < ia.W;
  const int64_t w = active ? gw : ia.W - 1;  // tail lanes shadow the last walker, never store
  const int64_t W = ia.W;
  double y[S], p[PMAX];
#pragma unroll
  for (int s = 0; s < S; ++s) y[s] = ia.y0[(int64_t)s * W + w];
#pragma unroll
  for (int j = 0; j < PMAX; ++j) p[j] = (j < pb.P) ? ia.theta[(int64_t)j * W + w] : 0.0;
  Acc a = acc_init();
  const bool handed = integrate_dopri5<M, PMAX, TRAJ, NT, true, false, true, false, true, MIX>(
      pb, y, p, ia.traj, W, (uint32_t)w * 8u, active, a, nullptr, nullptr, &hq);
  if (active && !handed) {
    if (ia.chi) ia.chi[w] = a.nvalid ? a.chi : __builtin_nan("");
    if (ia.ssres) ia.ssres[w] = a.ssres;
    if (ia.status) ia.status[w] = finish(a);
  }
#if OE_HQ_TRACE
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_fetch_max((uint64_t*)(hq.ctl + 8), __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
#endif
  // this wave's pass is over (its slots were published, each with its own release store; the
  // count only ends the BDF kernel's polling, so it needs no release — a release here writes
  // the XCD's L2 back, once per wave)
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(hq.ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kHandBdfWaves = OE_HQ_WAVES;  // k_bdf_hq's one-wave workgroups beside the DOPRI5 kernel, at most
// Slots are dealt statically: BDF wave g's lane l takes slot g + l·G (G = the kernel's waves;
// the host sizes G·64 >= W, so every slot has a lane: capi.hip oe_integrate), so each handed
// walker is alone in its wave while there are no more than G of them, and no
// wave claims anything (a CAS claim by a thousand waves on one counter serialised the claims:
// 655 walkers were picked up over 6.7 ms, r06n).  A lane waits until its slot is published or
// every producer wave is done without reaching it; no loop runs around the BDF pass, so the
// pass's loop-invariant constants are formed after the wait instead of in the prologue, where
// they lived across the polling in SGPRs spilled to VGPR lanes (111 spilled SGPRs -> 21).
// DREG (after the DOPRI5 kernel): the BDF pass's difference table in registers (DTab<S, 0>);
// beside it the table stays in LDS, within the co-residency budget.
template <class M, bool TRAJ, bool NT, bool DREG = false>
__global__ void __launch_bounds__(64) k_bdf_hq(const DevProblem pb, const IntegrateArgs ia, const HandQ hq) {
  constexpr int S = M::S;
  constexpr int PMAX = kPmax<M>;
  const int lane = (int)threadIdx.x;
  const int64_t W = ia.W, c = hq.cap;
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  const int64_t slot = (int64_t)blockIdx.x + (int64_t)lane * gridDim.x;
  bool part = slot < W;
  for (;;) {
    bool wait = false;
    if (part && hq_load(hq.n + 5 * c + slot) != hq.epoch) {
      // not (yet) published: a producer will, unless every producer wave is done without
      // having reserved this slot
      if (hq_load(hq.ctl + 2) >= hq.n_waves) {
        hq_acquire();
        if (hq_load(hq.ctl) <= slot) part = false;
        else wait = true;  // reserved: its data is on the way
      } else {
        wait = true;
      }
    }
    if (__ballot(wait) == 0ull) break;
    if (__builtin_amdgcn_s_memrealtime() - t_start > kHandTimeout) {
      if (lane == 0) __hip_atomic_store(hq.ctl + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    // ~OE_HQ_POLL x 8 000 cycles between polls: a few thousand pollers must not load the
    // queue's lines (or the memory side behind them) the DOPRI5 kernel also uses
    for (int z = 0; z < OE_HQ_POLL; ++z) __builtin_amdgcn_s_sleep(127);
  }
  if (__ballot(part) == 0ull) return;
  const int64_t j = part ? slot : 0;
  hq_acquire();  // the slots' data, published by their producers' release stores
  double y[S], p[PMAX];
#pragma unroll
  for (int s = 0; s < S; ++s) y[s] = hq.d[s * c + j];
  const double t = hq.d[S * c + j];
  Acc a{hq.d[(S + 1) * c + j], hq.d[(S + 2) * c + j], hq.d[(S + 3) * c + j], hq.d[(S + 4) * c + j],
        hq.n[2 * c + j], hq.n[3 * c + j]};
  const int i = hq.n[j], k = hq.n[c + j];
  const int64_t w = hq.n[4 * c + j];
#pragma unroll
  for (int q = 0; q < PMAX; ++q) p[q] = (q < pb.P) ? ia.theta[(int64_t)q * W + w] : 0.0;
#if OE_HQ_TRACE
  const uint64_t t_claim = __builtin_amdgcn_s_memrealtime();
#endif
  // The BDF pass is one lane's dependency chain (latency-bound, sparse issue); the DOPRI5
  // wave sharing its SIMD is issue-bound.  At a higher priority the BDF wave issues whenever
  // it is ready, taking few slots from the DOPRI5 wave, instead of waiting behind it.
  if (OE_HQ_PRIO) __builtin_amdgcn_s_setprio(3);
  integrate_bdf_lane<M, PMAX, TRAJ, NT, DREG ? 0 : 64>(pb, y, t, i, k, p, ia.traj, W, w, part, part, a);
#if OE_HQ_TRACE
  {
    // s_memrealtime: 100 MHz; chi = start·1e5 + the DOPRI5 kernel's last wave end, ssres =
    // claim·1e5 + BDF pass, all in whole µs from the DOPRI5 kernel's first wave
    const uint64_t t0 = __hip_atomic_load((const uint64_t*)(hq.ctl + 4 + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t_pend = __hip_atomic_load((const uint64_t*)(hq.ctl + 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.chi = (double)((int64_t)(t_start - t0) / 100) * 1e5 + (double)((int64_t)(t_pend - t0) / 100);
    a.ssres = (double)((int64_t)(t_claim - t0) / 100) * 1e5 + (double)((__builtin_amdgcn_s_memrealtime() - t_claim) / 100);
    a.nvalid = 1;
  }
#endif
  if (part) {
    if (ia.chi) ia.chi[w] = a.nvalid ? a.chi : __builtin_nan("");
    if (ia.ssres) ia.ssres[w] = a.ssres;
    if (ia.status) ia.status[w] = finish(a);
  }
}

// ---------------------------------------------------------------------------------
// Kernel 1c: DOPRI5 trajectory mode with store waves (C2; S <= 8).
//
// One workgroup = 4 COMPUTE waves (256 walkers, one per lane, the lockstep DOPRI5 of
// k_integrate with the same step sequences) + 4 STORE waves, store wave c serving compute
// wave c through that wave's slot ring (DpPipe): the dense output at the non-observed grid
// times, the running minimum and the row stores leave the compute wave, whose VALU issue
// sets the kernel time at one wave per SIMD.  Per-wave counters, no
// phase barrier; one workgroup barrier at the end merges the store waves' minima into the
// status bits.  Same outputs as k_integrate<M, DOPRI5, true, NT>, bit for bit.
// ---------------------------------------------------------------------------------
template <class M, bool NT>
__global__ void __launch_bounds__(512) k_integrate_dopri5_piped(const DevProblem pb, const IntegrateArgs ia) {
  constexpr int S = M::S;
  constexpr int PMAX = kPmax<M>;
  constexpr int R = dp_pipe_slots<S>();
  static_assert(R >= 2, "slot ring too small");
  __shared__ double ring[4][R][kDpPipeFields * S * 64];
  __shared__ double uni[4][R][4];
  __shared__ int produced[4], consumed[4];
  __shared__ double ymin_sh[4][64];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int c = wave & 3;  // the compute wave (and its store wave)
  if (threadIdx.x < 4) { produced[threadIdx.x] = 0; consumed[threadIdx.x] = 0; }
  __syncthreads();
  const int64_t blk = ia.xcd_remap ? xcd_block(blockIdx.x, gridDim.x, ia.xcd_remap) : (int64_t)blockIdx.x;
  const int64_t gw = blk * 256 + c * 64 + lane;
  const bool active = gw < ia.W;
  const int64_t w = active ? gw : ia.W - 1;
  const int64_t W = ia.W;
  const int T = pb.T;
  if (wave < 4) {
    // ------------------------------ compute waves ------------------------------
    double y[S], p[PMAX];
#pragma unroll
    for (int s = 0; s < S; ++s) y[s] = ia.y0[(int64_t)s * W + w];
#pragma unroll
    for (int j = 0; j < PMAX; ++j) p[j] = (j < pb.P) ? ia.theta[(int64_t)j * W + w] : 0.0;
    Acc a = acc_init();
    DpPipe<S> pp{&ring[c][0][0], &uni[c][0][0], &produced[c], &consumed[c], lane, R, 0, 0};
    integrate_dopri5<M, PMAX, true, NT, false, false, false, true>(pb, y, p, ia.traj, W, (uint32_t)w * 8u, active, a,
                                                                 nullptr, &pp);
    __syncthreads();  // the store waves' minima
    a.ymin = min_raw(a.ymin, ymin_sh[c][lane]);
    if (active) {
      if (ia.chi) ia.chi[w] = a.nvalid ? a.chi : __builtin_nan("");
      if (ia.ssres) ia.ssres[w] = a.ssres;
      if (ia.status) ia.status[w] = finish(a);
    }
  } else {
    // ------------------------------ store waves --------------------------------
    const double* times = pb.times;
    const uint32_t off = (uint32_t)w * 8u;
    const uint32_t row_bytes = (uint32_t)(S * W * 8);
    Acc a = acc_init();  // only its running minimum is used
    int i = 0;
    for (int n = 0; i < T; ++n) {
      while (*(volatile int*)&produced[c] <= n) __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");
      const int slot = n % R;
      const double* f = &ring[c][slot][0] + lane;
      const double t = uni[c][slot][0], tn = uni[c][slot][1], rh = uni[c][slot][2];
      double y[S], ydf[S], bsp[S], r4[S], r5[S], yn[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        y[s] = f[(0 * S + s) * 64];
        ydf[s] = f[(1 * S + s) * 64];
        bsp[s] = f[(2 * S + s) * 64];
        r4[s] = f[(3 * S + s) * 64];
        r5[s] = f[(4 * S + s) * 64];
        yn[s] = f[(5 * S + s) * 64];
      }
      lds_fence();  // the slot is read: release it
      if (lane == 0) *(volatile int*)&consumed[c] = n + 1;
      double ti = times[i];
      while (ti < tn) {  // the compute wave's dense output, operation for operation
        const double th = (ti - t) * rh;
        const double th1 = 1.0 - th;
        double yo[S];
#pragma unroll
        for (int s = 0; s < S; ++s)
          yo[s] = fma(th, fma(th1, fma(th, fma(th1, r5[s], r4[s]), bsp[s]), ydf[s]), y[s]);
        store_row_at<S, true, NT>(ia.traj + (int64_t)i * S * W, yo, W, off, active, a);
        ++i;
        ti = times[i];  // times[T] is the +inf sentinel
      }
      // (i < T: an all-evicted wave publishes a last slot reaching t = +inf, and the
      // sentinel times[T] = +inf equals it — that row would lie past the buffer)
      if (i < T && ti == tn) {
        store_row_at<S, true, NT>(ia.traj + (int64_t)i * S * W, yn, W, off, active, a);
        ++i;
      }
    }
    (void)row_bytes;
    ymin_sh[c][lane] = a.ymin;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------
// Kernel 1b: RK4 trajectory mode with producer/consumer waves (W even).
//
// One workgroup = 4 COMPUTE waves (256 walkers, one per lane) + NSW STORE waves (2, 4
// or 8).  Output rows are produced in phases of H rows into one half of a
// double-buffered LDS ring [2][H][S][256]; in the next phase the store waves read that
// half with ds_read_b128 (two consecutive walkers per lane) and write 1 KB per
// wave-instruction with buffer_store_dwordx4, while the compute waves fill the other
// half.  Store wave j covers walker half j & 1 and the states s ≡ j/2 (mod NSW/2).
// Phases are separated by a raw s_barrier behind an lgkmcnt(0) wait only, so
// the global stores stay in flight across barriers and the compute waves never wait on
// vmcnt.  Same arithmetic, same outputs as k_integrate<M, RK4, true, NT>.
// ---------------------------------------------------------------------------------
constexpr int kPipeWalkers = 256;  // walkers per workgroup (4 compute waves)
#ifndef OE_PIPE_LDS_BYTES
#define OE_PIPE_LDS_BYTES (160 * 1024)  // all of a CU's LDS: one workgroup per CU either way
#endif
constexpr int kPipeLdsBytes = OE_PIPE_LDS_BYTES;

template <int S>
constexpr int pipe_rows() { return (kPipeLdsBytes / (2 * S * kPipeWalkers * 8)) > 0 ? (kPipeLdsBytes / (2 * S * kPipeWalkers * 8)) : 1; }

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}


template <class M, bool NT, int NSW>
__global__ void __launch_bounds__(256 + 64 * NSW) k_integrate_rk4_piped(const DevProblem pb, const IntegrateArgs ia) {
  constexpr int S = M::S;
  constexpr int PMAX = kPmax<M>;
  constexpr int H = pipe_rows<S>();
  static_assert(2 * H * S * kPipeWalkers * 8 <= kPipeLdsBytes, "LDS ring too large");
  __shared__ double pipe_ring[2][H][S][kPipeWalkers];
  auto ring = [&](int half, int h, int s, int b) -> double* { return &pipe_ring[half][h][s][b]; };

  const int64_t W = ia.W;
  const int T = pb.T;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  // blockIdx order by default (the XCD-contiguous remap of the direct kernel measured 9 %
  // slower here: 0.400 vs 0.366 ms on C1, profiles/r02l_time_modes.log)
  const int64_t blk = ia.xcd_remap ? xcd_block(blockIdx.x, gridDim.x, ia.xcd_remap) : (int64_t)blockIdx.x;
  const int64_t base = blk * kPipeWalkers;
  const int nphase = (T + H - 1) / H;

  if (wave < 4) {
    // ------------------------------ compute waves ------------------------------
    const int b = wave * 64 + lane;  // walker slot in the block
    const int64_t gw = base + b;
    const bool active = gw < W;
    const int64_t w = active ? gw : W - 1;
    double y[S], p[PMAX];
#pragma unroll
    for (int s = 0; s < S; ++s) y[s] = ia.y0[(int64_t)s * W + w];
#pragma unroll
    for (int j = 0; j < PMAX; ++j) p[j] = (j < pb.P) ? ia.theta[(int64_t)j * W + w] : 0.0;
    Acc a = acc_init();
    int k = 0;
    const cptr<double> tab = kconst(pb.rk4);
    const cptr<Obs> obs = kconst(pb.obs);
    const int n = pb.substeps;
    auto put = [&](int half, int h, const double (&v)[S]) {
#pragma unroll
      for (int s = 0; s < S; ++s) *ring(half, h, s, b) = v[s];
#pragma unroll
      for (int s = 0; s < S; ++s) a.ymin = min_raw(a.ymin, v[s]);
    };
    auto interval = [&](int i) {
      const double h = tab[4 * (i - 1)], hh = tab[4 * (i - 1) + 1], h6 = tab[4 * (i - 1) + 2];
      const double t = tab[4 * (i - 1) + 3];
      for (int j = 0; j < n; ++j) rk4_step<M, PMAX>(y, t + (double)j * h, h, hh, h6, p);
    };
    for (int ph = 0; ph <= nphase; ++ph) {
      if (ph < nphase) {
        const int half = ph & 1;
        const int r0 = ph * H;
        const int r1 = (r0 + H < T) ? r0 + H : T;
        int r = r0;
        if (r == 0) {  // row 0 is the initial state
          put(half, 0, y);
          observe<S, true>(pb, 0, y, k, a);
          ++r;
        }
        while (r < r1) {
          int next = (k < pb.n_obs) ? obs[k].tidx : T;
          if (next > r1) next = r1;
          for (; r < next; ++r) {
            interval(r);
            put(half, r - r0, y);
          }
          if (r < r1) {  // observed row
            interval(r);
            put(half, r - r0, y);
            observe<S, true>(pb, r, y, k, a);
            ++r;
          }
        }
      }
      lds_barrier();
    }
    check_finite(y, a);
    if (active) {
      if (ia.chi) ia.chi[w] = a.nvalid ? a.chi : __builtin_nan("");
      if (ia.ssres) ia.ssres[w] = a.ssres;
      if (ia.status) ia.status[w] = finish(a);
    }
  } else {
    // ------------------------------ store waves --------------------------------
    const int sw = wave - 4;                 // store wave 0 .. NSW-1
    constexpr int G = NSW / 2;               // state groups
    const int sg = sw >> 1;                  // this wave's states: sg, sg + G, ...
    const int b = (sw & 1) * 128 + 2 * lane; // first of this lane's two walkers
    const bool active = base + b < W;        // W even: both or neither
    const uint32_t off = (uint32_t)(base + b) * 8u;
    const uint32_t row_bytes = (uint32_t)(S * W * 8);
    for (int ph = 0; ph <= nphase; ++ph) {
      if (ph >= 1) {
        const int half = (ph - 1) & 1;
        const int r0 = (ph - 1) * H;
        const int r1 = (r0 + H < T) ? r0 + H : T;
        for (int r = r0; r < r1; ++r) {
          const __amdgpu_buffer_rsrc_t rsrc =
              __builtin_amdgcn_make_buffer_rsrc((void*)(ia.traj + (int64_t)r * S * W), 0, row_bytes, 0x00020000);
#pragma unroll
          for (int s0 = 0; s0 < S; s0 += G) {
            const int s = s0 + sg;
            if (G > 1 && s >= S) break;
            const u32x4 v = *reinterpret_cast<const u32x4*>(ring(half, r - r0, s, b));
            if (active)
              __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, off, (uint32_t)(s * W * 8), NT ? OE_NT_AUX : 0);
          }
        }
      }
      lds_barrier();
    }
  }
}

// ---------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11) counter-based RNG for the MH proposals.
// ---------------------------------------------------------------------------------
struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1,
           (uint32_t)p0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// 53-bit uniform in [0,1) from two words (numpy random_sample construction)
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// Proposal draws of iterations [it0, it1) for every walker, in the layout of the
// replay streams: dz[it - it0][p][w] = step_sd * N(0,1), u[it - it0][w] = U[0,1).
// Counter (global walker id, iteration, pair index) under key = seed, so the draws do
// not depend on how walkers are sharded or iterations chunked.  Its own kernel, so the
// MH kernel carries no Box–Muller transcendentals (register pressure).
struct DrawArgs {
  int64_t W;
  int64_t walker_offset;
  int32_t it0, it1;
  int32_t P;
  uint32_t seed_lo, seed_hi;
  double step_sd;
  double* dz;  // [it1 - it0][P][W]
  double* u;   // [it1 - it0][W]
};

__device__ __forceinline__ void philox_draw_iteration(const DrawArgs d, int64_t w, int it) {
  const uint64_t gid = (uint64_t)(d.walker_offset + w);
  const int64_t W = d.W;
  {
    double* dz = d.dz + (int64_t)(it - d.it0) * d.P * W + w;
    for (int j = 0; j < d.P; j += 2) {
      const U4 r = philox4x32_10(U4{(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)it, (uint32_t)(j >> 1)},
                                 d.seed_lo, d.seed_hi);
      const double u1 = 1.0 - u53(r.x, r.y);
      const double u2 = u53(r.z, r.w);
      const double rad = sqrt(-2.0 * log(u1));
      const double ang = 6.283185307179586 * u2;
      dz[(int64_t)j * W] = d.step_sd * (rad * cos(ang));
      if (j + 1 < d.P) dz[(int64_t)(j + 1) * W] = d.step_sd * (rad * sin(ang));
    }
    const U4 r = philox4x32_10(U4{(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)it, 0x80000000u},
                               d.seed_lo, d.seed_hi);
    d.u[(int64_t)(it - d.it0) * W + w] = u53(r.x, r.y);
  }
}

// ---------------------------------------------------------------------------------
// Kernel 2: Metropolis–Hastings, iterations [it0, it1) for every walker
// (Samplers.py:104-153).  One lane = one chain; the chain state lives in HBM
// between chunked launches.
// ---------------------------------------------------------------------------------
struct MHArgs {
  int64_t W;
  int64_t walker_offset;
  int32_t it0, it1;        // iteration range of this launch (1-based, ref `it`)
  int32_t burnin;
  int32_t row0;            // iteration stored in samples row 0 (burnin+1, or later on resume)
  int32_t draw_it0;        // iteration whose draws sit at offset 0 of dz/u
  int32_t init;            // 1: compute the a-priori chi/R²/AIC only (Samplers.py:88-91)
  int32_t any_walk;
  uint64_t walk_mask;      // bit p: parameter p walks
  int32_t init_param[64];  // per state: -1 or parameter index
  const double* dz;        // [..][P][W] step_sd·N(0,1) (replay streams or philox_draws)
  const double* u;         // [..][W]
  double* theta;           // [P][W]
  double* y0;              // [S][W]
  double* samples;         // [kept][P+5][W]
  double* cur;             // [4][W]: chi, rsquared, aic, n_accepted
  int32_t* status;         // [W]
  int32_t n_rows;          // rows of samples (the kept iterations of this call)
};

// Integrity checks of the MH kernel's uniform state (below): compiled into the debug
// library (make debug -> libodelib_amd_debug.so), whose MH parity run is a GPU test.
// Off in the product library: even these few scalar compares move the register
// allocation of the chain20 DOPRI5 MH kernel (scratch 176 -> 240 B/lane).
#ifndef OE_MH_CHECKS
#define OE_MH_CHECKS 0
#endif

// Element w of a walker-minor row [W] through a buffer resource: row base and size in
// SGPRs, the lane's byte offset w*8 in one VGPR.  With plain pointers the compiler
// forms one 64-bit per-lane address per row, and since every row base is invariant in
// the MH iteration loop it hoists them: two VGPRs per row, dozens of rows — the
// register cost of a second wave per SIMD.
struct Row {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ Row(const double* row, int64_t W)
      // num_records is 32 bits: W = 2^29 (the ABI maximum) makes W*8 = 2^32, clamp it
      : r(__builtin_amdgcn_make_buffer_rsrc((void*)row, 0,
                                            (int)(uint32_t)(W * 8 > 0xffffffffll ? 0xffffffffll : W * 8),
                                            0x00020000)) {}
  __device__ __forceinline__ double ld(uint32_t off) const {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
  }
  __device__ __forceinline__ void st(uint32_t off, double v) const {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, 0);
  }
};

// A uniform pointer the compiler must treat as redefined here: row resources derived
// from it are rebuilt at their use (a few SALU) instead of hoisted out of the MH
// iteration loop, where S + 2P hoisted 4-SGPR descriptors (chain20: ~120 SGPRs) stay
// live across the whole integration and spill to VGPR lanes.
template <class T>
__device__ __forceinline__ T* opaque(T* p) {
  asm volatile("" : "+s"(p));
  return p;
}
// The same for a wave-uniform scalar (a kernel argument): the predicates the MH iteration
// derives from it — j < P, walk bit j, init_param[s] == j per state and parameter (the
// '<state>0' picks) — are formed at their use in each iteration instead of hoisted out of
// the iteration loop as 64-bit lane masks, ~50 of which lived across the whole integration
// in SGPR pairs spilled to VGPR lanes (k_mh<TwoI, auto>: 510 SGPRs spilled).
#ifndef OE_MH_W_OPAQUE
#define OE_MH_W_OPAQUE 0
#endif
template <class T>
__device__ __forceinline__ T uopaque(T v) {
  asm volatile("" : "+s"(v));
  return v;
}

// The stiff methods' Rosenbrock fallback (dual-number Jacobian, in-register LU) would set
// the register budget of the whole MH kernel (chain5 'auto': 300 VGPR+AGPR, one wave per
// SIMD, +49 % per iteration at 262 144 walkers); for S = 5, where the plain DOPRI5 MH
// kernel runs two waves per SIMD, asking for two keeps the DOPRI5 phase there (80 B of
// scratch, in the rare path).  S = 6..8 DOPRI5 MH kernels are at one wave per SIMD anyway.
// The stiff methods' MH with one lane per chain (S <= kStiffRegS) has no iteration-loop kernel:
// its chains run as rounds of k_mh_tree + k_mh_resolve (below), of one iteration when not
// speculating.  k_mh's loop around the per-lane DOPRI5 + BDF passes held ~160-380 SGPRs
// spilled to VGPR lanes (the regime of round 4's unexplained code-shape failures; DESIGN.md
// §3.6), where the loop-free tree kernel holds ~20; a round costs two launches.
#ifndef OE_MH_SPREAD  // measurement builds: 0 = MH rounds never spread one lane per wave
#define OE_MH_SPREAD 1
#endif
template <class M, int METHOD>
constexpr bool kMhRoundsOnly = (METHOD == kAuto || METHOD == kBdf) && M::S <= kStiffRegS;

// INIT: the a-priori fit's pass alone (ma.init, Samplers.py:88-91) — its own kernel, so k_mh's
// iteration loop is the kernel's only copy of the integrator (with the init branch inside
// k_mh, the two copies of a stiff method's BDF pass shared one register allocation: ~100 of
// k_mh<TwoI, auto>'s spilled SGPRs held values across both).
template <class M, int METHOD, bool INIT = false>
__global__ void __launch_bounds__(256)
    __attribute__((amdgpu_waves_per_eu((METHOD == kRosenbrock && M::S == 5) ? 2 : 1)))
    k_mh(const DevProblem pb, const MHArgs ma) {
  constexpr int S = M::S;
  constexpr int PMAX = kPmax<M>;
#if OE_BDF_CLOCKS
  if ((threadIdx.x & 63) == 0) bdf_clk_wave_start()[threadIdx.x >> 6] = __builtin_amdgcn_s_memtime();
#endif
  const int64_t gw = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = gw < ma.W;
  const int64_t w = active ? gw : ma.W - 1;
  const int64_t W0 = ma.W;
  const int P = pb.P;
  // The chain state θ [P][W] and y0 [S][W] stays in HBM between iterations (a few loads
  // per iteration against ~1000 integration steps): only the proposal is held in
  // registers while integrating, which keeps the DOPRI5 MH kernel within the register
  // budget of two waves per SIMD.  Tail lanes (w clamped to W-1) never store.
  double* __restrict__ theta = ma.theta;
  double* __restrict__ y0g = ma.y0;
  const uint32_t off = (uint32_t)w * 8u;  // W <= 2^29 (oe_mh_run)

  if constexpr (INIT) {  // a-priori fit (Samplers.py:88-91)
    const int64_t W = W0;
    double th[PMAX], y[S];
#pragma unroll
    for (int j = 0; j < PMAX; ++j) th[j] = (j < P) ? Row(theta + (int64_t)j * W, W).ld(off) : 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) y[s] = Row(y0g + (int64_t)s * W, W).ld(off);
    Acc a = acc_init();
    integrate_walker<M, PMAX, METHOD, false, false, false, kLaneSteps<M, METHOD>>(pb, y, th, nullptr, W, w, active, a);
    if (active) {
      const double chi = a.nvalid ? a.chi : __builtin_nan("");
      Row(ma.cur, W).st(off, chi);
      Row(ma.cur + W, W).st(off, 1.0 - a.ssres / pb.sstot);
      Row(ma.cur + 2 * W, W).st(off, -2.0 * (-chi) + 2.0 * (double)pb.pnum);
      Row(ma.cur + 3 * W, W).st(off, 0.0);
      if (ma.status) ma.status[w] = finish(a);
    }
  } else {
  // The current chain point (chi, R², AIC, acceptance count; status) also stays in
  // HBM (cur rows): read after the proposal's integration, written on accept, so none
  // of it holds registers across the integration.
  double* __restrict__ cur = ma.cur;
  const int PS = P + 5;

  for (int it = ma.it0; it < ma.it1; ++it) {
    // (W re-read per iteration: the row offsets j·W·8 are formed at their use, not hoisted
    // into the kernel's prologue and kept across the whole loop)
    int64_t W = OE_MH_W_OPAQUE ? uopaque(W0) : W0;
    // ---- proposal: θ' = exp(log θ + N(0, sd)) for walking parameters (Framework.py:107-122)
    double tn[PMAX];
    theta = opaque(theta);
    y0g = opaque(y0g);
    const double* dz = opaque(ma.dz + (int64_t)(it - ma.draw_it0) * P * W);
    {
      // one call site each for log and exp: a loop over the parameters, the result put in
      // place with selects.  Unrolled, every call site is a point where the caller-saved
      // SGPRs live across the call are spilled to VGPR lanes and restored — 2·PMAX of them.
      const int Pu = uopaque(P);
      const uint64_t wm = uopaque(ma.walk_mask);
#pragma unroll
      for (int j = 0; j < PMAX; ++j) tn[j] = 0.0;
#pragma unroll 1
      for (int j = 0; j < Pu; ++j) {
        const double thj = Row(theta + (int64_t)j * W, W).ld(off);
        const double v = ((wm >> j) & 1ull) ? oe_exp(oe_log(thj) + Row(dz + (int64_t)j * W, W).ld(off)) : thj;
#pragma unroll
        for (int q = 0; q < PMAX; ++q) tn[q] = (q == j) ? v : tn[q];
      }
    }
    // '<state>0' parameters drive initial states (Samplers.py:110-114)
    double y[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pi = uopaque(ma.init_param[s]);
      y[s] = (uopaque(ma.any_walk) && pi >= 0) ? pick(tn, pi) : Row(y0g + (int64_t)s * W, W).ld(off);
    }
    // ---- integrate + fused chi (Samplers.py:115-116)
    Acc a = acc_init();
    integrate_walker<M, PMAX, METHOD, false, false, false, kLaneSteps<M, METHOD>>(pb, y, tn, nullptr, W, w, active, a);
    const double chin = a.nvalid ? a.chi : __builtin_nan("");
    theta = opaque(theta);
    y0g = opaque(y0g);
    cur = opaque(cur);
    if (OE_MH_W_OPAQUE) W = uopaque(W0);
#if OE_MH_CHECKS
    // Integrity of the wave-uniform state every store below depends on:
    // the row pointers carried through the integration (live in SGPRs or spilled across
    // ~1000 steps) still equal the kernel arguments, the sample row lies inside the
    // buffer, linked initial states name a parameter.  Lane offsets are in range by
    // construction and range-checked by the buffer descriptors.  On a violation nothing
    // more is stored and the walker's status carries ST_INTERNAL (a recorded assert: a
    // device trap would take the process — and on this pool possibly the box — down).
    {
      bool sound = theta == ma.theta && y0g == ma.y0 && cur == ma.cur &&
                   (it <= ma.burnin || (it - ma.row0 >= 0 && it - ma.row0 < ma.n_rows));
#pragma unroll
      for (int s = 0; s < S; ++s) sound = sound && ma.init_param[s] < P;
      if (!sound) {
        if (active && ma.status) ma.status[w] = ST_INTERNAL;
        return;
      }
    }
#endif
    const double u = Row(opaque(ma.u + (int64_t)(it - ma.draw_it0) * W), W).ld(off);
    double chi = Row(cur, W).ld(off), rsq = Row(cur + W, W).ld(off), aic = Row(cur + 2 * W, W).ld(off);
    double nacc = Row(cur + 3 * W, W).ld(off);
    // ---- acceptance, in the reference's arithmetic (Samplers.py:124-127)
    const double lr = oe_exp(chi - chin);
    const double accp = oe_exp(oe_log(lr));
    const bool acc = accp > u;
    const int Pa = uopaque(P);
    if (acc) {
      chi = chin;
      rsq = 1.0 - a.ssres / pb.sstot;
      aic = -2.0 * (-chi) + 2.0 * (double)pb.pnum;
      nacc += 1.0;
      if (active) {
#pragma unroll
        for (int j = 0; j < PMAX; ++j)
          if (j < Pa) Row(theta + (int64_t)j * W, W).st(off, tn[j]);
        Row(cur, W).st(off, chi);
        Row(cur + W, W).st(off, rsq);
        Row(cur + 2 * W, W).st(off, aic);
        Row(cur + 3 * W, W).st(off, nacc);
        if (ma.status) ma.status[w] = finish(a);
      }
    }
    // linked initial states follow the current parameters: the accepted proposal, or
    // on reject the restored ones (Samplers.py:110-114, :137-143)
    if (uopaque(ma.any_walk) && active) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int pi = uopaque(ma.init_param[s]);
        if (pi >= 0) Row(y0g + (int64_t)s * W, W).st(off, acc ? pick(tn, pi) : Row(theta + (int64_t)pi * W, W).ld(off));
      }
    }
    // ---- keep the sample after burn-in (Samplers.py:147-153)
    if (it > ma.burnin && active) {
      double* row = ma.samples + (int64_t)(it - ma.row0) * PS * W;
#pragma unroll
      for (int j = 0; j < PMAX; ++j)
        if (j < Pa) Row(row + (int64_t)j * W, W).st(off, acc ? tn[j] : Row(theta + (int64_t)j * W, W).ld(off));
      Row(row + (int64_t)P * W, W).st(off, chi);
      Row(row + (int64_t)(P + 1) * W, W).st(off, rsq);
      Row(row + (int64_t)(P + 2) * W, W).st(off, aic);
      Row(row + (int64_t)(P + 3) * W, W).st(off, (double)it);
      Row(row + (int64_t)(P + 4) * W, W).st(off, nacc / (double)it);
    }
  }
  }
}

// ---------------------------------------------------------------------------------
// Kernel 2b: speculative Metropolis–Hastings for small ensembles (prefetching MH).
// A chain's proposal at iteration it depends on the chain state, i.e. on which of the
// earlier proposals were accepted, but its draws (dz[it], u[it]) do not.  One round
// covers iterations it0 .. it0+d-1: every outcome path of the first j accept/reject
// decisions gives one candidate state for iteration it0+j, so the 2^d - 1 nodes of the
// binary tree hold every proposal the chain can make in the round.  k_mh_tree integrates
// all of them at once (one lane per (node, chain)); k_mh_resolve then walks each chain's
// tree with the accept test and keeps the path the sequential chain takes.  Each node's
// proposal is formed by the same operations, in the same order, as k_mh forms it on that
// path (θ ← exp(log θ + dz) per accepted iteration), and RK4 integrates a lane on its own,
// so RK4 chains are bitwise those of k_mh; a DOPRI5 lane shares its step size with the 63
// lanes of its wave, which are other nodes here, so DOPRI5 chains agree within the
// integration tolerance.  For W chains the round keeps (2^d - 1)·W lanes busy: with few
// chains the GPU is mostly idle in k_mh, and d iterations cost about one.
// Node n (heap order): depth j = floor(log2(n + 1)), path bits p = n + 1 - 2^j, bit k of p
// = the decision at depth k; buffers node-major, [n][W]; 'auto' lanes chain-major (k_mh_tree).
// ---------------------------------------------------------------------------------
struct MHTreeArgs {
  MHArgs m;            // chain state, draws, masks; m.it0 = the round's first iteration
  int32_t depth;       // iterations of this round (the tree has 2^depth - 1 nodes)
  int64_t n_lanes;     // (2^depth - 1) * W
  double* node_th;     // [n][P][W] proposals
  double* node_chi;    // [n][W] chi of the proposal (NaN if no observation was finite)
  double* node_ss;     // [n][W] R² residual
  int32_t* node_st;    // [n][W] status bits
  int32_t spread;      // 1: one lane per wave (lane 0 of 64-thread workgroups; few lanes, idle device)
};

template <class M, int METHOD>
__global__ void __launch_bounds__(256)
    __attribute__((amdgpu_waves_per_eu((METHOD == kRosenbrock && M::S == 5) ? 2 : 1)))
    k_mh_tree(const DevProblem pb, const MHTreeArgs ta) {
  constexpr int S = M::S;
  constexpr int PMAX = kPmax<M>;
#if OE_BDF_CLOCKS
  if ((threadIdx.x & 63) == 0) bdf_clk_wave_start()[threadIdx.x >> 6] = __builtin_amdgcn_s_memtime();
#endif
  const MHArgs& ma = ta.m;
  const int64_t W = ma.W;
  const int P = pb.P;
  // spread: each lane alone in its wave (lane 0 of a 64-thread workgroup).  With few lanes
  // (sequential rounds of a small ensemble) the device is idle anyway, and a wave then costs
  // its own lane's DOPRI5 + BDF passes instead of its slowest DOPRI5 lane's plus its slowest
  // BDF lane's, at a uniform wave's pace per step (1.3-1.4x for mixed waves).
  const int64_t gl = ta.spread ? (int64_t)blockIdx.x : (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = gl < ta.n_lanes && (!ta.spread || threadIdx.x == 0);
  const int64_t gw = active ? gl : ta.n_lanes - 1;
  // 'auto': chain-major lanes — a wave holds consecutive nodes of one chain, near-identical
  // proposals that step alike, observe together at little cost and share the BDF pass's
  // lockstep with proposals of the same stiffness (notebook fit, same box: 0.229 -> 0.221 s,
  // 1 024 chains 0.706 -> 0.678 s); the other methods keep node-major lanes (a wave = 64 // W
  // nodes of every chain: synthetic RK4 rounds 7-9 % faster that way, profiles/NOTES.md r04x).
  // The node buffers are node-major (index g = n·W + c) either way.  n_lanes < 2^29.
  int64_t n, c;
  if constexpr (METHOD == kAuto) {
    const uint32_t nodes = (uint32_t)(ta.n_lanes / W);
    const uint32_t cq = (uint32_t)gw / nodes;
    n = (int64_t)((uint32_t)gw - cq * nodes);
    c = cq;
  } else {
    n = gw / W;
    c = gw - n * W;
  }
  const int64_t g = n * W + c;
  const int j = 31 - __builtin_clz((uint32_t)(n + 1));  // depth
  const uint32_t path = (uint32_t)(n + 1) - (1u << j);
  const uint32_t off = (uint32_t)c * 8u;
  // the chain state this path reaches at depth j: the round's start, moved on by every
  // accepted proposal of the path, each formed as k_mh forms it
  double th[PMAX];
#pragma unroll
  for (int q = 0; q < PMAX; ++q) th[q] = (q < P) ? Row(ma.theta + (int64_t)q * W, W).ld(off) : 0.0;
  for (int k = 0; k < j; ++k) {
    if (!((path >> k) & 1u)) continue;
    const double* dz = ma.dz + (int64_t)(ma.it0 + k - ma.draw_it0) * P * W;
#pragma unroll
    for (int q = 0; q < PMAX; ++q)
      if (q < P && ((ma.walk_mask >> q) & 1ull)) th[q] = oe_exp(oe_log(th[q]) + Row(dz + (int64_t)q * W, W).ld(off));
  }
  double tn[PMAX];
  {
    const double* dz = ma.dz + (int64_t)(ma.it0 + j - ma.draw_it0) * P * W;
#pragma unroll
    for (int q = 0; q < PMAX; ++q)
      tn[q] = (q < P && ((ma.walk_mask >> q) & 1ull)) ? oe_exp(oe_log(th[q]) + Row(dz + (int64_t)q * W, W).ld(off))
                                                      : th[q];
  }
  double y[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int pi = ma.init_param[s];
    y[s] = (ma.any_walk && pi >= 0) ? pick(tn, pi) : Row(ma.y0 + (int64_t)s * W, W).ld(off);
  }
  Acc a = acc_init();
  integrate_walker<M, PMAX, METHOD, false, false, false, kLaneSteps<M, METHOD>>(pb, y, tn, nullptr, ta.n_lanes, g, active, a);
  if (active) {
    const int64_t NW = ta.n_lanes;
    const uint32_t o = (uint32_t)g * 8u;
#pragma unroll
    for (int q = 0; q < PMAX; ++q)
      if (q < P) Row(ta.node_th + n * P * W + (int64_t)q * W, W).st(off, tn[q]);
    Row(ta.node_chi, NW).st(o, a.nvalid ? a.chi : __builtin_nan(""));
    Row(ta.node_ss, NW).st(o, a.ssres);
    ta.node_st[g] = finish(a);
  }
}

}  // namespace oe
#include "stiff_wave.cuh"
#include "split.cuh"
