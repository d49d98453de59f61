// split.cuh — DOPRI5 for wide chain models with a walker split over K adjacent lanes.
//
// A 20-state DOPRI5 walker in one lane needs ~100 doubles of stage vectors: the
// one-lane kernel sits at 256 VGPRs + 256 AGPRs with ~1 500 v_accvgpr moves in a
// 2 600-instruction step, one wave per SIMD.  Here K adjacent lanes of a
// quad share one walker, lane r holding states [r·m, r·m + m), m = S/K: the stage
// vectors shrink K-fold (no AGPR traffic, two or more waves per SIMD), and the work a
// walker does per step is the same elementwise arithmetic spread over K lanes.
//
// What crosses lanes (DPP quad_perm, no LDS):
//   * the chain RHS is nearest-neighbour: lane r needs the last state of
//     lane r-1, and every lane needs S (lane 0's first state) and V (lane K-1's last)
//     for the infection term — three broadcasts per RHS evaluation;
//   * the per-walker error norm: each lane's argmax of |e_s|/sk_s over its states, then
//     a tree over the K lanes (lower lanes win ties, as the sequential scan does);
//   * HINIT's norms (max, exact, any order), the observation sums (passed lane to lane
//     in state order, so the sum has the one-lane kernel's sequential order) and, at
//     the end, the status accumulators.
// Each state's arithmetic is the one-lane kernel's, operation for operation (the split
// RHS below is Chain::rhs element by element); a wave now holds 64/K walkers, which
// share one step size.  oracle/rk_ref.c restates exactly this (Prob.split = K).
#pragma once

namespace oe {

#ifndef OE_SPLIT_HOIST_M
#define OE_SPLIT_HOIST_M 6
#endif
constexpr int kSplitHoistM = OE_SPLIT_HOIST_M;  // dense coefficients per step up to this many states per lane

// quad_perm DPP controls for a group of K adjacent lanes (K = 2: lanes {0,1}, {2,3})
template <int K>
struct QuadCtl;
template <>
struct QuadCtl<2> {
  static constexpr int first = 0xA0;  // [0,0,2,2]: each lane gets its group's lane 0
  static constexpr int last = 0xF5;   // [1,1,3,3]: its group's last lane
  static constexpr int prev = 0xA0;   // lane r gets lane r-1 (lane 0: itself, unused)
};
template <>
struct QuadCtl<4> {
  static constexpr int first = 0x00;  // [0,0,0,0]
  static constexpr int last = 0xFF;   // [3,3,3,3]
  static constexpr int prev = 0x90;   // [0,0,1,2]
};
// butterfly partner at distance d (1: quad_perm [1,0,3,2], 2: [2,3,0,1])
template <int D>
__device__ __forceinline__ double partner(double v) {
  static_assert(D == 1 || D == 2, "groups of at most 4 lanes");
  return dpp_f64<D == 1 ? 0xB1 : 0x4E>(v);
}

// Chain<N>'s right-hand side for lane r's states [r·m, r·m + m): each element is the
// expression Chain::rhs evaluates for it, fma(A, B, -C), with the operands selected by
// the element's global index (a boundary role only on lane 0's first two and lane K-1's
// last two elements).
template <int N, int K>
__device__ __forceinline__ void chain_rhs_split(const double (&y)[N / K], const double* p, double (&dy)[N / K],
                                                bool first_lane, bool last_lane) {
  constexpr int m = N / K;
  const double mu = p[0], phi = p[1], beta = p[2], lam = p[3], tau = p[4];
  const double Sv = dpp_f64<QuadCtl<K>::first>(y[0]);
  const double V = dpp_f64<QuadCtl<K>::last>(y[m - 1]);
  const double prev = dpp_f64<QuadCtl<K>::prev>(y[m - 1]);
  const double inf = phi * Sv * V;
  const double bl = beta * lam;
  // roles by the element's GLOBAL index g = r·m + j (with m = 1 or 2 the I1 / I(N-2) roles sit
  // on inner lanes); r from the lane flags for K = 2, from the lane id otherwise
  const int r = (K == 2) ? (first_lane ? 0 : 1) : (int)(__lane_id() & (K - 1));
#pragma unroll
  for (int j = 0; j < m; ++j) {
    const int g = r * m + j;
    const double ym1 = (j == 0) ? prev : y[j - 1];
    double A = tau, B = ym1, C = tau * y[j];  // tau*I(k-1) - tau*Ik
    if (g == 0) { A = mu; B = Sv; C = inf; }                                      // mu*S - phi*S*V
    if (g == 1) { A = -tau; B = y[j]; C = -inf; }                                 // phi*S*V - tau*I1
    if (g == N - 2) C = lam * y[j];                                               // tau*I(N-3) - lam*I(N-2)
    if (g == N - 1) { A = bl; C = inf; }                                          // beta*lam*I(N-2) - phi*S*V
    dy[j] = fma(A, B, -C);
  }
}

// the lane-group reductions
template <int K>
__device__ __forceinline__ double group_fmax(double v) {
  v = fmax(v, partner<1>(v));
  if constexpr (K == 4) v = fmax(v, partner<2>(v));
  return v;
}
template <int K>
__device__ __forceinline__ double group_fmin(double v) {
  v = fmin(v, partner<1>(v));
  if constexpr (K == 4) v = fmin(v, partner<2>(v));
  return v;
}
template <int K>
__device__ __forceinline__ double group_sum(double v) {  // NaN iff any lane's is
  v = v + partner<1>(v);
  if constexpr (K == 4) v = v + partner<2>(v);
  return v;
}
// per-walker argmax of |e|/sk: lane-local (num, den), combined in a tree in which the
// lower lanes' candidate is kept unless the upper one is strictly larger
template <int K>
__device__ __forceinline__ void group_argmax(double& num, double& den, int r) {
#pragma unroll
  for (int d = 1; d < K; d <<= 1) {
    const double pn = d == 1 ? partner<1>(num) : partner<2>(num);
    const double pd = d == 1 ? partner<1>(den) : partner<2>(den);
    const bool upper_self = (r & d) != 0;
    const double ln = upper_self ? pn : num, ld = upper_self ? pd : den;
    const double un = upper_self ? num : pn, ud = upper_self ? den : pd;
    const bool take_upper = un * ld > ln * ud;
    num = take_upper ? un : ln;
    den = take_upper ? ud : ld;
  }
}

// Σ of the masked states in increasing state order, passed from lane to lane (lane r
// continues lane r-1's partial sum), then broadcast from the last lane: the one-lane
// kernel's sequential sum, bit for bit.
template <int S, int K>
__device__ __forceinline__ double group_masked_sum(const double (&y)[S / K], uint64_t mask, int r) {
  constexpr int m = S / K;
  const uint64_t mine = mask >> (r * m);
  double c = 0.0;
#pragma unroll
  for (int step = 0; step < K; ++step) {
    const double in = step == 0 ? 0.0 : dpp_f64<QuadCtl<K>::prev>(c);
    double cn = in;
#pragma unroll
    for (int j = 0; j < m; ++j)
      if ((mine >> j) & 1ull) cn = cn + y[j];
    c = (r == step) ? cn : c;
  }
  return dpp_f64<QuadCtl<K>::last>(c);
}

template <int S, int K, bool INLINE_LOG = false>
__device__ __forceinline__ void observe_split(const DevProblem& pb, int i, const double (&y)[S / K], int& k, int r,
                                              Acc& a) {
  const cptr<Obs> obs = kconst(pb.obs);
  if (!(k < pb.n_obs && obs[k].tidx == i)) return;
  check_finite(y, a);
  while (k < pb.n_obs && obs[k].tidx == i) {
    const double c = group_masked_sum<S, K>(y, obs[k].mask, r);
    const double O = obs[k].O, two_s2 = obs[k].two_s2, O_lin = obs[k].O_lin;
    const double d = O - (INLINE_LOG ? log(c) : oe_log(c));
    const double term = (d * d) / two_s2;
    if (__builtin_isfinite(term)) { a.chi += term; a.nvalid += 1; }
    const double rr = c - O_lin;
    const double r2 = rr * rr;
    if (!__builtin_isnan(r2)) a.ssres += r2;
    ++k;
  }
}

// Emit grid point i for lane r's states: row store through a descriptor of the whole
// S·W row (lane offset = w·8 + r·m·W·8, state offset j·W·8), minimum, observations.
template <int S, int K, bool TRAJ, bool NT>
__device__ __forceinline__ void emit_split(const DevProblem& pb, int i, const double (&y)[S / K], double* traj,
                                           int64_t W, uint32_t off, bool active, int& k, int r, Acc& a) {
  constexpr int m = S / K;
  track_min<m>(y, a);
  if constexpr (TRAJ) {
    if (active) {
      const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(traj + (int64_t)i * S * W), 0, (uint32_t)(S * W * 8), 0x00020000);
#pragma unroll
      for (int j = 0; j < m; ++j) st_row<NT>(rsrc, off, (uint32_t)(j * W * 8), y[j]);
    }
  }
  observe_split<S, K>(pb, i, y, k, r, a);
}

// DOPRI5 (the one-lane kernel's algorithm) for K lanes per walker.
template <int N, int K, bool TRAJ, bool NT>
__device__ __forceinline__ void integrate_dopri5_split(const DevProblem& pb, double (&y)[N / K], const double* p,
                                                       double* traj, int64_t W, uint32_t off, bool active, int r,
                                                       Acc& a) {
  using namespace dp;
  constexpr int m = N / K;
  const bool first_lane = r == 0, last_lane = r == K - 1;
  auto rhs = [&](const double (&yy)[m], double (&dy)[m]) { chain_rhs_split<N, K>(yy, p, dy, first_lane, last_lane); };
  int k = 0;
  emit_split<N, K, TRAJ, NT>(pb, 0, y, traj, W, off, active, k, r, a);
  const cptr<double> times = kconst(pb.times);
  const double t0 = times[0];
  const double tend = times[pb.T - 1];
  const double rtol = pb.rtol, atol = pb.atol;
  bool dead = !active;
  double t = t0;
  double k1[m], k2[m], k3[m], k4[m], k5[m], k6[m], k7[m], yt[m], yn[m];
  rhs(y, k1);

  double h;
  {  // HINIT per walker (max norms over the group's lanes), wave minimum
    double d0 = 0.0, d1v = 0.0;
#pragma unroll
    for (int s = 0; s < m; ++s) {
      const double sk = atol + rtol * fabs(y[s]);
      d0 = fmax(d0, fabs(y[s]) / sk);
      d1v = fmax(d1v, fabs(k1[s]) / sk);
    }
    d0 = group_fmax<K>(d0);
    d1v = group_fmax<K>(d1v);
    double h0 = (d0 <= 1e-5 || d1v <= 1e-5) ? 1e-6 : 0.01 * (d0 / d1v);
    h0 = fmin(h0, tend - t0);
#pragma unroll
    for (int s = 0; s < m; ++s) yt[s] = fma(h0, k1[s], y[s]);
    rhs(yt, k2);
    double d2 = 0.0;
#pragma unroll
    for (int s = 0; s < m; ++s) {
      const double sk = atol + rtol * fabs(y[s]);
      d2 = fmax(d2, fabs(k2[s] - k1[s]) / sk);
    }
    d2 = group_fmax<K>(d2) / h0;
    const double dm = fmax(d1v, d2);
    const double h1 = (dm <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : inv_fifth_root(dm / 0.01);
    double hl = fmin(100.0 * h0, h1);
    if (dead || !__builtin_isfinite(hl) || !(hl > 0.0)) hl = tend - t0;
    h = wave_min(hl);
    h = fmin(h, tend - t0);
  }
  const double span = tend - t0;
  const double hmin = 1e-14 * fmax(fabs(tend), fabs(t0)) + 1e-300;
  const cptr<double> fifth = kconst(kFifthScale.v);
  int i = 1, nst = 0;
  bool last_rej = false;
  while (i < pb.T) {
    bool last = false;
    if (t + h >= tend) { h = tend - t; last = true; }
    const double b21 = h * a21;
    const double b31 = h * a31, b32 = h * a32;
    const double b41 = h * a41, b42 = h * a42, b43 = h * a43;
    const double b51 = h * a51, b52 = h * a52, b53 = h * a53, b54 = h * a54;
    const double b61 = h * a61, b62 = h * a62, b63 = h * a63, b64 = h * a64, b65 = h * a65;
    const double b71 = h * a71, b73 = h * a73, b74 = h * a74, b75 = h * a75, b76 = h * a76;
#pragma unroll
    for (int s = 0; s < m; ++s) yt[s] = fma(b21, k1[s], y[s]);
    rhs(yt, k2);
#pragma unroll
    for (int s = 0; s < m; ++s) yt[s] = fma(b32, k2[s], fma(b31, k1[s], y[s]));
    rhs(yt, k3);
#pragma unroll
    for (int s = 0; s < m; ++s) yt[s] = fma(b43, k3[s], fma(b42, k2[s], fma(b41, k1[s], y[s])));
    rhs(yt, k4);
#pragma unroll
    for (int s = 0; s < m; ++s) yt[s] = fma(b54, k4[s], fma(b53, k3[s], fma(b52, k2[s], fma(b51, k1[s], y[s]))));
    rhs(yt, k5);
#pragma unroll
    for (int s = 0; s < m; ++s)
      yt[s] = fma(b65, k5[s], fma(b64, k4[s], fma(b63, k3[s], fma(b62, k2[s], fma(b61, k1[s], y[s])))));
    rhs(yt, k6);
#pragma unroll
    for (int s = 0; s < m; ++s)
      yn[s] = fma(b76, k6[s], fma(b75, k5[s], fma(b74, k4[s], fma(b73, k3[s], fma(b71, k1[s], y[s])))));
    rhs(yn, k7);
    const double g1 = h * e1, g3 = h * e3, g4 = h * e4, g5 = h * e5, g6 = h * e6, g7 = h * e7;
    double num = 0.0, den = 1.0, nfe = 0.0;
#pragma unroll
    for (int s = 0; s < m; ++s) {
      const double e = fma(g7, k7[s], fma(g6, k6[s], fma(g5, k5[s], fma(g4, k4[s], fma(g3, k3[s], g1 * k1[s])))));
      const double ae = fabs(e);
      const double sk = fma(rtol, max_abs_raw(y[s], yn[s]), atol);
      nfe = fma(ae, 0.0, nfe);
      if (s == 0 || ae * den > num * sk) { num = ae; den = sk; }
    }
    group_argmax<K>(num, den, r);
    nfe = group_sum<K>(nfe);
    double el = num / den;
    if (!__builtin_isfinite(el) || __builtin_isnan(nfe)) el = 1e30;
    if (dead) el = 0.0;
    const double err = wave_max(el);
    ++nst;
    if (err <= 1.0) {
      const double tn = last ? tend : t + h;
      const double rh = 1.0 / h;
      const double hd1 = h * d1, hd3 = h * d3, hd4 = h * d4, hd5 = h * d5, hd6 = h * d6, hd7 = h * d7;
      // Hairer's dense-output coefficients: with few states per lane (and a trajectory, so
      // a grid point nearly always falls in the step) formed once per accepted step, else
      // per output point (the registers of m > kSplitHoistM lanes are taken); same values
      constexpr bool kHoist = TRAJ && m <= kSplitHoistM;
      double ydf[kHoist ? m : 1], bsp[kHoist ? m : 1], r4[kHoist ? m : 1], r5[kHoist ? m : 1];
      if constexpr (kHoist) {
#pragma unroll
        for (int s = 0; s < m; ++s) {
          ydf[s] = yn[s] - y[s];
          bsp[s] = fma(h, k1[s], -ydf[s]);
          r4[s] = fma(-h, k7[s], ydf[s]) - bsp[s];
          r5[s] = fma(hd7, k7[s], fma(hd6, k6[s], fma(hd5, k5[s], fma(hd4, k4[s], fma(hd3, k3[s], hd1 * k1[s])))));
        }
      }
      while (i < pb.T && times[i] <= tn) {
        const double ti = times[i];
        if (grid_needs_emit<N, TRAJ>(pb, i, k)) {
          double yo[m];
          if (ti == tn) {
#pragma unroll
            for (int s = 0; s < m; ++s) yo[s] = yn[s];
          } else {
            const double th = (ti - t) * rh;
            const double th1 = 1.0 - th;
#pragma unroll
            for (int s = 0; s < m; ++s) {
              if constexpr (kHoist) {
                yo[s] = fma(th, fma(th1, fma(th, fma(th1, r5[s], r4[s]), bsp[s]), ydf[s]), y[s]);
              } else {
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
            for (int s = 0; s < m; ++s) yo[s] = __builtin_nan("");
          }
          emit_split<N, K, TRAJ, NT>(pb, i, yo, traj, W, off, active, k, r, a);
        }
        ++i;
        nst = 0;
      }
#pragma unroll
      for (int s = 0; s < m; ++s) { y[s] = yn[s]; k1[s] = k7[s]; }
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
    if (i < pb.T && (nst >= pb.max_steps || h < hmin)) {  // budget: evict the walkers that pin the wave
      if (!dead && el >= 0.5 * err) {
        dead = true;
        a.status |= ST_MAXSTEP;
      }
      nst = pb.max_steps / 2;
      if (__ballot(!dead) == 0ull) {
        double yo[m];
#pragma unroll
        for (int s = 0; s < m; ++s) yo[s] = __builtin_nan("");
        for (; i < pb.T; ++i)
          if (grid_needs_emit<N, TRAJ>(pb, i, k)) emit_split<N, K, TRAJ, NT>(pb, i, yo, traj, W, off, active, k, r, a);
        break;
      }
      if (h < hmin) h = fmin(1e-3 * span, tend - t);
    }
  }
  if (dead && active) a.status |= ST_MAXSTEP;
  check_finite(y, a);
  if (dead) a.nf = __builtin_nan("");  // an evicted walker's final state is NaN
  // the walker's status accumulators over its lanes
  a.nf = group_sum<K>(a.nf);
  a.ymin = group_fmin<K>(a.ymin);
}

// Kernel: batched DOPRI5 integrate of Chain<N> with K lanes per walker (64/K walkers per
// wave).  Lane offsets into a trajectory row are 32-bit (S·W·8 < 2^32, checked on the
// host).  The XCD block order is the one-lane kernel's, over blocks of 256/K walkers.
template <int N, int K, bool TRAJ, bool NT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
    k_integrate_split(const DevProblem pb, const IntegrateArgs ia) {
  constexpr int m = N / K;
  static_assert(N % K == 0 && (K == 2 || K == 4), "K lanes per walker, m states each");
  const int64_t blk = ia.xcd_remap ? xcd_block(blockIdx.x, gridDim.x, ia.xcd_remap) : (int64_t)blockIdx.x;
  const int64_t gt = blk * blockDim.x + threadIdx.x;
  const int r = (int)(threadIdx.x & (K - 1));
  const int64_t gw = gt / K;
  const bool active = gw < ia.W;
  const int64_t w = active ? gw : ia.W - 1;  // tail lanes shadow the last walker, never store
  const int64_t W = ia.W;
  double y[m], p[5];
#pragma unroll
  for (int j = 0; j < m; ++j) y[j] = ia.y0[(int64_t)(r * m + j) * W + w];
#pragma unroll
  for (int j = 0; j < 5; ++j) p[j] = ia.theta[(int64_t)j * W + w];
  Acc a = acc_init();
  const uint32_t off = (uint32_t)(w * 8 + (int64_t)r * m * W * 8);
  integrate_dopri5_split<N, K, TRAJ, NT>(pb, y, p, ia.traj, W, off, active, r, a);
  if (active && r == 0) {
    if (ia.chi) ia.chi[w] = a.nvalid ? a.chi : __builtin_nan("");
    if (ia.ssres) ia.ssres[w] = a.ssres;
    if (ia.status) ia.status[w] = finish(a);
  }
}

// lanes per walker of the split DOPRI5 integrate for a model (0: not split)
template <class M>
constexpr int split_lanes() { return 0; }
#ifdef OE_SPLIT_FORCE_K  // measurement builds (tools/split_ab.py): one K for every chain N >= 10
template <int N>
constexpr int split_lanes_chain() { return (N >= 10 && N % OE_SPLIT_FORCE_K == 0) ? OE_SPLIT_FORCE_K : 0; }
#else
template <int N>
constexpr int split_lanes_chain() { return (N >= 14 && N <= 22 && N % 2 == 0) ? 2 : (N >= 24 && N % 4 == 0) ? 4 : 0; }
#endif

}  // namespace oe

namespace oe {

// Metropolis–Hastings (Samplers.py:104-153) for the split DOPRI5 models: the chain of
// walker w lives on its K lanes.  The walker's chain state (θ, the current point) is read
// and written by lane 0 only and broadcast to the other lanes with DPP, so no lane ever
// reads a row another lane writes; every lane then holds the same proposal, integrates its
// states, sees the same chi (the observation sums are group-wide) and takes the same
// decision.  Each lane reads and writes its own linked '<state>0' initial states.
// Otherwise k_mh's structure (chain state in HBM between iterations, buffer-descriptor
// rows, opaque row pointers).
template <int N, int K>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
    k_mh_split(const DevProblem pb, const MHArgs ma) {
  constexpr int m = N / K;
  constexpr int PMAX = 5 + 4;  // kPmax<Chain<N>>: the model's 5 plus up to 4 '<state>0' parameters
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int r = (int)(threadIdx.x & (K - 1));
  const int64_t gw = gt / K;
  const bool active = gw < ma.W;
  const bool writer = active && r == 0;
  const int64_t w = active ? gw : ma.W - 1;
  const int64_t W = ma.W;
  const int P = pb.P;
  double* __restrict__ theta = ma.theta;
  double* __restrict__ y0g = ma.y0;
  const uint32_t off = (uint32_t)w * 8u;
  const uint32_t off_s = (uint32_t)(w * 8 + (int64_t)r * m * W * 8);  // this lane's first state in [S][W]
  const Row ys(y0g, (int64_t)N * W);
  // lane 0's value of a walker row, on all K lanes
  auto ld0 = [&](const double* row) { return dpp_f64<QuadCtl<K>::first>(Row(row, W).ld(off)); };
  // the '<state>0' parameter of local state j (a select over the K lanes' global indices)
  auto linked = [&](int j) {
    int pi = ma.init_param[j];
#pragma unroll
    for (int q = 1; q < K; ++q) pi = (r == q) ? ma.init_param[q * m + j] : pi;
    return pi;
  };
  bool any_linked = false;  // wave-uniform
#pragma unroll
  for (int s = 0; s < N; ++s) any_linked = any_linked || ma.init_param[s] >= 0;

  if (ma.init) {  // a-priori fit (Samplers.py:88-91)
    double th[PMAX], y[m];
#pragma unroll
    for (int j = 0; j < PMAX; ++j) th[j] = (j < P) ? ld0(theta + (int64_t)j * W) : 0.0;
#pragma unroll
    for (int j = 0; j < m; ++j) y[j] = ys.ld(off_s + (uint32_t)(j * W * 8));
    Acc a = acc_init();
    integrate_dopri5_split<N, K, false, false>(pb, y, th, nullptr, W, off_s, active, r, a);
    if (writer) {
      const double chi = a.nvalid ? a.chi : __builtin_nan("");
      Row(ma.cur, W).st(off, chi);
      Row(ma.cur + W, W).st(off, 1.0 - a.ssres / pb.sstot);
      Row(ma.cur + 2 * W, W).st(off, -2.0 * (-chi) + 2.0 * (double)pb.pnum);
      Row(ma.cur + 3 * W, W).st(off, 0.0);
      if (ma.status) ma.status[w] = finish(a);
    }
    return;
  }
  double* __restrict__ cur = ma.cur;
  const int PS = P + 5;
  // the proposal θ' = exp(log θ + dz) for walking parameters (Framework.py:107-122),
  // formed from lane 0's θ: identical values every time it is formed
  auto propose = [&](int it, double (&tn)[PMAX]) {
    const double* dz = opaque(ma.dz + (int64_t)(it - ma.draw_it0) * P * W);
#pragma unroll
    for (int j = 0; j < PMAX; ++j) {
      const double thj = (j < P) ? ld0(theta + (int64_t)j * W) : 0.0;
      tn[j] = (j < P && ((ma.walk_mask >> j) & 1ull)) ? oe_exp(oe_log(thj) + Row(dz + (int64_t)j * W, W).ld(off)) : thj;
    }
  };
  for (int it = ma.it0; it < ma.it1; ++it) {
    double y[m], p5[5];
    theta = opaque(theta);
    y0g = opaque(y0g);
    {
      double tn[PMAX];
      propose(it, tn);
#pragma unroll
      for (int j = 0; j < m; ++j) {
        const int pi = linked(j);
        y[j] = (ma.any_walk && pi >= 0) ? pick(tn, pi) : ys.ld(off_s + (uint32_t)(j * W * 8));
      }
#pragma unroll
      for (int j = 0; j < 5; ++j) p5[j] = tn[j];  // the RHS reads the model's 5 parameters only
    }
    Acc a = acc_init();
    integrate_dopri5_split<N, K, false, false>(pb, y, p5, nullptr, W, off_s, active, r, a);
    const double chin = a.nvalid ? a.chi : __builtin_nan("");
    theta = opaque(theta);
    y0g = opaque(y0g);
    cur = opaque(cur);
#if OE_MH_CHECKS
    {  // the debug library's integrity checks, as k_mh; wave-uniform
      bool sound = theta == ma.theta && y0g == ma.y0 && cur == ma.cur &&
                   (it <= ma.burnin || (it - ma.row0 >= 0 && it - ma.row0 < ma.n_rows));
#pragma unroll
      for (int s = 0; s < N; ++s) sound = sound && ma.init_param[s] < P;
      if (!sound) {
        if (writer && ma.status) ma.status[w] = ST_INTERNAL;
        return;
      }
    }
#endif
    double tn[PMAX];  // the proposal again (not held in registers across the integration)
    propose(it, tn);
    const double u = Row(opaque(ma.u + (int64_t)(it - ma.draw_it0) * W), W).ld(off);
    double chi = ld0(cur), rsq = ld0(cur + W), aic = ld0(cur + 2 * W);
    double nacc = ld0(cur + 3 * W);
    const double lr = oe_exp(chi - chin);
    const double accp = oe_exp(oe_log(lr));
    const bool acc = accp > u;
    // the current parameters (lane 0's, on every lane), for the rejected proposal's
    // linked states and the sample row
    double told[PMAX];
#pragma unroll
    for (int j = 0; j < PMAX; ++j) told[j] = (j < P) ? ld0(theta + (int64_t)j * W) : 0.0;
    if (acc) {
      chi = chin;
      rsq = 1.0 - a.ssres / pb.sstot;
      aic = -2.0 * (-chi) + 2.0 * (double)pb.pnum;
      nacc += 1.0;
      if (writer) {
#pragma unroll
        for (int j = 0; j < PMAX; ++j)
          if (j < P) Row(theta + (int64_t)j * W, W).st(off, tn[j]);
        Row(cur, W).st(off, chi);
        Row(cur + W, W).st(off, rsq);
        Row(cur + 2 * W, W).st(off, aic);
        Row(cur + 3 * W, W).st(off, nacc);
        if (ma.status) ma.status[w] = finish(a);
      }
    }
    if (ma.any_walk && any_linked && active) {
#pragma unroll
      for (int j = 0; j < m; ++j) {
        const int pi = linked(j);
        if (pi >= 0) ys.st(off_s + (uint32_t)(j * W * 8), acc ? pick(tn, pi) : pick(told, pi));
      }
    }
    if (it > ma.burnin && writer) {
      double* row = ma.samples + (int64_t)(it - ma.row0) * PS * W;
#pragma unroll
      for (int j = 0; j < PMAX; ++j)
        if (j < P) Row(row + (int64_t)j * W, W).st(off, acc ? tn[j] : told[j]);
      Row(row + (int64_t)P * W, W).st(off, chi);
      Row(row + (int64_t)(P + 1) * W, W).st(off, rsq);
      Row(row + (int64_t)(P + 2) * W, W).st(off, aic);
      Row(row + (int64_t)(P + 3) * W, W).st(off, (double)it);
      Row(row + (int64_t)(P + 4) * W, W).st(off, nacc / (double)it);
    }
  }
}

}  // namespace oe

namespace oe {

// Speculative MH rounds (k_mh_tree, ode_kernels.cuh) for the split DOPRI5 models: a
// (node, chain) pair on K adjacent lanes, node-major, every lane forming the node's
// proposal from the chain's θ (the same values on every lane) and integrating its m
// states; lane 0 stores the node's result.  k_mh_resolve is shared.
template <int N, int K>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
    k_mh_split_tree(const DevProblem pb, const MHTreeArgs ta) {
  constexpr int m = N / K;
  constexpr int PMAX = 5 + 4;
  const MHArgs& ma = ta.m;
  const int64_t W = ma.W;
  const int P = pb.P;
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int r = (int)(threadIdx.x & (K - 1));
  const int64_t gl = gt / K;
  const bool active = gl < ta.n_lanes;
  const int64_t g = active ? gl : ta.n_lanes - 1;
  const int64_t n = g / W;
  const int64_t c = g - n * W;
  const int j = 31 - __builtin_clz((uint32_t)(n + 1));
  const uint32_t path = (uint32_t)(n + 1) - (1u << j);
  const uint32_t off = (uint32_t)c * 8u;
  const uint32_t off_s = (uint32_t)(c * 8 + (int64_t)r * m * W * 8);  // this lane's first state in [N][W]
  const Row ys(ma.y0, (int64_t)N * W);
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
  double y[m], p5[5];
#pragma unroll
  for (int jj = 0; jj < m; ++jj) {
    int pi = ma.init_param[jj];
#pragma unroll
    for (int q = 1; q < K; ++q) pi = (r == q) ? ma.init_param[q * m + jj] : pi;
    y[jj] = (ma.any_walk && pi >= 0) ? pick(tn, pi) : ys.ld(off_s + (uint32_t)(jj * W * 8));
  }
#pragma unroll
  for (int q = 0; q < 5; ++q) p5[q] = tn[q];
  Acc a = acc_init();
  integrate_dopri5_split<N, K, false, false>(pb, y, p5, nullptr, ta.n_lanes, 0u, active, r, a);
  if (active && r == 0) {
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
