// lane.cuh — DOPRI5 with its own step size per lane, for the kernels that store no
// trajectory (k_mh, k_mh_tree): the Metropolis–Hastings chains of Samplers.py:104-155, where
// each chain's odeint call (Framework.py:656) integrates that chain alone.
//
// The trajectory kernels keep the wave-lockstep step (one h per wave): their
// 64 lanes must sit on the same output row for coalesced row stores.  Without rows to store
// nothing ties the lanes together, and a shared step makes every chain pay for the hardest
// one in its wave: on the notebook fit's chains (explosive phi·beta draws, accuracy-limited)
// a 32-chain wave takes ~900 lockstep steps against ~650 for its worst chain alone and ~215
// for the median one (oracle/rk_ref.c, tools/lane_steps.py).  Here every step-size decision
// is the lane's own: HINIT without the wave minimum, the error norm without the wave
// maximum, the budget eviction of the lane itself; the loop runs until the wave's last lane
// is done.  The arithmetic of a step is integrate_dopri5's, operation for operation, so a
// lane's result is the lockstep algorithm on a one-walker group — what the C restatement
// computes with lane_steps set (oracle/rk_ref.c integrate_group) — and no longer depends on
// its wave-mates (MH chains are the same whatever chains share their wave, and speculative
// DOPRI5 rounds reproduce the sequential chains bit for bit).
//
// Observations: lanes reach an observed time at different loop iterations, and an
// observation handled whenever any lane reaches one (a divergent block with per-lane record
// loads and a log call) ran in most iterations: the first version was 1.6-1.8x slower than
// the lockstep kernel.  So the loop runs in segments, one per observed grid index (a
// wave-uniform walk over the sorted observation records): every lane steps until its step
// has crossed the segment's time, keeping that step's dense-output coefficients, then the
// wave evaluates the observation together (uniform records through scalar loads).  A lane's
// step sequence is not touched — it only waits — so the bits stay those of a group of one.
// Grid points that are not observed only advance the lane's grid index (the step budget
// counts steps since the last grid point, as odeint's mxstep per output interval); they are
// counted on a window of kGridWin grid times loaded one step ahead.
#pragma once

#ifndef OE_LANE_TAB_VREG
#define OE_LANE_TAB_VREG false
#endif
#ifndef OE_LANE_TAB_PIN  // the tableau's SGPR immediates defined at each integration's start (load_tab PIN)
#define OE_LANE_TAB_PIN true
#endif
#ifndef OE_LANE_AUTO_TAB  // 'auto' lanes: 0 tableau immediates, 1 in VGPRs, 2 mixed (load_tab MIX)
#define OE_LANE_AUTO_TAB 1
#endif
namespace oe {


// AUTO (S <= kStiffRegS): the stiffness test of integrate_dopri5 hands the lane over at
// its eviction point, as does the step budget; the BDF pass at the end continues it from
// the loop's live state (t, y, grid index, observation index, accumulators) with a step
// size and an order of its own (integrate_bdf_lane, bdf.cuh), so a handed lane's result
// does not depend on its wave-mates.  The call sits inside the DOPRI5 loop's exit path
// rather than in the caller: round 4's copy of the state into a Resume struct for a BDF
// pass run by the caller miscompiled in the MH kernels (400+ SGPRs spilled to VGPR lanes).
// This shape is bitwise the C restatement (oracle/rk_ref.c, lane mode) in every kernel:
// tests/test_gpu_bdf_lane.py, test_gpu_stiff.py, test_gpu_speculative.py.
template <class M, int PMAX, bool AUTO>
__device__ __forceinline__ void integrate_dopri5_lane(const DevProblem& pb, double (&y)[M::S],
                                                      const double (&p)[PMAX], int64_t W, uint32_t off,
                                                      bool active, Acc& a) {
  using namespace dp;
  constexpr int S = M::S;
  static_assert(S <= 8, "per-lane DOPRI5: the register path (S <= 8)");
  int k = 0;  // wave-uniform: the next observation record
  emit<S, false, false>(pb, 0, y, nullptr, W, off, active, k, a);
  const cptr<double> times = kconst(pb.times);
  const cptr<Obs> obs = kconst(pb.obs);
  const double t0 = times[0];
  const double tend = times[pb.T - 1];
  const double rtol = pb.rtol, atol = pb.atol;
  double t = t0;
  const Tab tb = load_tab<OE_LANE_TAB_VREG || (AUTO && OE_LANE_AUTO_TAB > 0), AUTO && OE_LANE_AUTO_TAB == 2, OE_LANE_TAB_PIN>();
  double k1[S], k2[S], k3[S], k4[S], k5[S], k6[S], k7[S], yt[S], yn[S];
  M::rhs(y, t, p, k1);

  // ---- initial step: Hairer's HINIT (max norm), this lane's own ----
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
    if (!__builtin_isfinite(hl) || !(hl > 0.0)) hl = tend - t0;
    h = fmin(hl, tend - t0);
  }

  const double hmin = 1e-14 * fmax(fabs(tend), fabs(t0)) + 1e-300;
  int i = 1;  // next grid index: times[i] > t
  double wv[kGridWin];  // times[i .. i + kGridWin)
#pragma unroll
  for (int j = 0; j < kGridWin; ++j) wv[j] = times[i + j];
  int nst = 0;
  bool last_rej = false;
  bool done = !active;           // no more steps: at t_end, abandoned or handed over
  bool evicted = false, handed = false;
  double t_stop = __builtin_inf();  // abandoned / handed over at this time: later points are not ours
  int k_lane = k;                   // the records this lane has observed
  int n_stiff = 0, n_nonstiff = 0;
  // the last accepted step's dense-output coefficients (from t_c with 1/h = rh_c to the
  // current t, whose state is y), kept for the observation that ends the segment
  double cy[S], cydf[S], cbsp[S], cr4[S], cr5[S];
  double t_c = t0, rh_c = 0.0;
#pragma unroll
  for (int s = 0; s < S; ++s) { cy[s] = y[s]; cydf[s] = 0.0; cbsp[s] = 0.0; cr4[s] = 0.0; cr5[s] = 0.0; }

#if OE_LANE_CLOCKS  // measurement builds: s_memtime per phase of a lane's DOPRI5 step (bdf.cuh BdfClk)
  BdfClk lclk;
  lclk.start();
#endif
  bool more = true;
  while (more) {  // one segment per observed grid index, then the rest of the grid (uniform)
    const bool is_obs = k < pb.n_obs;
    more = is_obs;
    const int tidx = is_obs ? obs[k].tidx : pb.T - 1;
    const double t_seg = times[tidx];
    while (!done && t < t_seg) {  // this lane's steps until one has crossed t_seg
      bool last = false;
      if (t + h >= tend) { h = tend - t; last = true; }
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
      M::rhs(yn, t + h, p, k7);
#if OE_LANE_CLOCKS
      lclk.mark(0);
#endif
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
      double err = num / den;
      if (!__builtin_isfinite(err) || __builtin_isnan(nfe)) err = 1e30;
      ++nst;

      if (err <= 1.0) {
        if (AUTO && nst >= kBdfTestSteps && (tend - t) > kBdfSwitchSteps * h) {  // as integrate_dopri5
          double stnum = 0.0, stden = 0.0;
          const double thr2 = ((tend - t) > kBdfSwitchLong * h) ? kBdfThrLong2 : kBdfThr2;
#pragma unroll
          for (int s = 0; s < S; ++s) {
            const double r = 1.0 / fma(rtol, max_abs_raw(y[s], yn[s]), atol);
            const double dk = (k7[s] - k6[s]) * r;
            stnum = fma(dk, dk, stnum);
            const double dy = (yn[s] - yt[s]) * r;
            stden = fma(dy, dy, stden);
          }
          if (stden > 0.0 && (h * h) * stnum > thr2 * stden) {
            n_nonstiff = 0;
            ++n_stiff;
          } else if (++n_nonstiff >= 6) {
            n_stiff = 0;
          }
          if (n_stiff >= 15) {  // handed over at the start of this step: (t, y, i) stay as they are
            handed = done = true;
            t_stop = t;
          }
        }
      }
      // the controller's safe·err^(-1/5), shared by the accept and reject paths (a wave whose
      // lanes split between them would otherwise run the root twice)
      const double sfe = safe * inv_fifth_root(err > 0.0 ? err : 1.0);
#if OE_LANE_CLOCKS
      lclk.mark(1);
#endif
      if (!handed && err <= 1.0) {  // an accepted step (not handed over at its start)
        const double tn = last ? tend : t + h;
        if (tn >= t_seg) {  // the step that crosses the segment's time: keep its coefficients
          const double hd1 = h * tb.v[26], hd3 = h * tb.v[27], hd4 = h * tb.v[28], hd5 = h * tb.v[29],
                       hd6 = h * tb.v[30], hd7 = h * tb.v[31];
#pragma unroll
          for (int s = 0; s < S; ++s) {
            cy[s] = y[s];
            cydf[s] = yn[s] - y[s];
            cbsp[s] = fma(h, k1[s], -cydf[s]);
            cr4[s] = fma(-h, k7[s], cydf[s]) - cbsp[s];
            cr5[s] = fma(hd7, k7[s], fma(hd6, k6[s], fma(hd5, k5[s], fma(hd4, k4[s], fma(hd3, k3[s], hd1 * k1[s])))));
          }
          t_c = t;
          rh_c = 1.0 / h;
        }
        // grid points in (t, tn]: counted on the window, which then moves past them
        int c = count_le(wv, tn);
        if (c != 0) {
          nst = 0;
          i += c;
          while (c == kGridWin) {  // more grid points than the window in one step
#pragma unroll
            for (int j = 0; j < kGridWin; ++j) wv[j] = times[i + j];
            c = count_le(wv, tn);
            i += c;
          }
#pragma unroll
          for (int j = 0; j < kGridWin; ++j) wv[j] = times[i + j];  // used from the next step on
        }
#pragma unroll
        for (int s = 0; s < S; ++s) { y[s] = yn[s]; k1[s] = k7[s]; }
        t = tn;
        double fac = (err > 0.0) ? sfe : facmax;
        fac = fmin(facmax, fmax(facmin, fac));
        if (last_rej) fac = fmin(fac, 1.0);
        h = h * fac;
        last_rej = false;
        if (i >= pb.T) done = true;
      } else if (!handed) {
        h = h * fmax(facmin, sfe);
        last_rej = true;
      }
      // ---- budget: the lane leaves (not after the last grid point) ----
      // (an accepted step just before may have crossed t_seg: that point is still this
      // lane's, from the step's coefficients — t_stop = t)
      if (!done && i < pb.T && (nst >= pb.max_steps || h < hmin)) {
        done = true;
        t_stop = t;
        if constexpr (AUTO) {  // handed over at its current state
          handed = true;
        } else {  // abandoned: NaN at the later points (masked chi), as a lone lockstep lane
          evicted = true;
        }
      }
#if OE_LANE_CLOCKS
      lclk.mark(2);
#endif
    }
    // ---- the segment's observation, evaluated by the whole wave (uniform records) ----
    // Every lane runs it (full EXEC: the out-of-line log is called from uniform control
    // flow — called under a partial EXEC, inside a kernel with hundreds of SGPRs spilled to
    // VGPR lanes, the BDF pass after it computed garbage); the lanes the point is not for
    // (handed over before it, tail lanes) work on a copy and drop it.
    if (is_obs) {
      const bool ours = t_seg <= t_stop;
      const bool part = active && (ours || evicted);
      double yo[S];
      if (!ours) {
#pragma unroll
        for (int s = 0; s < S; ++s) yo[s] = __builtin_nan("");
      } else if (t_seg == t) {  // on the crossing step's end: its new state
#pragma unroll
        for (int s = 0; s < S; ++s) yo[s] = y[s];
      } else {
        const double th = (t_seg - t_c) * rh_c;
        const double th1 = 1.0 - th;
#pragma unroll
        for (int s = 0; s < S; ++s)
          yo[s] = fma(th, fma(th1, fma(th, fma(th1, cr5[s], cr4[s]), cbsp[s]), cydf[s]), cy[s]);
      }
      int kk = k;
      Acc at = a;
      store_row_at<S, false, false>(nullptr, yo, W, off, active, at);  // the running minimum
      observe<S>(pb, tidx, yo, kk, at);
      if (part) {
        a = at;
        k_lane = kk;
      }
    }
    while (k < pb.n_obs && obs[k].tidx == tidx) ++k;  // uniform
#if OE_LANE_CLOCKS
    lclk.mark(3);
#endif
  }
#if OE_LANE_CLOCKS
  if (active)
    printf("lane_clocks lane %d stages %lu %u error %lu %u accept %lu %u segment %lu %u\n", (int)(off >> 3),
           lclk.c[0], lclk.n[0], lclk.c[1], lclk.n[1], lclk.c[2], lclk.n[2], lclk.c[3], lclk.n[3]);
#endif
  if (evicted) {
    a.status |= ST_MAXSTEP;
#pragma unroll
    for (int s = 0; s < S; ++s) y[s] = __builtin_nan("");
  }
  if (!handed) check_finite(y, a);
  if constexpr (AUTO) {
    if (__ballot(handed) != 0ull) {  // wave-uniform: the BDF pass from each handed lane's (t, y, i, k)
      if (handed) a.status |= ST_STIFF;
      integrate_bdf_lane<M, PMAX, false, false>(pb, y, t, i, k_lane, p, nullptr, W, (int64_t)(off >> 3), active,
                                                handed, a);
    }
  }
}

}  // namespace oe
