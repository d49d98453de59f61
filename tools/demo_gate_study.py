"""Where the notebook fit's MH iterations spend their time, per proposal, on the C restatement
(CPU), and what the 'auto' hand-over knobs would change — a study tool, not product.

    python tools/demo_gate_study.py NAME [MACRO=VALUE ...]

Builds oracle/rk_ref.c with the given -D knobs (NSW_RESUME: the cost gate, hand over only
while (t_end - t) > NSW_RESUME·h, default 300 = ode_kernels.cuh kBdfSwitchSteps; GATE_ALL=1:
the stiffness test counts steps since the start instead of since the last grid point;
BDF_SWITCH_LONG / BDF_THR_LONG2) into a temporary library, replays the device's numpy-legacy
streams (one RandomState per chain, seed = chain index) over the demo fit's 32 LHS starts
for 300 iterations, integrates every 6th iteration's 32 proposals one lane at a time
('auto', lane mode) and prints the wave cost model: max DOPRI5 steps × 1.39 us + max BDF steps
× 4.5 us (the two phases of a wave run one after the other; per-step costs from the 32-chain
synthetic MH and a lone-wave BDF step).  Results: profiles/NOTES.md (r04t).
"""
import os, sys, subprocess, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import numpy as np
sys.path.insert(0, ROOT)
import bench
from oracle import rk_ref
variant = sys.argv[1]; defs = sys.argv[2:]
so = os.path.join(tempfile.mkdtemp(), f"librkref_{variant}.so")
subprocess.check_call(["gcc", "-O2", "-std=c11", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", "-shared",
                       "-o", so, os.path.join(ROOT, "oracle", "rk_ref.c"), "-lm"] + [f"-D{d}" for d in defs])
rk_ref.LIB = so
m = bench.demo_model()
starts = bench.demo_fit_starts(m, 32)
pn = m.get_pnames(); P = len(pn); W = 32; NIT = 301
th = np.array([[s[p] for s in starts] for p in pn])
fp = m.fit_problem(); fp.method = "auto"
y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
dz = np.zeros((NIT - 1, P, W)); u = np.zeros((NIT - 1, W))
for w in range(W):
    rs = np.random.RandomState(w)
    for it in range(NIT - 1):
        for j in range(P): dz[it, j, w] = rs.normal(0, 0.05)
        for k in range(P): rs.standard_normal()
        u[it, w] = rs.random_sample()
r = rk_ref.mh_run(fp, th, y0, nits=NIT, burnin=0, walk_mask=np.ones(P, np.uint8), rng="replay", replay=(dz, u))
DP, BD = 1.39, 4.5
maxes = []; nb = 0; wave = []
cur = th.copy()
for it in range(0, NIT - 1, 6):
    cur = th if it == 0 else r["samples"][it - 1, :P, :]
    T = np.exp(np.log(cur) + dz[it])
    costs = []
    for w in range(W):
        rk_ref.dopri5_stats(); rk_ref.bdf_detail()
        rk_ref.integrate(fp, y0[:, w:w+1].copy(), np.ascontiguousarray(T[:, w:w+1]), trajectory=False, lane=True)
        s = rk_ref.dopri5_stats(); b = rk_ref.bdf_detail()
        bd = b["accepted"] + b["rejected_error"] + b["rejected_newton"]
        nb += bd > 0
        costs.append(((s["accepted"] + s["rejected"]) * DP + bd * BD, s["accepted"] + s["rejected"], bd))
    maxes.append(max(costs))
    wave.append(max(c[1] for c in costs) * DP + max(c[2] for c in costs) * BD)
mm = np.array([c[0] for c in maxes])
wave = np.array(wave)
print(f"{variant}: wave model (max dopri5 + max bdf) mean {wave.mean():.0f} us p90 {np.percentile(wave,90):.0f}")
print(f"{variant}: mean max-lane cost {mm.mean():.0f} us (p90 {np.percentile(mm,90):.0f}); max lanes using BDF "
      f"{sum(c[2] > 0 for c in maxes)}/{len(maxes)}; lanes with BDF {nb}/{len(maxes)*W}; "
      f"mean max dopri5 {np.mean([c[1] for c in maxes]):.0f} bdf {np.mean([c[2] for c in maxes]):.0f}", flush=True)
