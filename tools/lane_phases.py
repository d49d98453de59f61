"""Where a lone lane's per-lane DOPRI5 step (lane.cuh, the MH kernels) spends its cycles
(measurement build: bash tools/build_alt.sh lclk -DOE_LANE_CLOCKS=1, then on the GPU box
ODELIB_AMD_LIB=alt_lib/lclk/odelib_amd/csrc/libodelib_amd.so python tools/lane_phases.py).

One walker, method 'dopri5', an mh_run with nits = 1 (the a-priori fit: one integration):
the notebook fit's slow-chain θ and a near-posterior θ.  Phases: the seven stages (six RHS
evaluations and their combinations), the error norm + stiffness test + step-size root, the
accept/reject bookkeeping (grid window, dense-output coefficients at an observed crossing,
budget), and the wave's observation segments.  Each s_memtime mark costs a few hundred cycles.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, numpy as np
sys.path.insert(0, %(root)r); sys.path.insert(0, %(tests)r)
from helpers import product_model
from oracle import rk_ref
th = np.array(%(theta)r)[:, None]
m = product_model("two_i", method="dopri5")
eng = m.engine()
y0 = np.asarray(m.get_inits(), float)[:, None]
for _ in range(2):
    eng.mh_run(th, y0, nits=1, burnin=0, walk_mask=np.ones(5, np.uint8))
    print("kernel_ms", eng.last_kernel_ms(), flush=True)
'''
CASES = {"slow_demo": [4.467e-09, 1.241e-05, 5.917e+01, 1.711e-01, 1.739e+00],
         "posterior": [7.475e-9, 1.069e-7, 19.73, 1.934, 2.799]}


def main():
    for case, theta in CASES.items():
        code = CHILD % {"root": ROOT, "tests": os.path.join(ROOT, "tests"), "theta": theta}
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300).stdout
        lines = [l for l in out.splitlines() if l.startswith("lane_clocks")]
        kms = [float(l.split()[1]) for l in out.splitlines() if l.startswith("kernel_ms")]
        if not lines:
            print(json.dumps({"case": case, "error": "no lane_clocks line", "tail": out[-400:]}))
            continue
        f = lines[-1].split()
        vals = {nm: (int(f[f.index(nm) + 1]), int(f[f.index(nm) + 2])) for nm in ("stages", "error", "accept", "segment")}
        att = vals["stages"][1]
        tot = sum(c for c, _ in vals.values())
        print(json.dumps({"case": case, "attempts": att, "kernel_ms": kms[-1] if kms else None,
                          "cycles_per_attempt": round(tot / max(att, 1), 1),
                          "per_attempt": {k: round(c / max(att, 1), 1) for k, (c, n) in vals.items()},
                          "per_visit": {k: round(c / n, 1) if n else None for k, (c, n) in vals.items()},
                          "visits": {k: n for k, (c, n) in vals.items()}}), flush=True)


if __name__ == "__main__":
    main()
