"""Where a lone lane's BDF step spends its cycles, by phase (measurement build with
-DOE_BDF_CLOCKS=1: bash tools/build_alt.sh clk -DOE_BDF_CLOCKS=1, then on the GPU box
ODELIB_AMD_LIB=alt_lib/clk/odelib_amd/csrc/libodelib_amd.so python tools/bdf_phases.py).

Runs one stiff walker (1) with method 'bdf' through the MH kernel's per-lane pass (an mh_run
with nits = 1: no trajectory) and (2) with 'auto' through k_integrate with a trajectory (the
hand-over pass of C2 + 0.1 % stiff).  The kernel prints per-phase shader cycles (s_memtime)
and visit counts; this script prints cycles per step and shares.  The clock reads serialise
a little, so the total is a few % above an uninstrumented step.
"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, numpy as np
sys.path.insert(0, %(root)r); sys.path.insert(0, %(tests)r)
from helpers import product_model
th = np.array([7.475e-9, 1.069e-7, 19.73, 1.934, 1e5])[:, None]
mode = sys.argv[1]
m = product_model("two_i", method="bdf" if mode == "mh_bdf" else "auto")
# modes: mh_bdf | integrate_auto_traj (NT row stores) | integrate_auto_traj_temporal |
# integrate_auto_nortraj (chi only) | stiffmix2
eng = m.engine()
y0 = np.asarray(m.get_inits(), float)[:, None]
if mode == "stiffmix":  # bench.py's C2-stiffmix: 65 536 synthetic walkers, 0.1 %% with tau = 1e5
    import bench
    W = 65536
    th = bench.synthetic_walkers(W, 5)
    th[4, np.random.RandomState(7).choice(W, 66, replace=False)] = 1e5
    y0 = np.repeat(y0, W, axis=1)
if mode == "stiffmix2":  # -DOE_BDF_CLOCKS=2 library: cycles in the chi / R² outputs
    import bench
    W = 65536
    th = bench.synthetic_walkers(W, 5)
    lanes = np.random.RandomState(7).choice(W, 66, replace=False)
    th[4, lanes] = 1e5
    y0 = np.repeat(y0, W, axis=1)
    for _ in range(3):
        out = eng.integrate(y0, th, trajectory=True, sync=True)
    chi, ss, st = (out[k].cpu().numpy() for k in ("chi", "ssres", "status"))
    stiff = np.nonzero(st & 8)[0]
    rows = sorted(((int(chi[w]), int(ss[w]), int(w), int(w) // 64) for w in stiff), key=lambda r: -(r[0] + r[1]))
    import json
    print("stiffmix2", eng.last_kernel_ms(), json.dumps(rows), flush=True)
    sys.exit(0)
for _ in range(2):
    if mode == "mh_bdf":
        eng.mh_run(th, y0, nits=1, burnin=0, walk_mask=np.ones(5, np.uint8))
    else:
        eng.integrate(y0, th, trajectory=mode != "integrate_auto_nortraj", sync=True,
                      nt_stores=mode != "integrate_auto_traj_temporal")
    print("kernel_ms", eng.last_kernel_ms(), flush=True)
'''


def main():
    names = ["predict", "factor", "newton", "err", "diff", "grid", "select", "fail"]
    modes = sys.argv[1:] or ["mh_bdf", "integrate_auto_traj"]
    for mode in modes:
        code = CHILD % {"root": ROOT, "tests": os.path.join(ROOT, "tests")}
        out = subprocess.run([sys.executable, "-c", code, mode], capture_output=True, text=True, timeout=300).stdout
        if mode == "stiffmix2":
            for l in out.splitlines():
                if l.startswith("stiffmix2"):
                    _, ms, rows = l.split(" ", 2)
                    rows = json.loads(rows)
                    print(json.dumps({"mode": mode, "kernel_ms": float(ms), "stiff_lanes": len(rows),
                                      "slowest_8 [cycles_to_pass, cycles_in_pass, walker, wave]": rows[:8],
                                      "median_cycles_to_pass": sorted(r[0] for r in rows)[len(rows) // 2],
                                      "median_cycles_in_pass": sorted(r[1] for r in rows)[len(rows) // 2]}))
            continue
        lines = [l for l in out.splitlines() if l.startswith("bdf_clocks")]
        kms = [float(l.split()[1]) for l in out.splitlines() if l.startswith("kernel_ms")]
        if not lines:
            print(json.dumps({"mode": mode, "error": "no bdf_clocks line (not a -DOE_BDF_CLOCKS=1 library?)",
                              "tail": out[-500:]}))
            continue
        if mode == "stiffmix":  # the last launch's lines: when each stiff lane's pass began and how long it ran
            n = len(lines) // 2
            rows = []
            for l in lines[-n:]:
                f = l.split()
                rows.append((int(f[f.index("since_wave_start") + 1]), int(f[f.index("bdf_pass") + 1]),
                             int(f[f.index("predict") + 2])))
            rows.sort(key=lambda r: -(r[0] + r[1]))
            print(json.dumps({"mode": mode, "kernel_ms": kms[-1] if kms else None, "stiff_lanes": n,
                              "slowest_5 [since_wave_start, bdf_pass, attempts]": rows[:5],
                              "median_since_wave_start": sorted(r[0] for r in rows)[n // 2],
                              "median_bdf_pass": sorted(r[1] for r in rows)[n // 2],
                              "median_cycles_per_attempt": sorted(r[1] / max(r[2], 1) for r in rows)[n // 2]}),
                  flush=True)
            continue
        f = lines[-1].split()
        vals = {}
        for nm in names:
            j = f.index(nm)
            vals[nm] = (int(f[j + 1]), int(f[j + 2]))
        steps = vals["predict"][1]
        tot = sum(c for c, _ in vals.values())
        print(json.dumps({"mode": mode, "attempts": steps, "kernel_ms": kms[-1] if kms else None,
                          "since_wave_start": int(f[f.index("since_wave_start") + 1]),
                          "bdf_pass": int(f[f.index("bdf_pass") + 1]),
                          "cycles_per_attempt": round(tot / max(steps, 1), 1),
                          "per_attempt": {k: round(c / max(steps, 1), 1) for k, (c, n) in vals.items()},
                          "per_visit": {k: round(c / n, 1) if n else None for k, (c, n) in vals.items()},
                          "visits": {k: n for k, (c, n) in vals.items()},
                          "share": {k: round(c / tot, 3) for k, (c, n) in vals.items()}}), flush=True)


if __name__ == "__main__":
    main()
