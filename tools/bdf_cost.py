"""What one BDF step costs on the device: the trajectory kernels' lockstep pass (bdf.cuh,
chi-only integrate) against the MH kernels' per-lane pass (bdf.cuh integrate_bdf_lane, the a-priori fit
of an mh_run with nits = 1), method 'bdf' (BDF from t0, no DOPRI5 phase), per step of the
slowest lane (C restatement's counts: accepted + rejected attempts).

    python tools/bdf_cost.py          (GPU box; the C library built in-tree)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    from helpers import product_model
    from oracle import rk_ref
    post = np.array([7.475e-9, 1.069e-7, 19.73, 1.934, 2.799])
    cases = {
        "tau1e5": np.array([7.475e-9, 1.069e-7, 19.73, 1.934, 1e5]),
        "slow_demo": np.array([4.467e-09, 1.241e-05, 5.917e+01, 1.711e-01, 1.739e+00]),
        "phi1e-4": np.array([7.475e-9, 1.06e-4, 19.73, 1.934, 2.799]),
        "posterior": post,
    }
    for method in ("bdf", "auto"):
        m = product_model("two_i", method=method)
        eng = m.engine()
        fp = m.fit_problem()
        for name, th1 in cases.items():
            for W in (1, 64):
                rs = np.random.RandomState(1)
                th = th1[:, None] * np.exp(0.02 * rs.standard_normal((5, W))) if W > 1 else th1[:, None].copy()
                th = np.ascontiguousarray(th)
                y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
                steps = []
                for w in range(W):
                    rk_ref.bdf_detail()
                    rk_ref.integrate(fp, y0[:, w:w + 1].copy(), th[:, w:w + 1].copy(), trajectory=False, lane=True)
                    b = rk_ref.bdf_detail()
                    steps.append(b["accepted"] + b["rejected_error"] + b["rejected_newton"])
                nmax = max(1, max(steps))
                for _ in range(2):
                    eng.integrate(y0, th, trajectory=False)
                lock_ms = eng.last_kernel_ms()
                for _ in range(2):
                    eng.mh_run(th, y0, nits=1, burnin=0, walk_mask=np.ones(5, np.uint8))
                lane_ms = eng.last_kernel_ms()
                print(json.dumps({"method": method, "case": name, "W": W, "max_bdf_steps": int(nmax),
                                  "lockstep_ms": round(lock_ms, 4), "lane_ms": round(lane_ms, 4),
                                  "lockstep_us_per_step": round(1e3 * lock_ms / nmax, 3),
                                  "lane_us_per_step": round(1e3 * lane_ms / nmax, 3)}), flush=True)


if __name__ == "__main__":
    main()
