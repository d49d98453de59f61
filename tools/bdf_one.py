"""One wave, one stiff lane: method 'bdf' on a single walker — the per-lane pass (bdf.cuh, the
a-priori fit of an mh_run with nits = 1, kernel k_mh) or the wave-lockstep pass (bdf_wave.cuh,
a chi-only integrate, k_integrate) — for rocprofv3 PMC passes (SQ counters per BDF step of a
lone lane) and wall timing.

    python tools/bdf_one.py --case tau1e5 --reps 5
    rocprofv3 --pmc SQ_INSTS_VALU ... --kernel-include-regex k_integrate -- python tools/bdf_one.py

Prints the C restatement's step count (accepted + rejected attempts) and the device's
kernel time per step; ODELIB_AMD_LIB selects a measurement build of the library.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

CASES = {"tau1e5": [7.475e-9, 1.069e-7, 19.73, 1.934, 1e5], "slow_demo": [4.467e-09, 1.241e-05, 5.917e+01, 1.711e-01, 1.739e+00],
         "posterior": [7.475e-9, 1.069e-7, 19.73, 1.934, 2.799]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="tau1e5", choices=list(CASES))
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--method", default="bdf")
    ap.add_argument("--kernel", default="lane", choices=["lane", "wave"])
    args = ap.parse_args()
    import numpy as np
    from helpers import product_model
    from oracle import rk_ref
    m = product_model("two_i", method=args.method)
    eng = m.engine()
    th = np.array(CASES[args.case], float)[:, None]
    y0 = np.asarray(m.get_inits(), float)[:, None]
    rk_ref.bdf_detail()
    rk_ref.integrate(m.fit_problem(), y0, th, trajectory=False, lane=True)
    b = rk_ref.bdf_detail()
    steps = b["accepted"] + b["rejected_error"] + b["rejected_newton"]
    ms = []
    for _ in range(args.reps):
        if args.kernel == "lane":
            eng.mh_run(th, y0, nits=1, burnin=0, walk_mask=np.ones(5, np.uint8))
        else:
            eng.integrate(y0, th, trajectory=False)
        ms.append(eng.last_kernel_ms())
    print(json.dumps({"case": args.case, "method": args.method, "kernel": args.kernel, "lib": os.environ.get("ODELIB_AMD_LIB", "default"),
                      "bdf_steps": steps, "detail": b, "kernel_ms_min": min(ms),
                      "us_per_step": 1e3 * min(ms) / max(steps, 1)}), flush=True)


if __name__ == "__main__":
    main()
