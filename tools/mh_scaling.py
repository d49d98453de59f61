"""MCMC-mode cost per iteration vs walker count: device Metropolis–Hastings (Philox
draws) against the bare integrate + fused chi of the same walkers (no trajectory), so
the MH overhead and the occupancy effect of larger ensembles are visible.

    python tools/mh_scaling.py --cases two_i:rk4 two_i:dopri5 chain20:rk4 --walkers 65536 262144 1048576
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", nargs="+", default=["two_i:rk4", "two_i:dopri5"])
    ap.add_argument("--walkers", nargs="+", type=int, default=[65536, 262144, 1048576])
    ap.add_argument("--nits", type=int, default=11)
    ap.add_argument("--onelane", action="store_true", help="also time one lane per chain (OE_NO_SPLIT)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    dev = torch.device("cuda:0")
    for case in args.cases:
        model, method = case.split(":")
        m, y0h = bench.build_problem(model, method, 1000)
        eng = m.engine()
        P = 5
        for W in args.walkers:
            theta = torch.as_tensor(bench.synthetic_walkers(W, P), device=dev).contiguous()
            y0 = torch.as_tensor(np.repeat(y0h[:, None], W, axis=1), device=dev).contiguous()
            for split in ((True, False) if args.onelane else (True,)):
                ms_int = []
                for r in range(5):
                    eng.integrate(y0, theta, trajectory=False, sync=True, split=split)
                    if r >= 2:
                        ms_int.append(eng.last_kernel_ms())
                walk = np.ones(P, np.uint8)
                eng.mh_run(theta, y0, nits=2, burnin=0, walk_mask=walk, rng="philox", seed=1, split=split)
                ms_mh = []
                for r in range(2):
                    eng.mh_run(theta, y0, nits=args.nits, burnin=args.nits // 2, walk_mask=walk, rng="philox",
                               seed=7, split=split)
                    ms_mh.append(eng.last_kernel_ms())
                integ = float(np.median(ms_int))
                per_it = min(ms_mh) / args.nits  # a-priori integrate + nits-1 proposals
                print(json.dumps({"case": case, "walkers": W, "split": split, "integrate_notraj_ms": round(integ, 4),
                                  "mh_ms_per_iteration": round(per_it, 4),
                                  "mh_overhead": round(per_it / integ - 1.0, 4),
                                  "walker_timesteps_per_s_mh": W * 999 / (per_it / 1e3)}), flush=True)
            del theta, y0
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
