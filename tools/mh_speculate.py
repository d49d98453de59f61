"""Wall time of Metropolis–Hastings chains with and without speculative rounds
(oe_mh_args.speculate), per method and chain count — the small ensembles of a real fit
(the notebook: 32 chains x 1000 iterations) up to a full device.

    python tools/mh_speculate.py --cases two_i:rk4 two_i:dopri5 two_i:auto --walkers 1 32 1024 65536
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", nargs="+", default=["two_i:rk4", "two_i:dopri5", "two_i:auto"])
    ap.add_argument("--walkers", nargs="+", type=int, default=[1, 32, 256, 1024, 8192, 65536])
    ap.add_argument("--nits", type=int, default=201)
    ap.add_argument("--depths", nargs="+", default=["0", "auto"])
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
        walk = np.ones(P, np.uint8)
        for W in args.walkers:
            theta = torch.as_tensor(bench.synthetic_walkers(W, P), device=dev).contiguous()
            y0 = torch.as_tensor(np.repeat(y0h[:, None], W, axis=1), device=dev).contiguous()
            row = {"case": case, "walkers": W, "nits": args.nits}
            res = {}
            for d in args.depths:
                spec = d if d == "auto" else int(d)
                eng.mh_run(theta, y0, nits=3, burnin=0, walk_mask=walk, rng="philox", seed=1, speculate=spec)
                best = None
                for _ in range(2):
                    t0 = time.perf_counter()
                    r = eng.mh_run(theta, y0, nits=args.nits, burnin=args.nits // 2, walk_mask=walk, rng="philox",
                                   seed=7, speculate=spec)
                    wall = time.perf_counter() - t0
                    best = wall if best is None else min(best, wall)
                res[d] = r
                row[f"s_{d}"] = round(best, 4)
                row[f"depth_{d}"] = eng.last_mh_depth()
                row[f"ms_per_it_{d}"] = round(best / (args.nits - 1) * 1e3, 4)
            if "0" in res and "auto" in res:
                a, b = res["0"], res["auto"]
                row["speedup"] = round(row["s_0"] / row["s_auto"], 2)
                row["same_params"] = bool(torch.equal(a["samples"][:, :P], b["samples"][:, :P]))
            print(json.dumps(row), flush=True)
            del theta, y0, res
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
