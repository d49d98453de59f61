"""Kernel time of one batched integrate with and without the trajectory store, per
model / method / walker count: separates the compute floor from the store floor.

    python tools/time_modes.py --cases two_i:rk4:65536 two_i:dopri5:65536 chain20:dopri5:262144
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", nargs="+", default=["two_i:rk4:65536", "two_i:dopri5:65536"])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--modes", nargs="+", default=["traj", "notraj", "traj_half", "traj_noxcd"],
                    help="traj/notraj + optional _half, _noxcd, _xcdrange (one walker range per XCD), _pipe / _pipe4 / _pipe8 (producer/consumer store waves), _auto (library choice; default: direct kernel)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    dev = torch.device("cuda:0")
    for case in args.cases:
        model, method, W = case.split(":")
        W = int(W)
        m, y0h = bench.build_problem(model, method, 1000)
        eng = m.engine()
        S, P = len(y0h), 5
        theta = torch.as_tensor(bench.synthetic_walkers(W, P), device=dev).contiguous()
        y0 = torch.as_tensor(np.repeat(y0h[:, None], W, axis=1), device=dev).contiguous()
        traj = eng.empty_traj(W)
        row = {"case": case}
        modes = tuple(args.modes)
        ms = {k: [] for k in modes}
        # interleaved rounds after a warm-up of every mode (clocks settle, pages mapped)
        for r in range(args.reps + 3):
            for mode in modes:
                eng.integrate(y0, theta, trajectory=mode.startswith("traj"),
                              traj_out=traj if mode.startswith("traj") else None, sync=True,
                              half_waves="half" in mode,
                              xcd_remap=False if "noxcd" in mode else "ranges" if "xcdrange" in mode else True,
                              pipelined=(8 if "pipe8" in mode else 4 if "pipe4" in mode else 2 if "pipe" in mode
                                         else None if "auto" in mode else False))
                if r >= 3:
                    ms[mode].append(eng.last_kernel_ms())
        for mode in modes:
            row[mode + "_ms"] = round(float(np.median(ms[mode])), 4)
        row["store_floor_ms"] = round(W * 999 * 8 * S / 6.3e12 * 1e3, 4)
        row["hbm_frac_traj"] = round(W * 999 * 8 * S / (row["traj_ms"] * 1e-3) / 8e12, 4)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
