"""Back-to-back vs interleaved kernel times of one trajectory configuration (diagnostic).

    python tools/b2b.py --case two_i:dopri5:65536
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="two_i:dopri5:65536")
    ap.add_argument("--reps", type=int, default=12)
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    dev = torch.device("cuda:0")
    model, method, W = args.case.split(":")
    W = int(W)
    m, y0h = bench.build_problem(model, method, 1000)
    eng = m.engine()
    theta = torch.as_tensor(bench.synthetic_walkers(W, 5), device=dev).contiguous()
    y0 = torch.as_tensor(np.repeat(y0h[:, None], W, axis=1), device=dev).contiguous()
    traj = eng.empty_traj(W)
    out = {"case": args.case}
    seqs = {
        "b2b_sync": lambda: [(eng.integrate(y0, theta, traj_out=traj, sync=True), eng.last_kernel_ms())[1]
                             for _ in range(args.reps)],
        "after_notraj": lambda: [(eng.integrate(y0, theta, trajectory=False, sync=True),
                                  eng.integrate(y0, theta, traj_out=traj, sync=True), eng.last_kernel_ms())[2]
                                 for _ in range(args.reps)],
        "b2b_sync_again": lambda: [(eng.integrate(y0, theta, traj_out=traj, sync=True), eng.last_kernel_ms())[1]
                                   for _ in range(args.reps)],
    }
    for name, f in seqs.items():
        f()  # warm
        ms = f()
        out[name] = [round(x, 4) for x in ms]
        out[name + "_median"] = round(float(np.median(ms)), 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
