"""One wave (64 walkers, demo draws) with one lane at tau = --tau, no trajectory, for the
methods given: a small workload for rocprofv3 --pmc passes comparing 'dopri5' and 'auto'
at the stability limit."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tau", type=float, default=3e3)
    ap.add_argument("--methods", nargs="+", default=["dopri5", "auto"])
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    dev = torch.device("cuda:0")
    W = 64
    for method in args.methods:
        m, y0h = bench.build_problem("two_i", method, 1000)
        eng = m.engine()
        th = bench.synthetic_walkers(W, 5)
        th[4, 17] = args.tau
        theta = torch.as_tensor(th, device=dev).contiguous()
        y0 = torch.as_tensor(np.repeat(y0h[:, None], W, axis=1), device=dev).contiguous()
        ms = []
        for _ in range(args.reps):
            eng.integrate(y0, theta, trajectory=False, sync=True)
            ms.append(eng.last_kernel_ms())
        print(method, args.tau, [round(x, 3) for x in ms], flush=True)


if __name__ == "__main__":
    main()
