"""Mean launch time of back-to-back series of different lengths (bench regime: a sync, then
K launches issued from Python between two events), interleaved, for one kernel — is there a
transient at the start of a series?

    python tools/series_len.py --kernel pipe4x --lengths 5 10 20 50 100
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
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--lengths", nargs="+", type=int, default=[5, 10, 20, 50, 100])
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--per-launch", action="store_true", help="also an event pair per launch (first 20)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    dev = torch.device("cuda:0")
    m, y0h = bench.build_problem("two_i", "rk4", 1000)
    eng = m.engine()
    W = 65536
    theta = torch.as_tensor(bench.synthetic_walkers(W, 5), device=dev).contiguous()
    y0 = torch.as_tensor(np.repeat(y0h[:, None], W, axis=1), device=dev).contiguous()
    traj = eng.empty_traj(W)
    s = torch.cuda.current_stream(dev)

    def launch():
        eng.integrate(y0, theta, traj_out=traj, sync=False, timing=False, kernel=args.kernel)

    launch()
    tw = time.perf_counter()
    while time.perf_counter() - tw < 0.2:
        for _ in range(5):
            launch()
        torch.cuda.synchronize(dev)
    res = {n: [] for n in args.lengths}
    for r in range(args.rounds):
        for n in args.lengths:
            torch.cuda.synchronize(dev)
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(s)
            for _ in range(n):
                launch()
            ev[1].record(s)
            torch.cuda.synchronize(dev)
            res[n].append(ev[0].elapsed_time(ev[1]) / n)
    out = {"kernel": eng.last_variant(), "mean_ms_by_length": {n: round(float(np.mean(v)), 4) for n, v in res.items()}}
    if args.per_launch:
        torch.cuda.synchronize(dev)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a, b in evs:
            a.record(s)
            launch()
            b.record(s)
        torch.cuda.synchronize(dev)
        out["per_launch_first20"] = [round(a.elapsed_time(b), 4) for a, b in evs]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
