"""CPU-baseline pool size vs throughput on the GPU box (no GPU use): the box reports 256
CPUs (affinity) under a cgroup quota of 16 cores; bench.py sizes its oracle pool by the
smaller.  This runs the same oracle leg with 8, 16, 32, 64 and 128 processes, a short
budget each, and prints walker-timesteps/s per pool size.

    python tools/cpu_scaling.py --budget 6
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget", type=float, default=6.0)
    ap.add_argument("--procs", type=int, nargs="+", default=[8, 16, 32, 64, 128])
    a = ap.parse_args()
    import bench
    m, y0 = bench.build_problem("two_i", "rk4", 1000)
    fp = m.fit_problem()
    print(json.dumps({"host_cores": bench.host_cores()}), flush=True)
    for n in a.procs:
        r = bench.cpu_baseline("two_i", fp, y0, a.budget, 5, procs=n)
        print(json.dumps({"procs": n, "value": r["value"], "sample": r["sample"]}), flush=True)


if __name__ == "__main__":
    main()
