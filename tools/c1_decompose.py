"""C1 on this box, decomposed (GPU box): the trajectory kernel, the same kernel without
the trajectory (its compute alone), and a plain fill of the same 2.1 GB buffer (the box's
write rate), each as K back-to-back launches after a warm-up, in one process.

    python tools/c1_decompose.py --rounds 3
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--walkers", type=int, default=65536)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--buffers", type=int, default=1,
                    help="time the trajectory kernel on this many separately allocated buffers")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    m, y0h = bench.build_problem("two_i", "rk4", 1000)
    eng = m.engine()
    W = a.walkers
    th = torch.as_tensor(bench.synthetic_walkers(W, 5), device=eng.dev).contiguous()
    y0 = torch.as_tensor(np.repeat(y0h[:, None], W, axis=1), device=eng.dev).contiguous()
    traj = eng.empty_traj(W)
    s = torch.cuda.current_stream()
    bufs = [traj] + [eng.empty_traj(W) for _ in range(a.buffers - 1)]
    cases = {f"traj_buf{j}": (lambda b=b: eng.integrate(y0, th, trajectory=True, traj_out=b, sync=False,
                                                         timing=False)) for j, b in enumerate(bufs)}
    cases.update({
        "compute_only": lambda: eng.integrate(y0, th, trajectory=False, sync=False, timing=False),
        "fill": lambda: traj.zero_(),
    })
    res = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, go in cases.items():
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.06:
                go()
                torch.cuda.synchronize()
            e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            e[0].record(s)
            for _ in range(a.launches):
                go()
            e[1].record(s)
            torch.cuda.synchronize()
            res[k].append(round(e[0].elapsed_time(e[1]) / a.launches, 4))
    addr = [hex(b.data_ptr()) for b in bufs]
    print(json.dumps({"walkers": W, "ms": res, "buffers": addr}), flush=True)


if __name__ == "__main__":
    main()
