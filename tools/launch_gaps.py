"""Wall time per back-to-back C1 launch with and without timing-event markers between
the launches (diagnostic for bench.py's ms_per_step vs kernel time).

    python tools/launch_gaps.py [--steps 50]
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
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    dev = torch.device("cuda:0")
    m, y0h = bench.build_problem("two_i", "rk4", 1000)
    eng = m.engine()
    W, P = 65536, 5
    theta = torch.as_tensor(bench.synthetic_walkers(W, P), device=dev).contiguous()
    y0 = torch.as_tensor(np.repeat(y0h[:, None], W, axis=1), device=dev).contiguous()
    traj = eng.empty_traj(W)
    stream = torch.cuda.current_stream(dev)

    def run(mode):
        K = args.steps
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        span = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        for _ in range(3):
            eng.integrate(y0, theta, trajectory=True, traj_out=traj, sync=False)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        span[0].record(stream)
        for k in range(K):
            if mode == "bench":
                ev[k][0].record(stream)
            eng.integrate(y0, theta, trajectory=True, traj_out=traj, sync=False, timing=(mode != "bare"))
            if mode == "bench":
                ev[k][1].record(stream)
        span[1].record(stream)
        torch.cuda.synchronize(dev)
        wall = (time.perf_counter() - t0) / K * 1e3
        out = {"mode": mode, "wall_ms_per_step": wall, "span_ms_per_step": span[0].elapsed_time(span[1]) / K}
        if mode == "bench":
            out["kernel_event_ms"] = sum(a.elapsed_time(b) for a, b in ev) / K
        return out

    for _ in range(args.reps):
        for mode in ("bench", "lib_events", "bare"):
            print(json.dumps(run(mode)), flush=True)


if __name__ == "__main__":
    main()
