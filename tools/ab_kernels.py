"""The RK4 trajectory kernels of one shape in long back-to-back series (the bench's regime),
interleaved, against the library's own choice (kernel="auto", OE_TUNE) — checks that the
tuner's short measurements pick the kernel that wins a long series.

    python tools/ab_kernels.py --cases two_i:65536 two_i:1048576 chain8:65536
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KERNELS = ("direct", "half", "pipe2", "pipe4", "pipe8", "pipe2x", "pipe4x", "pipe8x")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", nargs="+", default=["two_i:65536", "two_i:1048576"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--series-ms", type=float, default=40.0, help="length of one timed series")
    ap.add_argument("--substeps", type=int, default=1, help="rk4_substeps of the problem")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    dev = torch.device("cuda:0")
    for case in args.cases:
        model, W = case.split(":")
        W = int(W)
        m, y0h = bench.build_problem(model, "rk4", 1000, args.substeps)
        theta = torch.as_tensor(bench.synthetic_walkers(W, 5), device=dev).contiguous()
        y0 = torch.as_tensor(np.repeat(y0h[:, None], W, axis=1), device=dev).contiguous()
        eng = m.engine()
        traj = eng.empty_traj(W)
        # the library's choice first (a fresh engine: nothing tuned yet), timed as it would be
        t0 = time.perf_counter()
        eng.integrate(y0, theta, traj_out=traj, kernel="auto")
        tune_s = time.perf_counter() - t0
        row = {"case": case, "substeps": args.substeps, "auto_choice": eng.last_variant(), "tune_ms": eng.tune_times(),
               "tune_call_s": round(tune_s, 3)}
        avail = [k for k in KERNELS if k in row["tune_ms"]]

        def series(k, n):
            s = torch.cuda.current_stream(dev)
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            eng.integrate(y0, theta, traj_out=traj, kernel=k, sync=False, timing=False)
            ev[0].record(s)
            for _ in range(n):
                eng.integrate(y0, theta, traj_out=traj, kernel=k, sync=False, timing=False)
            ev[1].record(s)
            torch.cuda.synchronize(dev)
            return ev[0].elapsed_time(ev[1]) / n

        one = series("direct", 3)
        n = max(4, int(args.series_ms / one))
        tw = time.perf_counter()
        while time.perf_counter() - tw < 0.15:
            series("direct", n)
        ms = {k: [] for k in avail}
        for r in range(args.rounds):
            for k in (avail if r % 2 == 0 else avail[::-1]):
                ms[k].append(series(k, n))
        row["series_launches"] = n
        row["series_ms"] = {k: round(float(np.median(v)), 4) for k, v in ms.items()}
        best = min(row["series_ms"], key=row["series_ms"].get)
        row["series_best"] = best
        row["auto_vs_best"] = round(row["series_ms"][row["auto_choice"]] / row["series_ms"][best], 4)
        print(json.dumps(row), flush=True)
        del traj, eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
