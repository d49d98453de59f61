"""A/B of the split DOPRI5 kernel (split.cuh) against the one-lane kernel (OE_NO_SPLIT)
for the wide chain models, back-to-back launches timed with events (GPU box).

    python tools/split_ab.py --walkers 262144 --models 10 16 20 24 32
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
    ap.add_argument("--walkers", type=int, default=262144)
    ap.add_argument("--models", nargs="+", default=["10", "12", "16", "20", "24", "32"],
                    help="chain sizes (10) or model names (two_i)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    import numpy as np
    import torch
    from bench import HBM_PEAK_GBS, build_problem, synthetic_walkers
    W = args.walkers
    for name in args.models:
        name = f"chain{name}" if name.isdigit() else name
        m, y0h = build_problem(name, "dopri5", 1000)
        n = int(y0h.shape[0])
        eng = m.engine()
        th = torch.as_tensor(synthetic_walkers(W, 5), device=eng.dev).contiguous()
        y0 = torch.as_tensor(np.repeat(y0h[:, None], W, axis=1), device=eng.dev).contiguous()
        res = {"model": name, "walkers": W}
        for traj in (True, False):
            tr = eng.empty_traj(W) if traj else None
            for rnd in range(args.rounds):  # interleaved A/B rounds
                for split in (True, False):
                    def go():
                        return eng.integrate(y0, th, trajectory=traj, traj_out=tr, sync=False, timing=False,
                                             split=split)
                    t0 = time.perf_counter()
                    while time.perf_counter() - t0 < 0.06:
                        go()
                        torch.cuda.synchronize()
                    s = torch.cuda.current_stream()
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    ev[0].record(s)
                    for _ in range(args.reps):
                        go()
                    ev[1].record(s)
                    torch.cuda.synchronize()
                    ms = ev[0].elapsed_time(ev[1]) / args.reps
                    key = f"{'traj' if traj else 'chi'}_{'split' if split else 'onelane'}"
                    res.setdefault(key, []).append(round(ms, 4))
                    if traj and rnd == args.rounds - 1:
                        res[key + "_hbm_frac"] = round(W * 999 * 8 * n / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
            del tr
            torch.cuda.empty_cache()
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
