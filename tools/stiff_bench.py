"""Kernel time of the adaptive methods on the C2 workload (two_i, 65 536 walkers, demo
draws; --model chain<N> for the wider chains) with a fraction of the walkers made stiff (tau raised), per method:

    python tools/stiff_bench.py --fracs 0 0.001 0.01 --taus 1e5 1e6

'dopri5' keeps stiff walkers in the shared step (the wave crawls at the stability limit,
or evicts them as MAXSTEP after max_steps per interval); 'auto' hands them to BDF at
their eviction points after 15 stiff steps (n_states <= 8; wider models: a Rosenbrock redo);
'rosenbrock' integrates every walker with RODAS.  One JSON line per (fraction, tau, mode).
--contiguous makes the stiff walkers walkers 0..n-1 (one wave's lanes).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--walkers", type=int, default=65536)
    ap.add_argument("--model", default="two_i", help="two_i | chain<N> (same five parameters)")
    ap.add_argument("--fracs", type=float, nargs="+", default=[0.0, 0.001, 0.01])
    ap.add_argument("--taus", type=float, nargs="+", default=[1e5, 1e6])
    ap.add_argument("--methods", nargs="+", default=["dopri5", "auto", "rosenbrock"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--trajectory", type=int, default=1)
    ap.add_argument("--contiguous", action="store_true", help="the stiff walkers are walkers 0..n-1 (one wave's lanes)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    dev = torch.device("cuda:0")
    W = args.walkers
    engines = {}
    for method in args.methods:
        m, y0h = bench.build_problem(args.model, method, 1000)
        engines[method] = m.engine()
    y0 = torch.as_tensor(np.repeat(y0h[:, None], W, axis=1), device=dev).contiguous()
    base = bench.synthetic_walkers(W, 5)
    traj = engines[args.methods[0]].empty_traj(W) if args.trajectory else None
    for frac in args.fracs:
        for tau in (args.taus if frac > 0 else [None]):
            th = base.copy()
            n_stiff = int(round(frac * W))
            lanes = np.random.RandomState(7).choice(W, n_stiff, replace=False) if n_stiff else []
            if args.contiguous:
                lanes = np.arange(n_stiff)
            if n_stiff:
                th[4, lanes] = tau
            theta = torch.as_tensor(th, device=dev).contiguous()
            for method in args.methods:
                eng = engines[method]
                ms = []
                for r in range(args.reps + 1):
                    out = eng.integrate(y0, theta, trajectory=bool(args.trajectory), traj_out=traj, sync=True)
                    if r:
                        ms.append(eng.last_kernel_ms())
                st = out["status"].cpu().numpy()
                print(json.dumps({"model": args.model, "walkers": W, "stiff_frac": frac, "tau": tau, "method": method,
                                  "kernel_ms": round(float(np.median(ms)), 4),
                                  "stiff_flagged": int(((st & 8) != 0).sum()), "maxstep": int(((st & 4) != 0).sum()),
                                  "trajectory": bool(args.trajectory)}), flush=True)


if __name__ == "__main__":
    main()
