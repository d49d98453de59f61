"""DOPRI5 steps of a wave: the lockstep step (one h per wave, the trajectory kernels) against
every walker stepping on its own (lane.cuh, the MH kernels), on the C restatement (CPU).

    python tools/lane_steps.py [--iters 300] [--every 20]

Two ensembles: the notebook fit's 32 chains (the bench's demo-fit starts, then the chains of
a Philox MH run of the C restatement, sampled every --every iterations) and 64 synthetic
near-posterior walkers (the bench's C2 draws).  Prints, per sample, the lockstep group's
accepted steps and the per-walker step counts (accepted + rejected: a walker alone can
reject) — the wave's loop runs until its slowest lane is done.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_lane(fp, y0, th):
    import numpy as np
    from oracle import rk_ref
    steps = []
    for w in range(th.shape[1]):
        rk_ref.dopri5_stats()
        rk_ref.integrate(fp, y0[:, w:w + 1].copy(), th[:, w:w + 1].copy(), trajectory=False)
        s = rk_ref.dopri5_stats()
        steps.append(s["accepted"] + s["rejected"])
    return np.array(steps)


def lockstep(fp, y0, th):
    from oracle import rk_ref
    rk_ref.dopri5_stats()
    rk_ref.integrate(fp, y0, th, trajectory=False)
    s = rk_ref.dopri5_stats()
    return s["accepted"] + s["rejected"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--every", type=int, default=20)
    args = ap.parse_args()
    import numpy as np
    import bench
    from oracle import rk_ref

    m = bench.demo_model()
    starts = bench.demo_fit_starts(m, 32)
    pn = m.get_pnames()
    th = np.array([[s[p] for s in starts] for p in pn])
    fp = m.fit_problem()
    fp.method = "dopri5"
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], 32, axis=1)
    r = rk_ref.mh_run(fp, th, y0, nits=args.iters + 1, burnin=0, walk_mask=np.ones(len(pn), np.uint8),
                      rng="philox", seed=3)
    for it in range(0, args.iters, args.every):
        T = np.ascontiguousarray(r["samples"][it, :len(pn), :])
        per = per_lane(fp, y0, T)
        print(f"demo it {it:4d}: lockstep {lockstep(fp, y0, T):5d} | per walker max {per.max():4d} "
              f"median {int(np.median(per)):4d}")
    mc, y0h = bench.build_problem("two_i", "dopri5", 1000)
    fpc = mc.fit_problem()
    W = 64
    th = bench.synthetic_walkers(W, 5)
    y0 = np.repeat(y0h[:, None], W, axis=1)
    per = per_lane(fpc, y0, th)
    print(f"synthetic 64: lockstep {lockstep(fpc, y0, th)} | per walker max {per.max()} mean {per.mean():.1f}")


if __name__ == "__main__":
    main()
