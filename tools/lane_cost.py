"""Per-step cost of the MH kernel's per-lane DOPRI5 on fixed proposals (GPU) against the
step counts of the C restatement (CPU) — is a demo step dearer than a synthetic one?

    python tools/lane_cost.py            (on a GPU box; the C library is built in-tree)

Each case runs `nits` MH iterations whose proposals are the same θ every time (replay draws
dz = 0, u = 2: never accepted), so every iteration integrates exactly the given 32 θ; the
kernel time per iteration ÷ the slowest lane's steps (C restatement, lane mode) is the cost
of one step of a 32-lane wave.  The C counts come from `auto` lane mode for both kernels
(identical to `dopri5`'s without a hand-over; `dopri5` lane mode's stats also count the idle
padding lanes of a one-walker call).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import bench
    from oracle import rk_ref
    m = bench.demo_model()
    pn = m.get_pnames()
    starts = bench.demo_fit_starts(m, 32)
    th_demo = np.array([[s[p] for s in starts] for p in pn])
    slow = np.array([4.467e-09, 1.241e-05, 5.917e+01, 1.711e-01, 1.739e+00])
    post = np.array([7.475e-9, 1.069e-7, 19.73, 1.934, 2.799])
    cases = {"synthetic": bench.synthetic_walkers(32, 5), "demo_starts": th_demo,
             "slow_x32": np.repeat(slow[:, None], 32, axis=1), "posterior_x32": np.repeat(post[:, None], 32, axis=1)}
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], 32, axis=1)
    nits = 41
    for method in ("dopri5", "auto"):
        mm = bench.demo_model()
        mm.method = method
        eng = mm.engine() if hasattr(mm, "engine") else None
        fpc = mm.fit_problem()
        fpc.method = "auto"
        for name, th in cases.items():
            th = np.ascontiguousarray(th, dtype=float)
            steps = []
            for w in range(32):
                rk_ref.dopri5_stats()
                rk_ref.bdf_detail()
                rk_ref.integrate(fpc, y0[:, w:w + 1].copy(), th[:, w:w + 1].copy(), trajectory=False, lane=True)
                s = rk_ref.dopri5_stats()
                b = rk_ref.bdf_detail()
                steps.append((s["accepted"] + s["rejected"], b["accepted"] + b["rejected_error"] + b["rejected_newton"]))
            steps = np.array(steps)
            dz = np.zeros((nits - 1, 5, 32))
            u = np.full((nits - 1, 32), 2.0)
            eng.mh_run(th, y0, nits=nits, burnin=0, walk_mask=np.ones(5, np.uint8), rng="replay", replay=(dz, u))
            eng.mh_run(th, y0, nits=nits, burnin=0, walk_mask=np.ones(5, np.uint8), rng="replay", replay=(dz, u))
            ms = eng.last_kernel_ms() / (nits - 1)
            print(json.dumps({"method": method, "case": name, "ms_per_it": round(ms, 4),
                              "max_dopri5_steps": int(steps[:, 0].max()), "max_bdf_steps": int(steps[:, 1].max()),
                              "us_per_max_dopri5_step": round(1e3 * ms / max(1, steps[:, 0].max()), 3)}), flush=True)


if __name__ == "__main__":
    main()
