"""Correctness of a two_i split measurement build (OE_SPLIT_TWOI=K, ODELIB_AMD_LIB): its DOPRI5
trajectories against the C restatement with the same K-lane grouping (GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    from helpers import product_model, walker_thetas
    from oracle import rk_ref
    K = int(sys.argv[1])
    m = product_model("two_i", method="dopri5")
    W = 70
    th = walker_thetas("two_i", W, seed=3).T.copy()
    th[1, 5] = 1.5e-5
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    out = m.engine().integrate(y0, th, trajectory=True)
    ref = rk_ref.integrate(m.fit_problem(), y0, th, trajectory=True, split=K)
    same = np.array_equal(out["traj"].cpu().numpy(), ref["traj"], equal_nan=True)
    print("split", K, "traj bitwise vs C restatement:", same, "max|d|",
          float(np.nanmax(np.abs(out["traj"].cpu().numpy() - ref["traj"]))))


if __name__ == "__main__":
    main()
