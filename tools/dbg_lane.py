"""Debug helper (GPU): the a-priori chi of MH chains (k_mh's per-lane DOPRI5 + BDF
hand-over) for the stiff MH test's thetas, saved for comparison with the C restatement."""
import os
import sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
import numpy as np
from helpers import product_model
from test_gpu_stiff import _mixed_thetas
out = {}
for method in ("auto", "dopri5"):
    m = product_model("two_i", method=method)
    W = 128
    theta = _mixed_thetas("two_i", W, [1, 64, 65, 127])
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    walk = np.ones(5, np.uint8)
    r = m.engine().mh_run(theta, y0, nits=1, burnin=0, walk_mask=walk, rng="philox", seed=11)
    out[f"final_{method}"] = r["final"].cpu().numpy()
    out[f"status_{method}"] = r["status"].cpu().numpy()
    r = m.engine().mh_run(theta, y0, nits=3, burnin=0, walk_mask=walk, rng="philox", seed=11)
    out[f"samples3_{method}"] = r["samples"].cpu().numpy()
    out["theta"] = theta
np.savez("gpurun_out/dbg_lane.npz", **out)
print("saved")
