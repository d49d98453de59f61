"""Debug helper (GPU): MH chains with stiff proposals, sequential (k_mh) and speculative
(k_mh_tree), 'auto' and 'bdf', saved for comparison with the C restatement."""
import os
import sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
import numpy as np
from helpers import product_model
from test_gpu_stiff import _mixed_thetas
out = {}
W = 128
theta = _mixed_thetas("two_i", W, [1, 64, 65, 127])
out["theta"] = theta
for method in ("auto", "bdf"):
    m = product_model("two_i", method=method)
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    walk = np.ones(5, np.uint8)
    for spec in (0, 3):
        r = m.engine().mh_run(theta, y0, nits=4, burnin=0, walk_mask=walk, rng="philox", seed=11, speculate=spec)
        out[f"samples_{method}_{spec}"] = r["samples"].cpu().numpy()
        out[f"status_{method}_{spec}"] = r["status"].cpu().numpy()
np.savez("gpurun_out/dbg_lane3.npz", **out)
print("saved")
