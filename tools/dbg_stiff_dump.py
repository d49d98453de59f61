"""Debug helper (GPU): device 'auto' trajectories of the stiff bitwise test cases (W = 1, 70,
200) saved to gpurun_out/ for offline comparison with the C restatement."""
import os
import sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
import numpy as np
from helpers import product_model
from test_gpu_stiff import _mixed_thetas
m = product_model("two_i", method="auto")
eng = m.engine()
out = {}
for W, stiff in ((1, [0]), (70, [3, 64, 69]), (200, [0, 1, 2, 130, 199])):
    theta = _mixed_thetas("two_i", W, stiff)
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1).copy()
    o = eng.integrate(y0, theta, trajectory=True)
    out[f"theta_{W}"] = theta
    out[f"traj_{W}"] = o["traj"].cpu().numpy()
    out[f"chi_{W}"] = o["chi"].cpu().numpy()
    out[f"status_{W}"] = o["status"].cpu().numpy()
np.savez("gpurun_out/dbg_stiff.npz", **out)
print("saved")
