"""Debug helper (GPU): device 'auto' outputs of the bitwise test's W=1 case under several
store policies, saved for comparison with the C restatement."""
import os
import sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
import numpy as np
from helpers import product_model
from test_gpu_stiff import _mixed_thetas
tag = sys.argv[1] if len(sys.argv) > 1 else "prod"
m = product_model("two_i", method="auto")
eng = m.engine()
theta = _mixed_thetas("two_i", 1, [0])
y0 = np.asarray(m.get_inits(), float)[:, None].copy()
out = {"theta": theta}
for nt in (True, False):
    o = eng.integrate(y0, theta, trajectory=True, nt_stores=nt)
    out[f"traj_nt{int(nt)}"] = o["traj"].cpu().numpy()
    out[f"chi_nt{int(nt)}"] = o["chi"].cpu().numpy()
o = eng.integrate(y0, theta, trajectory=False)
out["chi_notraj"] = o["chi"].cpu().numpy()
np.savez(f"gpurun_out/dbg_{tag}.npz", **out)
print("saved", tag)
