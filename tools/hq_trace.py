"""Timeline of the hand-over queue on C2 + 0.1 % stiff (a build with -DOE_HQ_TRACE=1, via
ODELIB_AMD_LIB): per handed walker, when its BDF wave started, when it claimed the walker and
how long its BDF pass took, in µs from the DOPRI5 kernel's first wave (s_memrealtime)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-3
    dev = torch.device("cuda:0")
    m, y0h = bench.build_problem("two_i", "auto", 1000)
    eng = m.engine()
    th = bench.synthetic_walkers(W, 5)
    n = max(1, int(round(frac * W)))
    lanes = np.random.RandomState(7).choice(W, n, replace=False)
    th[4, lanes] = 1e5
    theta = torch.as_tensor(th, device=dev).contiguous()
    y0 = torch.as_tensor(np.repeat(y0h[:, None], W, axis=1), device=dev).contiguous()
    traj = eng.empty_traj(W)
    for rep in range(3):
        out = eng.integrate(y0, theta, trajectory=True, traj_out=traj, sync=True)
        ms = eng.last_kernel_ms()
    cc = out["chi"].cpu().numpy()[lanes]
    ss = out["ssres"].cpu().numpy()[lanes]
    chi = np.floor(cc / 1e5)
    pend = cc - chi * 1e5
    claim = np.floor(ss / 1e5)
    dur = ss - claim * 1e5
    order = np.argsort(claim + dur)
    print(json.dumps({"kernel_ms": ms, "n": int(n), "dopri5_end_us": float(np.max(pend)),
                      "claim_spread_us": float(np.max(claim) - np.min(claim)),
                      "wave_start_us": [float(np.min(chi)), float(np.median(chi)), float(np.max(chi))],
                      "claim_us": [float(np.min(claim)), float(np.median(claim)), float(np.max(claim))],
                      "bdf_us": [float(np.min(dur)), float(np.median(dur)), float(np.max(dur))],
                      "end_us_max": float(np.max(claim + dur))}))
    for j in order[-8:]:
        print(int(lanes[j]), round(float(chi[j]), 1), round(float(claim[j]), 1), round(float(dur[j]), 1))


if __name__ == "__main__":
    main()
