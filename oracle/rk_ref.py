"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of oracle/rk_ref.c (see its header).

Batched layouts as in include/odelib_amd.h: y0 [S][W], theta [P][W], traj [T][S][W].
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "librkref.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp, i32, i64, d, u64 = C.c_void_p, C.c_int, C.c_int64, C.c_double, C.c_uint64
        L.ref_integrate.restype = C.c_int
        L.ref_integrate.argtypes = [i32, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp, i32, i32, d, d, i32,
                                    i64, vp, vp, vp, vp, vp, vp, i32, i32]
        L.ref_mh.restype = C.c_int
        L.ref_mh.argtypes = [i32, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp, i32, i32, d, d, i32, d, i32,
                             i64, i64, i32, i32, i32, u64, d, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32]
        L.ref_inv_fifth_root.restype = d
        L.ref_inv_fifth_root.argtypes = [d]
        L.ref_inv_fourth_root.restype = d
        L.ref_inv_fourth_root.argtypes = [d]
        L.ref_philox4x32_10.restype = None
        L.ref_philox4x32_10.argtypes = [vp, vp, vp]
        L.ref_philox_draws.restype = None
        L.ref_philox_draws.argtypes = [u64, u64, i32, i32, vp, vp]
        L.ref_dopri5_stats.restype = None
        L.ref_dopri5_stats.argtypes = [vp, i32]
        L.ref_rosenbrock_stats.restype = None
        L.ref_rosenbrock_stats.argtypes = [vp, i32]
        L.ref_bdf_stats.restype = None
        L.ref_bdf_stats.argtypes = [vp, i32]
        L.ref_inv_root.restype = d
        L.ref_inv_root.argtypes = [d, i32]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


METHODS = {"rk4": 0, "dopri5": 1, "auto": 2, "rosenbrock": 3, "bdf": 4}


class Problem:
    """Host copy of a FitProblem-like object, observations sorted by grid index
    (stable), exactly as oe_problem_set orders them."""

    def __init__(self, fp):
        order = np.argsort(np.asarray(fp.obs_tidx), kind="stable")
        self.model = int(fp.model_id)
        self.S, self.P, self.T = int(fp.n_states), int(fp.n_params), len(fp.times)
        self.times = np.ascontiguousarray(fp.times, dtype=np.float64)
        self.tidx = np.ascontiguousarray(np.asarray(fp.obs_tidx, np.int32)[order])
        self.mask = np.ascontiguousarray(np.asarray(fp.obs_mask, np.uint64)[order])
        self.O = np.ascontiguousarray(np.asarray(fp.obs_log, np.float64)[order])
        s = np.asarray(fp.obs_logsigma, np.float64)[order]
        self.two_s2 = np.ascontiguousarray(2.0 * (s * s))
        self.lin = np.ascontiguousarray(np.asarray(fp.obs_lin, np.float64)[order])
        self.method = METHODS[fp.method]
        self.substeps = int(fp.rk4_substeps)
        self.rtol, self.atol, self.max_steps = float(fp.rtol), float(fp.atol), int(fp.max_steps)
        self.sstot, self.pnum = float(fp.sstot), int(fp.pnum)

    def args(self):
        return (self.model, self.S, self.P, self.T, _p(self.times), len(self.tidx), _p(self.tidx),
                _p(self.mask), _p(self.O), _p(self.two_s2), _p(self.lin), self.method, self.substeps,
                self.rtol, self.atol, self.max_steps)


def product_split(fp) -> int:
    """Lanes per walker of the product's DOPRI5 integrate for this problem (the rule in
    include/odelib_amd.h, OE_NO_SPLIT): the built-in chain with 14..22 states (even) runs
    2 lanes per walker, 24+ states (a multiple of 4) 4 lanes; everything else 1."""
    S = int(fp.n_states)
    if int(fp.model_id) != 3 or fp.method != "dopri5" or getattr(fp, "custom_source", None) is not None:
        return 1
    if 14 <= S <= 22 and S % 2 == 0:
        return 2
    if S >= 24 and S % 4 == 0:
        return 4
    return 1


def lane_steps(fp) -> bool:
    """Whether the product's MH kernels step every chain on its own (ode_kernels.cuh
    kLaneSteps, lane.cuh, bdf.cuh integrate_bdf_lane): DOPRI5 / 'auto' / 'bdf', one lane per walker, at most
    8 states — step sizes (and BDF orders) per walker, not per lockstep group."""
    return fp.method in ("dopri5", "auto", "bdf") and int(fp.n_states) <= 8 and product_split(fp) == 1


def integrate(fp, y0, theta, trajectory=True, split=None, lane=False):
    """The engine's integrate restated.  ``split``: lanes per walker of the DOPRI5 kernel
    being checked (None: the product's choice for this problem, ``product_split``; 1: the
    one-lane grouping, as the product's OE_NO_SPLIT).  ``lane``: every walker with its own
    DOPRI5 step sizes (the MH kernels' integrator, no trajectory; ``lane_steps``)."""
    pr = Problem(fp)
    split = product_split(fp) if split is None else int(split)
    y0 = np.ascontiguousarray(y0, dtype=np.float64)
    theta = np.ascontiguousarray(theta, dtype=np.float64)
    W = theta.shape[1]
    traj = np.empty((pr.T, pr.S, W)) if trajectory else None
    chi = np.empty(W)
    ssres = np.empty(W)
    status = np.empty(W, np.int32)
    rc = lib().ref_integrate(*pr.args(), W, _p(y0), _p(theta), _p(traj), _p(chi), _p(ssres), _p(status),
                             split if split > 1 else 0, int(bool(lane)))
    if rc:
        raise RuntimeError("ref_integrate failed")
    return {"traj": traj, "chi": chi, "ssres": ssres, "status": status}


def mh_run(fp, theta, y0, nits, burnin, walk_mask, init_param=None, rng="philox", seed=0, replay=None,
           step_sd=0.05, walker_offset=0, split=None):
    """oe_mh_run restated; ``split`` as in ``integrate`` (the product's MH splits a chain over
    the same lanes as its DOPRI5 integrate)."""
    pr = Problem(fp)
    split = product_split(fp) if split is None else int(split)
    theta = np.array(theta, dtype=np.float64, order="C", copy=True)
    y0 = np.array(y0, dtype=np.float64, order="C", copy=True)
    W = theta.shape[1]
    kept = max(0, nits - 1 - burnin)
    samples = np.empty((max(kept, 1), pr.P + 5, W))
    final = np.empty((4, W))
    status = np.zeros(W, np.int32)
    walk = np.ascontiguousarray(np.asarray(walk_mask, np.uint8))
    ip = np.full(pr.S, -1, np.int32) if init_param is None else np.ascontiguousarray(np.asarray(init_param, np.int32))
    dz = u = None
    if rng == "replay":
        dz = np.ascontiguousarray(replay[0], dtype=np.float64)
        u = np.ascontiguousarray(replay[1], dtype=np.float64)
    rc = lib().ref_mh(*pr.args(), pr.sstot, pr.pnum, W, int(walker_offset), int(nits), int(burnin),
                      0 if rng == "replay" else 1, int(seed), float(step_sd), _p(walk), _p(ip), _p(dz), _p(u),
                      _p(theta), _p(y0), _p(samples), _p(final), _p(status), split if split > 1 else 0)
    if rc:
        raise RuntimeError("ref_mh failed")
    return {"samples": samples[:kept], "theta": theta, "y0": y0, "final": final, "status": status}


def dopri5_stats(reset: bool = True) -> dict:
    """Accepted / rejected DOPRI5 lockstep steps and groups since the last reset."""
    out = np.zeros(3, np.int64)
    lib().ref_dopri5_stats(out.ctypes.data, int(reset))
    return {"accepted": int(out[0]), "rejected": int(out[1]), "groups": int(out[2])}


def rosenbrock_stats(reset: bool = True) -> dict:
    """Rosenbrock lockstep steps (accepted + rejected) and groups since the last reset."""
    out = np.zeros(2, np.int64)
    lib().ref_rosenbrock_stats(out.ctypes.data, int(reset))
    return {"steps": int(out[0]), "groups": int(out[1])}


def bdf_stats(reset: bool = True) -> dict:
    """BDF lockstep steps (accepted + rejected), Jacobian evaluations and groups since the last reset."""
    out = np.zeros(3, np.int64)
    lib().ref_bdf_stats(out.ctypes.data, int(reset))
    return {"steps": int(out[0]), "jacobians": int(out[1]), "groups": int(out[2])}


def bdf_detail(reset: bool = True) -> dict:
    """Per-phase counts of the BDF restatement since the last reset: accepted steps,
    rejections on the error and on Newton, Newton iterations, order/step selections and grid
    points emitted (where a BDF step's time goes; profiles/NOTES.md)."""
    L = lib()
    L.ref_bdf_detail.restype = None
    L.ref_bdf_detail.argtypes = [C.c_void_p, C.c_int]
    out = np.zeros(6, np.int64)
    L.ref_bdf_detail(out.ctypes.data, int(reset))
    return dict(zip(("accepted", "rejected_error", "rejected_newton", "newton_iterations", "selections",
                     "grid_points"), (int(v) for v in out)))


def inv_root(x: float, q: int) -> float:
    """x^(-1/q) as the BDF step controller computes it (oracle/rk_ref.c inv_root)."""
    return lib().ref_inv_root(float(x), int(q))


def inv_fifth_root(x: float) -> float:
    """x^(-1/5) as the DOPRI5 step controller computes it (oracle/rk_ref.c)."""
    return lib().ref_inv_fifth_root(float(x))


def inv_fourth_root(x: float) -> float:
    """x^(-1/4) as the Rosenbrock step controller computes it (oracle/rk_ref.c)."""
    return lib().ref_inv_fourth_root(float(x))


def philox4x32_10(ctr, key):
    c = np.ascontiguousarray(ctr, np.uint32)
    k = np.ascontiguousarray(key, np.uint32)
    out = np.empty(4, np.uint32)
    lib().ref_philox4x32_10(_p(c), _p(k), _p(out))
    return out


def philox_draws(seed, gid, it, P, step_sd):
    """(step_sd·z [P], u) of walker ``gid`` at iteration ``it`` (the MH kernel's Philox draws)."""
    z = np.empty(P + 1)
    u = np.empty(1)
    lib().ref_philox_draws(int(seed) & 0xFFFFFFFFFFFFFFFF, int(gid), int(it), int(P), _p(z), _p(u))
    return step_sd * z[:P], float(u[0])


def mh_tree_run(fp, theta, y0, nits, burnin, walk_mask, init_param=None, depth=3, rng="philox", seed=0,
                replay=None, step_sd=0.05, walker_offset=0, chunk=25, split=None):
    """The speculative MH rounds of oe_mh_run (oe_mh_args.speculate = depth; ode_kernels.cuh
    k_mh_tree / capi.hip k_mh_resolve) restated on top of this restatement's batched
    integrate: per round of d iterations the (2^d - 1)·W proposals (node-major lanes n·W + c,
    chain-major c·N + n for 'auto'; node n at depth floor(log2(n+1)), path bits
    n + 1 - 2^depth) are integrated in ONE call —
    the same lockstep grouping as the device lanes — then each chain walks its tree with
    the accept test exp(log(exp(chi - chin))) > u (Samplers.py:124-153).  Rounds restart at
    the device's chunk boundaries (chunk rounded down to a multiple of d).  Proposals use
    numpy's exp/log (the device: ocml), hence rtol-level, not bitwise, agreement.
    ``split`` as in ``mh_run`` (the split DOPRI5 models' rounds put a proposal on K lanes:
    64/K proposals per step size)."""
    pr = Problem(fp)
    split = product_split(fp) if split is None else int(split)
    S, P = pr.S, pr.P
    theta = np.array(theta, dtype=np.float64, copy=True)
    y0 = np.array(y0, dtype=np.float64, copy=True)
    W = theta.shape[1]
    walk = np.asarray(walk_mask, bool)
    ip = np.full(S, -1) if init_param is None else np.asarray(init_param)
    any_walk = walk.any()
    lane = lane_steps(fp) and split == 1
    a0 = integrate(fp, y0, theta, trajectory=False, split=split, lane=lane)
    chi = a0["chi"].copy()
    rsq = 1.0 - a0["ssres"] / pr.sstot
    aic = -2.0 * (-chi) + 2.0 * pr.pnum
    nacc = np.zeros(W)
    status = a0["status"].copy()
    dz = np.empty((nits, P, W))
    uu = np.empty((nits, W))
    for it in range(1, nits):
        if rng == "philox":
            for w in range(W):
                dz[it, :, w], uu[it, w] = philox_draws(seed, walker_offset + w, it, P, step_sd)
        else:
            dz[it], uu[it] = replay[0][it - 1], replay[1][it - 1]
    kept = max(0, nits - 1 - burnin)
    samples = np.empty((max(kept, 1), P + 5, W))
    chunk = max(depth, chunk // depth * depth)
    for c0 in range(1, nits, chunk):
        c1 = min(nits, c0 + chunk)
        r0 = c0
        while r0 < c1:
            d = min(depth, c1 - r0)
            N = (1 << d) - 1
            tn = np.empty((N, P, W))
            for n in range(N):
                j = int(np.floor(np.log2(n + 1)))
                path = n + 1 - (1 << j)
                th = theta.copy()
                for k in range(j):
                    if (path >> k) & 1:
                        th[walk] = np.exp(np.log(th[walk]) + dz[r0 + k][walk])
                t = th.copy()
                t[walk] = np.exp(np.log(th[walk]) + dz[r0 + j][walk])
                tn[n] = t
            ys = np.repeat(y0[None], N, axis=0)
            if any_walk:
                for s in range(S):
                    if ip[s] >= 0:
                        ys[:, s] = tn[:, ip[s]]
            if split == 1 and pr.method == METHODS["auto"]:  # 'auto' k_mh_tree lanes: chain-major (c·N + n), 64 a group
                res = integrate(fp, np.ascontiguousarray(ys.transpose(1, 2, 0).reshape(S, W * N)),
                                np.ascontiguousarray(tn.transpose(1, 2, 0).reshape(P, W * N)), trajectory=False,
                                split=split, lane=lane)
                nchi, nss, nst = (res[k].reshape(W, N).T for k in ("chi", "ssres", "status"))
            else:  # node-major lanes (the other methods; split.cuh's tree kernel)
                res = integrate(fp, np.ascontiguousarray(ys.transpose(1, 0, 2).reshape(S, N * W)),
                                np.ascontiguousarray(tn.transpose(1, 0, 2).reshape(P, N * W)), trajectory=False,
                                split=split, lane=lane)
                nchi = res["chi"].reshape(N, W)
                nss = res["ssres"].reshape(N, W)
                nst = res["status"].reshape(N, W)
            for w in range(W):
                path = 0
                for j in range(d):
                    it = r0 + j
                    n = (1 << j) - 1 + path
                    with np.errstate(over="ignore", invalid="ignore"):
                        acc = bool(np.exp(np.log(np.exp(chi[w] - nchi[n, w]))) > uu[it, w])
                    if acc:
                        chi[w] = nchi[n, w]
                        rsq[w] = 1.0 - nss[n, w] / pr.sstot
                        aic[w] = -2.0 * (-chi[w]) + 2.0 * pr.pnum
                        nacc[w] += 1.0
                        theta[:, w] = tn[n, :, w]
                        status[w] = nst[n, w]
                    if any_walk:
                        for s in range(S):
                            if ip[s] >= 0:
                                y0[s, w] = theta[ip[s], w]
                    if it > burnin:
                        row = samples[it - burnin - 1]
                        row[:P, w] = theta[:, w]
                        row[P:, w] = (chi[w], rsq[w], aic[w], it, nacc[w] / it)
                    path |= int(acc) << j
            r0 += d
    final = np.stack([chi, rsq, aic, nacc])
    return {"samples": samples[:kept], "theta": theta, "y0": y0, "final": final, "status": status}
