"""Proposal / acceptance draw streams for ``oe_mh_run``.

``legacy_replay_streams`` reproduces, per chain, the exact numpy legacy-RNG
consumption of the reference sampler, so a device chain in replay mode sees the
same increments and uniforms as ``Statistics.Samplers.MetropolisHastings``:

  np.random.seed(random_seed)                                  Samplers.py:70
  per iteration it = 1..nits-1:
    for p in walking parameters (pnames order):  normal(0, 0.05)  Framework.py:119/122
    for p in walking parameters:  pdf(oldval)  -> draws only if oldval is falsy
    for p in walking parameters:  pdf()        -> dist.rvs(**hp)  Framework.py:103
    np.random.rand()                                           Samplers.py:127

The prior densities themselves are never used (Samplers.py:118-121), so only the
draws' consumption is reproduced.  ``device_plan`` says when the device generator
(``oe_numpy_streams`` / rng mode OE_RNG_NUMPY, odelib_amd/csrc/numpy_rng.cuh) can
produce the same streams: priors that are absent or lognorm (one standard normal per
rvs) and no falsy old values.  Otherwise this host generator is used.
"""
from __future__ import annotations

import numpy as np


def _consume_rvs(dist, hp, rs):
    name = getattr(getattr(dist, "dist", dist), "name", None)
    if name == "lognorm":  # lognorm._rvs = exp(s * standard_normal) (one gauss)
        rs.standard_normal()
    else:
        dist.rvs(random_state=rs, **(hp or {}))


def _is_lognorm(dist):
    return getattr(getattr(dist, "dist", dist), "name", None) == "lognorm"


def device_plan(seeds, pnames, walking, dists, oldvals=None):
    """Number of prior standard normals per iteration if the device can generate the
    reference's streams for these chains, else None."""
    if any(not (0 <= int(s) < 2 ** 32) for s in seeds):
        return None
    prior = 0
    for i, p in enumerate(pnames):
        if p not in walking:
            continue
        d = dists.get(p, (None, None))[0]
        if d is None:
            continue
        if not _is_lognorm(d):
            return None
        if oldvals is not None and any(not ov[i] for ov in oldvals):
            return None  # pdf(oldval) would draw too (Framework.py:99)
        prior += 1
    return prior


def legacy_replay_streams(seeds, nits, pnames, walking, dists, oldvals=None, step_sd=0.05, shape_dims=None):
    """Build replay arrays for W chains.

    seeds   : [W] int seeds (MCMC uses chain index, Framework.py:1015/1020)
    pnames  : parameter names in order (P)
    walking : set of walking parameter names (non-static)
    dists   : name -> (scipy dist or None, hyperparameter dict)
    Returns dz [nits-1][P][W] (0 for static parameters), u [nits-1][W].
    """
    seeds = list(seeds)
    W, P = len(seeds), len(pnames)
    n = max(int(nits) - 1, 0)
    dz = np.zeros((n, P, W))
    u = np.zeros((n, W))
    walk_idx = [i for i, p in enumerate(pnames) if p in walking]
    with_dist = [i for i in walk_idx if dists.get(pnames[i], (None, None))[0] is not None]
    sd = np.full((), step_sd)
    for w, seed in enumerate(seeds):
        rs = np.random.RandomState(int(seed))
        for it in range(n):
            for i in walk_idx:
                dz[it, i, w] = rs.normal(0, sd)
            # pdf(oldval): no draw unless the old value is falsy (Framework.py:99)
            if oldvals is not None:
                for i in with_dist:
                    if not oldvals[w][i]:
                        d, hp = dists[pnames[i]]
                        _consume_rvs(d, hp, rs)
            for i in with_dist:
                d, hp = dists[pnames[i]]
                _consume_rvs(d, hp, rs)
            u[it, w] = rs.rand()
    return dz, u
