"""Samplers: Latin-hypercube survey and Metropolis–Hastings (ODElib/Statistics/Samplers.py).

``MetropolisHastings`` keeps the reference signature (Samplers.py:53) and runs the
chain on the device (one walker).  ``batched_metropolis_hastings`` is what
``ModelFramework.MCMC`` uses: every chain is a walker of ONE ``oe_mh_run``.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from ..rng import device_plan, legacy_replay_streams


def lhs_classic(n, samples):
    """Classic Latin hypercube (the algorithm of pyDOE2.lhs with no criterion, which the
    reference imports at Samplers.py:3 and which is absent from this image): one
    uniform draw per stratum and dimension, strata shuffled per dimension, global
    numpy RNG."""
    cut = np.linspace(0, 1, samples + 1)
    u = np.random.rand(samples, n)
    a = cut[:samples]
    b = cut[1:samples + 1]
    rdpoints = np.zeros_like(u)
    for j in range(n):
        rdpoints[:, j] = u[:, j] * (b - a) + a
    H = np.zeros_like(rdpoints)
    for j in range(n):
        order = np.random.permutation(range(samples))
        H[:, j] = rdpoints[order, j]
    return H


def sample_lhs(parameter_dict, samples):
    """LHS draws mapped through each prior's ppf (Samplers.py:6-51)."""
    total_ps = 0
    for p in parameter_dict:
        total_ps += np.count_nonzero(parameter_dict[p].val)
    lhd = lhs_classic(total_ps, samples=samples)
    var_samples = {}
    lhd_i = 0
    for p in parameter_dict:
        nump = np.count_nonzero(parameter_dict[p].val)
        s = lhd[:, lhd_i:lhd_i + nump]
        lhd_i += nump
        s = parameter_dict[p].dist.ppf(s, **parameter_dict[p].hp)
        if nump == 1:
            var_samples[p] = np.concatenate(s, axis=None)
        else:
            _sample = []
            _p = np.array(parameter_dict[p].val, dtype=float)
            for row in s:
                _p[np.where(_p != 0)] = row
                _sample.append(np.copy(_p))
            var_samples[p] = _sample
    return pd.DataFrame(var_samples)


def _posterior_frame(samples, pnames, static_parameters, chains, kept):
    """[kept][P+5][W] device block -> the reference's per-chain DataFrames
    (Samplers.py:160-172) concatenated with 'chain#' (Framework.py:1035-1038)."""
    P = len(pnames)
    W = len(chains)
    cols = list(pnames) + ["chi", "rsquared", "aic", "iteration", "acceptance_ratio"]
    if kept <= 0:
        frames = []
        for i in range(W):
            df = pd.DataFrame([[np.nan] * (P + 3)])
            df["chain#"] = i
            frames.append(df)
        out = pd.concat(frames)
        out.reset_index(drop=True, inplace=True)
        return out
    blk = np.ascontiguousarray(np.transpose(samples, (2, 0, 1))).reshape(W * kept, P + 5)
    out = pd.DataFrame(blk, columns=cols)
    out["iteration"] = out["iteration"].astype(np.int64)
    for p in static_parameters:  # Samplers.py:166-170 (reports hp['scale'])
        out[p] = [chains[c].parameters[p].hp['scale'] for c in range(W) for _ in range(kept)]
    out["chain#"] = np.repeat(np.arange(W), kept)
    out.reset_index(drop=True, inplace=True)
    return out


def batched_metropolis_hastings(chains, nits=1000, burnin=None, static_parameters=(), rng="replay", seed=0,
                                engine=None, walker_offset=0, return_device=False):
    """Run ``len(chains)`` Metropolis–Hastings chains as walkers of one device launch.

    chains : ModelFramework copies (one per chain, each with its own initial θ,
             initial states and ``random_seed``); they must share the fit problem."""
    m0 = chains[0]
    pnames = m0.get_pnames()
    snames = list(m0._snames)
    reject = set(static_parameters)
    if not burnin:
        burnin = int(nits / 2)
    W = len(chains)
    theta = np.array([[float(np.asarray(c.parameters[p].val)) for p in pnames] for c in chains]).T.copy()
    y0 = np.array([[float(np.asarray(c.istates[s])) for s in snames] for c in chains]).T.copy()
    walk = [p not in reject for p in pnames]
    init_param = [pnames.index(s + "0") if (s + "0") in pnames else -1 for s in snames]
    eng = engine if engine is not None else m0.engine()
    replay, numpy_seeds, prior_draws = None, None, 0
    if rng in ("replay", "replay-host"):
        # the reference's numpy streams: generated on the device when the priors allow
        # it (rng.device_plan), else on the host ('replay-host' forces the host)
        dists = {p: (m0.parameters[p].dist, m0.parameters[p].hp) for p in pnames}
        seeds = [c.random_seed for c in chains]
        walking = {p for p in pnames if p not in reject}
        plan = device_plan(seeds, pnames, walking, dists, oldvals=theta.T.tolist()) if rng == "replay" else None
        if plan is not None:
            rng, numpy_seeds, prior_draws = "numpy", seeds, plan
        else:
            rng = "replay"
            replay = legacy_replay_streams(seeds, nits, pnames, walking, dists, oldvals=theta.T.tolist())
    res = eng.mh_run(theta, y0, nits=nits, burnin=burnin, walk_mask=walk, init_param=init_param, rng=rng,
                     seed=seed, replay=replay, walker_offset=walker_offset, numpy_seeds=numpy_seeds,
                     prior_draws=prior_draws)
    kept = max(0, nits - 1 - burnin)
    if return_device:
        return res
    samples = res["samples"].cpu().numpy() if kept > 0 else None
    th = res["theta"].cpu().numpy()
    yf = res["y0"].cpu().numpy()
    for w, c in enumerate(chains):  # chains end at their last state, as the reference leaves them
        c.set_parameters(**{p: th[j, w] for j, p in enumerate(pnames) if p not in reject})
        c.set_inits(**{s: yf[k, w] for k, s in enumerate(snames)})
    return _posterior_frame(samples, pnames, static_parameters, chains, kept)


def MetropolisHastings(modelframework, nits=1000, burnin=None, static_parameters=set(), print_progress=True):
    """Single-chain drop-in of Samplers.MetropolisHastings (Samplers.py:53-174), on
    the device, with the reference's numpy draws replayed (seed = random_seed)."""
    if not burnin:
        burnin = int(nits / 2)
    df = batched_metropolis_hastings([modelframework], nits=nits, burnin=burnin,
                                     static_parameters=static_parameters, rng="replay")
    df = df.drop(columns=["chain#"])
    if print_progress:
        print("iteration; error; acceptance ratio")
        if len(df) and "chi" in df:
            print(int(df["iteration"].iloc[-1]), float(np.exp(-df["chi"].iloc[-1])),
                  float(df["acceptance_ratio"].iloc[-1]))
    return df
