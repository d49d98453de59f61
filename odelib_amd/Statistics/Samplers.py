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
    """Latin-hypercube samples of the parameters in ``parameter_dict`` (name -> parameter
    with a prior), mapped through each prior's ppf (Samplers.py:6-51).  An array-valued
    parameter takes one hypercube dimension per non-zero element and yields one array per
    sample (its zero elements stay zero).  Returns a DataFrame with one column per name."""
    width = {name: int(np.count_nonzero(par.val)) for name, par in parameter_dict.items()}
    unit = lhs_classic(sum(width.values()), samples=samples)
    columns, first = {}, 0
    for name, par in parameter_dict.items():
        block = par.dist.ppf(unit[:, first:first + width[name]], **par.hp)
        first += width[name]
        if width[name] == 1:
            columns[name] = block.ravel()
            continue
        template = np.array(par.val, dtype=float)
        slots = template != 0
        rows = []
        for draw in block:
            row = template.copy()
            row[slots] = draw
            rows.append(row)
        columns[name] = rows
    return pd.DataFrame(columns)


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


def _fmt(x):
    """How the reference's print shows a likelihood value: str of an np.float64, or '--'
    for an all-masked chi (np.ma.masked, NaN here)."""
    return "--" if np.isnan(x) else str(np.float64(x))


def _print_iterations(a_priori, chi_rows):
    """The line every reference chain prints on every iteration, before its decision
    (Samplers.py:123: ``print(it, np.exp(-chi))`` with chi the current state's):
    iteration 1 shows the a-priori chi, iteration it the chi after iteration it-1.
    a_priori [W], chi_rows [nits-1][W] (chain state after each iteration); chain after
    chain, as the reference's serial MCMC loop prints them."""
    import sys
    n, W = chi_rows.shape
    with np.errstate(over="ignore", invalid="ignore"):
        for w in range(W):
            prev = np.concatenate([[a_priori[w]], chi_rows[:-1, w]]) if n else np.zeros(0)
            err = np.exp(-prev)
            sys.stdout.write("".join(f"{it} {_fmt(e)}\n" for it, e in zip(range(1, n + 1), err)))
    sys.stdout.flush()


def batched_metropolis_hastings(chains, nits=1000, burnin=None, static_parameters=(), rng="replay", seed=0,
                                engine=None, walker_offset=0, return_device=False, iteration_log=False,
                                print_prior=False, speculate="auto"):
    """Run ``len(chains)`` Metropolis–Hastings chains as walkers of one device launch.

    chains : ModelFramework copies (one per chain, each with its own initial θ,
             initial states and ``random_seed``); they must share the fit problem.
    iteration_log : print the reference's per-iteration line of every chain (the run
             then keeps every iteration's row on the device and drops the burn-in rows
             on the host: same chains, the kernel's arithmetic does not depend on burnin).
    print_prior : print the reference's ``a priori error`` line and header first
             (MetropolisHastings with print_progress, Samplers.py:101-103).
    speculate : speculative MH rounds (``Engine.mh_run``): "auto" lets the library run
             several iterations per launch while the chains leave the device mostly idle
             (a few to a few thousand chains); 0 runs one iteration per step.  The chains
             are bitwise the same either way, for every method: the MH kernels integrate
             every proposal on its own (DOPRI5 step sizes per chain, csrc/lane.cuh; the BDF
             hand-over of 'auto' and method 'bdf' with step sizes and orders per chain,
             csrc/bdf.cuh integrate_bdf_lane), so a chain does not depend on the chains that share its
             wavefront, the speculation depth or the device's CU count."""
    m0 = chains[0]
    pnames = m0.get_pnames()
    snames = list(m0._snames)
    reject = set(static_parameters)
    if not burnin:
        burnin = int(nits / 2)
    W = len(chains)
    P = len(pnames)
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
    kw = dict(walk_mask=walk, init_param=init_param, rng=rng, seed=seed, replay=replay, walker_offset=walker_offset,
              numpy_seeds=numpy_seeds, prior_draws=prior_draws, speculate=speculate)
    logging = (iteration_log or print_prior) and not return_device
    a_priori = None
    if logging:  # the a-priori state's chi: the kernel's own first integration (nits = 1)
        a_priori = eng.mh_run(theta, y0, nits=1, burnin=0, **kw)["final"][0].cpu().numpy()
    res = eng.mh_run(theta, y0, nits=nits, burnin=0 if iteration_log and not return_device else burnin, **kw)
    kept = max(0, nits - 1 - burnin)
    if return_device:
        return res
    if print_prior:
        print('a priori error', _fmt(a_priori[0]) if W == 1 else a_priori)
        print('iteration; error; acceptance ratio')
    samples = res["samples"].cpu().numpy() if res["samples"].shape[0] > 0 else None
    if iteration_log:
        _print_iterations(a_priori, samples[:, P, :] if samples is not None else np.zeros((0, W)))
        samples = samples[burnin:] if (samples is not None and kept > 0) else None
    th = res["theta"].cpu().numpy()
    yf = res["y0"].cpu().numpy()
    for w, c in enumerate(chains):  # chains end at their last state, as the reference leaves them
        c.set_parameters(**{p: th[j, w] for j, p in enumerate(pnames) if p not in reject})
        c.set_inits(**{s: yf[k, w] for k, s in enumerate(snames)})
    return _posterior_frame(samples if kept > 0 else None, pnames, static_parameters, chains, kept)


def MetropolisHastings(modelframework, nits=1000, burnin=None, static_parameters=set(), print_progress=True):
    """Single-chain drop-in of Samplers.MetropolisHastings (Samplers.py:53-174), on the
    device, with the reference's numpy draws replayed (seed = random_seed).  Prints what
    the reference prints: with ``print_progress`` the a-priori chi and a header, and on
    every iteration ``it exp(-chi)`` (Samplers.py:101-103, :123)."""
    if not burnin:
        burnin = int(nits / 2)
    df = batched_metropolis_hastings([modelframework], nits=nits, burnin=burnin,
                                     static_parameters=static_parameters, rng="replay",
                                     iteration_log=True, print_prior=print_progress)
    return df.drop(columns=["chain#"])
