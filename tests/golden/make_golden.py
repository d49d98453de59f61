"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Run in the build container only (needs /root/reference, read-only):

    python tests/golden/make_golden.py

The reference (SEpapoulis/ODElib @ /root/reference) is imported as a Python package
with two import-time adjustments that do not touch the fitting arithmetic:
  * ``pyDOE2`` (requirements.txt:3) is not installed; ODElib/Statistics/Samplers.py:3
    imports it at module load.  A module object whose ``lhs`` RAISES is registered, so
    the LHS survey path can never feed a fixture (LHS outputs stay unpinned).
  * pandas 2.x removed ``Series.iteritems`` (used at Framework.py:247/276); it is
    aliased to ``Series.items``.
Parameters are passed as ``ODElib.parameter(init_value=...)`` objects because plain
floats crash at Framework.py:452 (value passed positionally as ``stats_gen``).

Outputs (all small; numbers only — no reference source is stored):
  demodata.csv    the demo data file (demo/demodata.csv), input data
  setup.npz       times grid, first-nearest pred_tindex, obs log/logsigma, y0, pnum
  integrate.npz   odeint trajectories [W][T][S], predictions, chi, R², AIC per walker
  mh.npz          seeded Metropolis–Hastings chains (posterior columns)
  mcmc.npz        ModelFramework.MCMC over three listed chain inits (+ report text)
  replicate.npz   data set-up of the replicate-dataframe path (Framework.py:287-298)
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import shutil
import sys
import types
import warnings

import numpy as np
import pandas as pd
import scipy.stats

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def import_reference():
    m = types.ModuleType("pyDOE2")

    def lhs(*a, **k):
        raise NotImplementedError("pyDOE2 is not installed; the LHS path is not pinned by fixtures")

    m.lhs = lhs
    sys.modules["pyDOE2"] = m
    pd.Series.iteritems = pd.Series.items
    sys.path.insert(0, REF)
    import ODElib  # noqa: E402
    return ODElib


# ---- demo models (Demo_InfectionStates.ipynb:60-128) ---------------------------------
def zero_i(y, t, ps):
    mu, phi, beta = ps[0], ps[1], ps[2]
    S, V = y[0], y[1]
    dSdt = mu * S - phi * S * V
    dVdt = beta * phi * S * V - phi * S * V
    return np.array([dSdt, dVdt])


def one_i(y, t, ps):
    mu, phi, beta, lam = ps[0], ps[1], ps[2], ps[3]
    S, I1, V = y[0], y[1], y[2]
    dSdt = mu * S - phi * S * V
    dI1dt = phi * S * V - lam * I1
    dVdt = beta * lam * I1 - phi * S * V
    return np.array([dSdt, dI1dt, dVdt])


def two_i(y, t, ps):
    mu, phi, beta, lam, tau = ps[0], ps[1], ps[2], ps[3], ps[4]
    S, I1, I2, V = y[0], y[1], y[2], y[3]
    dSdt = mu * S - phi * S * V
    dI1dt = phi * S * V - tau * I1
    dI2dt = tau * I1 - lam * I2
    dVdt = beta * lam * I2 - phi * S * V
    return np.array([dSdt, dI1dt, dI2dt, dVdt])


PRIORS = {  # notebook:8575-8578 / twoI cell
    "mu": (scipy.stats.lognorm, {"s": 3, "scale": 1e-8}),
    "phi": (scipy.stats.lognorm, {"s": 3, "scale": 1e-8}),
    "beta": (scipy.stats.lognorm, {"s": 1, "scale": 20}),
    "lam": (scipy.stats.lognorm, {"s": 2, "scale": .1}),
    "tau": (scipy.stats.lognorm, {"s": 2, "scale": 1}),
}
THETA = {  # twoI posterior medians; one_i start from SURVEY §8c
    "zero_i": {"mu": 7.475e-9, "phi": 1.069e-7, "beta": 19.73},
    "one_i": {"mu": 1.2e-8, "phi": 3.5e-8, "beta": 19.4, "lam": 1.8},
    "two_i": {"mu": 7.475e-9, "phi": 1.069e-7, "beta": 19.73, "lam": 1.934, "tau": 2.799},
}
CONFIGS = {
    "zero_i": dict(ode=zero_i, pnames=["mu", "phi", "beta"], snames=["S", "V"], rename={"virus": "V", "host": "S"},
                   sums=None, t_steps=288, extra={}),
    "one_i": dict(ode=one_i, pnames=["mu", "phi", "beta", "lam"], snames=["S", "I1", "V"],
                  rename={"virus": "V", "host": "H"}, sums={"H": ["S", "I1"]}, t_steps=1000, extra={"S": 5236900}),
    "two_i": dict(ode=two_i, pnames=["mu", "phi", "beta", "lam", "tau"], snames=["S", "I1", "I2", "V"],
                  rename={"virus": "V", "host": "H"}, sums={"H": ["S", "I1", "I2"]}, t_steps=1000,
                  extra={"S": 5236900}),
}


def build_model(ODElib, name, theta=None, seed=0, priors=True, extra_params=None):
    cfg = CONFIGS[name]
    df = pd.read_csv(os.path.join(HERE, "demodata.csv")).replace(cfg["rename"])
    th = dict(THETA[name] if theta is None else theta)
    pn = list(cfg["pnames"]) + list((extra_params or {}).keys())
    kw = {}
    for p in pn:
        v = th[p] if p in th else extra_params[p]
        if priors and p in PRIORS:
            d, hp = PRIORS[p]
            kw[p] = ODElib.parameter(stats_gen=d, hyperparameters=dict(hp), init_value=v)
        else:
            kw[p] = ODElib.parameter(init_value=v)
    kw.update(cfg["extra"])
    return ODElib.ModelFramework(ODE=cfg["ode"], parameter_names=pn, state_names=cfg["snames"], dataframe=df,
                                 state_summations=cfg["sums"], t_steps=cfg["t_steps"], random_seed=seed, **kw)


def walker_thetas(name, W=8, seed=0):
    rs = np.random.RandomState(seed)
    base = THETA[name]
    pn = CONFIGS[name]["pnames"]
    z = rs.standard_normal((W, len(pn)))
    return np.array([[base[p] * np.exp(0.05 * z[w, j]) for j, p in enumerate(pn)] for w in range(W)])


def main():
    shutil.copyfile(os.path.join(REF, "demo", "demodata.csv"), os.path.join(HERE, "demodata.csv"))
    ODElib = import_reference()
    warnings.filterwarnings("ignore")
    setup, integ, mh, meta = {}, {}, {}, {}

    for name, cfg in CONFIGS.items():
        m = build_model(ODElib, name)
        setup[f"{name}/times"] = m.times
        setup[f"{name}/y0"] = np.asarray(m.get_inits(), float)
        setup[f"{name}/pnum"] = np.array(m._pnum)
        names = m.get_snames(after_summation=True)
        with_obs = [s for s in names if s in m._pred_tindex]
        meta[f"{name}/obs_names"] = with_obs
        for s in with_obs:
            setup[f"{name}/tidx/{s}"] = np.asarray(m._pred_tindex[s], np.int64)
            setup[f"{name}/obs_log/{s}"] = m._obs_logabundance[s]
            setup[f"{name}/obs_logsigma/{s}"] = m._obs_logsigma[s]
        # batched integrate fixtures: the reference's own integrate() per walker
        TH = walker_thetas(name)
        integ[f"{name}/theta"] = TH
        trajs, preds, chis, rsqs, aics = [], [], [], [], []
        for w in range(TH.shape[0]):
            ps = list(TH[w])
            trajs.append(m.integrate(parameters=(ps,), as_dataframe=False, sum_subpopulations=False))
            d = m.integrate(parameters=(ps,), predict_obs=True, as_dataframe=False)
            preds.append(np.concatenate([d[s] for s in d]))
            c = m.get_chi(d)
            chis.append(float(c))
            rsqs.append(float(m.get_Rsqrd(d)))
            aics.append(float(m.get_AIC(c)))
        integ[f"{name}/traj"] = np.array(trajs)
        integ[f"{name}/pred"] = np.array(preds)
        integ[f"{name}/chi"] = np.array(chis)
        integ[f"{name}/rsq"] = np.array(rsqs)
        integ[f"{name}/aic"] = np.array(aics)

    # ---- Metropolis–Hastings chains (Samplers.py:53-174) ----
    chains = [
        ("one_i_s7", "one_i", 7, 100, [], None),
        ("two_i_s3", "two_i", 3, 60, [], None),
        ("zero_i_s0_static", "zero_i", 0, 50, ["beta"], None),
        ("one_i_V0_s5", "one_i", 5, 40, [], {"V0": 10981000.0}),
    ]
    for key, name, seed, nits, static, extra in chains:
        m = build_model(ODElib, name, seed=seed, extra_params=extra)
        with contextlib.redirect_stdout(io.StringIO()):
            post = ODElib.Statistics.Samplers.MetropolisHastings(m, nits=nits, static_parameters=set(static),
                                                                 print_progress=False)
        meta[f"mh/{key}"] = dict(model=name, seed=seed, nits=nits, static=static, extra=extra or {},
                                 columns=list(post.columns))
        for col in post.columns:
            mh[f"{key}/{col}"] = np.asarray(post[col].to_numpy(), dtype=float)

    # ---- MCMC over listed chain inits (Framework.py:946-1061) ----
    m = build_model(ODElib, "one_i")
    inits = [THETA["one_i"], {k: v * 1.1 for k, v in THETA["one_i"].items()},
             {k: v * 0.9 for k, v in THETA["one_i"].items()}]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        post = m.MCMC(chain_inits=inits, iterations_per_chain=40, cpu_cores=1, print_report=True)
    mcmc = {f"post/{c}": np.asarray(post[c].to_numpy(), dtype=float) for c in post.columns}
    meta["mcmc"] = dict(model="one_i", inits=inits, iterations=40, columns=list(post.columns),
                        report=buf.getvalue().split("Fitting Report")[-1])
    for c in ["mu", "phi", "beta", "lam"]:
        med, std = ODElib.Framework.rawstats(post[c])
        mcmc[f"rawstats/{c}"] = np.array([med, std])

    # ---- replicate-dataframe set-up (Framework.py:287-298) ----
    rs = np.random.RandomState(11)
    rows = []
    for org in ["V", "H"]:
        for t in [0.0, 0.5, 1.0, 2.0, 3.0]:
            for r in range(3):
                rows.append({"organism": org, "time": t, "abundance": float(1e6 * np.exp(rs.normal(0, 0.3))),
                             "replicate": r})
    rdf = pd.DataFrame(rows)
    rdf.to_csv(os.path.join(HERE, "replicate_data.csv"), index=False)
    mr = ODElib.ModelFramework(ODE=one_i, parameter_names=["mu", "phi", "beta", "lam"], state_names=["S", "I1", "V"],
                               dataframe=rdf, state_summations={"H": ["S", "I1"]}, t_steps=100,
                               mu=ODElib.parameter(init_value=1e-8), phi=ODElib.parameter(init_value=1e-7),
                               beta=ODElib.parameter(init_value=20.0), lam=ODElib.parameter(init_value=1.0))
    rep = {"times": mr.times, "y0": np.asarray(mr.get_inits(), float)}
    for s in mr._pred_tindex:
        rep[f"tidx/{s}"] = np.asarray(mr._pred_tindex[s], np.int64)
        rep[f"obs_log/{s}"] = mr._obs_logabundance[s]
        rep[f"obs_logsigma/{s}"] = mr._obs_logsigma[s]

    np.savez_compressed(os.path.join(HERE, "setup.npz"), **setup)
    np.savez_compressed(os.path.join(HERE, "integrate.npz"), **integ)
    np.savez_compressed(os.path.join(HERE, "mh.npz"), **mh)
    np.savez_compressed(os.path.join(HERE, "mcmc.npz"), **mcmc)
    np.savez_compressed(os.path.join(HERE, "replicate.npz"), **rep)
    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
