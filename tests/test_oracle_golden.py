"""Pin the oracle (oracle/cpu_ref.py) against golden vectors produced by the reference
itself (tests/golden/make_golden.py).  Everything here is bit-exact: the oracle issues
the same scipy/numpy calls in the same order as ODElib."""
import contextlib
import io

import numpy as np
import pytest

from helpers import CONFIGS, THETA, demo_df, oracle_model
from oracle import cpu_ref

MODELS = ["zero_i", "one_i", "two_i"]


@pytest.mark.parametrize("name", MODELS)
def test_setup_matches_reference(golden, name):
    cfg = CONFIGS[name]
    df = cpu_ref.format_df(demo_df(cfg["rename"]), cfg["snames"])
    times = cpu_ref.times_grid(max(df["time"]), cfg["t_steps"])
    assert np.array_equal(times, golden.setup[f"{name}/times"])
    ptidx, olog, osig = cpu_ref.fit_setup(df, times)
    for s in golden.meta[f"{name}/obs_names"]:
        assert np.array_equal(ptidx[s], golden.setup[f"{name}/tidx/{s}"])
        assert np.array_equal(olog[s], golden.setup[f"{name}/obs_log/{s}"])
        assert np.array_equal(osig[s], golden.setup[f"{name}/obs_logsigma/{s}"])


@pytest.mark.parametrize("name", MODELS)
def test_integrate_and_fit_stats_bit_exact(golden, name):
    m = oracle_model(name)
    TH = golden.integrate[f"{name}/theta"]
    y0 = [m.istates[s] for s in CONFIGS[name]["snames"]]
    assert np.array_equal(np.asarray(y0, float), golden.setup[f"{name}/y0"])
    for w in range(TH.shape[0]):
        traj = cpu_ref.odeint_traj(CONFIGS[name]["ode"], y0, m.times, TH[w])
        assert np.array_equal(traj, golden.integrate[f"{name}/traj"][w])
        for p, v in zip(m._pnames, TH[w]):
            m.parameters[p].val = np.array(v)
        d = m.integrate_obs()
        assert np.array_equal(np.concatenate([d[s] for s in d]), golden.integrate[f"{name}/pred"][w])
        c = m.get_chi(d)
        assert float(c) == golden.integrate[f"{name}/chi"][w]
        assert float(m.get_Rsqrd(d)) == golden.integrate[f"{name}/rsq"][w]
        assert float(m.get_AIC(c)) == golden.integrate[f"{name}/aic"][w]


def _chain_cfg(golden, key):
    meta = golden.meta[f"mh/{key}"]
    return meta, {c: golden.mh[f"{key}/{c}"] for c in meta["columns"]}


@pytest.mark.parametrize("key", ["one_i_s7", "two_i_s3", "zero_i_s0_static", "one_i_V0_s5"])
def test_metropolis_hastings_bit_exact(golden, key):
    meta, ref = _chain_cfg(golden, key)
    m = oracle_model(meta["model"], seed=meta["seed"], extra_params=meta["extra"] or None)
    out = cpu_ref.metropolis_hastings(m, nits=meta["nits"], static_parameters=meta["static"])
    for c in meta["columns"]:
        assert np.array_equal(out[c], ref[c]), c


def test_mcmc_pooling_and_rawstats(golden):
    meta = golden.meta["mcmc"]
    cols = [c for c in meta["columns"] if c != "chain#"]
    outs = []
    for i, init in enumerate(meta["inits"]):
        m = oracle_model("one_i", theta=init, seed=i)
        o = cpu_ref.metropolis_hastings(m, nits=meta["iterations"], burnin=int(meta["iterations"] / 2))
        o["chain#"] = np.full(len(o["chi"]), i, float)
        outs.append(o)
    for c in cols + ["chain#"]:
        assert np.array_equal(np.concatenate([o[c] for o in outs]), golden.mcmc[f"post/{c}"]), c
    import pandas as pd
    for p in ["mu", "phi", "beta", "lam"]:
        med, std = cpu_ref.rawstats(pd.Series(golden.mcmc[f"post/{p}"]))
        assert np.array_equal([med, std], golden.mcmc[f"rawstats/{p}"])


def test_replicate_dataframe_setup(golden):
    import os

    import pandas as pd
    from helpers import GOLDEN
    rdf = pd.read_csv(os.path.join(GOLDEN, "replicate_data.csv"))
    df = cpu_ref.format_df(rdf, ["S", "I1", "V"])
    times = cpu_ref.times_grid(max(df["time"]), 100)
    assert np.array_equal(times, golden.replicate["times"])
    ptidx, olog, osig = cpu_ref.fit_setup(df, times)
    for s in ptidx:
        assert np.array_equal(ptidx[s], golden.replicate[f"tidx/{s}"])
        assert np.array_equal(olog[s], golden.replicate[f"obs_log/{s}"])
        assert np.array_equal(osig[s], golden.replicate[f"obs_logsigma/{s}"])


def test_masked_chi_semantics():
    """stats.chi drops non-finite terms (stats.py:41); all-masked is np.ma.masked."""
    O = np.array([1., 2., 3., 4.])
    assert float(cpu_ref.chi(O, np.array([1.5, np.nan, np.inf, -np.inf]), np.ones(4))) == 0.125
    assert cpu_ref.chi(O, np.full(4, np.nan), np.ones(4)) is np.ma.masked
    assert float(cpu_ref.chi(O, np.array([1., 2, 3, 4.5]), np.array([0., 1, 1, 1]))) == 0.125
    # an all-masked proposal is never accepted (acc > u is masked -> falsy)
    acc = np.exp(0.0 - cpu_ref.chi(O, np.full(4, np.nan), np.ones(4)))
    assert not bool(acc > 0.5)


def _stiff_fixture():
    import os

    from helpers import GOLDEN
    return dict(np.load(os.path.join(GOLDEN, "stiff.npz")))


@pytest.mark.parametrize("group", ["near", "stiff"])
@pytest.mark.parametrize("tag,tol", [("default", None), ("tight", 1e-13)])
def test_stiff_and_near_posterior_fixtures_bit_exact(group, tag, tol):
    """tests/golden/stiff.npz (make_golden_stiff.py: the reference's integrate + get_chi at
    odeint's default tolerance and at rtol = atol = 1e-13, on 16 near-posterior walkers and
    on stiff draws where LSODA runs BDF): the oracle's odeint call and masked chi reproduce
    them bit for bit."""
    fx = _stiff_fixture()
    m = oracle_model("two_i")
    y0 = [m.istates[s] for s in CONFIGS["two_i"]["snames"]]
    TH = fx[f"{group}/theta"]
    for w in range(TH.shape[0]):
        traj = cpu_ref.odeint_traj(CONFIGS["two_i"]["ode"], y0, m.times, TH[w], rtol=tol, atol=tol)
        assert np.array_equal(traj, fx[f"{group}/{tag}/traj"][w]), w
        for p, v in zip(m._pnames, TH[w]):
            m.parameters[p].val = np.array(v)
        m.integrator = (lambda yy, ps, tr=traj: tr)
        d = m.integrate_obs()
        assert np.array_equal(np.concatenate([d[s] for s in d]), fx[f"{group}/{tag}/pred"][w])
        assert float(m.get_chi(d)) == fx[f"{group}/{tag}/chi"][w]
        assert float(m.get_Rsqrd(d)) == fx[f"{group}/{tag}/rsq"][w]


def _mh_stiff():
    import json
    import os

    from helpers import GOLDEN
    with open(os.path.join(GOLDEN, "mh_stiff.json")) as f:
        meta = json.load(f)
    return meta, dict(np.load(os.path.join(GOLDEN, "mh_stiff.npz")))


@pytest.mark.parametrize("key", ["slow_phi1.5e-5_s11", "slow_phi1.2e-5_s12", "tau1e3_s13"])
def test_stiff_region_metropolis_hastings_bit_exact(key):
    """tests/golden/mh_stiff.npz (make_golden_stiff.py: the reference's MetropolisHastings,
    LSODA for every proposal, from the notebook fit's slow starts phi ~ 1.5e-5 / beta ~ 50
    and from tau = 1e3, 200 iterations, seeded numpy stream): the oracle's chain is the
    reference's, every column bit for bit, and its stored decision margins are the oracle's."""
    meta, fx = _mh_stiff()
    cfg = meta[key]
    ref = cpu_ref.metropolis_hastings(oracle_model(cfg["model"], theta=cfg["theta"], seed=cfg["seed"]),
                                      nits=cfg["nits"])
    for c in cfg["columns"]:
        assert np.array_equal(np.asarray(ref[c], float), fx[f"{key}/{c}"], equal_nan=True), c
    assert np.array_equal(np.asarray(ref["margin"], float), fx[f"{key}/margin"], equal_nan=True)
