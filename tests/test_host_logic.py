"""CPU tests of the product's host-side logic (no GPU): data set-up parity with the
reference, the kernel's constant inputs, device-model binding, the replay RNG streams
and the posterior DataFrame assembly."""
import numpy as np
import pandas as pd
import pytest

from helpers import CONFIGS, THETA, oracle_model, product_model
from odelib_amd import models
from odelib_amd import _native as N
from odelib_amd.rng import legacy_replay_streams
from odelib_amd.Statistics import Samplers, stats
from oracle import cpu_ref

MODELS = ["zero_i", "one_i", "two_i"]


@pytest.mark.parametrize("name", MODELS)
def test_modelframework_setup_matches_reference(golden, name):
    m = product_model(name)
    assert np.array_equal(m.times, golden.setup[f"{name}/times"])
    assert np.array_equal(np.asarray(m.get_inits(), float), golden.setup[f"{name}/y0"])
    assert m._pnum == int(golden.setup[f"{name}/pnum"])
    for s in golden.meta[f"{name}/obs_names"]:
        assert np.array_equal(m._pred_tindex[s], golden.setup[f"{name}/tidx/{s}"])
        assert np.array_equal(m._obs_logabundance[s], golden.setup[f"{name}/obs_log/{s}"])
        assert np.array_equal(m._obs_logsigma[s], golden.setup[f"{name}/obs_logsigma/{s}"])


@pytest.mark.parametrize("name", MODELS)
def test_fit_problem_layout(golden, name):
    """Observation records in get_chi's concatenation order with the summation masks;
    sstot as stats.Rsqrd computes it."""
    m = product_model(name)
    fp = m.fit_problem()
    names = golden.meta[f"{name}/obs_names"]
    assert np.array_equal(fp.obs_tidx, np.concatenate([golden.setup[f"{name}/tidx/{s}"] for s in names]))
    assert np.array_equal(fp.obs_log, np.concatenate([golden.setup[f"{name}/obs_log/{s}"] for s in names]))
    assert np.array_equal(fp.obs_logsigma, np.concatenate([golden.setup[f"{name}/obs_logsigma/{s}"] for s in names]))
    # masks: H = S+I1(+I2) for summed models, else the state itself
    snames = CONFIGS[name]["snames"]
    sums = CONFIGS[name]["sums"] or {}
    for k, s in enumerate(np.repeat(names, [len(golden.setup[f"{name}/tidx/{s}"]) for s in names])):
        group = sums.get(s, [s])
        assert int(fp.obs_mask[k]) == sum(1 << snames.index(g) for g in group)
    sstot = 0
    for s in names:
        o = np.exp(golden.setup[f"{name}/obs_log/{s}"])
        sstot += len(o) * np.var(o)
    assert fp.sstot == sstot
    assert fp.n_states == len(snames) and fp.n_params == len(CONFIGS[name]["pnames"])
    # R² from the kernel's ssres form reproduces stats.Rsqrd on the reference predictions
    for w in range(3):
        pred = golden.integrate[f"{name}/pred"][w]
        ssres = np.nansum((pred - fp.obs_lin) ** 2)
        assert np.isclose(1 - ssres / fp.sstot, golden.integrate[f"{name}/rsq"][w], rtol=1e-12)


def test_model_resolution():
    assert models.resolve(CONFIGS["two_i"]["ode"], 4, 5) == (N.OE_MODEL_TWO_I, 4)
    assert models.resolve(CONFIGS["one_i"]["ode"], 3, 4) == (N.OE_MODEL_ONE_I, 3)
    assert models.resolve(CONFIGS["zero_i"]["ode"], 2, 3) == (N.OE_MODEL_ZERO_I, 2)
    # extra '<state>0' parameters are allowed (P = model P + k)
    assert models.resolve(CONFIGS["one_i"]["ode"], 3, 5) == (N.OE_MODEL_ONE_I, 3)
    # two_i IS chain<4>; explicit selection validates the callable
    assert models.resolve(CONFIGS["two_i"]["ode"], 4, 5, device_model="chain") == (N.OE_MODEL_CHAIN, 4)
    assert models.resolve(models.chain_rhs(20), 20, 5) == (N.OE_MODEL_CHAIN, 20)

    def zero_i_bad_etiquette(y, t, ps):  # notebook's alternative spelling of zero_i
        return np.array([ps[0] * y[0] - ps[1] * y[0] * y[1], ps[2] * ps[1] * y[0] * y[1] - ps[1] * y[0] * y[1]])
    assert models.resolve(zero_i_bad_etiquette, 2, 3) == (N.OE_MODEL_ZERO_I, 2)

    def other(y, t, ps):
        return np.array([-ps[0] * y[0], ps[1] * y[1]])
    with pytest.raises(NotImplementedError):
        models.resolve(other, 2, 3)
    with pytest.raises(ValueError):
        models.resolve(other, 2, 3, device_model="zero_i")


@pytest.mark.parametrize("key", ["one_i_s7", "two_i_s3", "zero_i_s0_static", "one_i_V0_s5"])
def test_replay_streams_reproduce_reference_chain(golden, key):
    """The product's replay stream (rng.py) drives the oracle chain to the reference's
    posterior bit-exactly: same increments, same uniforms, same consumption."""
    meta = golden.meta[f"mh/{key}"]
    m = oracle_model(meta["model"], seed=meta["seed"], extra_params=meta["extra"] or None)
    pn = m.get_pnames()
    walking = {p for p in pn if p not in meta["static"]}
    dists = {p: (m.parameters[p].dist, m.parameters[p].hp) for p in pn}
    oldvals = [[float(m.parameters[p].val) for p in pn]]
    dz, u = legacy_replay_streams([meta["seed"]], meta["nits"], pn, walking, dists, oldvals=oldvals)
    out = cpu_ref.metropolis_hastings(m, nits=meta["nits"], static_parameters=meta["static"],
                                      replay=(dz[:, :, 0], u[:, 0]))
    for c in meta["columns"]:
        assert np.array_equal(out[c], golden.mh[f"{key}/{c}"]), c


def test_posterior_frame_layout(golden):
    """[kept][P+5][W] device block → the reference's MCMC DataFrame layout."""
    meta = golden.meta["mcmc"]
    W, kept, P = 3, 19, 4
    cols = meta["columns"]
    block = np.zeros((kept, P + 5, W))
    for w in range(W):
        rows = golden.mcmc["post/chain#"] == w
        for j, c in enumerate(cols[:-1]):
            block[:, j, w] = golden.mcmc[f"post/{c}"][rows]
    chains = [product_model("one_i") for _ in range(W)]
    df = Samplers._posterior_frame(block, chains[0].get_pnames(), [], chains, kept)
    assert list(df.columns) == cols
    for c in cols:
        assert np.array_equal(df[c].to_numpy(dtype=float), golden.mcmc[f"post/{c}"]), c
    assert df["iteration"].dtype == np.int64
    empty = Samplers._posterior_frame(None, chains[0].get_pnames(), [], chains, 0)
    assert len(empty) == W and empty.drop(columns=["chain#"]).isna().all().all()


def test_lhs_classic_is_stratified():
    np.random.seed(3)
    H = Samplers.lhs_classic(4, 50)
    assert H.shape == (50, 4)
    for j in range(4):
        assert np.array_equal(np.sort(np.floor(H[:, j] * 50)), np.arange(50))


def test_stats_formulas_match_oracle(golden):
    rs = np.random.RandomState(1)
    O, C, S = rs.rand(37) + 1, rs.rand(37) + 1, rs.rand(37) + 0.1
    C[3] = np.nan
    assert stats.chi(O, C, S) == cpu_ref.chi(O, C, S)
    assert stats.AIC(3.5, 5) == cpu_ref.aic(3.5, 5)
    d = {"H": rs.rand(18), "V": rs.rand(19)}
    o = {"H": rs.rand(18), "V": rs.rand(19)}
    assert stats.Rsqrd(d, o) == cpu_ref.rsqrd(d, o)
    assert np.isclose(stats.get_adjusted_rsquared(0.9, 37, 5), 1 - 0.1 * 36 / 31)


def test_parameter_api():
    import scipy.stats
    from odelib_amd import parameter
    p = parameter(stats_gen=scipy.stats.lognorm, hyperparameters={"s": 1, "scale": 2.0}, init_value=3.0)
    assert p.has_distribution() and float(p.val) == 3.0
    q = p.copy()
    assert q.dist is p.dist and float(q.val) == 3.0
    np.random.seed(0)
    p.rwalk()
    np.random.seed(0)
    assert float(p.val) == float(np.exp(np.log(3.0) + np.random.normal(0, 0.05)))
    with pytest.raises(ValueError):
        parameter()
    r = parameter(init_value=2.0)
    assert not r.has_distribution() and r.pdf() == 1.0
    f = parameter(stats_gen=scipy.stats.norm, hyperparameters={}, init_value=1.0)
    f.fit(np.random.RandomState(0).normal(5.0, 2.0, 2000))
    assert abs(f.hp["loc"] - 5.0) < 0.2 and abs(f.hp["scale"] - 2.0) < 0.2


def test_engine_options_do_not_shadow_names():
    m = product_model("two_i", method="rk4", rk4_substeps=2)
    assert m.method == "rk4" and m.rk4_substeps == 2
    fp = m.fit_problem()
    assert fp.method == "rk4" and fp.rk4_substeps == 2
    m2 = m.copy(overwrite={"mu": 1e-8, "S": 5.0})
    assert float(m2.parameters["mu"].val) == 1e-8 and m2.istates["S"] == 5.0
    assert float(m.parameters["mu"].val) == THETA["two_i"]["mu"]
    with pytest.raises(Exception):
        m.set_parameters(nope=1.0)
    with pytest.raises(Exception):
        m.set_inits(nope=1.0)
    assert "Current State Summations" in repr(m)


def test_compute_without_gpu_fails_loudly():
    """No CPU fallback: on a machine without a HIP device every compute call raises."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    m = product_model("two_i")
    with pytest.raises(N.NativeUnavailable):
        m.integrate()
    with pytest.raises(N.NativeUnavailable):
        m.MCMC(chain_inits=[THETA["two_i"]], iterations_per_chain=4, print_report=False)


def test_lazy_mt19937_twist_and_polar_gauss_reproduce_numpy_legacy_stream():
    """The device generator's algorithm (odelib_amd/csrc/numpy_rng.cuh: init_genrand,
    one-word-per-draw lazy twist, 53-bit doubles, polar gauss with its cached value),
    restated in Python, reproduces numpy's legacy RandomState bit for bit."""
    import math

    def stream(seed, n_gauss, n_dbl):
        key = [0] * 624
        s = seed
        for i in range(624):
            key[i] = s
            s = (1812433253 * (s ^ (s >> 30)) + i + 1) & 0xFFFFFFFF
        st = {"pos": 0, "has": False, "g": 0.0}

        def next32():
            i = st["pos"]
            i1 = 0 if i + 1 == 624 else i + 1
            im = i + 397 - 624 if i + 397 >= 624 else i + 397
            y = (key[i] & 0x80000000) | (key[i1] & 0x7FFFFFFF)
            v = key[im] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            key[i] = v
            st["pos"] = i1
            t = v ^ (v >> 11)
            t ^= (t << 7) & 0x9D2C5680
            t ^= (t << 15) & 0xEFC60000
            return t ^ (t >> 18)

        def dbl():
            a, b = next32() >> 5, next32() >> 6
            return (a * 67108864.0 + b) / 9007199254740992.0

        def gauss():
            if st["has"]:
                st["has"] = False
                return st["g"]
            while True:
                x1 = 2.0 * dbl() - 1.0
                x2 = 2.0 * dbl() - 1.0
                r2 = x1 * x1 + x2 * x2
                if r2 < 1.0 and r2 != 0.0:
                    break
            f = math.sqrt(-2.0 * math.log(r2) / r2)
            st["g"], st["has"] = f * x1, True
            return f * x2

        out = []
        for _ in range(n_gauss):
            out.append(gauss())
        for _ in range(n_dbl):
            out.append(dbl())
        return out

    for seed in (0, 1, 7, 123456789):
        rs = np.random.RandomState(seed)
        want = [rs.standard_normal() for _ in range(701)] + [rs.rand() for _ in range(650)]
        got = stream(seed, 701, 650)
        assert got == want, seed


def test_checkpoint_roundtrip(tmp_path):
    from odelib_amd import checkpoint
    rs = np.random.RandomState(3)
    res = {"theta": rs.rand(5, 7), "y0": rs.rand(4, 7), "final": rs.rand(4, 7),
           "status": np.arange(7, dtype=np.int32), "next_it": 12}
    checkpoint.save(tmp_path / "c.npz", res, meta={"seed": 3})
    back = checkpoint.load(tmp_path / "c.npz")
    for k in ("theta", "y0", "final", "status"):
        assert np.array_equal(back[k], res[k])
    assert back["next_it"] == 12 and back["meta"] == {"seed": 3}


def test_engine_binds_torch_current_device(monkeypatch):
    """Without device=, the engine is built on torch's current device (the rank's GPU
    under torchrun after torch.cuda.set_device), not on GPU 0; device= overrides it."""
    import torch
    import odelib_amd.Framework as F

    class FakeEngine:
        def __init__(self, fp, device=0):
            self.device = device
            self.key = None

        def set_problem(self, fp, key=None):
            self.key = key

    monkeypatch.setattr(F, "Engine", FakeEngine)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 3)
    m = product_model("two_i")
    assert m.engine().device == 3
    m.device = 1
    assert m.engine().device == 1


class _RecordingEngine:
    """Engine stand-in recording the uploaded FitProblem (no GPU)."""
    uploads = 0

    def __init__(self, fp, device=0):
        self.device = device
        self.key = None
        self.problem = fp
        _RecordingEngine.uploads += 1

    def set_problem(self, fp, key=None):
        self.problem = fp
        self.key = key
        _RecordingEngine.uploads += 1


def test_copy_with_other_data_does_not_leak_into_original(monkeypatch):
    """copies share one Engine; a copy that resets its dataframe must not
    leave the original integrating on the copy's grid / scoring the copy's data."""
    import odelib_amd.Framework as F
    from helpers import CONFIGS, demo_df
    monkeypatch.setattr(F, "Engine", _RecordingEngine)
    m = product_model("two_i", device=0)
    e0 = m.engine()
    t_orig, obs_orig = e0.problem.times.copy(), e0.problem.obs_log.copy()
    m2 = m.copy()
    assert m2.engine() is e0 and e0.problem.times[-1] == t_orig[-1]  # same data: no re-upload needed
    n_up = _RecordingEngine.uploads
    df2 = demo_df(CONFIGS["two_i"]["rename"])
    df2["time"] = df2["time"] * 2.0
    df2["abundance"] = df2["abundance"] * 3.0
    m2.reset_dataframe(df2)
    assert m2.engine().problem.times[-1] == 2.0 * t_orig[-1]
    # the original re-uploads its own problem before its next use
    p = m.engine().problem
    assert np.array_equal(p.times, t_orig) and np.array_equal(p.obs_log, obs_orig)
    assert np.array_equal(m.times, t_orig)
    assert _RecordingEngine.uploads == n_up + 2
    # and the copy again
    assert m2.engine().problem.times[-1] == 2.0 * t_orig[-1]
    # an unchanged model reuses the upload
    n_up = _RecordingEngine.uploads
    m2.engine()
    assert _RecordingEngine.uploads == n_up


def test_checkpoint_records_rng_state_and_resume_checks_it(tmp_path):
    """a checkpoint carries what the chains' draws depend on, and a resume
    with other draws (rng mode, Philox seed / walker offset, numpy seeds, prior draws,
    replay streams) is refused instead of silently producing a different chain."""
    from odelib_amd import checkpoint
    from odelib_amd.engine import check_resume, rng_record
    rs = np.random.RandomState(3)
    W, P = 6, 5
    base = {"theta": rs.rand(P, W), "y0": rs.rand(4, W), "final": rs.rand(4, W),
            "status": np.zeros(W, np.int32), "next_it": 9}
    walk = np.ones(P, np.uint8)

    # philox
    res = dict(base, rng_state=rng_record("philox", 11, 64, 0.05, walk, 20, nits=9))
    checkpoint.save(tmp_path / "p.npz", res)
    back = checkpoint.load(tmp_path / "p.npz")
    assert back["rng_state"] == res["rng_state"]
    check_resume(back, rng_record("philox", 11, 64, 0.05, walk, 20, nits=30))
    for bad in (rng_record("philox", 12, 64, 0.05, walk, 20), rng_record("philox", 11, 0, 0.05, walk, 20),
                rng_record("numpy", 11, 64, 0.05, walk, 20), rng_record("philox", 11, 64, 0.1, walk, 20),
                rng_record("philox", 11, 64, 0.05, walk, 21)):
        with pytest.raises(ValueError):
            check_resume(back, bad)

    # numpy: seeds and prior draws saved; seeds taken from the checkpoint when omitted
    seeds = np.arange(W) * 3
    res = dict(base, rng_state=rng_record("numpy", 0, 0, 0.05, walk, 20, prior_draws=P), numpy_seeds=seeds)
    checkpoint.save(tmp_path / "n.npz", res)
    back = checkpoint.load(tmp_path / "n.npz")
    assert np.array_equal(check_resume(back, rng_record("numpy", 0, 0, 0.05, walk, 20, prior_draws=P)), seeds)
    with pytest.raises(ValueError):
        check_resume(back, rng_record("numpy", 0, 0, 0.05, walk, 20, prior_draws=P), numpy_seeds=seeds + 1)
    with pytest.raises(ValueError):
        check_resume(back, rng_record("numpy", 0, 0, 0.05, walk, 20, prior_draws=0), numpy_seeds=seeds)

    # replay: rows used by the checkpointed run must be unchanged in the resuming streams
    dz, u = rs.rand(40, P, W), rs.rand(40, W)
    res = dict(base, rng_state=rng_record("replay", 0, 0, 0.05, walk, 20, replay=(dz, u), nits=9))
    checkpoint.save(tmp_path / "r.npz", res)
    back = checkpoint.load(tmp_path / "r.npz")
    ok = rng_record("replay", 0, 0, 0.05, walk, 20, replay=(dz, u), nits=40)
    check_resume(back, dict(ok, _replay=(dz, u)))
    dz2 = dz.copy()
    dz2[7, 1, 2] += 1e-12
    with pytest.raises(ValueError):
        check_resume(back, dict(rng_record("replay", 0, 0, 0.05, walk, 20, replay=(dz2, u), nits=40),
                                _replay=(dz2, u)))
    # a checkpoint without recorded state cannot be verified: refused, unless the caller
    # vouches for the draws, then resumed with a warning
    checkpoint.save(tmp_path / "old.npz", dict(base, numpy_seeds=seeds))
    old = checkpoint.load(tmp_path / "old.npz")
    with pytest.raises(ValueError, match="allow_unverified"):
        check_resume(old, ok)
    with pytest.warns(UserWarning, match="not verified"):
        got = check_resume(old, rng_record("numpy", 0, 0, 0.05, walk, 20, prior_draws=P), allow_unverified=True)
    assert np.array_equal(got, seeds)


def test_resolution_never_binds_a_builtin_by_probing_alone():
    """callables that agree with a built-in on probe points but differ by a
    term switched on by t (dosing after t=3) or by a state threshold must NOT be
    replaced by the built-in; they go to the exact transpiled (hipRTC) path."""
    two_i = CONFIGS["two_i"]["ode"]

    def dosed(y, t, ps):  # forcing only at t > 3 (outside the old probe window)
        mu, phi, beta, lam, tau = ps[0], ps[1], ps[2], ps[3], ps[4]
        S, I1, I2, V = y[0], y[1], y[2], y[3]
        dose = 1e6 if t > 3.5 else 0.0
        return np.array([mu * S - phi * S * V, phi * S * V - tau * I1, tau * I1 - lam * I2,
                         beta * lam * I2 - phi * S * V + dose])

    def threshold(y, t, ps):  # extra decay only for tiny susceptible populations
        mu, phi, beta, lam, tau = ps[0], ps[1], ps[2], ps[3], ps[4]
        S, I1, I2, V = y[0], y[1], y[2], y[3]
        dS = mu * S - phi * S * V - (0.5 * S if S < 1e-3 else 0.0)
        return np.array([dS, phi * S * V - tau * I1, tau * I1 - lam * I2, beta * lam * I2 - phi * S * V])

    def reordered(y, t, ps):  # algebraically two_i, written differently: still the built-in
        S, I1, I2, V = y
        mu, phi, beta, lam, tau = ps
        inf = phi * V * S
        return [S * mu - inf, inf - I1 * tau, -(lam * I2) + tau * I1, (beta * I2) * lam - inf]

    times = np.linspace(0, 6, 1000)
    for f in (dosed, threshold):
        dm = models.resolve_model(f, 4, 5, times=times)
        assert dm.model_id is None and dm.source is not None, f.__name__
        with pytest.raises(NotImplementedError):
            models.resolve(f, 4, 5, times=times)
        with pytest.raises(ValueError):  # an explicit claim is checked exactly too
            models.resolve_model(f, 4, 5, device_model="two_i", times=times)
    assert models.resolve(reordered, 4, 5) == (N.OE_MODEL_TWO_I, 4)
    assert models.resolve_model(two_i, 4, 5).model_id == N.OE_MODEL_TWO_I


def test_untranspilable_callable_is_bound_only_on_request():
    """A callable outside the transpilable subset cannot be proven equal to a built-in:
    it is refused unless the caller names the built-in (numerically checked over the
    whole time grid, with a warning)."""
    import functools

    def _inf(phi, S, V):
        return phi * S * V

    def helper_style(y, t, ps):  # calls a user helper: not transpilable
        mu, phi, beta, lam, tau = ps[0], ps[1], ps[2], ps[3], ps[4]
        S, I1, I2, V = y[0], y[1], y[2], y[3]
        i = _inf(phi, S, V)
        return np.array([mu * S - i, i - tau * I1, tau * I1 - lam * I2, beta * lam * I2 - i])

    with pytest.raises(NotImplementedError, match="cannot be transpiled"):
        models.resolve_model(helper_style, 4, 5)
    with pytest.warns(UserWarning, match="numerically only"):
        assert models.resolve(helper_style, 4, 5, device_model="two_i") == (N.OE_MODEL_TWO_I, 4)
    late = functools.partial(lambda y, t, ps, k: helper_style(y, t, ps) + (k if t > 4 else 0.0), k=1.0)
    with pytest.raises(ValueError):
        models.resolve(late, 4, 5, device_model="two_i", times=np.linspace(0, 6, 100))


def test_worker_order_matches_reference_packaging():
    """fit_survey / explore_equilibriums return rows in the order and with the index the
    reference's cpu_cores workers produce (round-robin packaging, Framework.py:787-798;
    jobs popped last-first and concatenated, :800-816)."""
    from odelib_amd.Framework import _worker_order
    for n, cores in [(10, 1), (10, 3), (7, 4), (3, 5), (0, 2)]:
        worklist = [list() for _ in range(cores)]
        for i in range(n):
            worklist[i % cores].append(i)
        order, index = [], []
        while worklist:
            rows = worklist.pop()
            order += rows
            index += range(len(rows))
        o, ix = _worker_order(n, cores)
        assert list(o) == order and list(ix) == index


def test_sample_lhs_maps_the_hypercube_through_each_prior():
    """Samplers.sample_lhs: one hypercube column per scalar parameter, in dict order,
    through the prior's ppf (Samplers.py:6-51)."""
    import scipy.stats
    from odelib_amd import parameter
    pars = {"a": parameter(stats_gen=scipy.stats.lognorm, hyperparameters={"s": 1, "scale": 2.0}, init_value=1.0),
            "b": parameter(stats_gen=scipy.stats.norm, hyperparameters={"loc": 5, "scale": 0.1}, init_value=5.0)}
    np.random.seed(4)
    df = Samplers.sample_lhs(pars, samples=40)
    np.random.seed(4)
    u = Samplers.lhs_classic(2, 40)
    assert list(df.columns) == ["a", "b"]
    np.testing.assert_array_equal(df["a"].to_numpy(), scipy.stats.lognorm.ppf(u[:, 0], s=1, scale=2.0))
    np.testing.assert_array_equal(df["b"].to_numpy(), scipy.stats.norm.ppf(u[:, 1], loc=5, scale=0.1))
