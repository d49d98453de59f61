"""GPU tests of user right-hand sides compiled at run time with hipRTC."""
import numpy as np
import pandas as pd
import pytest

from helpers import CONFIGS, THETA, demo_df, product_model, walker_thetas
from oracle import cpu_ref
from test_transpile import chain_loop, sat_infection, vec_chain

pytestmark = pytest.mark.gpu

ONE_I_FMA_BODY = """
    const double mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3];
    const double S = y[0], I1 = y[1], V = y[2];
    const double inf = phi * S * V;
    dy[0] = fma(mu, S, -inf);
    dy[1] = fma(-lam, I1, inf);
    dy[2] = fma(beta * lam, I1, -inf);
"""


def _run(m, theta):
    W = theta.shape[1]
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    out = m.engine().integrate(y0, theta)
    return y0, {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("method", ["rk4", "dopri5"])
def test_rtc_copy_of_builtin_is_bitwise_identical(method):
    """C source identical to the built-in one_i RHS, compiled at run time: same kernel
    templates, same bits as the ahead-of-time library."""
    theta = walker_thetas("one_i", 130).T.copy()
    a = product_model("one_i", method=method)
    b = product_model("one_i", method=method, device_rhs=ONE_I_FMA_BODY)
    _, ra = _run(a, theta)
    _, rb = _run(b, theta)
    for k in ("traj", "chi", "ssres", "status"):
        assert np.array_equal(ra[k], rb[k]), k


@pytest.mark.parametrize("method", ["rk4", "dopri5"])
def test_transpiled_demo_model_matches_builtin_and_odeint(method):
    theta = walker_thetas("two_i", 100).T.copy()
    a = product_model("two_i", method=method)
    b = product_model("two_i", method=method, device_model="rtc")
    y0, ra = _run(a, theta)
    _, rb = _run(b, theta)
    # Python operand order vs fused form: a few ulps per RHS evaluation
    np.testing.assert_allclose(rb["traj"], ra["traj"], rtol=1e-10, atol=1e-6)
    for w in (0, 63, 99):
        tight = cpu_ref.odeint_traj(CONFIGS["two_i"]["ode"], y0[:, w], a.times, theta[:, w], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(rb["traj"][:, :, w], tight, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("method,substeps", [("rk4", 2), ("dopri5", 1)])
def test_non_builtin_model_vs_odeint(method, substeps):
    """A model that is not compiled in (saturating infection, logistic host, time
    forcing): transpiled from Python, compiled with hipRTC, fitted to the demo data."""
    from odelib_amd import ModelFramework, parameter
    df = demo_df({"virus": "V", "host": "S"})
    th = {"mu": 0.5, "phi": 2e-7, "beta": 20.0, "delta": 0.3}
    m = ModelFramework(ODE=sat_infection, parameter_names=list(th), state_names=["S", "V"], dataframe=df,
                       method=method, rk4_substeps=substeps,
                       **{k: parameter(init_value=v) for k, v in th.items()})
    fp = m.fit_problem()
    assert fp.custom_source is not None
    W = 70
    theta = np.array(list(th.values()))[:, None] * np.exp(0.05 * np.random.RandomState(4).standard_normal((4, W)))
    y0, out = _run(m, theta)
    for w in (0, 35, 69):
        tight = cpu_ref.odeint_traj(sat_infection, y0[:, w], m.times, theta[:, w], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(out["traj"][:, :, w], tight, rtol=1e-6, atol=1e-6)
        # fused in-kernel chi == the reference's get_chi on the same trajectory
        tr = out["traj"][:, :, w]
        d = {"S": tr[m._pred_tindex["S"], 0], "V": tr[m._pred_tindex["V"], 1]}
        np.testing.assert_allclose(out["chi"][w], float(m.get_chi(d)), rtol=1e-12)
    # the drop-in single-walker path and MCMC run on the compiled RHS too
    traj = m.integrate(as_dataframe=False)
    assert traj.shape == (len(m.times), 2)
    post = m.MCMC(chain_inits=[th, th], iterations_per_chain=10, print_report=False)
    assert len(post) == 2 * 4 and np.isfinite(post["chi"]).all()


def test_transpiled_mh_matches_builtin_mh():
    theta = np.repeat(np.array(list(THETA["two_i"].values()))[:, None], 96, axis=1)
    a = product_model("two_i", method="rk4")
    b = product_model("two_i", method="rk4", device_model="rtc")
    y0 = np.repeat(np.asarray(a.get_inits(), float)[:, None], 96, axis=1)
    walk = np.ones(5, np.uint8)
    ra = a.engine().mh_run(theta, y0, nits=20, burnin=8, walk_mask=walk, rng="philox", seed=9)
    rb = b.engine().mh_run(theta, y0, nits=20, burnin=8, walk_mask=walk, rng="philox", seed=9)
    np.testing.assert_allclose(rb["samples"].cpu().numpy(), ra["samples"].cpu().numpy(), rtol=1e-9)


@pytest.mark.parametrize("ode", [chain_loop, vec_chain], ids=["loop", "slices"])
@pytest.mark.parametrize("method", ["rk4", "dopri5"])
def test_loop_written_chain_model_via_rtc(method, ode):
    """The chain model written with a loop and a local array, forced onto the hipRTC
    path (device_model='rtc'): same trajectories as the compiled Chain<12> up to the
    fused vs separate multiply-subtract rounding, and within 1e-6 of tight odeint.
    Without the force, the callable resolves to the compiled chain by probing."""
    from helpers import chain_problem
    n = 12
    a = chain_problem(n, method=method)
    b = chain_problem(n, method=method, ode=ode, device_model="rtc")
    assert b.fit_problem().custom_source is not None
    assert chain_problem(n, method=method, ode=ode, device_model=None).fit_problem().custom_source is None
    theta = walker_thetas("two_i", 96).T.copy()
    y0, ra = _run(a, theta)
    _, rb = _run(b, theta)
    np.testing.assert_allclose(rb["traj"], ra["traj"], rtol=1e-9, atol=1e-4)
    np.testing.assert_allclose(rb["chi"], ra["chi"], rtol=1e-9)
    for w in (0, 50, 95):
        tight = cpu_ref.odeint_traj(ode, y0[:, w], a.times, theta[:, w], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(rb["traj"][:, :, w], tight, rtol=1e-6, atol=1e-4)


@pytest.mark.parametrize("method", ["rk4", "auto"])
def test_rtc_model_speculative_mh(method):
    """A hipRTC user model (one_i transpiled from the Python callable, forced onto the
    run-time path) runs the speculative MH rounds too (k_mh_tree from the module,
    k_mh_resolve from the library): RK4 bitwise its sequential chain, 'auto' (the module's
    stiff part: the body instantiated with dual numbers) the same decisions; both within
    the transpiled operand order's rounding of the ahead-of-time model's chains."""
    a = product_model("one_i", method=method)
    b = product_model("one_i", method=method, device_model="rtc")
    W = 12
    theta = walker_thetas("one_i", W).T.copy()
    y0 = np.repeat(np.asarray(a.get_inits(), float)[:, None], W, axis=1)
    walk = np.ones(theta.shape[0], np.uint8)
    kw = dict(nits=30, burnin=10, walk_mask=walk, rng="philox", seed=4)
    eb = b.engine()
    seq = eb.mh_run(theta, y0, **kw)
    spec = eb.mh_run(theta, y0, speculate="auto", **kw)
    assert eb.last_mh_depth() >= 8
    aot = a.engine().mh_run(theta, y0, speculate="auto", **kw)
    P = theta.shape[0]
    s_seq, s_spec, s_aot = (r["samples"].cpu().numpy() for r in (seq, spec, aot))
    if method == "rk4":
        assert np.array_equal(s_spec, s_seq)
    else:
        assert np.array_equal(s_spec[:, :P], s_seq[:, :P])
        np.testing.assert_allclose(s_spec, s_seq, rtol=1e-7)
    np.testing.assert_allclose(s_spec, s_aot, rtol=1e-7)
