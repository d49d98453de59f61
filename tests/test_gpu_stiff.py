"""GPU parity of the stiff methods (OE_METHOD_AUTO: DOPRI5 + stiffness test, evicted lanes
continue with BDF (S <= 8) or restart with RODAS (wider); OE_METHOD_BDF; OE_METHOD_ROSENBROCK)
through the C-ABI:

* same algorithm (oracle/rk_ref.c): trajectories and status bitwise, chi rtol 1e-12
  (ocml vs libm log), on waves that mix the demo draws with stiff ones;
* reference algorithm: within 1e-6·|y| + 1e-6 of a tight implicit solution (scipy Radau,
  rtol 1e-13) where odeint's LSODA would have switched to BDF (Framework.py:656);
* with no stiff walker 'auto' is DOPRI5 bit for bit (C2 size);
* MH with 'auto' against the C restatement; a user model compiled with hipRTC gets the
  stiff methods (its Jacobian from dual numbers, including ∂f/∂t of a time forcing).
"""
import numpy as np
import pytest
from scipy.integrate import solve_ivp

from helpers import CONFIGS, THETA, demo_df, product_model, walker_thetas
from oracle import rk_ref
from test_stiff_oracle import STIFF_SETS
from test_transpile import sat_infection

pytestmark = pytest.mark.gpu

TWO_I_TEMPLATED_BODY = """
    const R mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3], tau = ps[4];
    const R Sv = y[0], I1 = y[1], I2 = y[2], V = y[3];
    const R inf = phi * Sv * V;
    dy[0] = fma(mu, Sv, -inf);
    dy[1] = fma(-tau, I1, inf);
    dy[2] = fma(tau, I1, -(lam * I2));
    dy[3] = fma(beta * lam, I2, -inf);
"""


def _mixed_thetas(name, W, stiff_lanes, seed=0):
    """demo draws with a few lanes replaced by stiff parameter sets (two_i: tau/lam)"""
    theta = walker_thetas(name, W, seed).T.copy()
    sets = [v for k, v in STIFF_SETS.items() if k != "nonstiff"]
    for j, w in enumerate(stiff_lanes):
        theta[:, w] = sets[j % len(sets)][:theta.shape[0]]
    return theta


def _run(m, theta, trajectory=True):
    W = theta.shape[1]
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    out = m.engine().integrate(y0, theta, trajectory=trajectory)
    return y0, {k: (v.cpu().numpy() if v is not None else None) for k, v in out.items()}


def _radau(ode, y0, times, th):
    sol = solve_ivp(lambda t, y: ode(y, t, th), (times[0], times[-1]), y0, method="Radau", t_eval=times,
                    rtol=1e-13, atol=1e-10)
    assert sol.success
    return sol.y.T


@pytest.mark.parametrize("method", ["auto", "rosenbrock", "bdf"])
@pytest.mark.parametrize("W,stiff", [(1, [0]), (70, [3, 64, 69]), (200, [0, 1, 2, 130, 199])])
def test_stiff_methods_bitwise_vs_c_restatement(method, W, stiff):
    m = product_model("two_i", method=method)
    theta = _mixed_thetas("two_i", W, stiff)
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert np.array_equal(out["traj"], ref["traj"], equal_nan=True)
    np.testing.assert_allclose(out["chi"], ref["chi"], rtol=1e-12)
    np.testing.assert_allclose(out["ssres"], ref["ssres"], rtol=1e-12)
    assert np.array_equal(out["status"], ref["status"])
    if method == "auto":
        assert sorted(np.nonzero(out["status"] & 8)[0].tolist()) == sorted(stiff)
    assert not (out["status"] & 4).any()


def test_auto_moderately_stiff_walkers_bitwise_vs_c_restatement():
    """The weighted, cost-gated stiffness test (tau = 1e3 .. 3e4 lanes in demo waves): the
    same walkers flagged as the C restatement — every one of them, the hand-over to BDF
    being cheap — handed over at their own times, trajectories bitwise."""
    m = product_model("two_i", method="auto")
    W = 130
    theta = walker_thetas("two_i", W).T.copy()
    lanes = {5: 1e3, 40: 3e3, 64: 1e4, 100: 3e4, 129: 1e4}
    for w, tau in lanes.items():
        theta[4, w] = tau
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert np.array_equal(out["traj"], ref["traj"], equal_nan=True)
    assert np.array_equal(out["status"], ref["status"])
    np.testing.assert_allclose(out["chi"], ref["chi"], rtol=1e-12)
    assert sorted(np.nonzero(out["status"] & 8)[0].tolist()) == [5, 40, 64, 100, 129]


@pytest.mark.parametrize("W,trajectory", [(600, True), (600, False), (8192, True)])
def test_auto_hand_over_queue_many_walkers_bitwise(W, trajectory):
    """'auto' hands stiff walkers through the hand-over queue (ode_kernels.cuh HandQ: the DOPRI5
    kernel publishes each at its eviction point, the BDF kernel beside it takes them): many
    handed walkers in one workgroup (150 of block 1's 256),
    handed at different times (tau from 1e3 to 1e5), one in the partial last block, blocks
    without any — the same bits as the C restatement, whatever wave ran a walker's BDF pass;
    at 600 walkers the BDF kernel runs beside the DOPRI5 kernel, at 8 192 after it."""
    m = product_model("two_i", method="auto")
    theta = walker_thetas("two_i", W, seed=5).T.copy()
    rs = np.random.RandomState(11)
    lanes = sorted(set(rs.choice(np.arange(256, 512), 150, replace=False).tolist()) | {3, W - 1})
    taus = (1e3, 3e3, 1e4, 1e5)
    for j, w in enumerate(lanes):
        theta[4, w] = taus[j % len(taus)]
    y0, out = _run(m, theta, trajectory=trajectory)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta, trajectory=trajectory)
    if trajectory:
        assert np.array_equal(out["traj"], ref["traj"], equal_nan=True)
    assert np.array_equal(out["status"], ref["status"])
    np.testing.assert_allclose(out["chi"], ref["chi"], rtol=1e-12)
    np.testing.assert_allclose(out["ssres"], ref["ssres"], rtol=1e-12)
    assert sorted(np.nonzero(out["status"] & 8)[0].tolist()) == lanes


@pytest.mark.parametrize("name,W", [("one_i", 300), ("one_i", 5000), ("chain4", 300)])
def test_auto_hand_over_queue_other_models_bitwise(name, W):
    """The hand-over queue's kernels for the other models it serves (S <= 4): one_i (3 states)
    with a fast infected-cell decay (lam = 1e4) and the synthetic 4-state chain (tau = 1e4) in
    a few lanes — beside the DOPRI5 kernel (300 walkers) and after it (5 000) — the C
    restatement's bits, trajectories included."""
    from helpers import chain_problem
    if name == "chain4":
        m = chain_problem(4, method="auto")
        theta = walker_thetas("two_i", W, seed=2).T.copy()
        k = 4
    else:
        m = product_model(name, method="auto")
        theta = walker_thetas(name, W, seed=2).T.copy()
        k = 3
    lanes = [1, 64, 200, W - 1]
    theta[k, lanes] = 1e4
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert np.array_equal(out["traj"], ref["traj"], equal_nan=True)
    assert np.array_equal(out["status"], ref["status"])
    np.testing.assert_allclose(out["chi"], ref["chi"], rtol=1e-12)
    assert np.all(out["status"][lanes] & 8), out["status"][lanes]


def test_auto_hand_over_queue_more_handed_walkers_than_one_lane_each():
    """81 920 walkers, every one stiff (tau = 1e3): more handed walkers than the BDF kernel
    has lanes in one round of its waves (65 536 at one 4-wave workgroup per CU), so the grid
    must cover every slot.  Every walker comes back from the BDF pass (status STIFF, finite
    chi), and three aligned lockstep groups — first, middle, last — are the C restatement's
    bits (a DOPRI5 walker's bits depend on its 64-walker group only)."""
    W = 81920
    m = product_model("two_i", method="auto")
    theta = walker_thetas("two_i", W, seed=9).T.copy()
    theta[4, :] = 1e3
    y0, out = _run(m, theta, trajectory=False)
    assert np.all(out["status"] & 8), np.count_nonzero((out["status"] & 8) == 0)
    assert np.all(np.isfinite(out["chi"]))
    for a in (0, W // 2, W - 64):
        sl = slice(a, a + 64)
        ref = rk_ref.integrate(m.fit_problem(), y0[:, sl], np.ascontiguousarray(theta[:, sl]), trajectory=False)
        assert np.array_equal(out["status"][sl], ref["status"]), a
        np.testing.assert_allclose(out["chi"][sl], ref["chi"], rtol=1e-12, err_msg=str(a))
        np.testing.assert_allclose(out["ssres"][sl], ref["ssres"], rtol=1e-12, err_msg=str(a))


@pytest.mark.parametrize("method", ["rosenbrock", "bdf"])
@pytest.mark.parametrize("name", ["zero_i", "one_i"])
def test_rosenbrock_other_models_bitwise(name, method):
    m = product_model(name, method=method)
    theta = walker_thetas(name, 66).T.copy()
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert np.array_equal(out["traj"], ref["traj"])
    assert np.array_equal(out["status"], ref["status"])


@pytest.mark.parametrize("method", ["auto", "rosenbrock", "bdf"])
def test_stiff_walkers_vs_tight_implicit_solution(method):
    m = product_model("two_i", method=method)
    W = 64
    lanes = [5, 21, 40]
    theta = _mixed_thetas("two_i", W, lanes)
    y0, out = _run(m, theta)
    for w in lanes + [0, 63]:
        ref = _radau(CONFIGS["two_i"]["ode"], y0[:, w], m.times, theta[:, w])
        np.testing.assert_allclose(out["traj"][:, :, w], ref, rtol=1e-6, atol=1e-6, err_msg=str(w))


def test_auto_is_dopri5_without_stiff_walkers_at_c2_size():
    """65 536 demo draws: nothing is evicted, so 'auto' gives DOPRI5's bits."""
    W = 65536
    theta = walker_thetas("two_i", W, seed=3).T.copy()
    a = product_model("two_i", method="dopri5")
    b = product_model("two_i", method="auto")
    _, ra = _run(a, theta)
    _, rb = _run(b, theta)
    for k in ("traj", "chi", "ssres", "status"):
        assert np.array_equal(ra[k], rb[k]), k


def test_auto_chi_only_mode_equals_trajectory_mode():
    """MCMC mode (no trajectory) and trajectory mode step identically (steps end on every
    grid time either way), so the fused chi agrees bitwise."""
    m = product_model("two_i", method="auto")
    theta = _mixed_thetas("two_i", 130, [7, 100])
    _, a = _run(m, theta, trajectory=True)
    _, b = _run(m, theta, trajectory=False)
    for k in ("chi", "ssres", "status"):
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("method", ["auto", "rosenbrock", "bdf"])
def test_mh_stiff_methods_vs_c_restatement(method):
    """Philox MH chains where some proposals are stiff: the device chain equals the C
    restatement's (rtol 1e-8 as for DOPRI5 MH: ocml vs libm exp/log in the proposal)."""
    W = 8 if method == "rosenbrock" else 128  # (the C restatement of RODAS for every chain is slow)
    m = product_model("two_i", method=method)
    theta = _mixed_thetas("two_i", W, [1] if method == "rosenbrock" else [1, 64, 65, 127])
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    walk = np.ones(5, np.uint8)
    dev = m.engine().mh_run(theta, y0, nits=12, burnin=4, walk_mask=walk, rng="philox", seed=11)
    ref = rk_ref.mh_run(m.fit_problem(), theta, y0, 12, 4, walk, rng="philox", seed=11)
    np.testing.assert_allclose(dev["samples"].cpu().numpy(), ref["samples"], rtol=1e-8)


@pytest.mark.parametrize("method", ["auto", "bdf"])
def test_rtc_templated_body_gets_stiff_methods_bitwise(method):
    """A user C body written over the scalar type R compiles for dual numbers: the RTC
    module has the stiff methods and reproduces the built-in kernels bitwise."""
    theta = _mixed_thetas("two_i", 96, [2, 50])
    a = product_model("two_i", method=method)
    b = product_model("two_i", method=method, device_rhs=TWO_I_TEMPLATED_BODY)
    _, ra = _run(a, theta)
    _, rb = _run(b, theta)
    for k in ("traj", "chi", "ssres", "status"):
        assert np.array_equal(ra[k], rb[k], equal_nan=True), k


def test_rtc_double_only_body_reports_no_stiff_methods():
    """A body with `double` temporaries has no dual-number Jacobian: RK4/DOPRI5 work,
    the stiff methods are refused with OE_ERR_UNSUPPORTED (never silently replaced)."""
    from test_gpu_rtc import ONE_I_FMA_BODY
    m = product_model("one_i", method="dopri5", device_rhs=ONE_I_FMA_BODY)
    _run(m, walker_thetas("one_i", 8).T.copy())
    m2 = product_model("one_i", method="auto", device_rhs=ONE_I_FMA_BODY)
    with pytest.raises(Exception, match="dual numbers"):
        _run(m2, walker_thetas("one_i", 8).T.copy())


def test_transpiled_time_forced_model_with_stiff_methods():
    """A transpiled non-built-in model with a time forcing (∂f/∂t from the dual t):
    'rosenbrock' and 'auto' within tolerance of the tight implicit solution."""
    from odelib_amd import ModelFramework, parameter
    df = demo_df({"virus": "V", "host": "S"})
    th = {"mu": 0.5, "phi": 2e-7, "beta": 20.0, "delta": 0.3}
    W = 70
    theta = np.array(list(th.values()))[:, None] * np.exp(0.05 * np.random.RandomState(4).standard_normal((4, W)))
    theta[3, 9] = 1e5  # a stiff virus decay in one lane
    for method in ("rosenbrock", "auto"):
        m = ModelFramework(ODE=sat_infection, parameter_names=list(th), state_names=["S", "V"], dataframe=df,
                           method=method, **{k: parameter(init_value=v) for k, v in th.items()})
        y0, out = _run(m, theta)
        for w in (0, 9, 69):
            ref = _radau(sat_infection, y0[:, w], m.times, theta[:, w])
            np.testing.assert_allclose(out["traj"][:, :, w], ref, rtol=1e-6, atol=1e-6, err_msg=f"{method} {w}")


@pytest.mark.parametrize("method", ["rosenbrock", "auto"])
def test_transpiled_power_of_zero_state_has_finite_jacobian(method):
    """y**p with y starting at 0 (hill_power: X(0) = 0, exponent n a parameter): the
    dual-number Jacobian must not carry 0·log(0) = NaN from the parameter's zero tangent
    into the row — every walker finishes within tolerance of the tight implicit solution
    (before the fix every Rosenbrock step was rejected and the walkers were evicted)."""
    from odelib_amd import ModelFramework, parameter
    from test_transpile import hill_power
    th = {"k": 2.0, "K": 1.5, "n": 2.5, "d": 0.7}
    W = 70
    theta = np.array(list(th.values()))[:, None] * np.exp(0.05 * np.random.RandomState(6).standard_normal((4, W)))
    theta[3, [9, 64]] = 1e5  # stiff decay lanes (the stiff path under 'auto')
    m = ModelFramework(ODE=hill_power, parameter_names=list(th), state_names=["X", "Y"], t_end=3.0, t_steps=300,
                       method=method, **{k: parameter(init_value=v) for k, v in th.items()})
    assert m.fit_problem().custom_source is not None
    y0, out = _run(m, theta)
    assert not (out["status"] & 5).any(), out["status"]
    if method == "auto":
        assert sorted(np.nonzero(out["status"] & 8)[0].tolist()) == [9, 64]
    for w in (0, 9, 64, 69):
        ref = _radau(hill_power, y0[:, w], m.times, theta[:, w])
        np.testing.assert_allclose(out["traj"][:, :, w], ref, rtol=1e-6, atol=1e-6, err_msg=f"{method} {w}")


def test_transpiled_wide_model_auto_uses_stiff_wave_kernel():
    """A 12-state user model (loop-written chain, forced onto hipRTC) under 'auto': its
    stiff lanes go through the hipRTC module's k_stiff_wave (one wave per stiff walker)
    and agree with the built-in Chain<12> (same algorithm; the fused vs separate
    multiply-subtract of the RHS moves the last bits)."""
    from helpers import chain_problem
    from test_transpile import chain_loop
    a = chain_problem(12, method="auto")
    b = chain_problem(12, method="auto", ode=chain_loop, device_model="rtc")
    assert b.fit_problem().custom_source is not None
    theta = _mixed_thetas("two_i", 70, [3, 64])
    _, ra = _run(a, theta)
    _, rb = _run(b, theta)
    assert np.array_equal(ra["status"], rb["status"])
    assert sorted(np.nonzero(rb["status"] & 8)[0].tolist()) == [3, 64]
    np.testing.assert_allclose(rb["traj"], ra["traj"], rtol=1e-6, atol=1e-4)
    np.testing.assert_allclose(rb["chi"], ra["chi"], rtol=1e-6)


def test_default_method_is_auto_with_dopri5_fallback():
    """The drop-in default is 'auto' (LSODA-like) up to 8 states.  Wider models default
    to 'dopri5' (their stiff path keeps the matrices in private memory, ~20x slower per
    stiff walker) but take an explicit method='auto'; a C body without a dual-number
    instantiation falls back to 'dopri5' by default and refuses an explicit 'auto'."""
    from helpers import chain_problem
    from test_gpu_rtc import ONE_I_FMA_BODY
    from odelib_amd import _native as N
    m = product_model("two_i")
    assert m.method == "auto" and m.engine().problem.method == "auto"
    d = chain_problem(10, method="auto")
    d._method_default = True  # as if no method had been given
    assert d.engine().problem.method == "dopri5"
    assert chain_problem(10, method="auto").engine().problem.method == "auto"
    d = product_model("one_i", method="auto", device_rhs=ONE_I_FMA_BODY)
    d._method_default = True
    assert d.engine().problem.method == "dopri5"
    e = product_model("one_i", method="auto", device_rhs=ONE_I_FMA_BODY)
    with pytest.raises(N.NativeUnsupported):
        e.engine()


@pytest.mark.parametrize("n,method", [(6, "auto"), (10, "auto"), (20, "auto"), (6, "rosenbrock"), (10, "rosenbrock"),
                                      (20, "rosenbrock"), (6, "bdf"), (8, "bdf")])
def test_wide_chain_stiff_methods_bitwise_vs_c_restatement(n, method):
    """S = 6: the register path (wave-shared step); S = 10, 20: one wave per stiff
    walker (k_stiff_wave, the walker's own step; the C restatement redoes wide walkers one
    per group) — trajectories and status bitwise equal to the C restatement on a ragged
    two-wave ensemble with stiff lanes in both waves."""
    from helpers import chain_problem
    m = chain_problem(n, method=method)
    W, stiff = (70, [3, 64, 69]) if method in ("auto", "bdf") else (6, [1, 4])
    theta = _mixed_thetas("two_i", W, stiff)
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert np.array_equal(out["traj"], ref["traj"], equal_nan=True)
    np.testing.assert_allclose(out["chi"], ref["chi"], rtol=1e-12)
    assert np.array_equal(out["status"], ref["status"])
    if method == "auto":
        assert sorted(np.nonzero(out["status"] & 8)[0].tolist()) == sorted(stiff)
    assert not (out["status"] & 4).any()


def test_wide_chain_mh_auto_vs_c_restatement():
    """MH with 'auto' on a 10-state chain (in-kernel redo, matrices in private memory),
    stiff proposals in both waves."""
    from helpers import chain_problem
    W = 70
    m = chain_problem(10, method="auto")
    theta = _mixed_thetas("two_i", W, [2, 66])
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    walk = np.ones(5, np.uint8)
    dev = m.engine().mh_run(theta, y0, nits=6, burnin=2, walk_mask=walk, rng="philox", seed=5)
    ref = rk_ref.mh_run(m.fit_problem(), theta, y0, 6, 2, walk, rng="philox", seed=5)
    np.testing.assert_allclose(dev["samples"].cpu().numpy(), ref["samples"], rtol=1e-8)


def test_auto_demo_fit_region_bitwise_and_vs_tight_solution():
    """The draws that made the notebook's fit slow (phi ~ 1e-4: the host is infected within
    ~1e-3 time units and its relative decay then sets DOPRI5 to crawl at h|lambda| ~ 3.3
    for the rest of the span; tau ~ 1e2 .. 2e2, beta up to 4e2) in waves of demo draws:
    bitwise the C restatement (lanes handed to BDF at their own times), within 1e-6 of
    tight Radau."""
    m = product_model("two_i", method="auto")
    W = 130
    theta = walker_thetas("two_i", W, seed=9).T.copy()
    theta[1, [2, 70, 129]] = [1.06e-4, 8.8e-5, 5.0e-6]
    theta[4, [10, 71]] = [99.0, 218.0]
    theta[2, 40] = 415.0
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert np.array_equal(out["traj"], ref["traj"], equal_nan=True)
    assert np.array_equal(out["status"], ref["status"])
    np.testing.assert_allclose(out["chi"], ref["chi"], rtol=1e-12)
    assert {2, 70} <= set(np.nonzero(out["status"] & 8)[0].tolist())
    for w in (2, 10, 40, 70, 71, 129, 0):
        r = _radau(CONFIGS["two_i"]["ode"], y0[:, w], m.times, theta[:, w])
        np.testing.assert_allclose(out["traj"][:, :, w], r, rtol=1e-6, atol=1e-6, err_msg=str(w))


def test_bdf_refused_above_register_path():
    """'bdf' is the register path's (n_states <= 8): a wider model is refused, not replaced."""
    from helpers import chain_problem
    from odelib_amd import _native as N
    with pytest.raises(N.NativeUnsupported):
        chain_problem(10, method="bdf").engine()
    chain_problem(6, method="bdf").engine()


@pytest.mark.parametrize("method", ["rk4", "dopri5", "auto", "bdf", "rosenbrock"])
def test_two_point_time_grid_bitwise(method):
    """The smallest grid the ABI takes (T = 2: the initial state and one output row; every
    look-ahead load then reads the +inf sentinels): every method, stiff lanes included, the C
    restatement's bits."""
    from helpers import chain_problem
    m = chain_problem(4, method=method, T=2)
    W = 70
    theta = _mixed_thetas("two_i", W, [3, 64, 69])
    y0, out = _run(m, theta)
    assert out["traj"].shape[0] == 2
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert np.array_equal(out["traj"], ref["traj"], equal_nan=True)
    assert np.array_equal(out["status"], ref["status"])
    np.testing.assert_allclose(out["chi"], ref["chi"], rtol=1e-12)
