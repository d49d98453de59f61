"""GPU parity: the HIP kernels (through the C-ABI) against the oracle.

* same algorithm  (oracle/rk_ref.c): RK4 and DOPRI5 trajectories bitwise (the DOPRI5
  step controller uses no libm/ocml transcendental); chi / R² residual rtol 1e-12
  (ocml vs libm log);
* reference algorithm (scipy odeint, tight rtol=atol=1e-13): |Δ| <= 1e-6·|y| + 1e-6
  for the 4-state model (BASELINE.json: "trajectories within rtol=1e-6 of scipy"),
  atol 1e-4 for the 20-state chain (downstream compartments start at 0);
* the reference itself (golden vectors, odeint at its default 1.49e-8 tolerances,
  itself ~1e-6 accurate): rtol 5e-6 on trajectories and fit statistics;
* Metropolis–Hastings: replay mode reproduces the reference chains wherever the
  acceptance margin |acc - u| exceeds 1e-3 (the reference's own integration error
  moves acc by ~1e-5).
"""
import numpy as np
import pandas as pd
import pytest

from helpers import CONFIGS, THETA, chain_problem, oracle_model, product_model, walker_thetas
from odelib_amd import _native as N
from odelib_amd.models import chain_rhs
from oracle import cpu_ref, rk_ref

pytestmark = pytest.mark.gpu

RHS = {"zero_i": CONFIGS["zero_i"]["ode"], "one_i": CONFIGS["one_i"]["ode"], "two_i": CONFIGS["two_i"]["ode"]}


def _model(spec, method="rk4", substeps=1, **kw):
    if spec.startswith("chain"):
        return chain_problem(int(spec[5:]), method=method, substeps=substeps, **kw)
    return product_model(spec, method=method, rk4_substeps=substeps, **kw)


def _rhs(spec):
    return chain_rhs(int(spec[5:])) if spec.startswith("chain") else RHS[spec]


def _walkers(spec, W, seed=0):
    base = "two_i" if spec.startswith("chain") else spec
    return walker_thetas(base, W, seed).T.copy()


def _run(m, theta, y0=None, trajectory=True):
    W = theta.shape[1]
    if y0 is None:
        y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    out = m.engine().integrate(y0, theta, trajectory=trajectory)
    return y0, {k: (v.cpu().numpy() if v is not None else None) for k, v in out.items()}


# --------------------------------------------------------------------- same algorithm
@pytest.mark.parametrize("spec", ["zero_i", "one_i", "two_i", "chain4", "chain5", "chain8", "chain20"])
@pytest.mark.parametrize("W", [1, 65, 300])
def test_rk4_bitwise_vs_c_restatement(spec, W):
    m = _model(spec, "rk4")
    theta = _walkers(spec, W)
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert np.array_equal(out["traj"], ref["traj"])
    np.testing.assert_allclose(out["chi"], ref["chi"], rtol=1e-12)
    np.testing.assert_allclose(out["ssres"], ref["ssres"], rtol=1e-12)
    assert np.array_equal(out["status"], ref["status"])


@pytest.mark.parametrize("spec", ["zero_i", "one_i", "two_i", "chain5", "chain8", "chain12", "chain20", "chain32"])
@pytest.mark.parametrize("W", [2, 258, 4098])
def test_rk4_pipelined_kernel_matches_direct_kernel(spec, W):
    """The producer/consumer trajectory kernel (4 compute + 2 store waves, LDS ring)
    gives the same bits as the one-lane-per-walker kernel, incl. ragged tail blocks."""
    m = _model(spec, "rk4")
    theta = _walkers(spec, W)
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    eng = m.engine()
    b = eng.integrate(y0, theta, pipelined=False)
    for nsw in (2, 4, 8):  # store waves per 4 compute waves
        a = eng.integrate(y0, theta, pipelined=nsw)
        for key in ("traj", "chi", "ssres", "status"):
            assert np.array_equal(a[key].cpu().numpy(), b[key].cpu().numpy(), equal_nan=True), (nsw, key)
    for nt in (False, True):
        c = eng.integrate(y0, theta, pipelined=True, nt_stores=nt)
        assert np.array_equal(c["traj"].cpu().numpy(), b["traj"].cpu().numpy())


@pytest.mark.parametrize("spec", ["two_i", "chain5", "chain20"])
@pytest.mark.parametrize("W", [7, 4098])
def test_rk4_tuned_kernel_choice(spec, W):
    """kernel="auto" (OE_TUNE): the library times the available RK4 trajectory kernels for
    the shape, keeps the fastest, reuses the choice, and the result is the bits of the
    default kernel and of the C restatement.  Odd W has no piped kernel."""
    m = _model(spec, "rk4")
    theta = _walkers(spec, W)
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    eng = m.engine()
    b = eng.integrate(y0, theta)
    assert eng.last_variant() in ("direct", "half")
    a = eng.integrate(y0, theta, kernel="auto")
    tuned = eng.tune_times()
    chosen = eng.last_variant()
    assert chosen in tuned and set(tuned) >= {"direct", "half"}
    assert all(0 < v < 1e3 for v in tuned.values()), tuned
    piped = {"pipe2", "pipe4", "pipe8", "pipe2x", "pipe4x", "pipe8x"}
    assert piped & set(tuned) == (set() if W % 2 else piped)
    for k in sorted(piped & set(tuned)):  # each piped kernel by name, incl. the XCD-ordered ones
        d = eng.integrate(y0, theta, kernel=k)
        assert eng.last_variant() == k
        assert np.array_equal(d["traj"].cpu().numpy(), b["traj"].cpu().numpy()), k
    for key in ("traj", "chi", "ssres", "status"):
        assert np.array_equal(a[key].cpu().numpy(), b[key].cpu().numpy(), equal_nan=True), key
    c = eng.integrate(y0, theta, kernel="auto")  # cached: same choice, same numbers reported
    assert eng.last_variant() == chosen and eng.tune_times() == tuned
    assert np.array_equal(c["traj"].cpu().numpy(), rk_ref.integrate(m.fit_problem(), y0, theta)["traj"])
    eng.integrate(y0, theta, kernel="auto", trajectory=False)
    assert eng.last_variant() == "other"
    with pytest.raises(RuntimeError):
        eng.tune_times()


@pytest.mark.parametrize("spec", ["two_i", "chain8", "chain20"])
@pytest.mark.parametrize("W", [1, 33, 4099])
def test_rk4_half_waves_match_full_waves(spec, W):
    """32 walkers per wavefront (OE_HALF_WAVES; automatic for S >= 8 trajectories) gives
    the bits of the 64-walker layout, incl. ragged tails; C restatement as the anchor."""
    m = _model(spec, "rk4")
    theta = _walkers(spec, W)
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    eng = m.engine()
    a = eng.integrate(y0, theta, half_waves=True)
    b = eng.integrate(y0, theta, trajectory=False)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert np.array_equal(a["traj"].cpu().numpy(), ref["traj"])
    for key in ("chi", "ssres", "status"):
        assert np.array_equal(a[key].cpu().numpy(), b[key].cpu().numpy(), equal_nan=True), key


@pytest.mark.parametrize("method", ["rk4", "dopri5"])
@pytest.mark.parametrize("spec", ["zero_i", "one_i", "two_i", "chain5", "chain20"])
@pytest.mark.parametrize("W", [1, 100, 4099, 5000, 8192])
def test_xcd_block_order_matches_blockidx_order(method, spec, W):
    """XCD runs of 512 walkers (the default) and one walker range per XCD give the bits of
    blockIdx-order blocks (trajectory, chi, R² residual, status), incl. ragged tails, grids
    that are not whole rounds of runs, half waves (chain5 RK4) and odd S."""
    m = _model(spec, method)
    theta = _walkers(spec, W)
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    eng = m.engine()
    a = eng.integrate(y0, theta)
    b = eng.integrate(y0, theta, xcd_remap="ranges")
    c = eng.integrate(y0, theta, xcd_remap=False)
    for key in ("traj", "chi", "ssres", "status"):
        ref = c[key].cpu().numpy()
        assert np.array_equal(ref, a[key].cpu().numpy(), equal_nan=True), key
        assert np.array_equal(ref, b[key].cpu().numpy(), equal_nan=True), key


@pytest.mark.parametrize("spec", ["zero_i", "one_i", "two_i", "chain8"])
def test_rk4_substeps_bitwise(spec):
    m = _model(spec, "rk4", substeps=3)
    theta = _walkers(spec, 70)
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert np.array_equal(out["traj"], ref["traj"])


@pytest.mark.parametrize("spec", ["zero_i", "one_i", "two_i", "chain6", "chain10", "chain20", "chain24", "chain32"])
@pytest.mark.parametrize("W", [64, 200])
def test_dopri5_vs_c_restatement(spec, W):
    """Bitwise DOPRI5 vs the C restatement (chain10..chain32: the S > 8 register-limit
    code path), and the chi of a no-trajectory launch (lazy dense output at observed
    points only) equals the trajectory one.  The NEGATIVE status bit is "negative at an
    output time", and a no-trajectory launch outputs observed times only, so only the
    NONFINITE and MAXSTEP bits must agree between the two launches."""
    m = _model(spec, "dopri5")
    theta = _walkers(spec, W)
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert np.array_equal(out["traj"], ref["traj"])
    np.testing.assert_allclose(out["chi"], ref["chi"], rtol=1e-12)
    assert np.array_equal(out["status"], ref["status"])
    _, lean = _run(m, theta, y0=y0, trajectory=False)
    for key in ("chi", "ssres"):
        assert np.array_equal(lean[key], out[key], equal_nan=True), key
    assert np.array_equal(lean["status"] & 5, out["status"] & 5)


@pytest.mark.parametrize("spec", ["chain10", "chain16", "chain20", "chain24", "chain32"])
@pytest.mark.parametrize("W", [1, 33, 200])
def test_split_dopri5_bitwise_vs_c_restatement(spec, W):
    """The split DOPRI5 kernel (a walker over 2 lanes for chain16/20, 4 for chain24/32;
    chain10 stays one lane per walker; split.cuh): bitwise
    against the C restatement of the same grouping (64/K walkers per step size, the lane
    tree of the error norm), chi-only launch equal to the trajectory one; and with
    OE_NO_SPLIT the one-lane kernel, bitwise against the 64-walker grouping."""
    m = _model(spec, "dopri5")
    fp = m.fit_problem()
    assert rk_ref.product_split(fp) == {"chain10": 1, "chain16": 2, "chain20": 2, "chain24": 4, "chain32": 4}[spec]
    theta = _walkers(spec, W, seed=7)
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(fp, y0, theta)
    assert np.array_equal(out["traj"], ref["traj"])
    np.testing.assert_allclose(out["chi"], ref["chi"], rtol=1e-12)
    assert np.array_equal(out["status"], ref["status"])
    _, lean = _run(m, theta, y0=y0, trajectory=False)
    for key in ("chi", "ssres"):
        assert np.array_equal(lean[key], out[key], equal_nan=True), key
    one = m.engine().integrate(y0, theta, split=False)
    ref1 = rk_ref.integrate(fp, y0, theta, split=1)
    assert np.array_equal(one["traj"].cpu().numpy(), ref1["traj"])
    # both groupings meet the tolerance: same solution to well within rtol
    np.testing.assert_allclose(out["traj"], ref1["traj"], rtol=1e-6, atol=1e-4)


def test_split_dopri5_evicts_a_pinning_walker():
    """A walker that cannot finish within max_steps is evicted in the split kernel too
    (status MAXSTEP on both of its lanes' outputs, NaN rows), bitwise as the C oracle."""
    m = _model("chain20", "dopri5", max_steps=150)
    theta = _walkers("chain20", 70, seed=5)
    theta[4, 3] = 1e9
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert out["status"][3] & N.OE_STATUS_MAXSTEP and np.isnan(out["traj"][-1, :, 3]).all()
    assert np.array_equal(out["traj"], ref["traj"], equal_nan=True)
    assert np.array_equal(out["status"], ref["status"])


# --------------------------------------------------------------------- reference algorithm
@pytest.mark.parametrize("spec,method,substeps,atol", [
    ("zero_i", "rk4", 4, 1e-6), ("one_i", "rk4", 1, 1e-6), ("two_i", "rk4", 1, 1e-6),
    ("zero_i", "dopri5", 1, 1e-6), ("one_i", "dopri5", 1, 1e-6), ("two_i", "dopri5", 1, 1e-6),
    ("chain20", "rk4", 4, 1e-4), ("chain20", "dopri5", 1, 1e-4)])
def test_vs_tight_odeint(spec, method, substeps, atol):
    m = _model(spec, method, substeps)
    theta = _walkers(spec, 96, seed=3)
    y0, out = _run(m, theta)
    for w in (0, 17, 63, 64, 95):
        tight = cpu_ref.odeint_traj(_rhs(spec), y0[:, w], m.times, theta[:, w], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(out["traj"][:, :, w], tight, rtol=1e-6, atol=atol)


@pytest.mark.parametrize("name", ["zero_i", "one_i", "two_i"])
def test_dropin_integrate_matches_reference_golden(golden, name):
    """ModelFramework.integrate (default DOPRI5 at odeint's tolerances) vs the reference's
    own integrate() output.  zero_i drives S down to ~1e-9, where atol = 1.49e-8
    dominates BOTH solvers' error control and log-space chi carries 1e-4..3e-4 error in
    the reference itself (vs the converged solution, measured); its fit statistics are
    therefore compared at 5e-3 here, and at 1e-6 against the converged solution in
    test_fused_chi_matches_converged_reference_chi."""
    m = product_model(name)
    TH = golden.integrate[f"{name}/theta"]
    fs_tol = 5e-3 if name == "zero_i" else 5e-6
    for w in range(TH.shape[0]):
        traj = m.integrate(parameters=(list(TH[w]),), as_dataframe=False, sum_subpopulations=False)
        np.testing.assert_allclose(traj, golden.integrate[f"{name}/traj"][w], rtol=5e-6, atol=1e-6)
        d = m.integrate(parameters=(list(TH[w]),), predict_obs=True, as_dataframe=False)
        fs = m.get_fitstats(d)
        np.testing.assert_allclose(fs["Chi"], golden.integrate[f"{name}/chi"][w], rtol=fs_tol)
        np.testing.assert_allclose(fs["R^2"], golden.integrate[f"{name}/rsq"][w], rtol=5e-6)
        np.testing.assert_allclose(fs["AIC"], golden.integrate[f"{name}/aic"][w], rtol=fs_tol)
    # the fused in-kernel likelihood of the batched path agrees too
    res = m.integrate_batch(TH, trajectory=False)
    np.testing.assert_allclose(res["chi"].cpu().numpy(), golden.integrate[f"{name}/chi"], rtol=fs_tol)
    df = m.integrate(parameters=(list(TH[0]),))
    assert list(df.columns) == m.get_snames() + ["time"]
    po = m.integrate(parameters=(list(TH[0]),), predict_obs=True)
    assert len(po) == len(m.df)


@pytest.mark.parametrize("name", ["zero_i", "one_i", "two_i"])
def test_fused_chi_matches_converged_reference_chi(golden, name):
    """At tight tolerances the fused in-kernel chi equals the reference's get_chi on the
    converged odeint solution (rtol=atol=1e-13) to 1e-6."""
    m = product_model(name, rtol=1e-12, atol=1e-12)
    om = oracle_model(name)
    TH = golden.integrate[f"{name}/theta"]
    chi = m.integrate_batch(TH, trajectory=False)["chi"].cpu().numpy()
    y0 = [om.istates[s] for s in CONFIGS[name]["snames"]]
    for w in range(TH.shape[0]):
        tr = cpu_ref.odeint_traj(RHS[name], y0, om.times, TH[w], rtol=1e-13, atol=1e-13)
        om.integrator = lambda y, ps, tr=tr: tr
        np.testing.assert_allclose(chi[w], float(om.get_chi(om.integrate_obs())), rtol=1e-6)


# --------------------------------------------------------------------- full size (C1)
def test_full_size_c1_bitwise_and_properties():
    """BASELINE configs[1]: two_i, 65 536 walkers, RK4 — bitwise against the C
    restatement over the whole ensemble, plus size-independent properties."""
    W = 65536
    m = _model("two_i", "rk4")
    rs = np.random.RandomState(0)
    theta = np.asarray([THETA["two_i"][p] for p in CONFIGS["two_i"]["pnames"]])[:, None] * \
        np.exp(0.05 * rs.standard_normal((5, W)))
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta, trajectory=True)
    assert np.array_equal(out["traj"], ref["traj"])
    np.testing.assert_allclose(out["chi"], ref["chi"], rtol=1e-12)
    assert np.array_equal(out["traj"][0], y0)
    assert np.isfinite(out["chi"]).all() and (out["status"] == 0).all()
    # determinism and batch-composition invariance
    _, again = _run(m, theta)
    assert np.array_equal(again["traj"], out["traj"])
    sub = np.array([0, 1, 4097, 30000, 65535])
    _, part = _run(m, theta[:, sub].copy(), y0[:, sub].copy())
    assert np.array_equal(part["traj"], out["traj"][:, :, sub])
    # RK4 vs DOPRI5 (tight) agree at full size
    md = _model("two_i", "dopri5", rtol=1e-10, atol=1e-10)
    _, dp = _run(md, theta)
    np.testing.assert_allclose(out["traj"], dp["traj"], rtol=1e-6, atol=1e-6)


def test_full_size_c2_dopri5_bitwise():
    """BASELINE configs[2]: two_i, 65 536 walkers, DOPRI5 with the wavefront error norm at
    odeint's tolerances — bitwise against the C restatement (64-walker lockstep groups)
    over the whole ensemble."""
    W = 65536
    m = _model("two_i", "dopri5")
    rs = np.random.RandomState(2)
    theta = np.asarray([THETA["two_i"][p] for p in CONFIGS["two_i"]["pnames"]])[:, None] * \
        np.exp(0.05 * rs.standard_normal((5, W)))
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta, trajectory=True)
    assert np.array_equal(out["traj"], ref["traj"])
    np.testing.assert_allclose(out["chi"], ref["chi"], rtol=1e-12)
    assert np.array_equal(out["status"], ref["status"]) and (out["status"] == 0).all()


def test_c3_chain20_dopri5_groups_bitwise():
    """configs[3] with DOPRI5: 20-state chain, 262 144 walkers; three whole lockstep groups
    (64 consecutive walkers share the step size) against the C restatement, bitwise."""
    W = 262144
    m = _model("chain20", "dopri5")
    rs = np.random.RandomState(3)
    theta = np.asarray(list(THETA["two_i"].values()))[:, None] * np.exp(0.05 * rs.standard_normal((5, W)))
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    out = m.engine().integrate(y0, theta, trajectory=True)
    for g in (0, 2049, W // 64 - 1):
        sl = slice(64 * g, 64 * g + 64)
        ref = rk_ref.integrate(m.fit_problem(), y0[:, sl].copy(), theta[:, sl].copy())
        assert np.array_equal(out["traj"][:, :, sl].cpu().numpy(), ref["traj"]), g
        np.testing.assert_allclose(out["chi"][sl].cpu().numpy(), ref["chi"], rtol=1e-12)
    del out


def test_c3_chain20_size_properties():
    """configs[3] size: 20-state chain, 262 144 walkers (42 GB trajectory in HBM)."""
    W = 262144
    m = _model("chain20", "rk4", substeps=2)
    rs = np.random.RandomState(1)
    theta = np.asarray(list(THETA["two_i"].values()))[:, None] * np.exp(0.05 * rs.standard_normal((5, W)))
    eng = m.engine()
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    out = eng.integrate(y0, theta, trajectory=True)
    chi = out["chi"].cpu().numpy()
    last = out["traj"][-1].cpu().numpy()
    first = out["traj"][0].cpu().numpy()
    del out
    assert np.isfinite(chi).all() and np.array_equal(first, y0)
    sub = np.array([0, 123457, W - 1])
    ref = rk_ref.integrate(m.fit_problem(), y0[:, sub].copy(), theta[:, sub].copy())
    assert np.array_equal(last[:, sub], ref["traj"][-1])
    np.testing.assert_allclose(chi[sub], ref["chi"], rtol=1e-12)
    # population conservation check of the chain: total mass changes only by growth/burst
    assert (last[0] > 0).all()


# --------------------------------------------------------------------- edge cases
def test_status_and_masking_edge_cases():
    from odelib_amd.engine import Engine, FitProblem
    m = _model("two_i", "rk4")
    fp = m.fit_problem()
    # observation of I1 at t=0 (I1 = 0): log(0) -> non-finite term -> masked
    fp2 = FitProblem(model_id=fp.model_id, n_states=4, n_params=5, times=fp.times, obs_tidx=[0],
                     obs_mask=np.array([2], np.uint64), obs_log=[1.0], obs_logsigma=[0.5], obs_lin=[np.e],
                     sstot=1.0, pnum=5, method="rk4")
    eng = Engine(fp2)
    theta = _walkers("two_i", 3)
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], 3, axis=1)
    y0[0, 1] = -1.0          # walker 1 starts negative
    theta[1, 2] = np.nan     # walker 2 has a NaN rate
    out = eng.integrate(y0, theta)
    chi = out["chi"].cpu().numpy()
    st = out["status"].cpu().numpy()
    assert np.isnan(chi).all()
    assert st[0] == 0
    assert st[1] & N.OE_STATUS_NEGATIVE
    assert st[2] & N.OE_STATUS_NONFINITE
    ref = rk_ref.integrate(fp2, y0, theta)
    assert np.array_equal(st, ref["status"])
    # no observations at all: chi is NaN, trajectory still produced
    fp3 = FitProblem(model_id=fp.model_id, n_states=4, n_params=5, times=fp.times, method="rk4")
    out3 = Engine(fp3).integrate(y0[:, :1], theta[:, :1])
    assert np.isnan(out3["chi"].item()) and np.isfinite(out3["traj"].cpu().numpy()).all()


def test_dopri5_evicts_walker_that_pins_the_wave():
    """A stiff walker (tau = 1e9) cannot finish within max_steps; it is evicted (status
    MAXSTEP, NaN output) and the other 63 walkers of its wave still meet tolerance."""
    m = _model("two_i", "dopri5", max_steps=200)
    theta = _walkers("two_i", 64, seed=5)
    theta[4, 7] = 1e9
    y0, out = _run(m, theta)
    st = out["status"]
    assert st[7] & N.OE_STATUS_MAXSTEP
    assert np.isnan(out["traj"][-1, :, 7]).all()
    ok = [w for w in range(64) if w != 7]
    assert (st[ok] & N.OE_STATUS_MAXSTEP == 0).all()
    for w in (0, 30, 63):
        tight = cpu_ref.odeint_traj(RHS["two_i"], y0[:, w], m.times, theta[:, w], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(out["traj"][:, :, w], tight, rtol=1e-6, atol=1e-6)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert np.array_equal(ref["status"], st)


# --------------------------------------------------------------------- Metropolis–Hastings
def _mh_inputs(spec, W, method="rk4", extra=None):
    m = _model(spec, method) if extra is None else product_model(spec, method=method, extra_params=extra)
    P = len(m.get_pnames())
    theta = np.repeat(np.array([float(m.parameters[p].val) for p in m.get_pnames()])[:, None], W, axis=1)
    theta = theta * np.exp(0.02 * np.random.RandomState(9).standard_normal(theta.shape))
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    return m, P, theta, y0


@pytest.mark.parametrize("spec,method", [("one_i", "rk4"), ("two_i", "rk4"), ("two_i", "dopri5"), ("chain8", "rk4"),
                                         ("chain20", "rk4"), ("chain20", "dopri5")])
def test_mh_philox_vs_c_restatement(spec, method):
    m, P, theta, y0 = _mh_inputs(spec, 130, method)
    walk = np.ones(P, np.uint8)
    walk[2] = 0  # one static parameter
    dev = m.engine().mh_run(theta, y0, nits=30, burnin=12, walk_mask=walk, rng="philox", seed=77, walker_offset=5)
    ref = rk_ref.mh_run(m.fit_problem(), theta, y0, 30, 12, walk, rng="philox", seed=77, walker_offset=5)
    tol = 1e-11 if method == "rk4" else 1e-8
    np.testing.assert_allclose(dev["samples"].cpu().numpy(), ref["samples"], rtol=tol)
    np.testing.assert_allclose(dev["theta"].cpu().numpy(), ref["theta"], rtol=tol)
    np.testing.assert_allclose(dev["final"].cpu().numpy(), ref["final"], rtol=tol)
    assert np.array_equal(dev["status"].cpu().numpy(), ref["status"])
    assert (dev["samples"].cpu().numpy()[:, 2, :] == theta[2]).all()  # static parameter never moves


@pytest.mark.parametrize("n,linked", [(16, (0, 8, 15)), (24, (0, 11, 23)), (32, (0, 17, 31))])
def test_split_mh_state0_params_vs_c_restatement(n, linked):
    """Split DOPRI5 MH (k_mh_split: 2 lanes per chain for chain16, 4 for chain24/32):
    '<state>0' parameters linking states held by the first, a middle and the last lane,
    one static parameter, Philox draws — vs the C restatement, which groups 64/K chains
    per lockstep wave as the kernel does."""
    from odelib_amd import ModelFramework, parameter
    from helpers import THETA, chain_rhs, demo_df
    snames = ["S"] + [f"I{k}" for k in range(1, n - 1)] + ["V"]
    th = dict(THETA["two_i"])
    extra = {f"{snames[s]}0": v for s, v in zip(linked, (5236900.0, 10.0, 10981000.0))}
    pn = list(th) + list(extra)
    m = ModelFramework(ODE=chain_rhs(n), parameter_names=pn, state_names=snames, dataframe=demo_df({"virus": "V", "host": "H"}),
                       state_summations={"H": snames[:-1]}, t_steps=1000, S=5236900, method="dopri5",
                       device_model="chain", **{p: parameter(init_value=v) for p, v in {**th, **extra}.items()})
    fp = m.fit_problem()
    assert rk_ref.product_split(fp) == (2 if n == 16 else 4)
    W, P = 70, len(pn)
    theta = np.array([float(m.parameters[p].val) for p in pn])[:, None] * np.exp(
        0.02 * np.random.RandomState(4).standard_normal((P, W)))
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    init_param = np.full(n, -1, np.int32)
    for j, s in enumerate(linked):
        init_param[s] = 5 + j
    walk = np.ones(P, np.uint8)
    walk[2] = 0
    dev = m.engine().mh_run(theta, y0, nits=16, burnin=5, walk_mask=walk, init_param=init_param, rng="philox",
                            seed=31, walker_offset=3)
    ref = rk_ref.mh_run(fp, theta, y0, 16, 5, walk, init_param=init_param, rng="philox", seed=31, walker_offset=3)
    np.testing.assert_allclose(dev["samples"].cpu().numpy(), ref["samples"], rtol=1e-8)
    np.testing.assert_allclose(dev["theta"].cpu().numpy(), ref["theta"], rtol=1e-8)
    np.testing.assert_allclose(dev["y0"].cpu().numpy(), ref["y0"], rtol=1e-8)
    np.testing.assert_allclose(dev["final"].cpu().numpy(), ref["final"], rtol=1e-8)
    assert np.array_equal(dev["status"].cpu().numpy(), ref["status"])
    acc = dev["final"].cpu().numpy()[3]
    assert (acc > 0).any()  # some chains moved: the linked states were exercised
    yd, td = dev["y0"].cpu().numpy(), dev["theta"].cpu().numpy()
    for j, s in enumerate(linked):  # a linked state follows its parameter
        np.testing.assert_array_equal(yd[s], td[5 + j])


def test_mh_replay_and_state0_params_vs_c_restatement():
    m, P, theta, y0 = _mh_inputs("one_i", 67, "rk4", extra={"V0": 10981000.0})
    nits = 25
    rs = np.random.RandomState(2)
    dz = 0.05 * rs.standard_normal((nits - 1, P, 67))
    u = rs.rand(nits - 1, 67)
    init_param = [-1, -1, 4]  # V <- V0
    walk = np.ones(P, np.uint8)
    dev = m.engine().mh_run(theta, y0, nits=nits, burnin=10, walk_mask=walk, init_param=init_param,
                            rng="replay", replay=(dz, u))
    ref = rk_ref.mh_run(m.fit_problem(), theta, y0, nits, 10, walk, init_param=init_param, rng="replay",
                        replay=(dz, u))
    np.testing.assert_allclose(dev["samples"].cpu().numpy(), ref["samples"], rtol=1e-11)
    np.testing.assert_allclose(dev["y0"].cpu().numpy(), ref["y0"], rtol=1e-11)
    # V follows V0 after the first proposal
    np.testing.assert_allclose(dev["y0"].cpu().numpy()[2], dev["theta"].cpu().numpy()[4], rtol=0)


@pytest.mark.parametrize("method", ["rk4", "dopri5"])
@pytest.mark.parametrize("T", [2, 3, 17])
def test_short_grids_bitwise_vs_c_restatement(method, T):
    """Grids of 2, 3 and 17 output times (every observation folded onto few rows; the
    DOPRI5 step spans many rows or ends exactly on the last one) — same bits as C."""
    from helpers import chain_problem
    m = chain_problem(4, method=method, T=T)
    theta = _walkers("chain4", 70)
    y0, out = _run(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta)
    assert np.array_equal(out["traj"], ref["traj"])
    np.testing.assert_allclose(out["chi"], ref["chi"], rtol=1e-12)
    assert np.array_equal(out["status"], ref["status"])


@pytest.mark.parametrize("method", ["rk4", "dopri5"])
def test_mh_all_parameters_static_vs_c_restatement(method):
    """static_parameters = every parameter: the chains never move, every proposal is
    the current state (accepted: exp(0) > u), samples repeat it — as in the C oracle."""
    m, P, theta, y0 = _mh_inputs("two_i", 70, method)
    walk = np.zeros(P, np.uint8)
    dev = m.engine().mh_run(theta, y0, nits=8, burnin=2, walk_mask=walk, rng="philox", seed=2)
    ref = rk_ref.mh_run(m.fit_problem(), theta, y0, 8, 2, walk, rng="philox", seed=2)
    np.testing.assert_allclose(dev["samples"].cpu().numpy(), ref["samples"], rtol=1e-11)
    assert np.array_equal(dev["theta"].cpu().numpy(), theta)


def test_mh_degenerate_lengths():
    m, P, theta, y0 = _mh_inputs("two_i", 10)
    walk = np.ones(P, np.uint8)
    r = m.engine().mh_run(theta, y0, nits=1, burnin=0, walk_mask=walk, rng="philox")
    assert r["samples"].shape[0] == 0
    np.testing.assert_allclose(r["theta"].cpu().numpy(), theta, rtol=0)
    r = m.engine().mh_run(theta, y0, nits=6, burnin=10, walk_mask=walk, rng="philox")
    assert r["samples"].shape[0] == 0


def test_mh_shards_are_invariant_to_partitioning():
    """Philox keyed by global walker id: running walkers [0, W) at once or as two shards
    with walker_offset gives identical chains (what makes results GPU-count invariant)."""
    m, P, theta, y0 = _mh_inputs("two_i", 200)
    walk = np.ones(P, np.uint8)
    eng = m.engine()
    full = eng.mh_run(theta, y0, nits=16, burnin=5, walk_mask=walk, rng="philox", seed=3)["samples"].cpu().numpy()
    a = eng.mh_run(theta[:, :72], y0[:, :72], nits=16, burnin=5, walk_mask=walk, rng="philox", seed=3,
                   walker_offset=0)["samples"].cpu().numpy()
    b = eng.mh_run(theta[:, 72:], y0[:, 72:], nits=16, burnin=5, walk_mask=walk, rng="philox", seed=3,
                   walker_offset=72)["samples"].cpu().numpy()
    assert np.array_equal(np.concatenate([a, b], axis=2), full)


def _decisive_prefix(margins, thr=1e-3):
    bad = np.nonzero(~(np.abs(np.nan_to_num(margins, nan=1.0)) > thr))[0]
    return int(bad[0]) if len(bad) else len(margins)


@pytest.mark.parametrize("key", ["one_i_s7", "two_i_s3", "zero_i_s0_static", "one_i_V0_s5"])
def test_dropin_metropolis_hastings_vs_reference_chain(golden, key):
    """Samplers.MetropolisHastings on the device (replay of the reference's numpy draws)
    reproduces the reference's posterior up to the first near-tie acceptance."""
    from odelib_amd.Statistics import Samplers
    meta = golden.meta[f"mh/{key}"]
    om = oracle_model(meta["model"], seed=meta["seed"], extra_params=meta["extra"] or None)
    margins = cpu_ref.metropolis_hastings(om, nits=meta["nits"], static_parameters=meta["static"])["margin"]
    n_ok = _decisive_prefix(margins)
    m = product_model(meta["model"], seed=meta["seed"], extra_params=meta["extra"] or None,
                      rtol=1e-10, atol=1e-10)
    post = Samplers.MetropolisHastings(m, nits=meta["nits"], static_parameters=set(meta["static"]),
                                       print_progress=False)
    assert list(post.columns) == meta["columns"]
    burnin = meta["nits"] // 2
    rows = max(0, n_ok - burnin)  # kept rows fully decided by decisive iterations
    # every acceptance of these chains is decisive (|acc - u| > 1e-3), so every kept row
    # is compared — the bound is stated, not just "some rows"
    assert rows == meta["nits"] - 1 - burnin == len(post)
    for c in meta["columns"]:
        np.testing.assert_allclose(post[c].to_numpy(dtype=float)[:rows], golden.mh[f"{key}/{c}"][:rows],
                                   rtol=2e-5, err_msg=c)


@pytest.mark.parametrize("key", ["one_i_s7", "zero_i_s0_static"])
def test_dropin_metropolis_hastings_prints_the_reference_progress(golden, capsys, key):
    """What the reference prints (Samplers.py:101-103, :123): 'a priori error <chi>', the
    header, then ``it exp(-chi)`` on every iteration (chi of the current state before the
    decision) — line for line, values to the integration accuracy (rtol 2e-5, as the
    posterior rows)."""
    from odelib_amd.Statistics import Samplers
    meta = golden.meta[f"mh/{key}"]
    om = oracle_model(meta["model"], seed=meta["seed"], extra_params=meta["extra"] or None)
    ref = cpu_ref.metropolis_hastings(om, nits=meta["nits"], static_parameters=meta["static"])
    m = product_model(meta["model"], seed=meta["seed"], extra_params=meta["extra"] or None, rtol=1e-10, atol=1e-10)
    Samplers.MetropolisHastings(m, nits=meta["nits"], static_parameters=set(meta["static"]), print_progress=True)
    lines = capsys.readouterr().out.strip().splitlines()
    head, chi0 = lines[0].rsplit(" ", 1)
    assert head == "a priori error" and lines[1] == "iteration; error; acceptance ratio"
    # zero_i drives S to ~1e-9, where odeint's atol dominates and the reference's own chi
    # carries 1e-4..3e-4 relative error (test_dropin_integrate_matches_reference_golden)
    np.testing.assert_allclose(float(chi0), ref["a_priori"], rtol=5e-3 if meta["model"] == "zero_i" else 2e-5)
    body = [ln.split() for ln in lines[2:]]
    assert [int(b[0]) for b in body] == list(range(1, meta["nits"]))
    got = np.array([float(b[1]) for b in body])
    np.testing.assert_allclose(got, ref["printed"], rtol=2e-5)
    # MCMC's chains print the same per-iteration lines (print_progress=False there)
    Samplers.MetropolisHastings(m.copy(), nits=5, print_progress=False)
    quiet = capsys.readouterr().out.strip().splitlines()
    assert [q.split()[0] for q in quiet] == ["1", "2", "3", "4"]


def _ulps(a, b):
    a = np.ascontiguousarray(a, dtype=np.float64).view(np.int64)
    b = np.ascontiguousarray(b, dtype=np.float64).view(np.int64)
    return np.abs(a - b)


def test_device_numpy_streams_match_numpy_legacy():
    """oe_numpy_streams (MT19937 + polar gauss per chain on the device) gives the
    reference's draws: uniforms bit-exact (the MT19937 stream and its consumption order
    are exact), normals within a few ulp in rare draws (the polar method's log is ocml on
    the device, glibc in numpy)."""
    import scipy.stats as st
    from odelib_amd.rng import device_plan, legacy_replay_streams
    m = _model("two_i", "rk4")
    pn = m.get_pnames()
    P = len(pn)
    W, nits = 257, 140
    seeds = list(range(W - 1)) + [4000000000]
    walking = {p for p in pn if p != pn[2]}
    dists = {p: ((st.lognorm, {"s": 0.5, "scale": 1.0}) if p in pn[:3] else (None, None)) for p in pn}
    prior = device_plan(seeds, pn, walking, dists)
    assert prior == 2  # walking lognorm priors: pn[0], pn[1]
    dz_h, u_h = legacy_replay_streams(seeds, nits, pn, walking, dists)
    walk = np.array([p in walking for p in pn], np.uint8)
    dz_d, u_d = m.engine().numpy_streams(seeds, nits, walk, prior_draws=prior)
    assert np.array_equal(u_d.cpu().numpy(), u_h)
    d = _ulps(dz_d.cpu().numpy(), dz_h)
    assert d.max() <= 16 and (d > 0).mean() < 1e-2, (d.max(), (d > 0).mean())
    assert (dz_d.cpu().numpy()[:, 2, :] == 0).all()


@pytest.mark.parametrize("method", ["rk4", "dopri5"])
def test_mh_device_numpy_rng_equals_host_replay(method):
    """rng='numpy' (draws generated on the device per chunk) runs the same chains as
    rng='replay' fed with the host numpy streams."""
    import scipy.stats as st
    from odelib_amd.rng import legacy_replay_streams
    m, P, theta, y0 = _mh_inputs("two_i", 200, method)
    pn = m.get_pnames()
    walk = np.ones(P, np.uint8)
    walk[3] = 0
    walking = {p for j, p in enumerate(pn) if walk[j]}
    dists = {p: (st.lognorm, {"s": 1.0, "scale": 1.0}) for p in pn}
    seeds = np.arange(200) * 7 + 3
    nits = 60
    eng = m.engine()
    host = eng.mh_run(theta, y0, nits=nits, burnin=20, walk_mask=walk, rng="replay",
                      replay=legacy_replay_streams(seeds, nits, pn, walking, dists), chunk=7)
    dev = eng.mh_run(theta, y0, nits=nits, burnin=20, walk_mask=walk, rng="numpy", numpy_seeds=seeds,
                     prior_draws=len(walking), chunk=7)
    for k in ("samples", "theta", "final"):
        np.testing.assert_allclose(dev[k].cpu().numpy(), host[k].cpu().numpy(), rtol=1e-12, err_msg=k)


@pytest.mark.parametrize("rng", ["philox", "numpy", "replay"])
@pytest.mark.parametrize("split", [5, 17, 40])
def test_mh_checkpoint_resume_equals_one_run(tmp_path, rng, split):
    """Stop after iteration split-1, checkpoint to disk, resume to nits: the same chains,
    samples and final state as one uninterrupted run (split before / after burn-in)."""
    from odelib_amd import checkpoint
    from odelib_amd.rng import legacy_replay_streams
    import scipy.stats as st
    m, P, theta, y0 = _mh_inputs("two_i", 130, "rk4")
    pn = m.get_pnames()
    walk = np.ones(P, np.uint8)
    nits, burnin = 50, 25
    seeds = np.arange(130)
    kw = dict(walk_mask=walk, rng=rng, seed=11, numpy_seeds=seeds, prior_draws=P, chunk=6)
    if rng == "replay":
        kw["replay"] = legacy_replay_streams(seeds, nits, pn, set(pn), {p: (st.lognorm, {"s": 1}) for p in pn})
    eng = m.engine()
    full = eng.mh_run(theta, y0, nits=nits, burnin=burnin, **kw)
    part = eng.mh_run(theta, y0, nits=split, burnin=burnin, **kw)
    path = tmp_path / "chains.npz"
    checkpoint.save(path, part, meta={"rng": rng})
    rest = eng.mh_run(None, None, nits=nits, burnin=burnin, resume=checkpoint.load(path), **kw)
    for k in ("theta", "y0", "final", "status"):
        assert np.array_equal(rest[k].cpu().numpy(), full[k].cpu().numpy()), k
    s_full = full["samples"].cpu().numpy()
    s_rest = rest["samples"].cpu().numpy()
    first = max(split, burnin + 1)
    assert np.array_equal(s_rest, s_full[first - burnin - 1:])
    if split > burnin + 1:
        assert np.array_equal(part["samples"].cpu().numpy(), s_full[:split - burnin - 1])


def test_dropin_mcmc_vs_reference(golden, capsys):
    meta = golden.meta["mcmc"]
    m = product_model("one_i", rtol=1e-10, atol=1e-10)
    post = m.MCMC(chain_inits=meta["inits"], iterations_per_chain=meta["iterations"], cpu_cores=8,
                  print_report=True)
    report = capsys.readouterr().out
    assert "Fitting Report" in report and "R-squared" in report
    assert list(post.columns) == meta["columns"]
    nits = meta["iterations"]
    for i, init in enumerate(meta["inits"]):
        om = oracle_model("one_i", theta=init, seed=i)
        n_ok = _decisive_prefix(cpu_ref.metropolis_hastings(om, nits=nits)["margin"])
        rows = max(0, n_ok - nits // 2)
        assert rows == nits - 1 - nits // 2  # all kept rows of every chain are compared
        sel = golden.mcmc["post/chain#"] == i
        mine = post[post["chain#"] == i]
        for c in meta["columns"]:
            np.testing.assert_allclose(mine[c].to_numpy(dtype=float)[:rows], golden.mcmc[f"post/{c}"][sel][:rows],
                                       rtol=2e-5, err_msg=f"chain {i} {c}")


def _oracle_chi(name, rows, tight=False):
    """The reference's per-sample chi (_Fit_worker, Framework.py:41-48): odeint + the
    masked chi of get_chi; NaN where every term is masked."""
    om = oracle_model(name)
    y0 = [om.istates[s] for s in CONFIGS[name]["snames"]]
    tol = dict(rtol=1e-13, atol=1e-13) if tight else {}
    out = []
    for row in rows:
        tr = cpu_ref.odeint_traj(RHS[name], y0, om.times, row, **tol)
        om.integrator = lambda y, ps, tr=tr: tr
        c = om.get_chi(om.integrate_obs())
        out.append(np.nan if np.ma.is_masked(c) else float(c))
    return np.array(out)


@pytest.mark.parametrize("tight", [False, True])
def test_fit_survey_chi_matches_oracle(tight):
    """f1: fit_survey's per-sample chi (one batched launch) against the reference's
    per-sample odeint + get_chi on the same LHS samples (seeded), at odeint's default
    tolerances (measured max rel 9.5e-8) and at tight ones (2.8e-12)."""
    kw = dict(rtol=1e-12, atol=1e-12) if tight else {}
    m = product_model("two_i", **kw)
    pn = m.get_pnames()
    np.random.seed(11)
    fs = m.fit_survey(samples=256)
    assert list(fs.columns) == pn + ["chi"] and len(fs) == 256
    assert np.array_equal(fs.index.to_numpy(), np.arange(256))
    ref = _oracle_chi("two_i", fs[pn].to_numpy(dtype=float), tight=tight)
    got = fs["chi"].to_numpy()
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_allclose(got, ref, rtol=1e-10 if tight else 1e-6)
    # the batched survey is the batched integrate's chi, bit for bit
    res = m.integrate_batch(fs[pn].to_numpy(), trajectory=False)
    np.testing.assert_array_equal(res["chi"].cpu().numpy(), got)
    # cpu_cores only reorders: the reference's round-robin workers, started last-first
    np.random.seed(11)
    fs3 = m.fit_survey(samples=256, cpu_cores=3)
    assert np.array_equal(fs3["chi"].to_numpy(), np.concatenate([got[2::3], got[1::3], got[0::3]]))
    assert list(fs3.index[:3]) == [0, 1, 2] and fs3.index[len(got[2::3])] == 0


def test_mcmc_int_chain_starts_follow_the_cutchi_filter(monkeypatch):
    """f1: MCMC(chain_inits=<int>) starts its chains from the survey samples whose chi
    beats the shifted-data chi (Framework.py:993-1012): the same rows the reference's
    filter keeps (oracle chi on the same seeded LHS samples; no sample within 1e-5 of
    the threshold) and the same pandas ``sample`` draws from numpy's global RNG."""
    from odelib_amd.Statistics import Samplers
    m = product_model("two_i")
    pn = m.get_pnames()
    n_chains, n_samples, sd = 8, 2000, 6.0
    # the oracle's selection, replaying the same global-RNG consumption
    np.random.seed(21)
    ps = m._lhs_samples(n_samples)[pn].reset_index(drop=True)
    chi = _oracle_chi("two_i", ps.to_numpy(dtype=float))
    shifted = {s: np.exp(m._obs_logabundance[s] + sd * m._obs_logsigma[s]) for s in m._obs_logabundance}
    cut = float(m.get_chi(shifted))
    assert np.nanmin(np.abs(chi - cut)) / cut > 1e-5
    ps["chi"] = chi
    good = ps.dropna()
    good = good[good["chi"] < cut]
    assert len(good) >= 20
    want = good.sample(n_chains, replace=True)[pn].to_numpy(dtype=float)
    seen = {}

    def capture(chains, **kw):
        seen["theta"] = np.array([[float(np.asarray(c.parameters[p].val)) for p in pn] for c in chains])
        seen["seeds"] = [c.random_seed for c in chains]
        return pd.DataFrame({"chi": [0.0]})
    monkeypatch.setattr(Samplers, "batched_metropolis_hastings", capture)
    np.random.seed(21)
    m.MCMC(chain_inits=n_chains, iterations_per_chain=10, fitsurvey_samples=n_samples, sd_fitdistance=sd,
           print_report=False)
    np.testing.assert_array_equal(seen["theta"], want)
    assert seen["seeds"] == list(range(n_chains))


@pytest.mark.parametrize("name", ["one_i", "two_i"])
def test_explore_equilibriums_final_rows_match_odeint(name, capsys):
    """f3: explore_equilibriums' final states (one batched launch) against the reference's
    _Equilibrium_worker rows (odeint's last row per LHS sample, Framework.py:24-38):
    within rtol = atol = 1e-6 of odeint at its default tolerances (measured 0.42 of that
    budget) and of tight odeint (0.01)."""
    m = product_model(name)
    pn, sn = m.get_pnames(), m.get_snames(after_summation=False)
    np.random.seed(5)
    eq = m.explore_equilibriums(samples=128)
    assert capsys.readouterr().out.startswith("Sampling with a Latin Hypercube scheme")
    assert list(eq.columns) == sn + pn and len(eq) == 128
    rows = eq[pn].to_numpy(dtype=float)
    y0 = np.asarray(m.get_inits(), float)
    for w in range(len(eq)):
        for tol in ({}, dict(rtol=1e-13, atol=1e-13)):
            final = cpu_ref.odeint_traj(RHS[name], y0, m.times, rows[w], **tol)[-1]
            np.testing.assert_allclose(eq[sn].to_numpy()[w], final, rtol=1e-6, atol=1e-6, err_msg=f"{w} {tol}")


# --------------------------------------------------------------------- C-ABI host pointers
@pytest.mark.parametrize("method", ["rk4", "dopri5"])
def test_c_abi_host_pointers_match_device_path(method):
    """oe_integrate with OE_HOST_PTRS and plain numpy buffers — the binding a maintainer
    would add to ODElib itself — returns the device path's bits."""
    import ctypes as C
    m = _model("two_i", method)
    W = 300
    theta = np.ascontiguousarray(_walkers("two_i", W))
    y0 = np.ascontiguousarray(np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1))
    fp = m.fit_problem()
    ctx = N.Context(0)
    try:
        ctx.problem_set(fp.to_c())
        T, S = fp.n_times, fp.n_states
        traj = np.empty((T, S, W))
        chi = np.empty(W)
        ssres = np.empty(W)
        st = np.empty(W, np.int32)
        ptr = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
        ctx.integrate(W, ptr(y0), ptr(theta), ptr(traj), ptr(chi), ptr(ssres), ptr(st), N.OE_HOST_PTRS)
        # without a trajectory buffer (MCMC-style call)
        chi2 = np.empty(W)
        ctx.integrate(W, ptr(y0), ptr(theta), None, ptr(chi2), None, None, N.OE_HOST_PTRS)
    finally:
        ctx.close()
    dev = m.engine().integrate(y0, theta)
    assert np.array_equal(traj, dev["traj"].cpu().numpy())
    assert np.array_equal(chi, dev["chi"].cpu().numpy(), equal_nan=True)
    assert np.array_equal(ssres, dev["ssres"].cpu().numpy())
    assert np.array_equal(st, dev["status"].cpu().numpy())
    assert np.array_equal(chi2, chi, equal_nan=True)


def test_tuned_choice_is_shared_by_contexts_on_the_device():
    """OE_TUNE's table of the built-in models is process-wide: a second engine (its own
    context) with the same model and shape reuses the first one's measurements instead of
    tuning again (no ~0.1-0.3 s settle and rounds), and launches the same kernel."""
    import time
    theta = _walkers("two_i", 4096)
    m1, m2 = _model("two_i", "rk4"), _model("two_i", "rk4")
    y0 = np.repeat(np.asarray(m1.get_inits(), float)[:, None], 4096, axis=1)
    e1, e2 = m1.engine(), m2.engine()
    assert e1.ctx is not e2.ctx
    e1.integrate(y0, theta, kernel="auto")  # tunes (or reuses an earlier test's table entry)
    t0 = time.perf_counter()
    r2 = e2.integrate(y0, theta, kernel="auto")
    dt = time.perf_counter() - t0
    assert e2.tune_times() == e1.tune_times() and e2.last_variant() == e1.last_variant()
    assert dt < 0.05, dt  # one launch, no tuning (the settle alone is >= 60 ms of launches)
    r1 = e1.integrate(y0, theta, kernel="direct")
    assert np.array_equal(r2["traj"].cpu().numpy(), r1["traj"].cpu().numpy())


def test_c_abi_error_codes_leave_the_context_usable():
    """The boundary's error behaviour (include/odelib_amd.h, INTEGRATION.md "Error behaviour"):
    a call before oe_problem_set is OE_ERR_STATE, walker counts outside [1, 2^29], a missing y0
    and a one-point time grid are OE_ERR_ARG, each with a message naming the entry point — and
    the context then integrates as if nothing had happened (the device path's bits)."""
    import ctypes as C
    m = _model("two_i", "dopri5")
    W = 64
    theta = np.ascontiguousarray(_walkers("two_i", W))
    y0 = np.ascontiguousarray(np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1))
    fp = m.fit_problem()
    ptr = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
    chi = np.full(W, -1.0)
    ctx = N.Context(0)
    try:
        with pytest.raises(RuntimeError, match=r"oe_integrate failed \(-3\)"):
            ctx.integrate(W, ptr(y0), ptr(theta), None, ptr(chi), None, None, N.OE_HOST_PTRS)
        prob = fp.to_c()
        ctx.problem_set(prob)
        for bad_w in (0, -5, (1 << 29) + 1):
            with pytest.raises(RuntimeError, match=r"oe_integrate failed \(-1\).*n_walkers"):
                ctx.integrate(bad_w, ptr(y0), ptr(theta), None, ptr(chi), None, None, N.OE_HOST_PTRS)
        with pytest.raises(RuntimeError, match=r"oe_integrate failed \(-1\).*y0"):
            ctx.integrate(W, None, ptr(theta), None, ptr(chi), None, None, N.OE_HOST_PTRS)
        assert np.all(chi == -1.0)  # nothing was written
        bad = fp.to_c()
        bad.n_times = 1
        with pytest.raises(RuntimeError, match=r"oe_problem_set failed \(-1\)"):
            ctx.problem_set(bad)
        ctx.problem_set(prob)
        ctx.integrate(W, ptr(y0), ptr(theta), None, ptr(chi), None, None, N.OE_HOST_PTRS)
    finally:
        ctx.close()
    dev = m.engine().integrate(y0, theta)
    assert np.array_equal(chi, dev["chi"].cpu().numpy(), equal_nan=True)
