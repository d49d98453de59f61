"""Speculative Metropolis–Hastings rounds (oe_mh_args.speculate; k_mh_tree + k_mh_resolve)
against the one-iteration-per-step MH kernel, the C restatement and themselves.

The chain a round keeps is the sequential chain: same draws, same proposals (formed by the
same operations on the same path), same accept test.  RK4 integrates a lane on its own, so
RK4 chains must be bitwise those of speculate=0; DOPRI5 lanes share a step size with their
wave, which holds other proposals in a round, so DOPRI5/auto chains take the same
decisions — hence bitwise the same parameters — with chi, R², AIC within the integration
tolerance (rtol 1e-7 written below).
"""
import numpy as np
import pytest

from helpers import product_model
from oracle import rk_ref

pytestmark = pytest.mark.gpu


def _inputs(spec, W, method="rk4", extra=None, seed=9):
    m = product_model(spec, method=method, extra_params=extra) if extra else product_model(spec, method=method)
    P = len(m.get_pnames())
    theta = np.repeat(np.array([float(m.parameters[p].val) for p in m.get_pnames()])[:, None], W, axis=1)
    theta = theta * np.exp(0.02 * np.random.RandomState(seed).standard_normal(theta.shape))
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    return m, P, theta, y0


def _np(r):
    return {k: r[k].cpu().numpy() for k in ("samples", "theta", "y0", "final", "status")}


def _equal(a, b):
    for k in a:
        assert np.array_equal(a[k], b[k], equal_nan=True), k


@pytest.mark.parametrize("W", [1, 5, 70])
@pytest.mark.parametrize("depth", [2, 3, "auto"])
@pytest.mark.parametrize("rng", ["philox", "replay", "numpy"])
def test_rk4_speculative_chains_are_the_sequential_chains(W, depth, rng):
    """two_i RK4, one static parameter: every output bitwise equal to speculate=0, for
    fixed and library-chosen depths, a chunk that is not a multiple of the depth, and all
    three RNG modes (the draws do not depend on the chain state, so a round may consume
    them ahead)."""
    m, P, theta, y0 = _inputs("two_i", W)
    walk = np.ones(P, np.uint8)
    walk[2] = 0
    nits, burnin = 31, 9
    kw = dict(nits=nits, burnin=burnin, walk_mask=walk, chunk=7)
    if rng == "philox":
        kw.update(rng="philox", seed=5, walker_offset=3)
    elif rng == "replay":
        rs = np.random.RandomState(4)
        kw.update(rng="replay", replay=(0.05 * rs.standard_normal((nits - 1, P, W)), rs.rand(nits - 1, W)))
    else:
        kw.update(rng="numpy", numpy_seeds=np.arange(W) + 11, prior_draws=2)
    eng = m.engine()
    seq = _np(eng.mh_run(theta, y0, **kw))
    assert eng.last_mh_depth() == 0
    spec = _np(eng.mh_run(theta, y0, speculate=depth, **kw))
    d = eng.last_mh_depth()
    assert d == depth if depth != "auto" else d >= 8
    _equal(spec, seq)
    acc = seq["final"][3]
    assert (acc > 0).any() and (acc < nits - 1).any()  # both branches of the tree were taken


def test_rk4_speculative_state0_parameter_vs_c_restatement():
    """one_i with a 'V0' initial-condition parameter (the linked state follows the
    accepted parameter), replay draws: speculative rounds vs the C restatement of the
    sequential chain (rtol 1e-11: ocml vs libm log/exp) and bitwise vs speculate=0."""
    m, P, theta, y0 = _inputs("one_i", 67, extra={"V0": 10981000.0})
    nits = 25
    rs = np.random.RandomState(2)
    dz = 0.05 * rs.standard_normal((nits - 1, P, 67))
    u = rs.rand(nits - 1, 67)
    init_param = [-1, -1, 4]
    walk = np.ones(P, np.uint8)
    kw = dict(nits=nits, burnin=10, walk_mask=walk, init_param=init_param, rng="replay", replay=(dz, u))
    eng = m.engine()
    spec = _np(eng.mh_run(theta, y0, speculate=4, **kw))
    seq = _np(eng.mh_run(theta, y0, **kw))
    _equal(spec, seq)
    # depth 9: the one-wave-per-chain resolve (LDS tree), linked state included
    _equal(_np(eng.mh_run(theta, y0, speculate="auto", **kw)), seq)
    assert eng.last_mh_depth() == 9
    ref = rk_ref.mh_run(m.fit_problem(), theta, y0, nits, 10, walk, init_param=init_param, rng="replay",
                        replay=(dz, u))
    np.testing.assert_allclose(spec["samples"], ref["samples"], rtol=1e-11)
    np.testing.assert_allclose(spec["y0"], ref["y0"], rtol=1e-11)
    np.testing.assert_array_equal(spec["y0"][2], spec["theta"][4])


@pytest.mark.parametrize("method", ["dopri5", "auto"])
def test_dopri5_speculative_chains_are_the_sequential_chains(method):
    """DOPRI5 / auto: the MH integrator steps every proposal on its own (lane.cuh), so a
    proposal's chi does not depend on the other proposals in its wave and the speculative
    chains are the sequential ones bit for bit (near-posterior draws: no walker is handed to
    the BDF pass, whose step is shared by the wave's handed walkers)."""
    m, P, theta, y0 = _inputs("two_i", 24, method)
    walk = np.ones(P, np.uint8)
    kw = dict(nits=40, burnin=15, walk_mask=walk, rng="philox", seed=21)
    eng = m.engine()
    seq = _np(eng.mh_run(theta, y0, **kw))
    spec = _np(eng.mh_run(theta, y0, speculate="auto", **kw))
    assert eng.last_mh_depth() >= 8
    assert not (seq["status"] & 8).any()
    _equal(spec, seq)


@pytest.mark.parametrize("method", ["dopri5", "auto"])
def test_mh_chains_do_not_depend_on_their_wave_mates(method):
    """The same chains (same global ids, so the same Philox draws) run in a 40-chain and a
    17-chain ensemble: chains 0..16 are bitwise the same — a DOPRI5 chain no longer shares
    its step size with whichever chains fill its wave."""
    m, P, theta, y0 = _inputs("two_i", 40, method, seed=4)
    walk = np.ones(P, np.uint8)
    kw = dict(nits=25, burnin=5, walk_mask=walk, rng="philox", seed=2)
    eng = m.engine()
    big = _np(eng.mh_run(theta, y0, **kw))
    small = _np(eng.mh_run(theta[:, :17].copy(), y0[:, :17].copy(), **kw))
    for k in small:
        assert np.array_equal(small[k], big[k][..., :17], equal_nan=True), k
    acc = small["final"][3]
    assert (acc > 0).any()


def test_speculative_resume_equals_one_run():
    """A speculative run stopped at iteration 12 and resumed gives the uninterrupted run
    (rounds restart at the resume point; draws are indexed by iteration)."""
    m, P, theta, y0 = _inputs("two_i", 9)
    walk = np.ones(P, np.uint8)
    kw = dict(walk_mask=walk, rng="philox", seed=8, speculate=3)
    eng = m.engine()
    full = _np(eng.mh_run(theta, y0, nits=30, burnin=5, **kw))
    part = eng.mh_run(theta, y0, nits=12, burnin=5, **kw)
    rest = _np(eng.mh_run(None, None, nits=30, burnin=5, resume=part, **kw))
    np.testing.assert_array_equal(np.concatenate([part["samples"].cpu().numpy(), rest["samples"]]), full["samples"])
    for k in ("theta", "y0", "final", "status"):
        np.testing.assert_array_equal(rest[k], full[k])


def test_speculation_depth_rule_and_edges():
    """The library's depth: (2^d - 1)·W lanes within about one wave per SIMD, none when the
    chains fill the device; all-static chains and burn-in past the end behave as
    speculate=0."""
    m, P, theta, y0 = _inputs("two_i", 4096)
    eng = m.engine()
    walk = np.ones(P, np.uint8)
    eng.mh_run(theta, y0, nits=3, burnin=0, walk_mask=walk, speculate="auto")
    assert 2 <= eng.last_mh_depth() <= 5
    big = np.repeat(theta[:, :1], 131072, axis=1)
    eng.mh_run(big, np.repeat(y0[:, :1], 131072, axis=1), nits=2, burnin=0, walk_mask=walk, speculate="auto")
    assert eng.last_mh_depth() == 0
    th, yy = theta[:, :6], y0[:, :6]
    for walk_mask, burnin in ((np.zeros(P, np.uint8), 2), (walk, 40)):
        kw = dict(nits=9, burnin=burnin, walk_mask=walk_mask, rng="philox", seed=1)
        _equal(_np(eng.mh_run(th, yy, speculate=3, **kw)), _np(eng.mh_run(th, yy, **kw)))


@pytest.mark.parametrize("method", ["rk4", "dopri5", "auto"])
def test_speculative_rounds_vs_c_restatement(method):
    """Device rounds vs their C restatement (rk_ref.mh_tree_run: the round's proposals
    integrated by the restatement's batched integrate in the device's node-major lane order,
    hence the same DOPRI5 lockstep groups): rtol 1e-11 for RK4, 1e-8 for DOPRI5 / auto
    (ocml vs libm exp/log in the proposals), status bitwise; one static parameter, a chunk
    of 9 iterations (rounded down to 8 = two rounds of 4, then a last round of 3)."""
    m, P, theta, y0 = _inputs("two_i", 21, method)
    walk = np.ones(P, np.uint8)
    walk[3] = 0
    dev = _np(m.engine().mh_run(theta, y0, nits=20, burnin=6, walk_mask=walk, rng="philox", seed=13, walker_offset=4,
                                speculate=4, chunk=9))
    ref = rk_ref.mh_tree_run(m.fit_problem(), theta, y0, 20, 6, walk, depth=4, rng="philox", seed=13,
                             walker_offset=4, chunk=9)
    tol = 1e-11 if method == "rk4" else 1e-8
    for k in ("samples", "theta", "y0", "final"):
        np.testing.assert_allclose(dev[k], ref[k], rtol=tol, err_msg=k)
    assert np.array_equal(dev["status"], ref["status"])


@pytest.mark.parametrize("n,K", [(20, 2), (24, 4)])
def test_split_dopri5_speculative_rounds(n, K):
    """The wide chain models' split DOPRI5 MH (a chain on K lanes) in speculative rounds
    (k_mh_split_tree): the same decisions as the sequential split kernel, chi / R² / AIC
    within rtol 1e-7, and vs the C restatement of the rounds with the same 64/K grouping
    at rtol 1e-8; a '<state>0' parameter linking the last state (held by lane K-1)."""
    from odelib_amd import ModelFramework, parameter
    from helpers import THETA, chain_rhs, demo_df
    snames = ["S"] + [f"I{k}" for k in range(1, n - 1)] + ["V"]
    th = dict(THETA["two_i"], V0=10981000.0)
    m = ModelFramework(ODE=chain_rhs(n), parameter_names=list(th), state_names=snames,
                       dataframe=demo_df({"virus": "V", "host": "H"}), state_summations={"H": snames[:-1]},
                       t_steps=1000, S=5236900, method="dopri5", device_model="chain",
                       **{p: parameter(init_value=v) for p, v in th.items()})
    fp = m.fit_problem()
    assert rk_ref.product_split(fp) == K
    W, P = 9, len(th)
    theta = np.array(list(th.values()))[:, None] * np.exp(0.02 * np.random.RandomState(6).standard_normal((P, W)))
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    init_param = np.full(n, -1, np.int32)
    init_param[n - 1] = 5
    walk = np.ones(P, np.uint8)
    kw = dict(nits=18, burnin=5, walk_mask=walk, init_param=init_param, rng="philox", seed=17, chunk=8)
    eng = m.engine()
    seq = _np(eng.mh_run(theta, y0, **kw))
    spec = _np(eng.mh_run(theta, y0, speculate=4, **kw))
    assert eng.last_mh_depth() == 4
    for c in list(range(P)) + [P + 3, P + 4]:
        assert np.array_equal(spec["samples"][:, c], seq["samples"][:, c]), c
    np.testing.assert_allclose(spec["samples"], seq["samples"], rtol=1e-7)
    np.testing.assert_array_equal(spec["y0"][n - 1], spec["theta"][5])
    ref = rk_ref.mh_tree_run(fp, theta, y0, 18, 5, walk, init_param=init_param, depth=4, rng="philox", seed=17,
                             chunk=8)
    for k in ("samples", "theta", "y0", "final"):
        np.testing.assert_allclose(spec[k], ref[k], rtol=1e-8, err_msg=k)
    assert (seq["final"][3] > 0).any()


@pytest.mark.parametrize("method", ["auto", "bdf"])
def test_speculative_rounds_with_stiff_proposals_vs_c_restatement(method):
    """Rounds whose proposals include stiff draws (tau = 1e5, 1e6 / lam = 1e4, 1e9): 'auto'
    hands them to BDF from each lane's own eviction point, 'bdf' integrates every proposal
    with it — the device rounds take the C restatement's decisions and values (rtol 1e-8, the
    proposals' exp/log), status bitwise.  (The MH kernels sit at the register limit: this is
    the case that caught a code-generation fragility of the BDF hand-over, lane.cuh.)"""
    from test_gpu_stiff import _mixed_thetas
    W = 128
    m = product_model("two_i", method=method)
    theta = _mixed_thetas("two_i", W, [1, 64, 65, 127])
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    walk = np.ones(5, np.uint8)
    dev = _np(m.engine().mh_run(theta, y0, nits=4, burnin=0, walk_mask=walk, rng="philox", seed=11, speculate=3))
    ref = rk_ref.mh_tree_run(m.fit_problem(), theta, y0, 4, 0, walk, depth=3, rng="philox", seed=11)
    for k in ("samples", "theta", "final"):
        np.testing.assert_allclose(dev[k], ref[k], rtol=1e-8, err_msg=k)
    assert np.array_equal(dev["status"], ref["status"])


@pytest.mark.parametrize("method", ["rk4", "dopri5", "auto"])
@pytest.mark.parametrize("nits", [2, 3])
def test_smallest_mh_runs_on_a_two_point_grid(method, nits):
    """The smallest runs the ABI takes: one or two MH iterations (nits = 2, 3), one and three
    chains, on a two-point time grid — speculative rounds (a round then covers at most the
    iterations left) give the sequential chains bit for bit, every chain's chi finite."""
    from helpers import chain_problem
    m = chain_problem(4, method=method, T=2)
    P = len(m.get_pnames())
    for W in (1, 3):
        theta = np.repeat(np.array([float(m.parameters[p].val) for p in m.get_pnames()])[:, None], W, axis=1)
        y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
        kw = dict(nits=nits, burnin=0, walk_mask=np.ones(P, np.uint8), rng="philox", seed=3)
        eng = m.engine()
        seq = _np(eng.mh_run(theta, y0, **kw))
        spec = _np(eng.mh_run(theta, y0, speculate="auto", **kw))
        _equal(spec, seq)
        assert seq["samples"].shape[0] == nits - 1
        assert np.all(np.isfinite(seq["final"][0]))
