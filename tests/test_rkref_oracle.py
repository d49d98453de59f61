"""Pin the C restatement (oracle/rk_ref.c) — the same-algorithm checker of the HIP
kernels — against the reference-algorithm oracle (scipy odeint) and known answers."""
import numpy as np
import pytest

from helpers import CONFIGS, chain_problem, oracle_model, product_model, walker_thetas
from odelib_amd.models import chain_rhs
from oracle import cpu_ref, rk_ref


def test_philox_known_answers():
    """Random123 philox4x32_10 known-answer vectors."""
    assert list(rk_ref.philox4x32_10([0, 0, 0, 0], [0, 0])) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert list(rk_ref.philox4x32_10([0xffffffff] * 4, [0xffffffff] * 2)) == \
        [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert list(rk_ref.philox4x32_10([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344],
                                     [0xa4093822, 0x299f31d0])) == [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_inv_fifth_root_accuracy():
    """The step controller's x^(-1/5) (exact scalings + mul/fma only, so host and device
    agree bitwise) is within 1e-9 of the true value from denormals to 1e30."""
    xs = np.concatenate([[5e-324, 1e-310, 2.2250738585072014e-308, 1e-30, 1.0, 1e30],
                         np.logspace(-300, 300, 4001), np.random.RandomState(1).uniform(0.5, 40.0, 2000)])
    for x in xs:
        got = rk_ref.inv_fifth_root(x)
        want = float(np.float64(x) ** -0.2) if x > 1e-300 else float(np.exp(-0.2 * np.log(np.longdouble(x))))
        assert abs(got / want - 1.0) < 1e-9, (x, got, want)


def _inputs(name, W=8):
    m = product_model(name)
    fp = m.fit_problem()
    theta = walker_thetas(name, W).T.copy()
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    return m, fp, theta, y0


@pytest.mark.parametrize("name", ["zero_i", "one_i", "two_i"])
@pytest.mark.parametrize("method", ["rk4", "dopri5"])
def test_c_integrators_match_tight_odeint(name, method):
    m, fp, theta, y0 = _inputs(name)
    fp.method = method
    fp.rk4_substeps = 4 if name == "zero_i" else 1  # zero_i's grid is 288 points: keep h <= 3/999
    out = rk_ref.integrate(fp, y0, theta)
    for w in range(theta.shape[1]):
        tight = cpu_ref.odeint_traj(CONFIGS[name]["ode"], y0[:, w], fp.times, theta[:, w], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(out["traj"][:, :, w], tight, rtol=1e-6, atol=1e-6)
    assert (out["status"] == 0).all()


@pytest.mark.parametrize("name", ["zero_i", "one_i", "two_i"])
def test_c_fused_likelihood_matches_reference_formulas(name):
    m, fp, theta, y0 = _inputs(name)
    out = rk_ref.integrate(fp, y0, theta)
    om = oracle_model(name)
    for w in range(theta.shape[1]):
        traj = out["traj"][:, :, w].copy()
        om.integrator = lambda y, ps, tr=traj: tr
        d = om.integrate_obs()
        assert np.isclose(out["chi"][w], float(om.get_chi(d)), rtol=1e-13, atol=0)
        pred = np.concatenate([d[s] for s in d])
        assert np.isclose(out["ssres"][w], np.nansum((pred - fp.obs_lin) ** 2), rtol=1e-13)


def test_c_chain20_rk4_substeps_vs_odeint():
    m = chain_problem(20, method="rk4", substeps=4)
    fp = m.fit_problem()
    W = 4
    theta = walker_thetas("two_i", W).T.copy()
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    out = rk_ref.integrate(fp, y0, theta)
    for w in range(W):
        tight = cpu_ref.odeint_traj(chain_rhs(20), y0[:, w], fp.times, theta[:, w], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(out["traj"][:, :, w], tight, rtol=1e-6, atol=1e-4)


def test_c_mh_replay_matches_oracle_chain_with_same_integrator():
    """Batched C MH in replay mode == the reference MH loop (cpu_ref) when both use the
    C RK4 integrator and the same replay draws: the batched restatement of
    Samplers.py:104-153 is the reference's loop."""
    name, nits, seed = "one_i", 40, 4
    m, fp, _, _ = _inputs(name)
    fp.method = "rk4"
    om = oracle_model(name, seed=seed)
    pn = om.get_pnames()
    th0 = np.array([[float(om.parameters[p].val)] for p in pn])
    y0 = np.array([[float(om.istates[s])] for s in om._snames])
    from odelib_amd.rng import legacy_replay_streams
    dz, u = legacy_replay_streams([seed], nits, pn, set(pn),
                                  {p: (om.parameters[p].dist, om.parameters[p].hp) for p in pn})

    def c_integrator(yy, ps):
        r = rk_ref.integrate(fp, np.asarray(yy, float)[:, None], np.asarray(ps, float)[:, None])
        return r["traj"][:, :, 0]
    om.integrator = c_integrator
    ref = cpu_ref.metropolis_hastings(om, nits=nits, replay=(dz[:, :, 0], u[:, 0]))
    out = rk_ref.mh_run(fp, th0, y0, nits, nits // 2, np.ones(len(pn), np.uint8), rng="replay", replay=(dz, u))
    s = out["samples"][:, :, 0]
    for j, c in enumerate(pn + ["chi", "rsquared", "aic", "iteration", "acceptance_ratio"]):
        np.testing.assert_allclose(s[:, j], ref[c], rtol=1e-11, err_msg=c)


@pytest.mark.parametrize("method", ["rk4", "dopri5"])
def test_c_speculative_rounds_are_the_sequential_chain(method):
    """The restatement of the speculative MH rounds (rk_ref.mh_tree_run: all 2^d - 1
    proposals of a round integrated in one batched call, then each chain's path walked)
    gives the sequential batched MH chain: RK4 to rtol 1e-11 (numpy vs libm exp/log in the
    proposals); DOPRI5 too (rtol 1e-9): the MH integrator steps every proposal on its own
    (lane_steps), so a proposal's chi no longer depends on which proposals share its wave."""
    m, fp, _, _ = _inputs("two_i")
    fp.method = method
    W, nits, burnin = 5, 14, 4
    P = len(m.get_pnames())
    theta = np.array([[float(m.parameters[p].val)] for p in m.get_pnames()]) * np.exp(
        0.02 * np.random.RandomState(3).standard_normal((P, W)))
    y0 = np.repeat(np.array([[float(m.istates[s])] for s in m._snames]), W, axis=1)
    walk = np.ones(P, np.uint8)
    walk[1] = 0
    seq = rk_ref.mh_run(fp, theta, y0, nits, burnin, walk, rng="philox", seed=6, walker_offset=2)
    tree = rk_ref.mh_tree_run(fp, theta, y0, nits, burnin, walk, depth=3, rng="philox", seed=6, walker_offset=2,
                              chunk=7)
    P5 = P + 5
    tol = 1e-11 if method == "rk4" else 1e-9
    for k in ("samples", "theta", "final"):
        np.testing.assert_allclose(tree[k], seq[k], rtol=tol, err_msg=k)
    assert tree["samples"].shape == (nits - 1 - burnin, P5, W)
    assert np.array_equal(tree["status"], seq["status"])
    acc = seq["final"][3]
    assert (acc > 0).any() and (acc < nits - 1).any()


def test_c_speculative_rounds_split_grouping():
    """The restated rounds with the split DOPRI5 grouping (chain16: 2 lanes per chain, 32
    proposals per step size) take the sequential split chain's decisions: parameters equal,
    chi / R² / AIC within rtol 1e-7."""
    m = chain_problem(16, method="dopri5")
    fp = m.fit_problem()
    assert rk_ref.product_split(fp) == 2
    P = len(m.get_pnames())
    W, nits, burnin = 4, 10, 3
    theta = np.array([[float(m.parameters[p].val)] for p in m.get_pnames()]) * np.exp(
        0.02 * np.random.RandomState(5).standard_normal((P, W)))
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    walk = np.ones(P, np.uint8)
    seq = rk_ref.mh_run(fp, theta, y0, nits, burnin, walk, rng="philox", seed=3)
    tree = rk_ref.mh_tree_run(fp, theta, y0, nits, burnin, walk, depth=3, rng="philox", seed=3)
    np.testing.assert_allclose(tree["samples"][:, :P], seq["samples"][:, :P], rtol=1e-12)
    np.testing.assert_allclose(tree["samples"][:, P:], seq["samples"][:, P:], rtol=1e-7)
    assert (seq["final"][3] > 0).any()


@pytest.mark.parametrize("method", ["dopri5", "auto"])
def test_c_lane_steps_are_a_group_of_one(method):
    """The MH kernels' per-lane DOPRI5 (lane.cuh; rk_ref lane_steps): a walker of a 70-walker
    batch gives the bits of the same walker integrated alone (a lockstep group of one), so
    its result does not depend on the other walkers; 'auto' with two stiff walkers (tau = 1e5,
    1e4): the hand-over happens at each walker's own eviction point, and the BDF pass (one
    group) stays within 1e-6 of the walker integrated alone.  (A group of one is the lockstep
    algorithm's own case, held to tight odeint by test_c_integrators_match_tight_odeint.)"""
    m, fp, _, _ = _inputs("two_i")
    fp.method = method
    W = 70
    theta = walker_thetas("two_i", W, seed=4).T.copy()
    stiff = [9, 40] if method == "auto" else []
    for w, tau in zip(stiff, (1e5, 1e4)):
        theta[4, w] = tau
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    assert rk_ref.lane_steps(fp)
    lane = rk_ref.integrate(fp, y0, theta, trajectory=False, lane=True)
    lock = rk_ref.integrate(fp, y0, theta, trajectory=False)
    assert not np.array_equal(lane["chi"], lock["chi"])  # the lockstep grouping differs
    for w in range(W):
        one = rk_ref.integrate(fp, y0[:, w:w + 1].copy(), theta[:, w:w + 1].copy(), trajectory=False)
        if w in stiff:
            assert lane["status"][w] & 8
            np.testing.assert_allclose(lane["chi"][w], one["chi"][0], rtol=1e-6)
        else:
            assert lane["chi"][w] == one["chi"][0] and lane["ssres"][w] == one["ssres"][0], w
            assert lane["status"][w] == one["status"][0]
    with pytest.raises(RuntimeError):  # the per-lane mode has no trajectory
        rk_ref.integrate(fp, y0, theta, trajectory=True, lane=True)


@pytest.mark.parametrize("method", ["dopri5", "auto"])
def test_c_speculative_decision_agreement_over_many_chains(method):
    """How often speculative rounds change a DOPRI5 / 'auto' chain: a proposal's
    chi moves at the tolerance level when its lockstep group changes (other proposals share
    its step size), so an accept/reject whose margin |accp - u| is below ~1e-7 can flip, and
    the chain then diverges.  Measured on the restatement over 96 chains x 30 iterations x
    3 seeds, depth 3 and 5 (the depth the device picks depends on its CU count): every chain
    takes the sequential chain's decisions (asserted >= 99 % of chains, the documented bar;
    a flip needs a margin ~1e-7, probability ~1e-6 per decision)."""
    m, fp, _, _ = _inputs("two_i")
    fp.method = method
    W, nits, burnin = 96, 31, 0
    P = len(m.get_pnames())
    same = total = 0
    for seed in (1, 2, 3):
        theta = np.array([[float(m.parameters[p].val)] for p in m.get_pnames()]) * np.exp(
            0.3 * np.random.RandomState(seed).standard_normal((P, W)))
        y0 = np.repeat(np.array([[float(m.istates[s])] for s in m._snames]), W, axis=1)
        walk = np.ones(P, np.uint8)
        seq = rk_ref.mh_run(fp, theta, y0, nits, burnin, walk, rng="philox", seed=seed)
        for depth in (3, 5):
            tree = rk_ref.mh_tree_run(fp, theta, y0, nits, burnin, walk, depth=depth, rng="philox", seed=seed)
            # same decisions = the same parameters up to the proposals' exp/log (numpy in the
            # tree restatement, libm in the sequential one: ~1e-15); a flipped decision moves a
            # parameter by a whole random-walk step (~5 %)
            rel = np.abs(tree["samples"][:, :P] / seq["samples"][:, :P] - 1)
            eq = np.all(rel < 1e-9, axis=(0, 1))
            same += int(eq.sum())
            total += W
    print("same decisions", same, "of", total)
    assert same >= 0.99 * total, (same, total)
