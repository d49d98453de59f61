"""The MH kernels' BDF pass with a step size and an order per lane (csrc/bdf.cuh): the
hand-over of 'auto' and method 'bdf' in k_mh / k_mh_tree.

The reference integrates every proposal with its own odeint call (Framework.py:656, one
chain per process at :779-780), so no chain depends on another.  Here:

* a lane's chi / R² / status equal the C restatement's BDF on a group of one
  (oracle/rk_ref.c bdf_group with lane_steps) — chi rtol 1e-12 (ocml vs libm log), status
  bitwise — for the stiff sets, the notebook fit's slow region and demo draws, 1..8 states;
* speculative rounds reproduce the sequential chains bit for bit with stiff proposals;
* a chain's bits do not depend on the chains that share its wavefront.
"""
import numpy as np
import pytest

from helpers import chain_problem, product_model, walker_thetas
from oracle import rk_ref
from test_gpu_stiff import _mixed_thetas

pytestmark = pytest.mark.gpu

# the notebook fit's slow chains (LHS starts): phi ~ 1.5e-5, beta ~ 50; and
# the phi ~ 1e-4 / large-tau draws of test_gpu_stiff
SLOW = [(6.1e-9, 1.5e-5, 50.0, 2.0, 3.0), (9.0e-9, 1.4e-5, 47.0, 1.7, 1e3), (7.5e-9, 1.06e-4, 19.7, 1.9, 2.8),
        (7.5e-9, 1.07e-7, 19.7, 1.9, 99.0), (7.5e-9, 8.8e-5, 415.0, 1.9, 218.0)]


def _thetas(name, W, seed=0):
    theta = _mixed_thetas(name, W, [w for w in (1, 5, 9, 33, 64) if w < W] or [0], seed=seed)
    if name == "two_i":
        for j, th in enumerate(SLOW):
            w = (11 + 7 * j) % W
            theta[:, w] = th
    return theta


def _a_priori(m, theta):
    """one MH call with nits = 1: the a-priori fit of every chain (Samplers.py:88-91)"""
    W = theta.shape[1]
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    r = m.engine().mh_run(theta, y0, nits=1, burnin=0, walk_mask=np.ones(theta.shape[0], np.uint8))
    return y0, r["final"].cpu().numpy(), r["status"].cpu().numpy()


@pytest.mark.parametrize("method", ["auto", "bdf"])
@pytest.mark.parametrize("name,W", [("two_i", 70), ("two_i", 1), ("one_i", 66), ("zero_i", 40)])
def test_lane_bdf_vs_c_restatement(method, name, W):
    m = product_model(name, method=method)
    theta = _thetas(name, W)
    y0, fin, st = _a_priori(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta, trajectory=False, lane=True)
    np.testing.assert_allclose(fin[0], ref["chi"], rtol=1e-12)
    np.testing.assert_allclose(fin[1], 1.0 - ref["ssres"] / m.fit_problem().sstot, rtol=1e-12)
    assert np.array_equal(st, ref["status"])
    if method == "auto" and name == "two_i" and W > 1:
        assert (st & 8).sum() >= 5  # handed to BDF at their own eviction points


@pytest.mark.parametrize("n", [5, 6, 8])
@pytest.mark.parametrize("method", ["auto", "bdf"])
def test_lane_bdf_chain_models_vs_c_restatement(n, method):
    """The register path's widest models (the difference table in LDS, the LU in registers)."""
    m = chain_problem(n, method=method)
    W = 70
    theta = _mixed_thetas("two_i", W, [3, 64, 69])
    y0, fin, st = _a_priori(m, theta)
    ref = rk_ref.integrate(m.fit_problem(), y0, theta, trajectory=False, lane=True)
    np.testing.assert_allclose(fin[0], ref["chi"], rtol=1e-12)
    assert np.array_equal(st, ref["status"])


@pytest.mark.parametrize("method", ["auto", "bdf"])
def test_stiff_speculative_chains_are_the_sequential_chains(method):
    """Speculative rounds whose proposals are stiff (the stiff sets, the notebook fit's slow
    region): the chains kept are the sequential chains, every output bit for bit."""
    m = product_model("two_i", method=method)
    W = 24
    theta = _thetas("two_i", W, seed=3)
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    walk = np.ones(5, np.uint8)
    kw = dict(nits=14, burnin=4, walk_mask=walk, rng="philox", seed=21)
    eng = m.engine()
    seq = eng.mh_run(theta, y0, **kw)
    spec = eng.mh_run(theta, y0, speculate="auto", **kw)
    assert eng.last_mh_depth() >= 6
    for k in ("samples", "theta", "y0", "final", "status"):
        assert np.array_equal(seq[k].cpu().numpy(), spec[k].cpu().numpy(), equal_nan=True), k
    if method == "auto":
        assert (seq["status"].cpu().numpy() & 8).any()
    for d in (2, 3):
        s2 = eng.mh_run(theta, y0, speculate=d, **kw)
        assert np.array_equal(seq["samples"].cpu().numpy(), s2["samples"].cpu().numpy(), equal_nan=True), d


@pytest.mark.parametrize("method", ["auto", "bdf"])
def test_stiff_mh_chains_do_not_depend_on_their_wave_mates(method):
    """The same chains (same global ids, hence the same Philox draws) run among 70 chains and
    among 17: chains 0..16, stiff ones included, are bitwise the same."""
    m = product_model("two_i", method=method)
    theta = _thetas("two_i", 70, seed=4)
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], 70, axis=1)
    walk = np.ones(5, np.uint8)
    kw = dict(nits=8, burnin=2, walk_mask=walk, rng="philox", seed=2)
    eng = m.engine()
    big = eng.mh_run(theta, y0, **kw)
    small = eng.mh_run(theta[:, :17].copy(), y0[:, :17].copy(), **kw)
    for k in ("samples", "theta", "y0", "final", "status"):
        assert np.array_equal(small[k].cpu().numpy(), big[k].cpu().numpy()[..., :17], equal_nan=True), k
    if method == "auto":
        assert (small["status"].cpu().numpy() & 8).any()
