"""The DOPRI5 trajectory kernel with store waves (k_integrate_dopri5_piped, OE_PIPE with
OE_METHOD_DOPRI5): the dense output at non-observed grid times, the running minimum and the
row stores move to a store wave per compute wave, fed through an LDS slot ring — the same
operations, so trajectories, chi, R² residual and status must equal the direct DOPRI5 kernel
(k_integrate<M, DOPRI5, true, NT>) bit for bit, which the other DOPRI5 tests pin to the C
restatement and to tight odeint."""
import numpy as np
import pytest

from helpers import chain_problem, product_model, walker_thetas

pytestmark = pytest.mark.gpu


def _both(m, theta, nt=True):
    eng = m.engine()
    W = theta.shape[1]
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    a = eng.integrate(y0, theta, trajectory=True, nt_stores=nt)
    b = eng.integrate(y0, theta, trajectory=True, nt_stores=nt, kernel="pipe2")
    return ({k: v.cpu().numpy() for k, v in a.items()}, {k: v.cpu().numpy() for k, v in b.items()})


def _assert_same(a, b):
    for k in ("traj", "chi", "ssres", "status"):
        assert np.array_equal(a[k], b[k], equal_nan=True), k


@pytest.mark.parametrize("W", [65536, 300, 70, 1])
@pytest.mark.parametrize("nt", [True, False])
def test_piped_dopri5_bitwise_two_i(W, nt):
    m = product_model("two_i", method="dopri5")
    theta = walker_thetas("two_i", W, seed=5).T.copy()
    a, b = _both(m, theta, nt)
    _assert_same(a, b)


def test_piped_dopri5_evicted_lanes_and_all_dead_wave():
    """A lane over the step budget (tau = 1e9: evicted, NaN rows, MAXSTEP) in a wave of demo
    draws, and a wave whose only walker is evicted (every row after the eviction NaN, the
    compute wave's early exit through one slot that reaches t = +inf)."""
    m = product_model("two_i", method="dopri5")
    theta = walker_thetas("two_i", 70, seed=2).T.copy()
    theta[4, [3, 66]] = 1e9
    a, b = _both(m, theta)
    assert (a["status"][[3, 66]] & 4).all()
    _assert_same(a, b)
    a, b = _both(m, theta[:, 3:4].copy())
    _assert_same(a, b)


def test_piped_dopri5_all_dead_wave_stays_inside_the_buffer():
    """The all-evicted wave's last slot reaches t = +inf, which the sentinel times[T] equals:
    the store wave must not write a row T.  A canary row after the trajectory stays as it
    was."""
    import torch

    m = product_model("two_i", method="dopri5")
    theta = walker_thetas("two_i", 1, seed=2).T.copy()
    theta[4, 0] = 1e9
    eng = m.engine()
    T, S = eng.problem.n_times, eng.problem.n_states
    y0 = np.asarray(m.get_inits(), float)[:, None].copy()
    for kernel in (None, "pipe2"):
        buf = torch.full((T + 1, S, 1), 12345.0, dtype=torch.float64, device=eng.dev)
        out = eng.integrate(y0, theta, trajectory=True, traj_out=buf[:T], kernel=kernel)
        assert (out["status"].cpu().numpy()[0] & 4), kernel
        assert (buf[T].cpu().numpy() == 12345.0).all(), kernel


@pytest.mark.parametrize("name", ["zero_i", "one_i"])
def test_piped_dopri5_other_models(name):
    m = product_model(name, method="dopri5")
    a, b = _both(m, walker_thetas(name, 200, seed=1).T.copy())
    _assert_same(a, b)


@pytest.mark.parametrize("n", [5, 6])
def test_piped_dopri5_chain_models(n):
    m = chain_problem(n, method="dopri5")
    theta = walker_thetas("two_i", 130, seed=4).T.copy()
    a, b = _both(m, theta)
    _assert_same(a, b)
