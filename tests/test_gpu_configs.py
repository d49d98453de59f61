"""BASELINE.json configs at the sizes and settings bench.py runs them.

* C4 (configs[4]): 1 048 576 two_i walkers sharded over 8 GPUs.  On one GPU the eight
  shards run one after another (walker_offset = r·131 072, Philox keyed by the global
  walker id, the bench's C4 leg and ``distributed.sharded_mh``); they must equal ONE
  1 048 576-walker launch bitwise (integrate and MH), and sampled 64-walker lockstep
  groups must match the C restatement (oracle/rk_ref.c).
* C3 (configs[3]): the 20-state chain at the bench's settings: RK4 with
  rk4_substeps = 1 within rtol 1e-6 / atol 1e-4 of tight odeint (SURVEY §8c's
  20-state RK4 tolerance), rk4_substeps = 3 within rtol = atol = 1e-6 (C restatement over 32
  bench walkers: substeps 1 / 2 / 3 reach 0.44 of the 1e-4 budget / 1.09 and 0.21 of the 1e-6 one).
"""
import numpy as np
import pytest

from helpers import chain_problem, product_model
from odelib_amd.distributed import shard
from odelib_amd.models import chain_rhs
from oracle import cpu_ref, rk_ref

pytestmark = pytest.mark.gpu

THETA_STAR = [7.475e-9, 1.069e-7, 19.73, 1.934, 2.799]  # bench.py's synthetic walkers
C4_W, C4_RANKS = 1 << 20, 8


def _bench_walkers(W):
    z = np.random.RandomState(0).standard_normal((5, W))
    return np.asarray(THETA_STAR)[:, None] * np.exp(0.05 * z)


def test_c4_eight_shards_equal_one_launch_and_c_restatement():
    import torch
    m = product_model("two_i", method="rk4", priors=False)
    fp = m.fit_problem()
    eng = m.engine()
    dev = eng.dev
    theta_h = _bench_walkers(C4_W)
    y0_h = np.repeat(np.asarray(m.get_inits(), float)[:, None], C4_W, axis=1)
    theta = torch.as_tensor(theta_h, device=dev)
    y0 = torch.as_tensor(y0_h, device=dev)
    P = theta.shape[0]
    walk = np.ones(P, np.uint8)
    nits, burnin, seed = 12, 6, 4242
    groups = (0, 8191, 12345, C4_W // 64 - 1)  # lockstep groups checked against the C oracle

    # (1) trajectory integrate: one launch vs eight shards
    full = eng.integrate(y0, theta, trajectory=True)
    for g in groups:
        sl = slice(64 * g, 64 * g + 64)
        ref = rk_ref.integrate(fp, y0_h[:, sl].copy(), theta_h[:, sl].copy())
        assert np.array_equal(full["traj"][:, :, sl].cpu().numpy(), ref["traj"]), g
        np.testing.assert_allclose(full["chi"][sl].cpu().numpy(), ref["chi"], rtol=1e-12)
    for r in range(C4_RANKS):
        off, cnt = shard(C4_W, r, C4_RANKS)
        assert cnt == C4_W // C4_RANKS
        part = eng.integrate(y0[:, off:off + cnt], theta[:, off:off + cnt], trajectory=True)
        assert torch.equal(part["traj"], full["traj"][:, :, off:off + cnt]), r
        for k in ("chi", "ssres", "status"):
            assert torch.equal(part[k], full[k][off:off + cnt]), (r, k)
        del part
    assert bool(torch.isfinite(full["chi"]).all()) and int(full["status"].abs().sum()) == 0
    del full
    torch.cuda.empty_cache()

    # (2) Metropolis–Hastings, Philox keyed by the global walker id
    one = eng.mh_run(theta, y0, nits=nits, burnin=burnin, walk_mask=walk, rng="philox", seed=seed)
    for r in range(C4_RANKS):
        off, cnt = shard(C4_W, r, C4_RANKS)
        sh = eng.mh_run(theta[:, off:off + cnt], y0[:, off:off + cnt], nits=nits, burnin=burnin, walk_mask=walk,
                        rng="philox", seed=seed, walker_offset=off)
        assert torch.equal(sh["samples"], one["samples"][..., off:off + cnt]), r
        for k in ("theta", "y0", "final", "status"):
            assert torch.equal(sh[k], one[k][..., off:off + cnt]), (r, k)
        del sh
    for g in groups:
        sl = slice(64 * g, 64 * g + 64)
        ref = rk_ref.mh_run(fp, theta_h[:, sl], y0_h[:, sl], nits, burnin, walk, rng="philox", seed=seed,
                            walker_offset=64 * g)
        np.testing.assert_allclose(one["samples"][..., sl].cpu().numpy(), ref["samples"], rtol=1e-11)
        np.testing.assert_allclose(one["final"][:, sl].cpu().numpy(), ref["final"], rtol=1e-11)
    # the posterior block one rank all-gathers: [kept][P+5][W/8]
    assert tuple(one["samples"].shape) == (nits - 1 - burnin, P + 5, C4_W)


@pytest.mark.parametrize("substeps,atol", [(1, 1e-4), (3, 1e-6)])
def test_c3_rk4_bench_accuracy(substeps, atol):
    """The C3 line's RK4 accuracy, at the bench's size and draws: walkers of the
    262 144-walker launch against tight odeint (rtol = atol = 1e-13)."""
    W = 262144
    m = chain_problem(20, method="rk4", substeps=substeps)
    theta = _bench_walkers(W)
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    out = m.engine().integrate(y0, theta, trajectory=True)
    sel = (0, 1, 77777, W // 2, W - 1)
    got = {w: out["traj"][:, :, w].cpu().numpy() for w in sel}
    assert bool(np.isfinite(out["chi"].cpu().numpy()).all())
    del out
    worst = 0.0
    for w in sel:
        tight = cpu_ref.odeint_traj(chain_rhs(20), y0[:, w], m.times, theta[:, w], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(got[w], tight, rtol=1e-6, atol=atol)
        worst = max(worst, float(np.max(np.abs(got[w] - tight) / (atol + 1e-6 * np.abs(tight)))))
    print(f"C3 rk4_substeps={substeps}: worst error {worst:.3f} of the rtol 1e-6 / atol {atol:g} budget")
