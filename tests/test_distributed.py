"""world_size-2 gloo tests of the sharding + posterior all-gather (CPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from odelib_amd.distributed import allgather_walkers, pooled_rawstats, shard, sharded_mh


def test_shard_partitions():
    for W in (1, 7, 64, 65536, 1048577):
        for world in (1, 2, 3, 8):
            spans = [shard(W, r, world) for r in range(world)]
            assert spans[0][0] == 0
            for (o1, c1), (o2, _) in zip(spans, spans[1:]):
                assert o1 + c1 == o2
            assert sum(c for _, c in spans) == W
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _OracleEngine:
    """Stands in for the device engine in a CPU test: the C restatement of oe_mh_run."""

    def __init__(self, fp):
        self.fp = fp

    def mh_run(self, theta, y0, nits, burnin, walk_mask, init_param=None, rng="philox", seed=0, step_sd=0.05,
               walker_offset=0, **_):
        from oracle import rk_ref
        r = rk_ref.mh_run(self.fp, np.asarray(theta), np.asarray(y0), nits, burnin, walk_mask, init_param,
                          rng=rng, seed=seed, step_sd=step_sd, walker_offset=walker_offset)
        return {k: torch.as_tensor(v) for k, v in r.items()}


def _worker(rank, world, port, W, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # 1. uneven all-gather in global order
        off, cnt = shard(W, rank, world)
        blk = torch.arange(off, off + cnt, dtype=torch.float64).repeat(3, 2, 1)
        g = allgather_walkers(blk, W)
        assert torch.equal(g[1, 1], torch.arange(W, dtype=torch.float64))
        # 2. sharded MH == unsharded MH (Philox keyed by global walker id)
        from helpers import product_model
        m = product_model("two_i", method="rk4")
        fp = m.fit_problem()
        P = 5
        theta = np.repeat(np.array([float(m.parameters[p].val) for p in m.get_pnames()])[:, None], W, axis=1)
        y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
        pooled, _ = sharded_mh(_OracleEngine(fp), theta, y0, nits=6, burnin=2, walk_mask=np.ones(P, np.uint8),
                               seed=11)
        # 3. rawstats of the pooled posterior from all-reduced sufficient statistics
        off, cnt = shard(W, rank, world)
        med, sd = pooled_rawstats(pooled[..., off:off + cnt], P)
        if rank == 0:
            q.put(pooled.numpy())
            q.put((med, sd))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_sharded_mh_matches_single_process():
    W = 67  # ragged: 34 + 33 walkers, one shard not a multiple of 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, W, q)) for r in range(2)]
    for p in procs:
        p.start()
    pooled = q.get(timeout=240)
    med, sd = q.get(timeout=60)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from helpers import product_model
    from oracle import rk_ref
    m = product_model("two_i", method="rk4")
    theta = np.repeat(np.array([float(m.parameters[p].val) for p in m.get_pnames()])[:, None], W, axis=1)
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    ref = rk_ref.mh_run(m.fit_problem(), theta, y0, 6, 2, np.ones(5, np.uint8), rng="philox", seed=11)
    assert np.array_equal(pooled, ref["samples"])
    import pandas as pd
    from odelib_amd.Framework import rawstats
    for j in range(5):  # Framework.py:11-17 on the concatenated posterior column
        m_ref, s_ref = rawstats(pd.Series(pooled[:, j, :].reshape(-1)))
        np.testing.assert_allclose([med[j], sd[j]], [m_ref, s_ref], rtol=1e-12)


def test_collective_watch_names_a_stalled_call_and_exits():
    """bench.py's C4 pooling and barriers run inside distributed.watch: a call that does not
    return within its bound is named on stderr with the rank, and the rank exits 87 instead of
    hanging (a failing first 8-rank RCCL run must be diagnosable from the
    driver's tail alone)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, time; sys.path.insert(0, %r)\n"
            "from odelib_amd.distributed import watch\n"
            "with watch('C4 oe_allgather_samples, timed', 3, 0.5):\n"
            "    pass\n"
            "with watch('C4 barrier after the timed gather', 3, 0.5):\n"
            "    time.sleep(30)\n") % root
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 87, (r.returncode, r.stderr)
    assert "[rank 3" in r.stderr and "C4 oe_allgather_samples, timed: exit" in r.stderr, r.stderr
    assert "C4 barrier after the timed gather: did not return within" in r.stderr, r.stderr
