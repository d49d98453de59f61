"""The RCCL ("nccl" backend) code path of the posterior pooling on one GPU.

The multi-GPU runs (bench.py under torchrun, N = 2..8) pool posterior blocks with
``all_gather_into_tensor`` on device tensors and reduce ``rawstats`` sufficient
statistics with ``all_reduce``; the CPU tests cover the same functions over gloo.  Two
ranks cannot share one GPU under RCCL, so this runs a world-size-1 RCCL group in a child
process: the device engine's sharded MH, the RCCL all-gather and the pooled rawstats
must equal the single-process results exactly.
"""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent(r"""
    import os, sys
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.environ["ROOT"], "tests"))
    sys.path.insert(0, os.environ["ROOT"])
    from helpers import product_model
    from odelib_amd.distributed import allgather_walkers, pooled_rawstats, sharded_mh
    from odelib_amd.Framework import rawstats
    import pandas as pd

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        m = product_model("two_i", method="rk4")
        eng = m.engine()
        P = len(m.get_pnames())
        W = 333
        theta = np.repeat(np.array([float(m.parameters[p].val) for p in m.get_pnames()])[:, None], W, axis=1)
        theta = theta * np.exp(0.02 * np.random.RandomState(3).standard_normal(theta.shape))
        y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
        th = torch.as_tensor(theta, device=dev)
        yy = torch.as_tensor(y0, device=dev)
        walk = np.ones(P, np.uint8)
        pooled, r = sharded_mh(eng, th, yy, nits=12, burnin=4, walk_mask=walk, seed=5)
        ref = eng.mh_run(th, yy, nits=12, burnin=4, walk_mask=walk, rng="philox", seed=5)
        assert pooled.device.type == "cuda"
        assert torch.equal(pooled, ref["samples"])
        # the all-gather itself, with a ragged walker axis
        blk = torch.arange(W, dtype=torch.float64, device=dev).repeat(2, 1)
        assert torch.equal(allgather_walkers(blk, W), blk)
        # pooled rawstats over RCCL == rawstats of the same posterior (Framework.py:11-17)
        med, std = pooled_rawstats(ref["samples"], P)
        s = ref["samples"].cpu().numpy()
        for j in range(P):
            rm, rs = rawstats(pd.Series(s[:, j, :].ravel()))
            np.testing.assert_allclose(med[j], rm, rtol=1e-12)
            np.testing.assert_allclose(std[j], rs, rtol=1e-9)
        print("NCCL OK")
    finally:
        dist.destroy_process_group()
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_rccl_world1_pooling_equals_single_process():
    env = dict(os.environ, ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0 and "NCCL OK" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
