"""The MH kernel's integrity checks (debug library, OE_MH_CHECKS): DESIGN.md §3.4.

Round 1 saw the DOPRI5 MH kernel return corrupted chain state once, under heavy SGPR
spilling, after an unrelated integrator change.  Every store of chain state goes through
a buffer descriptor with an in-range lane offset, so a corrupted store needs a corrupted
wave-uniform value: a row pointer carried through the integration, the sample row index,
or a linked-state parameter index.  The debug library checks exactly those on every
iteration (a failed check stores nothing more and sets OE_STATUS_INTERNAL).  Here the MH
parity cases — including the register-heaviest kernels (chain20 RK4, chain20 DOPRI5 on
one lane and split over two, all spilling) — run on the debug library against the C restatement, with no check firing; a self-test
hook proves a check does fire.
"""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEBUG_LIB = os.path.join(ROOT, "odelib_amd", "csrc", "libodelib_amd_debug.so")

CHILD = textwrap.dedent(r"""
    import os, sys
    import numpy as np
    sys.path.insert(0, os.path.join(os.environ["ROOT"], "tests"))
    sys.path.insert(0, os.environ["ROOT"])
    from helpers import chain_problem, product_model
    from odelib_amd import _native as N
    from oracle import rk_ref
    selftest = bool(os.environ.get("OE_MH_CHECK_SELFTEST"))
    cases = [("two_i", "rk4", True), ("chain20", "dopri5", True)] if selftest else [
        ("two_i", "rk4", True), ("two_i", "dopri5", True), ("chain20", "rk4", True), ("chain20", "dopri5", True),
        ("chain20", "dopri5", False), ("one_i_V0", "rk4", True)]
    for spec, method, split in cases:
        if spec == "one_i_V0":
            m = product_model("one_i", method=method, extra_params={"V0": 10981000.0})
            init_param = [-1, -1, 4]
        elif spec.startswith("chain"):
            m = chain_problem(int(spec[5:]), method=method)
            init_param = None
        else:
            m = product_model(spec, method=method)
            init_param = None
        P = len(m.get_pnames())
        W = 130
        theta = np.repeat(np.array([float(m.parameters[p].val) for p in m.get_pnames()])[:, None], W, axis=1)
        theta = theta * np.exp(0.02 * np.random.RandomState(9).standard_normal(theta.shape))
        y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
        walk = np.ones(P, np.uint8)
        walk[2] = 0
        dev = m.engine().mh_run(theta, y0, nits=30, burnin=12, walk_mask=walk, init_param=init_param,
                                rng="philox", seed=77, walker_offset=5, split=split)
        st = dev["status"].cpu().numpy()
        if selftest:
            assert (st & N.OE_STATUS_INTERNAL).all(), st
            print("SELFTEST FIRED", spec, method)
            continue
        assert not (st & N.OE_STATUS_INTERNAL).any(), (spec, method, st)
        ref = rk_ref.mh_run(m.fit_problem(), theta, y0, 30, 12, walk, init_param=init_param, rng="philox",
                            seed=77, walker_offset=5, split=None if split else 1)
        tol = 1e-11 if method == "rk4" else 1e-8
        np.testing.assert_allclose(dev["samples"].cpu().numpy(), ref["samples"], rtol=tol)
        np.testing.assert_allclose(dev["final"].cpu().numpy(), ref["final"], rtol=tol)
        assert np.array_equal(st, ref["status"])
        print("CHECKED", spec, method, "split" if split else "one lane")
    maps = open("/proc/self/maps").read()
    assert "libodelib_amd_debug.so" in maps
    print("DEBUG OK")
""")


def _run(extra_env):
    env = dict(os.environ, ROOT=ROOT, ODELIB_AMD_LIB=DEBUG_LIB, **extra_env)
    return subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=240)


@pytest.mark.gpu
def test_mh_integrity_checks_hold_on_the_debug_library():
    assert os.path.exists(DEBUG_LIB), "build the debug library (make -C odelib_amd/csrc)"
    r = _run({})
    assert r.returncode == 0 and "DEBUG OK" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
    assert r.stdout.count("CHECKED") == 6


@pytest.mark.gpu
def test_mh_integrity_check_fires_on_a_bad_row_bound():
    r = _run({"OE_MH_CHECK_SELFTEST": "1"})
    assert r.returncode == 0 and r.stdout.count("SELFTEST FIRED") == 2, (r.stdout[-3000:], r.stderr[-3000:])
