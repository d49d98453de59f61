"""The C-ABI library loads and exports every symbol include/odelib_amd.h declares
(no compute calls without a GPU)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from helpers import ROOT
from odelib_amd import _native as N

HEADER = os.path.join(ROOT, "include", "odelib_amd.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(oe_[a-z_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert declared_functions() == sorted(N.EXPORTED)


def test_library_exports_every_declared_symbol():
    lib = N.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (oe_\w+)", out))
    assert set(declared_functions()) <= exported


def test_abi_version_and_model_registry():
    lib = N.load_library()
    assert lib.oe_abi_version() == N.OE_ABI_VERSION
    assert N.model_info(N.OE_MODEL_ZERO_I) == (2, 3)
    assert N.model_info(N.OE_MODEL_ONE_I) == (3, 4)
    assert N.model_info(N.OE_MODEL_TWO_I) == (4, 5)
    from odelib_amd.models import CHAIN_SIZES
    for n in CHAIN_SIZES:
        assert N.model_info(N.OE_MODEL_CHAIN, n) == (n, 5)
    with pytest.raises(ValueError):
        N.model_info(N.OE_MODEL_CHAIN, 7)
    with pytest.raises(ValueError):
        N.model_info(42)


def test_errors_are_codes_not_crashes():
    lib = N.load_library()
    assert lib.oe_ctx_create(0, None) == -1  # OE_ERR_ARG
    assert lib.oe_integrate(None, 1, None, None, None, None, None, None, 0) == -3  # OE_ERR_STATE
    assert lib.oe_problem_set(None, None) == -3
    assert lib.oe_mh_run(None, None, 0) == -3
    assert lib.oe_last_error(None) == b"null context"
    ms = C.c_double()
    assert lib.oe_last_kernel_ms(None, C.byref(ms)) == -1
    v = C.c_int32()
    assert lib.oe_last_variant(None, C.byref(v)) == -1
    buf = (C.c_double * 5)()
    assert lib.oe_tune_times(None, buf, 5) == -1
    s, p = C.c_int32(0), C.c_int32(0)
    assert lib.oe_model_info(99, C.byref(s), C.byref(p)) == -4
    # the pooling entry points validate before touching RCCL or the device
    h = C.c_void_p()
    uid = (C.c_uint8 * 128)()
    assert lib.oe_comm_init(0, 0, 0, C.cast(uid, C.c_void_p), 128, C.byref(h)) == -1  # n_ranks < 1
    assert lib.oe_comm_init(0, 2, 2, C.cast(uid, C.c_void_p), 128, C.byref(h)) == -1  # rank out of range
    assert lib.oe_comm_init(0, 1, 0, C.cast(uid, C.c_void_p), 64, C.byref(h)) == -1   # wrong id size
    assert b"rank" in lib.oe_comm_last_error(None)
    assert lib.oe_comm_unique_id(None, 128) == -1
    assert lib.oe_allgather_samples(None, 1, None, None, None, 0) == -1
    assert lib.oe_comm_set_stream(None, None) == -1
    lib.oe_comm_destroy(None)


def test_context_creation_reports_missing_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    with pytest.raises(N.NativeUnavailable, match="no HIP device"):
        N.Context(0)
