"""ctypes binding of libodelib_amd.so (include/odelib_amd.h).

This is the whole host↔device boundary: plain C pointers and sizes.  The library is
built in-tree (``odelib_amd/csrc/libodelib_amd.so``, see ``__graft_entry__.build``).
There is no CPU fallback anywhere in the package: if the library is missing or no
HIP device is visible, every compute entry point raises ``NativeUnavailable``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ODELIB_AMD_LIB", os.path.join(_HERE, "csrc", "libodelib_amd.so"))

# --- constants mirrored from include/odelib_amd.h -----------------------------------
OE_ABI_VERSION = 6
OE_COMM_ID_BYTES = 128
OE_OK = 0
OE_ERR_ARG, OE_ERR_HIP, OE_ERR_STATE, OE_ERR_UNSUPPORTED, OE_ERR_NOMEM = -1, -2, -3, -4, -5
OE_METHOD_RK4, OE_METHOD_DOPRI5, OE_METHOD_AUTO, OE_METHOD_ROSENBROCK, OE_METHOD_BDF = 0, 1, 2, 3, 4
OE_MODEL_ZERO_I, OE_MODEL_ONE_I, OE_MODEL_TWO_I, OE_MODEL_CHAIN = 0, 1, 2, 3
OE_MODEL_CUSTOM = 1000
OE_STATUS_NONFINITE, OE_STATUS_NEGATIVE, OE_STATUS_MAXSTEP, OE_STATUS_STIFF, OE_STATUS_INTERNAL = 1, 2, 4, 8, 16
OE_HOST_PTRS, OE_ASYNC, OE_NT_STORES, OE_PIPE, OE_HALF_WAVES, OE_NO_XCD_REMAP, OE_NO_TIMING = 1, 2, 4, 8, 16, 64, 128
OE_PIPE_4, OE_PIPE_8, OE_XCD_RANGES, OE_NO_SPLIT, OE_TUNE, OE_PIPE_XCD = 512, 1024, 2048, 4096, 8192, 16384
OE_KERNEL_DIRECT, OE_KERNEL_HALF, OE_KERNEL_PIPE2, OE_KERNEL_PIPE4, OE_KERNEL_PIPE8 = range(5)
OE_KERNEL_PIPE2X, OE_KERNEL_PIPE4X, OE_KERNEL_PIPE8X, OE_KERNEL_OTHER = range(5, 9)
OE_KERNEL_COUNT = 9
KERNEL_NAMES = ("direct", "half", "pipe2", "pipe4", "pipe8", "pipe2x", "pipe4x", "pipe8x", "other")
OE_RNG_REPLAY, OE_RNG_PHILOX, OE_RNG_NUMPY = 0, 1, 2

# every symbol include/odelib_amd.h declares (checked by tests/test_abi.py)
EXPORTED = (
    "oe_abi_version",
    "oe_model_info",
    "oe_model_compile",
    "oe_rtc_check",
    "oe_ctx_create",
    "oe_ctx_destroy",
    "oe_last_error",
    "oe_ctx_set_stream",
    "oe_ctx_use_own_stream",
    "oe_problem_set",
    "oe_integrate",
    "oe_mh_run",
    "oe_numpy_streams",
    "oe_last_kernel_ms",
    "oe_comm_unique_id",
    "oe_comm_init",
    "oe_comm_destroy",
    "oe_comm_last_error",
    "oe_comm_set_stream",
    "oe_allgather_samples",
    "oe_pool_pad",
    "oe_pool_relayout",
    "oe_last_variant",
    "oe_tune_times",
    "oe_last_mh_depth",
)


class NativeUnsupported(RuntimeError):
    """OE_ERR_UNSUPPORTED: the model / method combination is not available (e.g. a stiff
    method for n_states > 32, or for a C body that does not compile for dual numbers)."""


class NativeUnavailable(RuntimeError):
    """The HIP library or a HIP device is missing.  Raised instead of falling back."""


class OEProblem(C.Structure):
    _fields_ = [
        ("model_id", C.c_int32),
        ("n_states", C.c_int32),
        ("n_params", C.c_int32),
        ("n_times", C.c_int32),
        ("times", C.c_void_p),
        ("n_obs", C.c_int32),
        ("obs_tidx", C.c_void_p),
        ("obs_mask", C.c_void_p),
        ("obs_log", C.c_void_p),
        ("obs_logsigma", C.c_void_p),
        ("obs_lin", C.c_void_p),
        ("method", C.c_int32),
        ("rk4_substeps", C.c_int32),
        ("rtol", C.c_double),
        ("atol", C.c_double),
        ("max_steps", C.c_int32),
        ("sstot", C.c_double),
        ("pnum", C.c_int32),
    ]


class OEMHArgs(C.Structure):
    _fields_ = [
        ("n_walkers", C.c_int64),
        ("walker_offset", C.c_int64),
        ("nits", C.c_int32),
        ("burnin", C.c_int32),
        ("rng_mode", C.c_int32),
        ("chunk", C.c_int32),
        ("seed", C.c_uint64),
        ("step_sd", C.c_double),
        ("walk_mask", C.c_void_p),
        ("init_param", C.c_void_p),
        ("replay_dz", C.c_void_p),
        ("replay_u", C.c_void_p),
        ("theta", C.c_void_p),
        ("y0", C.c_void_p),
        ("samples", C.c_void_p),
        ("final_stats", C.c_void_p),
        ("status", C.c_void_p),
        ("numpy_seeds", C.c_void_p),
        ("numpy_prior_draws", C.c_int32),
        ("it_start", C.c_int32),
        ("speculate", C.c_int32),
    ]


_lib = None
_lib_lock = threading.Lock()


def load_library(path: str | None = None):
    """Load (once) and type the shared library.  Importing torch first makes the
    library bind to the same libamdhip64 instance as PyTorch (same SONAME), so
    torch device pointers are valid in it."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise NativeUnavailable(
                f"libodelib_amd.so not found at {p}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C odelib_amd/csrc`")
        try:
            import torch  # noqa: F401  (share the HIP runtime with torch)
        except Exception:  # pragma: no cover - torch is part of the image
            pass
        lib = C.CDLL(p, mode=C.RTLD_GLOBAL)
        vp, i32, i64, u32 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32
        lib.oe_abi_version.restype = C.c_int
        lib.oe_abi_version.argtypes = []
        lib.oe_model_info.restype = C.c_int
        lib.oe_model_info.argtypes = [i32, C.POINTER(i32), C.POINTER(i32)]
        lib.oe_model_compile.restype = C.c_int
        lib.oe_model_compile.argtypes = [vp, C.c_char_p, i32, i32, C.POINTER(i32)]
        lib.oe_rtc_check.restype = C.c_int
        lib.oe_rtc_check.argtypes = [C.c_char_p, i32, i32, C.c_char_p]
        lib.oe_ctx_create.restype = C.c_int
        lib.oe_ctx_create.argtypes = [i32, C.POINTER(vp)]
        lib.oe_ctx_destroy.restype = None
        lib.oe_ctx_destroy.argtypes = [vp]
        lib.oe_last_error.restype = C.c_char_p
        lib.oe_last_error.argtypes = [vp]
        lib.oe_ctx_set_stream.restype = C.c_int
        lib.oe_ctx_set_stream.argtypes = [vp, vp]
        lib.oe_ctx_use_own_stream.restype = C.c_int
        lib.oe_ctx_use_own_stream.argtypes = [vp]
        lib.oe_problem_set.restype = C.c_int
        lib.oe_problem_set.argtypes = [vp, C.POINTER(OEProblem)]
        lib.oe_integrate.restype = C.c_int
        lib.oe_integrate.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, u32]
        lib.oe_mh_run.restype = C.c_int
        lib.oe_mh_run.argtypes = [vp, C.POINTER(OEMHArgs), u32]
        lib.oe_numpy_streams.restype = C.c_int
        lib.oe_numpy_streams.argtypes = [vp, i64, vp, C.c_int32, C.c_int32, vp, C.c_int32, C.c_double, vp, vp]
        lib.oe_last_kernel_ms.restype = C.c_int
        lib.oe_last_kernel_ms.argtypes = [vp, C.POINTER(C.c_double)]
        lib.oe_comm_unique_id.restype = C.c_int
        lib.oe_comm_unique_id.argtypes = [vp, i32]
        lib.oe_comm_init.restype = C.c_int
        lib.oe_comm_init.argtypes = [i32, i32, i32, vp, i32, C.POINTER(vp)]
        lib.oe_comm_destroy.restype = None
        lib.oe_comm_destroy.argtypes = [vp]
        lib.oe_comm_last_error.restype = C.c_char_p
        lib.oe_comm_last_error.argtypes = [vp]
        lib.oe_comm_set_stream.restype = C.c_int
        lib.oe_comm_set_stream.argtypes = [vp, vp]
        lib.oe_allgather_samples.restype = C.c_int
        lib.oe_allgather_samples.argtypes = [vp, i64, vp, vp, vp, u32]
        lib.oe_pool_pad.restype = C.c_int
        lib.oe_pool_pad.argtypes = [i64, vp, i64, i64, vp, vp, u32]
        lib.oe_pool_relayout.restype = C.c_int
        lib.oe_pool_relayout.argtypes = [i32, i64, vp, vp, vp, vp, u32]
        lib.oe_last_variant.restype = C.c_int
        lib.oe_last_variant.argtypes = [vp, C.POINTER(i32)]
        lib.oe_last_mh_depth.restype = C.c_int
        lib.oe_last_mh_depth.argtypes = [vp, C.POINTER(i32)]
        lib.oe_tune_times.restype = C.c_int
        lib.oe_tune_times.argtypes = [vp, C.POINTER(C.c_double), i32]
        if lib.oe_abi_version() != OE_ABI_VERSION:
            raise NativeUnavailable("libodelib_amd.so ABI version mismatch; rebuild it")
        if path is None:
            _lib = lib
        return lib


def model_info(model_id: int, n_states: int = 0) -> tuple[int, int]:
    lib = load_library()
    s, p = C.c_int32(n_states), C.c_int32(0)
    rc = lib.oe_model_info(model_id, C.byref(s), C.byref(p))
    if rc != OE_OK:
        raise ValueError(f"model {model_id} with S={n_states} is not compiled into libodelib_amd.so")
    return s.value, p.value


def rtc_check(rhs_body: str, n_states: int, n_params: int, arch: str = "gfx950"):
    """Compile-only check of a user RHS body with hipRTC (no GPU needed)."""
    lib = load_library()
    rc = lib.oe_rtc_check(rhs_body.encode(), int(n_states), int(n_params), arch.encode())
    if rc != OE_OK:
        raise ValueError(lib.oe_last_error(None).decode())


class Context:
    """One oe_ctx (device, stream, events, device copy of the problem)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = C.c_void_p()
        rc = self.lib.oe_ctx_create(int(device), C.byref(h))
        self._h = h
        if rc != OE_OK:
            msg = self.lib.oe_last_error(h).decode() if h.value else f"error {rc}"
            if h.value:
                self.lib.oe_ctx_destroy(h)
            self._h = C.c_void_p()
            raise NativeUnavailable(f"oe_ctx_create({device}) failed: {msg}")
        self.device = device

    def _check(self, rc: int, what: str):
        if rc != OE_OK:
            cls = NativeUnsupported if rc == OE_ERR_UNSUPPORTED else RuntimeError
            raise cls(f"{what} failed ({rc}): {self.lib.oe_last_error(self._h).decode()}")

    def set_stream(self, stream_handle: int):
        """Launch on this hipStream_t handle (0 = the null stream)."""
        self._check(self.lib.oe_ctx_set_stream(self._h, C.c_void_p(int(stream_handle))), "oe_ctx_set_stream")

    def use_own_stream(self):
        self._check(self.lib.oe_ctx_use_own_stream(self._h), "oe_ctx_use_own_stream")

    def model_compile(self, rhs_body: str, n_states: int, n_params: int) -> int:
        """hipRTC-compile a user RHS for this device; returns its model id."""
        mid = C.c_int32(0)
        self._check(self.lib.oe_model_compile(self._h, rhs_body.encode(), int(n_states), int(n_params),
                                              C.byref(mid)), "oe_model_compile")
        return mid.value

    def problem_set(self, prob: OEProblem):
        self._check(self.lib.oe_problem_set(self._h, C.byref(prob)), "oe_problem_set")

    def integrate(self, n_walkers, y0, theta, traj, chi, ssres, status, flags=0):
        self._check(self.lib.oe_integrate(self._h, int(n_walkers), y0, theta, traj, chi, ssres, status,
                                          int(flags)), "oe_integrate")

    def mh_run(self, args: OEMHArgs, flags=0):
        self._check(self.lib.oe_mh_run(self._h, C.byref(args), int(flags)), "oe_mh_run")

    def numpy_streams(self, n_walkers, seeds, nits, n_params, walk_mask, prior_draws, step_sd, dz, u):
        self._check(self.lib.oe_numpy_streams(self._h, int(n_walkers), seeds, int(nits), int(n_params), walk_mask,
                                              int(prior_draws), float(step_sd), dz, u), "oe_numpy_streams")

    def last_kernel_ms(self) -> float:
        ms = C.c_double(0.0)
        self._check(self.lib.oe_last_kernel_ms(self._h, C.byref(ms)), "oe_last_kernel_ms")
        return ms.value

    def last_variant(self) -> int:
        """OE_KERNEL_* of the last oe_integrate."""
        v = C.c_int32(-1)
        self._check(self.lib.oe_last_variant(self._h, C.byref(v)), "oe_last_variant")
        return v.value

    def last_mh_depth(self) -> int:
        """Iterations per speculative round of the last oe_mh_run (0: sequential)."""
        v = C.c_int32(0)
        self._check(self.lib.oe_last_mh_depth(self._h, C.byref(v)), "oe_last_mh_depth")
        return v.value

    def tune_times(self) -> dict:
        """OE_TUNE's per-kernel ms for the last oe_integrate's shape (measured kernels only)."""
        n = OE_KERNEL_COUNT - 1
        buf = (C.c_double * n)()
        self._check(self.lib.oe_tune_times(self._h, buf, n), "oe_tune_times")
        return {KERNEL_NAMES[k]: buf[k] for k in range(n) if buf[k] == buf[k]}

    def close(self):
        if self._h and self._h.value:
            self.lib.oe_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id() -> bytes:
    """RCCL unique id (128 bytes) for ``Comm``: made on rank 0, handed to every rank."""
    lib = load_library()
    buf = (C.c_uint8 * OE_COMM_ID_BYTES)()
    rc = lib.oe_comm_unique_id(C.cast(buf, C.c_void_p), OE_COMM_ID_BYTES)
    if rc != OE_OK:
        raise RuntimeError(f"oe_comm_unique_id failed ({rc}): {lib.oe_comm_last_error(None).decode()}")
    return bytes(buf)


def pool_pad(rows: int, block_ptr, count: int, cmax: int, padded_ptr, stream: int = 0, flags: int = 0):
    """``oe_pool_pad``: a rank's block [rows][count] padded to [rows][cmax] (device)."""
    lib = load_library()
    rc = lib.oe_pool_pad(int(rows), block_ptr, int(count), int(cmax), padded_ptr, C.c_void_p(int(stream)), int(flags))
    if rc != OE_OK:
        raise RuntimeError(f"oe_pool_pad failed ({rc}): {lib.oe_comm_last_error(None).decode()}")


def pool_relayout(counts, rows: int, gathered_ptr, out_ptr, stream: int = 0, flags: int = 0):
    """``oe_pool_relayout``: the rank-major gathered [n][rows][max(counts)] -> [rows][sum(counts)]
    in global walker order (device)."""
    import numpy as np
    lib = load_library()
    cnt = np.ascontiguousarray(np.asarray(counts, dtype=np.int64))
    rc = lib.oe_pool_relayout(len(cnt), int(rows), C.c_void_p(cnt.ctypes.data), gathered_ptr, out_ptr,
                              C.c_void_p(int(stream)), int(flags))
    if rc != OE_OK:
        raise RuntimeError(f"oe_pool_relayout failed ({rc}): {lib.oe_comm_last_error(None).decode()}")


class Comm:
    """An RCCL communicator of the C-ABI (oe_comm): one rank per GPU, used to pool the
    ranks' posterior sample blocks with ``oe_allgather_samples`` (Framework.py:1037)."""

    def __init__(self, device: int, n_ranks: int, rank: int, unique_id: bytes):
        self.lib = load_library()
        if len(unique_id) != OE_COMM_ID_BYTES:
            raise ValueError("unique_id must be 128 bytes")
        buf = (C.c_uint8 * OE_COMM_ID_BYTES).from_buffer_copy(unique_id)
        h = C.c_void_p()
        rc = self.lib.oe_comm_init(int(device), int(n_ranks), int(rank), C.cast(buf, C.c_void_p), OE_COMM_ID_BYTES,
                                   C.byref(h))
        if rc != OE_OK:
            raise RuntimeError(f"oe_comm_init failed ({rc}): {self.lib.oe_comm_last_error(None).decode()}")
        self._h = h
        self.device, self.n_ranks, self.rank = int(device), int(n_ranks), int(rank)

    def set_stream(self, stream_handle: int):
        self.lib.oe_comm_set_stream(self._h, C.c_void_p(int(stream_handle)))

    def allgather_samples(self, rows: int, block_ptr, counts, out_ptr, flags: int = 0):
        import numpy as np
        cnt = np.ascontiguousarray(np.asarray(counts, dtype=np.int64))
        if len(cnt) != self.n_ranks:
            raise ValueError("counts must have one entry per rank")
        rc = self.lib.oe_allgather_samples(self._h, int(rows), block_ptr, C.c_void_p(cnt.ctypes.data), out_ptr,
                                           int(flags))
        if rc != OE_OK:
            raise RuntimeError(f"oe_allgather_samples failed ({rc}): {self.lib.oe_comm_last_error(self._h).decode()}")

    def close(self):
        if self._h and self._h.value:
            self.lib.oe_comm_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
