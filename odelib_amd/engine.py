"""Batched engine: device-resident walkers over the C-ABI.

``FitProblem`` is the host description of one fit (what ``ModelFramework.__init__``
derives from the data, ODElib/Framework.py:226-258); ``Engine`` owns an ``oe_ctx``
with that problem uploaded and runs

* ``integrate``  — W walkers through ``oe_integrate`` (Framework.py:622-697 batched):
  trajectory ``[T][S][W]``, fused chi / R² residual, status;
* ``mh_run``     — W independent Metropolis–Hastings chains through ``oe_mh_run``
  (Statistics/Samplers.py:53-174 batched, one chain per walker).

Tensors are torch tensors on ``cuda:<device>`` (PyTorch provides device memory and the
stream); the arithmetic happens in the HIP kernels only.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _native as N

METHODS = {"rk4": N.OE_METHOD_RK4, "dopri5": N.OE_METHOD_DOPRI5, "auto": N.OE_METHOD_AUTO,
           "rosenbrock": N.OE_METHOD_ROSENBROCK, "bdf": N.OE_METHOD_BDF}
ODEINT_TOL = 1.49012e-8  # scipy.integrate.odeint default rtol/atol (Framework.py:656)
# widest model for which a defaulted method 'auto' stays 'auto' (the register-resident
# stiff path, ode_kernels.cuh kStiffRegS); wider models default to 'dopri5'
AUTO_DEFAULT_MAX_STATES = 8


@dataclass
class FitProblem:
    """Wave-uniform inputs of the fused integrate+likelihood kernel."""
    model_id: int
    n_states: int
    n_params: int
    times: np.ndarray                       # [T] float64
    obs_tidx: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    obs_mask: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint64))
    obs_log: np.ndarray = field(default_factory=lambda: np.zeros(0))
    obs_logsigma: np.ndarray = field(default_factory=lambda: np.zeros(0))
    obs_lin: np.ndarray = field(default_factory=lambda: np.zeros(0))
    sstot: float = 1.0
    pnum: int = 0
    method: str = "rk4"
    rk4_substeps: int = 1
    rtol: float = ODEINT_TOL
    atol: float = ODEINT_TOL
    max_steps: int = 500
    custom_source: str | None = None        # user RHS body for hipRTC (model_id ignored)
    auto_fallback: bool = False             # method 'auto' was a default: use 'dopri5' where
                                            # the stiff methods are unavailable (S > 32, C body
                                            # without a dual-number instantiation) or slow
                                            # (S > AUTO_DEFAULT_MAX_STATES)

    def __post_init__(self):
        self.times = np.ascontiguousarray(self.times, dtype=np.float64)
        self.obs_tidx = np.ascontiguousarray(self.obs_tidx, dtype=np.int32)
        self.obs_mask = np.ascontiguousarray(self.obs_mask, dtype=np.uint64)
        self.obs_log = np.ascontiguousarray(self.obs_log, dtype=np.float64)
        self.obs_logsigma = np.ascontiguousarray(self.obs_logsigma, dtype=np.float64)
        self.obs_lin = np.ascontiguousarray(self.obs_lin, dtype=np.float64)
        n = len(self.obs_tidx)
        for a in (self.obs_mask, self.obs_log, self.obs_logsigma, self.obs_lin):
            if len(a) != n:
                raise ValueError("observation arrays must have equal length")
        if self.method not in METHODS:
            raise ValueError(f"method must be one of {sorted(METHODS)}")

    @property
    def n_times(self) -> int:
        return len(self.times)

    @property
    def n_obs(self) -> int:
        return len(self.obs_tidx)

    def to_c(self) -> N.OEProblem:
        p = N.OEProblem()
        p.model_id = int(self.model_id)
        p.n_states = int(self.n_states)
        p.n_params = int(self.n_params)
        p.n_times = int(self.n_times)
        p.times = self.times.ctypes.data
        p.n_obs = int(self.n_obs)
        p.obs_tidx = self.obs_tidx.ctypes.data if self.n_obs else None
        p.obs_mask = self.obs_mask.ctypes.data if self.n_obs else None
        p.obs_log = self.obs_log.ctypes.data if self.n_obs else None
        p.obs_logsigma = self.obs_logsigma.ctypes.data if self.n_obs else None
        p.obs_lin = self.obs_lin.ctypes.data if self.n_obs else None
        p.method = METHODS[self.method]
        p.rk4_substeps = int(self.rk4_substeps)
        p.rtol = float(self.rtol)
        p.atol = float(self.atol)
        p.max_steps = int(self.max_steps)
        p.sstot = float(self.sstot)
        p.pnum = int(self.pnum)
        return p


def _torch():
    import torch
    return torch


def _row_digest(a, k: int) -> str:
    """blake2b of row ``k`` of a replay stream (numpy array or tensor on any device)."""
    import hashlib
    r = a[k]
    r = r.detach().cpu().numpy() if hasattr(r, "detach") else np.asarray(r)
    return hashlib.blake2b(np.ascontiguousarray(r, dtype=np.float64).tobytes(), digest_size=16).hexdigest()


def rng_record(rng, seed, walker_offset, step_sd, walk_mask, burnin, prior_draws=0, replay=None, nits=0):
    """What a chain's random draws depend on, saved with a checkpoint (``checkpoint.save``)
    and checked when the chains are resumed (``check_resume``).  Replay streams are
    identified by digests of their first and last used rows."""
    rec = {"rng": str(rng), "seed": int(seed) & 0xFFFFFFFFFFFFFFFF, "walker_offset": int(walker_offset),
           "step_sd": float(step_sd), "walk_mask": [int(v) for v in np.asarray(walk_mask).reshape(-1)],
           "burnin": int(burnin), "prior_draws": int(prior_draws) if rng == "numpy" else 0}
    n = int(nits) - 1
    if rng == "replay" and replay is not None and n > 0:
        rec["replay_rows"] = [0, n - 1]
        rec["replay_digest"] = [_row_digest(replay[0], 0), _row_digest(replay[1], 0),
                                _row_digest(replay[0], n - 1), _row_digest(replay[1], n - 1)]
    return rec


def check_resume(resume, rec, numpy_seeds=None, allow_unverified=False):
    """Raise ValueError unless resuming ``resume`` with the draws described by ``rec``
    (``rng_record`` of the resuming call) continues the checkpointed chains exactly as
    one uninterrupted run would.  Returns the numpy seeds to use (the call's, else the
    checkpoint's).  A checkpoint written before random-stream records existed cannot be
    checked: it is refused unless ``allow_unverified=True`` (then resumed with a warning,
    on the caller's word that the draws are the original ones)."""
    old = resume.get("rng_state")
    if old is None:
        if not allow_unverified:
            raise ValueError("the checkpoint records no random-stream state (written by an older version); "
                             "cannot verify that resuming reproduces one uninterrupted run — pass "
                             "allow_unverified=True to resume it with the draws given")
        import warnings
        warnings.warn("resuming a checkpoint without a random-stream record: the draws are not verified")
        return numpy_seeds if numpy_seeds is not None else resume.get("numpy_seeds")
    for k in ("rng", "step_sd", "walk_mask", "burnin"):
        if old.get(k) != rec.get(k):
            raise ValueError(f"resume: {k}={rec.get(k)!r} differs from the checkpoint's {old.get(k)!r}")
    if rec["rng"] == "philox":
        for k in ("seed", "walker_offset"):
            if old[k] != rec[k]:
                raise ValueError(f"resume: philox {k}={rec[k]} differs from the checkpoint's {old[k]}")
    saved_seeds = resume.get("numpy_seeds")
    if rec["rng"] == "numpy":
        if old["prior_draws"] != rec["prior_draws"]:
            raise ValueError(f"resume: prior_draws={rec['prior_draws']} differs from the checkpoint's "
                             f"{old['prior_draws']}")
        if numpy_seeds is None:
            numpy_seeds = saved_seeds
        elif saved_seeds is not None and not np.array_equal(np.asarray(numpy_seeds, np.int64),
                                                            np.asarray(saved_seeds, np.int64)):
            raise ValueError("resume: numpy_seeds differ from the checkpoint's")
    if rec["rng"] == "replay" and "replay_digest" in old:
        if "replay_digest" not in rec:
            raise ValueError("resume: rng='replay' needs the replay streams")
        # rows the checkpointed run consumed must be the same rows in the resuming streams
        first, last = old["replay_rows"]
        if rec.get("_replay") is not None:
            dz, u = rec["_replay"]
            if len(dz) <= last or len(u) <= last:
                raise ValueError("resume: replay streams are shorter than the checkpointed run")
            got = [_row_digest(dz, first), _row_digest(u, first), _row_digest(dz, last), _row_digest(u, last)]
            if got != old["replay_digest"]:
                raise ValueError("resume: replay streams differ from the ones the checkpointed run used")
    return numpy_seeds


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class Engine:
    """A device context with one FitProblem uploaded."""

    def __init__(self, problem: FitProblem, device: int = 0, use_torch_stream: bool = True):
        torch = _torch()
        if not torch.cuda.is_available():
            raise N.NativeUnavailable("no HIP device visible to torch; the engine has no CPU path")
        self.torch = torch
        self.device = int(device)
        self.dev = torch.device("cuda", self.device)
        self.ctx = N.Context(self.device)
        self.use_torch_stream = use_torch_stream
        self.problem = None
        self.key = None
        self.set_problem(problem)

    # -- problem ---------------------------------------------------------------------------
    def set_problem(self, problem: FitProblem, key=None):
        """Upload ``problem``; ``key`` is an owner's label for it (``ModelFramework``
        compares it before reusing a shared engine) and is cleared by an unlabelled upload."""
        self.key = None
        self._sync_stream()
        c = problem.to_c()
        if problem.custom_source is not None:  # compiled once per context (cached by source)
            c.model_id = self.ctx.model_compile(problem.custom_source, problem.n_states, problem.n_params)
        if problem.method == "auto" and problem.auto_fallback and problem.n_states > AUTO_DEFAULT_MAX_STATES:
            # a defaulted 'auto' on a wide model: the MH kernel's stiff redo there keeps
            # its matrices in private memory (~20x slower per stiff walker than the
            # register path; the batched integrate uses one wave per stiff walker), so the
            # default stays the non-stiff integrator; method='auto' asks for it
            problem.method = "dopri5"
            c.method = METHODS["dopri5"]
        try:
            self.ctx.problem_set(c)
        except N.NativeUnsupported:
            if not (problem.method == "auto" and problem.auto_fallback):
                raise
            problem.method = "dopri5"
            c.method = METHODS["dopri5"]
            self.ctx.problem_set(c)
        self.problem = problem
        self.key = key

    def _sync_stream(self):
        if self.use_torch_stream:
            s = self.torch.cuda.current_stream(self.dev)
            self.ctx.set_stream(s.cuda_stream)

    # -- helpers -----------------------------------------------------------------------------
    def _dev(self, a, shape, dtype=None):
        torch = self.torch
        dtype = dtype or torch.float64
        if isinstance(a, torch.Tensor):
            t = a.to(device=self.dev, dtype=dtype)
        else:
            t = torch.as_tensor(np.asarray(a), dtype=dtype, device=self.dev)
        t = t.contiguous()
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"expected shape {tuple(shape)}, got {tuple(t.shape)}")
        return t

    def empty_traj(self, n_walkers: int):
        pb = self.problem
        return self.torch.empty((pb.n_times, pb.n_states, n_walkers), dtype=self.torch.float64, device=self.dev)

    # -- batched integrate -------------------------------------------------------------------
    def integrate(self, y0, theta, trajectory: bool = True, traj_out=None, nt_stores: bool = True,
                  sync: bool = True, pipelined=None, half_waves: bool = False,
                  xcd_remap=True, timing: bool = True, split: bool = True, kernel=None):
        """y0 [S][W], theta [P][W] → dict(traj [T][S][W] | None, chi [W], ssres [W], status [W]).

        ``pipelined=True`` (or 2, 4, 8: store waves per 4 compute waves) selects the
        opt-in producer/consumer RK4 trajectory kernel (same results).  ``half_waves=True`` runs
        32 walkers per wavefront (twice the waves; same results).
        ``xcd_remap=False`` keeps blockIdx-order walker blocks instead of runs of 512
        walkers dealt to the XCDs in turn; ``xcd_remap="ranges"`` gives each XCD one
        contiguous walker range (same results either way).  ``timing=False`` records no library events
        around the launch (``last_kernel_ms`` is then unavailable for this call).
        ``split=False`` keeps one lane per walker in DOPRI5 for the models whose kernel
        otherwise spreads a walker over 2 or 4 lanes (OE_NO_SPLIT; the wide built-in chain).
        ``kernel`` names the RK4 trajectory kernel instead: "direct" (the library's default
        rule: 32 walkers per wave for 5+ states at <= 1 wave per SIMD), "half", "pipe2",
        "pipe4", "pipe8" (blockIdx order), "pipe2x", "pipe4x", "pipe8x" (XCD runs), or "auto" (OE_TUNE: the library measures the available ones for
        this shape on the first call and keeps the fastest; ``last_variant()`` says which
        ran).  All of them produce the same bits."""
        torch = self.torch
        if kernel is not None:
            if kernel not in ("auto",) + N.KERNEL_NAMES[:-1]:
                raise ValueError(f"unknown kernel {kernel!r}")
            if kernel != "auto":
                pipelined = {"direct": False, "half": False, "pipe2": 2, "pipe4": 4, "pipe8": 8}[kernel.rstrip("x")]
                half_waves = (kernel == "half")
        pb = self.problem
        theta_t = theta if isinstance(theta, torch.Tensor) else np.asarray(theta)
        W = int(theta_t.shape[1])
        y0 = self._dev(y0, (pb.n_states, W))
        theta = self._dev(theta, (pb.n_params, W))
        traj = None
        if trajectory:
            traj = traj_out if traj_out is not None else self.empty_traj(W)
            if tuple(traj.shape) != (pb.n_times, pb.n_states, W) or traj.dtype != torch.float64 \
                    or not traj.is_contiguous() or traj.device != self.dev:
                raise ValueError("traj_out must be a contiguous float64 [T][S][W] tensor on the engine device")
        chi = torch.empty(W, dtype=torch.float64, device=self.dev)
        ssres = torch.empty(W, dtype=torch.float64, device=self.dev)
        status = torch.empty(W, dtype=torch.int32, device=self.dev)
        self._sync_stream()
        pipe = {None: 0, False: 0, True: N.OE_PIPE, 2: N.OE_PIPE, 4: N.OE_PIPE_4, 8: N.OE_PIPE_8}[pipelined]
        flags = N.OE_ASYNC | (N.OE_NT_STORES if nt_stores else 0) | pipe \
            | (N.OE_HALF_WAVES if half_waves else 0) \
            | (N.OE_XCD_RANGES if xcd_remap == "ranges" else 0 if xcd_remap else N.OE_NO_XCD_REMAP) \
            | (0 if timing else N.OE_NO_TIMING) | (0 if split else N.OE_NO_SPLIT) \
            | (N.OE_TUNE if kernel == "auto" else 0) \
            | (N.OE_PIPE_XCD if kernel is not None and kernel.endswith("x") else 0)
        self.ctx.integrate(W, _ptr(y0), _ptr(theta), _ptr(traj), _ptr(chi), _ptr(ssres), _ptr(status), flags)
        if sync:
            torch.cuda.synchronize(self.dev)
        return {"traj": traj, "chi": chi, "ssres": ssres, "status": status}

    def last_kernel_ms(self) -> float:
        return self.ctx.last_kernel_ms()

    def last_variant(self) -> str:
        """Name of the kernel the last ``integrate`` launched ("direct", "half", "pipe2",
        "pipe4", "pipe8", "pipe2x", "pipe4x", "pipe8x"; "other" for DOPRI5, the stiff
        methods, no trajectory)."""
        return N.KERNEL_NAMES[self.ctx.last_variant()]

    def last_mh_depth(self) -> int:
        """Iterations per speculative round of the last ``mh_run`` (0: one per step)."""
        return self.ctx.last_mh_depth()

    def tune_times(self) -> dict:
        """What ``kernel="auto"`` measured for the last ``integrate``'s shape: ms per kernel."""
        return self.ctx.tune_times()

    # -- batched Metropolis–Hastings ---------------------------------------------------------
    def numpy_streams(self, seeds, nits: int, walk_mask, prior_draws: int = 0, step_sd: float = 0.05):
        """The reference's per-chain numpy legacy draws, generated on the device
        (``oe_numpy_streams``): dz [nits-1][P][W], u [nits-1][W] — what
        ``odelib_amd.rng.legacy_replay_streams`` computes on the host."""
        torch = self.torch
        P = self.problem.n_params
        seeds = torch.as_tensor(np.asarray(seeds, dtype=np.int64).astype(np.uint32).view(np.int32),
                                device=self.dev).contiguous()
        W = int(seeds.numel())
        n = max(int(nits) - 1, 0)
        dz = torch.empty((max(n, 1), P, W), dtype=torch.float64, device=self.dev)
        u = torch.empty((max(n, 1), W), dtype=torch.float64, device=self.dev)
        wm = np.ascontiguousarray(np.asarray(walk_mask, dtype=np.uint8).reshape(P))
        self._sync_stream()
        self.ctx.numpy_streams(W, seeds.data_ptr(), int(nits), P, wm.ctypes.data, int(prior_draws), float(step_sd),
                               dz.data_ptr(), u.data_ptr())
        return dz[:n], u[:n]

    def mh_run(self, theta, y0, nits: int, burnin: int, walk_mask, init_param=None, rng: str = "philox",
               seed: int = 0, replay=None, step_sd: float = 0.05, walker_offset: int = 0, chunk: int = 0,
               sync: bool = True, numpy_seeds=None, prior_draws: int = 0, resume=None,
               allow_unverified: bool = False, split: bool = True, speculate=0):
        """Run W chains; returns dict(samples [kept][P+5][W], theta, y0, final [4][W], status).

        rng='replay' takes ``replay=(dz [nits-1][P][W], u [nits-1][W])`` (e.g. from
        ``odelib_amd.rng.legacy_replay_streams``) and reproduces the reference's numpy
        draws; rng='numpy' generates those same draws on the device from ``numpy_seeds``
        [W] (chain random_seed) with ``prior_draws`` prior normals per iteration;
        rng='philox' draws on device, keyed by (seed, walker_offset + w).

        ``resume`` continues a previous run's chains (a result dict of this method, or
        one loaded by ``odelib_amd.checkpoint.load``): its theta, y0, final and status
        are the chain state after iteration ``resume['next_it'] - 1``; iterations
        next_it..nits-1 run with the same draws as one uninterrupted run, and samples
        holds the kept rows from max(next_it, burnin+1) on.  ``allow_unverified`` resumes a
        checkpoint that predates the random-stream record (see ``check_resume``).
        ``split=False``: one lane per chain for the models whose DOPRI5 MH kernel otherwise
        spreads a chain over 2 or 4 lanes (OE_NO_SPLIT).
        ``speculate``: speculative rounds for small ensembles (oe_mh_args.speculate): 0 off,
        "auto" (or -1) the library's depth (off when the chains fill the device), d >= 2
        iterations per round — every proposal the next d decisions can lead to is integrated
        at once and each chain keeps its own path: RK4, and DOPRI5 / ``auto`` / ``bdf`` chains
        of models with <= 8 states, are bitwise those of ``speculate=0`` (every MH lane takes
        its own steps, BDF ones included).  ``last_mh_depth()``
        reports the depth used."""
        torch = self.torch
        pb = self.problem
        P, S = pb.n_params, pb.n_states
        nits = int(nits)
        burnin = int(burnin)
        it_start = 1
        rec = rng_record(rng, seed, walker_offset, step_sd, walk_mask, burnin, prior_draws, replay, nits)
        if resume is not None:
            chk = dict(rec, _replay=replay if rng == "replay" else None)
            numpy_seeds = check_resume(resume, chk, numpy_seeds, allow_unverified=allow_unverified)
            it_start = int(resume["next_it"])
            theta, y0 = resume["theta"], resume["y0"]
        W = int((theta if isinstance(theta, torch.Tensor) else np.asarray(theta)).shape[1])
        theta = self._dev(theta, (P, W)).clone()
        y0 = self._dev(y0, (S, W)).clone()
        kept = max(0, nits - max(it_start, burnin + 1))
        samples = torch.empty((max(kept, 1), P + 5, W), dtype=torch.float64, device=self.dev)
        if resume is not None:
            final = self._dev(resume["final"], (4, W)).clone()
            st = resume["status"]
            status = (st if isinstance(st, torch.Tensor) else torch.as_tensor(np.asarray(st, np.int32))).to(
                device=self.dev, dtype=torch.int32).clone()
        else:
            final = torch.empty((4, W), dtype=torch.float64, device=self.dev)
            status = torch.zeros(W, dtype=torch.int32, device=self.dev)
        wm = np.ascontiguousarray(np.asarray(walk_mask, dtype=np.uint8).reshape(P))
        ip = np.full(S, -1, np.int32) if init_param is None else np.ascontiguousarray(
            np.asarray(init_param, dtype=np.int32).reshape(S))
        a = N.OEMHArgs()
        a.n_walkers = W
        a.walker_offset = int(walker_offset)
        a.nits = nits
        a.burnin = burnin
        a.it_start = it_start
        a.chunk = int(chunk)
        a.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        a.step_sd = float(step_sd)
        a.walk_mask = wm.ctypes.data
        a.init_param = ip.ctypes.data
        # "auto" / True: the library's depth rule; an integer (False = 0) is the depth itself, and
        # 0 or 1 means one iteration per step (ints are tested before bools: 1 == True)
        if isinstance(speculate, str):
            if speculate != "auto":
                raise ValueError("speculate must be 'auto', True/False or an integer depth")
            a.speculate = -1
        elif speculate is True:
            a.speculate = -1
        else:
            a.speculate = int(speculate or 0)
        keep = []
        if rng == "replay":
            if replay is None:
                raise ValueError("rng='replay' needs replay=(dz, u)")
            n = max(nits - 1, 0)  # streams may be longer (a run stopped early for a checkpoint)
            dz = self._dev(replay[0][:n], (n, P, W))
            u = self._dev(replay[1][:n], (n, W))
            keep += [dz, u]
            a.rng_mode = N.OE_RNG_REPLAY
            a.replay_dz = dz.data_ptr() if nits > 1 else None
            a.replay_u = u.data_ptr() if nits > 1 else None
        elif rng == "philox":
            a.rng_mode = N.OE_RNG_PHILOX
        elif rng == "numpy":
            if numpy_seeds is None:
                raise ValueError("rng='numpy' needs numpy_seeds")
            sd = torch.as_tensor(np.asarray(numpy_seeds, dtype=np.int64).astype(np.uint32).view(np.int32),
                                 device=self.dev).contiguous()
            if sd.numel() != W:
                raise ValueError("numpy_seeds must have one seed per walker")
            keep.append(sd)
            a.rng_mode = N.OE_RNG_NUMPY
            a.numpy_seeds = sd.data_ptr()
            a.numpy_prior_draws = int(prior_draws)
        else:
            raise ValueError("rng must be 'replay', 'numpy' or 'philox'")
        a.theta = theta.data_ptr()
        a.y0 = y0.data_ptr()
        a.samples = samples.data_ptr()
        a.final_stats = final.data_ptr()
        a.status = status.data_ptr()
        self._sync_stream()
        self.ctx.mh_run(a, N.OE_ASYNC | (0 if split else N.OE_NO_SPLIT))
        if sync:
            torch.cuda.synchronize(self.dev)
        out = {"samples": samples[:kept], "theta": theta, "y0": y0, "final": final, "status": status,
               "next_it": max(nits, it_start), "rng_state": rec, "_keep": keep}
        if rng == "numpy":
            out["numpy_seeds"] = np.asarray(numpy_seeds, dtype=np.int64)
        return out

    def close(self):
        self.ctx.close()
