"""bench.py — walker-timesteps/s of the batched ODE integrate + fused likelihood on MI355X.

Contract (see task README): ``python bench.py --gpus N --steps K --warmup W``.  N > 1 runs
one rank per GPU under torchrun: when ``--gpus N > 1`` is given without ``WORLD_SIZE`` in
the environment, this process starts ``python -m torch.distributed.run --nproc-per-node N
bench.py ...`` as a child (before anything touches the GPU) and exits with its code; a
``WORLD_SIZE`` different from N is refused.  The reported throughput is always the
walkers the ranks actually ran ÷ the max-over-ranks wall time.

One *step* = one batched integrate of the rank's walkers in trajectory mode (writes
traj[T][S][W] fp64, the odeint [T,S] output of ODElib/Framework.py:656, plus the fused
chi / R² residual of :685-706).

Workload (BASELINE.json configs[1]): 4-state SEIV ``two_i``, 65 536
walkers per GPU, fixed-step RK4, t = linspace(0, 3, 1000), y0 = demo data
(S 5 236 900, V 10 981 000), θ_w = θ*·exp(0.05 z_w) with numpy RandomState(0),
observations = demo data (H = S+I1+I2, V).  Walkers shard across ranks by contiguous
global id with no data-path collective ("scaling": "weak").

Legs after the headline (all in the same JSON line):
* ``mcmc``  — device Metropolis–Hastings (RK4, Philox) over the rank's walkers; its FP64
  roofline counts the kernel's fp64 operations with rocprofv3 PMC
  (SQ_INSTS_VALU_{FMA,ADD,MUL}_F64) in a child pass of the same MH call.
* ``other_configs.C4`` — BASELINE.json configs[4]: 1 048 576 walkers sharded over the
  N ranks (131 072 per GPU at N = 8): trajectory integrate, MH (nits = 100) and the ONE
  posterior all-gather (RCCL over xGMI; Framework.py:1037's pd.concat), each timed
  between barriers, max over ranks.
* ``other_configs.C2/C3`` (N = 1 only) — the other single-GPU configs, kernel time.

Timing: W untimed warm-up steps, extended (untimed) to at least --warmup-ms (60 ms) of
launches so the chip's clocks have settled (``warmup_launches`` in the line), then exactly
K back-to-back steps between a barrier + synchronize on both sides; max over ranks.

Roofline: HBM, algorithmic bytes per walker-timestep = 8·S (trajectory store),
kernel time from HIP events recorded on the stream the kernel is launched on.
cpu_baseline: the oracle's scipy-odeint restatement of Framework.py:656-697
(oracle/cpu_ref.py) on the host cores available to this process, bounded sample,
rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

THETA_STAR = [7.475e-9, 1.069e-7, 19.73, 1.934, 2.799]  # twoI posterior medians (notebook:15120-15128)
HBM_PEAK_GBS = 8000.0    # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_VALU_TFS = 78.6     # MI355X FP64 vector spec
C4_WALKERS = 1 << 20     # BASELINE.json configs[4]: 1 048 576 walkers over 8 GPUs
C4_NITS = 100            # posterior block [49][P+5][W/G] per rank
MH_FP64_COUNTERS = ["SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                    "SQ_INSTS_VALU_TRANS_F64"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--warmup-ms", type=float, default=60.0,
                    help="continue the untimed warm-up until this much wall time has passed")
    ap.add_argument("--walkers", type=int, default=65536, help="walkers per GPU")
    ap.add_argument("--model", default="two_i", help="two_i | chain<N>")
    ap.add_argument("--method", default="rk4", choices=["rk4", "dopri5", "auto", "bdf", "rosenbrock"])
    ap.add_argument("--times", type=int, default=1000)
    ap.add_argument("--cached-stores", action="store_true", help="plain (cached) trajectory stores")
    ap.add_argument("--kernel", default="auto", choices=["auto", "direct", "half", "pipe2", "pipe4", "pipe8", "pipe2x", "pipe4x", "pipe8x"],
                    help="RK4 trajectory kernel: auto = the library times the bitwise-identical kernels on "
                         "this device (OE_TUNE, during the warm-up) and keeps the fastest; or a fixed one (A/B)")
    ap.add_argument("--half-waves", action="store_true", help="same as --kernel half")
    ap.add_argument("--xcd", default="runs", choices=["runs", "ranges", "off"],
                    help="walker blocks per XCD: runs of 512 walkers (default), one range, blockIdx order")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline budget (wall seconds)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mcmc-iters", type=int, default=21, help="MCMC leg iterations (0 = skip)")
    ap.add_argument("--mcmc-only", action="store_true",
                    help="run only one MCMC-leg mh_run (the PMC child pass of the MCMC roofline)")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC child passes")
    ap.add_argument("--no-extra-configs", action="store_true", help="skip the C2/C3 kernel timings")
    ap.add_argument("--no-split", action="store_true",
                    help="wide chain models' DOPRI5: one lane per walker instead of the split kernel")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 leg (1 048 576 walkers over the ranks)")
    ap.add_argument("--c4-steps", type=int, default=10, help="C4 leg: timed trajectory integrates")
    ap.add_argument("--comm-timeout", type=float, default=180.0,
                    help="C4 leg: a rank whose communicator set-up, all-gather or barrier has not returned "
                         "after this many seconds names the call on stderr and exits 87 (no hang)")
    ap.add_argument("--pool", default="cabi", choices=["cabi", "torch"],
                    help="C4 posterior pooling: the C-ABI's RCCL communicator (oe_allgather_samples, what "
                         "ODElib binds) or torch.distributed's all_gather_into_tensor")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def relaunch_under_torchrun(n: int) -> int:
    """``--gpus N > 1`` without a torchrun environment: run N ranks as a child
    ``torch.distributed.run`` (this process has not touched the GPU) and return its exit
    code.  Never multiply one process's throughput by N."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__), *sys.argv[1:]]
    print(f"bench.py: --gpus {n} without WORLD_SIZE; launching {n} ranks: {' '.join(cmd)}", file=sys.stderr,
          flush=True)
    return subprocess.run(cmd).returncode


def workload_args(args):
    out = ["--model", args.model, "--method", args.method, "--walkers", str(args.walkers), "--times", str(args.times)]
    if args.cached_stores:
        out.append("--cached-stores")
    return out


def _pmc_dir():
    import tempfile
    return tempfile.mkdtemp(prefix="bench_pmc_", dir=os.path.join(ROOT, "gpurun_out")
                            if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else None)


def _profiler_usable():
    import shutil
    if shutil.which("rocprofv3") is None:
        return "rocprofv3 not found"
    if any(k.startswith("ROCPROF") for k in os.environ):
        # already running under rocprofv3, whose library has initialised the GPU in this
        # process: a child launched from here would be an exec after GPU initialisation
        return "skipped (running under rocprofv3)"
    return None


def pmc_traffic(args):
    """HBM bytes per dispatch of the integrate kernel from two separate rocprofv3 PMC
    passes (FETCH_SIZE, WRITE_SIZE) of this same workload, run as child processes
    before this process touches the GPU.  gfx950 correction: FETCH_SIZE x2
    (MI355X_MICROARCH.md §HBM).  Returns (bytes or None, note)."""
    why = _profiler_usable()
    if why:
        return None, why
    try:
        from tools.profile import pmc_pass
        out = _pmc_dir()
        wl = workload_args(args) + ["--no-pmc"]
        f = pmc_pass(out, "FETCH_SIZE", wl, "k_integrate", 240)
        w = pmc_pass(out, "WRITE_SIZE", wl, "k_integrate", 240)
        # per kernel (with --kernel auto the child runs every candidate while it tunes)
        by = {n: {"bytes": f["by_kernel"][n]["mean"] * 1024 * 2 + w["by_kernel"][n]["mean"] * 1024,
                  "dispatches": f["by_kernel"][n]["dispatches"]}
              for n in f["by_kernel"] if n in w["by_kernel"]}
        return by, "rocprofv3 PMC FETCH_SIZE(x2)+WRITE_SIZE, separate passes, per dispatch of the kernel that ran"
    except BaseException as e:  # never let profiling break the bench line
        return None, f"PMC pass failed: {e!r}"[:200]


def traffic_of(by_kernel, variant, method):
    """The PMC bytes per dispatch of the kernel the timed region ran (by demangled name)."""
    if not by_kernel:
        return None
    meth = {"rk4": 0, "dopri5": 1}[method]
    want = (("k_integrate_rk4_piped<", f", true, {variant[4:].rstrip('x')}>") if variant.startswith("pipe")
            else ("k_integrate<", f", {meth}, true, true>"))
    hits = [v["bytes"] for n, v in by_kernel.items() if all(x in n for x in want)]
    return hits[0] if hits else None


def pmc_mh_flops(args):
    """fp64 operations of ONE MCMC-leg mh_run (the same call the line times), from one
    rocprofv3 PMC pass over a child ``bench.py --mcmc-only``: SQ_INSTS_VALU_*_F64 count
    wave-instructions, so flops = 64 lanes x (2·FMA + ADD + MUL) summed over the k_mh
    dispatches (rocprofv3's TOTAL_64_OPS without the int64 term; every lane of a wave is
    a walker at these walker counts).  Transcendental helper instructions (TRANS_F64:
    rcp/rsq/sqrt approximations inside log/exp) are reported, not counted as flops."""
    why = _profiler_usable()
    if why:
        return None, why
    try:
        from tools.profile import pmc_counts
        base = ["--mcmc-only", "--no-cpu-baseline", "--no-extra-configs", "--no-c4", "--no-pmc",
                "--mcmc-iters", str(args.mcmc_iters)]
        r = pmc_counts(_pmc_dir(), MH_FP64_COUNTERS, workload_args(args), "k_mh", 240, base=base, tag="mh_fp64")
        c = {k: v["sum"] for k, v in r.items()}
        flops = 64.0 * (2.0 * c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"])
        return {"flops": flops, "counters_sum": c, "k_mh_dispatches": r["SQ_INSTS_VALU_FMA_F64"]["dispatches"]}, \
            "rocprofv3 PMC SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F64, one pass, child bench.py --mcmc-only"
    except BaseException as e:  # never let profiling break the bench line
        return None, f"PMC pass failed: {e!r}"[:200]


XCD_ARG = {"runs": True, "ranges": "ranges", "off": False}


def build_problem(model: str, method: str, T: int, rk4_substeps: int = 1):
    """FitProblem for the bench workload (host-side set-up only)."""
    import numpy as np
    import pandas as pd
    from odelib_amd import ModelFramework, parameter
    from odelib_amd.models import BUILTIN, chain_rhs
    df = pd.read_csv(os.path.join(ROOT, "tests", "golden", "demodata.csv")).replace({"virus": "V", "host": "H"})
    if model == "two_i":
        n, ode = 4, BUILTIN["two_i"][3]
    elif model.startswith("chain"):
        n = int(model[5:])
        ode = chain_rhs(n)
    else:
        raise SystemExit(f"unknown bench model {model}")
    snames = ["S"] + [f"I{k}" for k in range(1, n - 1)] + ["V"]
    pn = ["mu", "phi", "beta", "lam", "tau"]
    m = ModelFramework(ODE=ode, parameter_names=pn, state_names=snames, dataframe=df,
                       state_summations={"H": snames[:-1]}, t_steps=T, S=5236900, method=method,
                       rk4_substeps=rk4_substeps, device_model="two_i" if model == "two_i" else "chain",
                       **{p: parameter(init_value=v) for p, v in zip(pn, THETA_STAR)})
    return m, np.asarray(m.get_inits(), float)


def synthetic_walkers(n_total: int, P: int):
    import numpy as np
    z = np.random.RandomState(0).standard_normal((P, n_total))
    return np.asarray(THETA_STAR)[:, None] * np.exp(0.05 * z)


# ------------------------------------------------------------------ CPU baseline (oracle)
def host_cores():
    """CPU cores this process may use: its affinity set, bounded by a cgroup v2 CPU quota
    if one is set (``/sys/fs/cgroup/cpu.max``).  Returns (cores, detail)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(q) // int(per))
    except (OSError, ValueError):
        pass
    cores = min(aff, quota) if quota else aff
    return cores, {"sched_getaffinity": aff, "cgroup_cpu_max_cores": quota, "os_cpu_count": os.cpu_count(),
                   "OMP_NUM_THREADS_env": os.environ.get("OMP_NUM_THREADS")}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_worker(args):
    model, times, wall_budget, theta_cols, y0, tidx, mask, O, Ssig = args
    import numpy as np
    from oracle import cpu_ref
    from odelib_amd.models import BUILTIN, chain_rhs
    ode = BUILTIN["two_i"][3] if model == "two_i" else chain_rhs(int(model[5:]))
    S = len(y0)
    done, t0 = 0, time.perf_counter()
    for th in theta_cols:
        traj = cpu_ref.odeint_traj(ode, y0, times, th)  # Framework.py:656
        # summation + gather at pred_tindex + masked chi (Framework.py:659-697)
        C = np.array([sum(traj[i, s] for s in range(S) if (int(mk) >> s) & 1) for i, mk in zip(tidx, mask)])
        cpu_ref.chi(O, np.log(C), Ssig)
        done += 1
        if time.perf_counter() - t0 > wall_budget:
            break
    return done, time.perf_counter() - t0


def cpu_baseline(model, fp, y0, budget_s, P, procs=None):
    """Oracle (scipy odeint, the reference's integrator) on every host core available to
    this process (``Pool(processes=cores)`` as Framework.py:779); fork-based pool started
    before this process initialises the GPU.  ``procs`` overrides the pool size
    (tools/cpu_scaling.py: does a pool larger than the cgroup quota gain anything?)."""
    import multiprocessing as mp
    cores, detail = host_cores()
    cores = procs or cores
    theta = synthetic_walkers(cores * 16384, P)
    jobs = [(model, fp.times, budget_s, [theta[:, w] for w in range(c, theta.shape[1], cores)], y0,
             fp.obs_tidx, fp.obs_mask, fp.obs_log, fp.obs_logsigma) for c in range(cores)]
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(cores) as pool:
        res = pool.map(_cpu_worker, jobs)
    wall = time.perf_counter() - t0
    walkers = sum(r[0] for r in res)
    T = len(fp.times)
    return {"value": walkers * (T - 1) / wall, "unit": "walker-timesteps/s", "cores": cores, "kind": "port",
            "cores_detail": detail,
            "sample": f"{walkers} walkers x {T - 1} intervals: scipy odeint (LSODA, default tol) + summation + "
                      f"masked chi (oracle/cpu_ref.py), multiprocessing.Pool({cores}) for {wall:.1f} s wall; "
                      f"CPU: {_cpu_model()}"}


NOTEBOOK_PRIORS = {"mu": {"s": 3, "scale": 1e-8}, "phi": {"s": 3, "scale": 1e-8}, "beta": {"s": 1, "scale": 20},
                   "lam": {"s": 2, "scale": .1}, "tau": {"s": 2, "scale": 1}}


def _oracle_mh_model(m):
    """oracle.cpu_ref.Model (the reference's MH loop, Samplers.py:53-174) for the product
    model ``m`` with the notebook's lognorm priors (their pdf/rvs calls are part of the
    reference's iteration cost)."""
    import scipy.stats
    from oracle import cpu_ref
    from odelib_amd.models import BUILTIN
    snames = list(m._snames)
    sidx, out_names, keep, _ = cpu_ref.summation_index(snames, {"H": snames[:-1]})
    params = {p: cpu_ref.Param(float(v), scipy.stats.lognorm, dict(NOTEBOOK_PRIORS[p]))
              for p, v in zip(m.get_pnames(), THETA_STAR)}
    return cpu_ref.Model(BUILTIN["two_i"][3], m.get_pnames(), snames, params, dict(zip(snames, m.get_inits())),
                         m.times, m._pred_tindex, m._obs_logabundance, m._obs_logsigma, sum_index=sidx,
                         sumkeep=keep, out_names=out_names)


_MH_ORACLE = None


def _cpu_mh_worker(args):
    chains, nits = args
    from oracle import cpu_ref
    t0 = time.perf_counter()
    for c in chains:
        _MH_ORACLE.random_seed = c
        cpu_ref.metropolis_hastings(_MH_ORACLE, nits=nits)
    return len(chains) * (nits - 1), time.perf_counter() - t0


def cpu_mcmc_baseline(m, chains=32, nits=101, full_nits=1001):
    """The reference's MCMC for the small-ensemble entries, on the host cores: the
    notebook's ``chains`` chains, each the reference's Metropolis-Hastings loop with
    scipy odeint (oracle/cpu_ref.py), one chain per pool task as Framework.py:779;
    a bounded sample of ``nits`` iterations per chain, scaled to ``full_nits``."""
    import multiprocessing as mp
    global _MH_ORACLE
    _MH_ORACLE = _oracle_mh_model(m)
    cores, _ = host_cores()
    jobs = [([c for c in range(chains) if c % cores == k], nits) for k in range(min(cores, chains))]
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(len(jobs)) as pool:
        res = pool.map(_cpu_mh_worker, jobs)
    wall = time.perf_counter() - t0
    its = sum(r[0] for r in res)
    return {"wall_s_sample": wall, "chain_iterations_sample": its, "cores": len(jobs),
            "wall_s_scaled_to_full_run": wall * (full_nits - 1) / (nits - 1),
            "sample": f"{chains} chains x {nits - 1} iterations of the reference MH loop (scipy odeint, "
                      f"lognorm priors' pdf/rvs), Pool({len(jobs)}); scaled to {full_nits - 1} iterations"}


DEMO_CHAINS, DEMO_NITS = 32, 1001  # the notebook's fit: MCMC(chain_inits=32), 1000 iterations


def demo_model():
    """The notebook's fit model (Demo_InfectionStates.ipynb: two_i, lognorm priors, demodata,
    H = S + I1 + I2), as tools/demo_fit.py builds it."""
    import pandas as pd
    import scipy.stats
    from odelib_amd import ModelFramework, parameter
    from odelib_amd.models import BUILTIN
    df = pd.read_csv(os.path.join(ROOT, "tests", "golden", "demodata.csv")).replace({"virus": "V", "host": "H"})
    pn = ["mu", "phi", "beta", "lam", "tau"]
    pars = {p: parameter(stats_gen=scipy.stats.lognorm, hyperparameters=dict(NOTEBOOK_PRIORS[p]), init_value=v)
            for p, v in zip(pn, THETA_STAR)}
    return ModelFramework(ODE=BUILTIN["two_i"][3], parameter_names=pn, state_names=["S", "I1", "I2", "V"],
                          dataframe=df, state_summations={"H": ["S", "I1", "I2"]}, S=5236900, **pars)


def demo_fit_starts(m, n=DEMO_CHAINS):
    """The notebook fit's chain starts, on the host (no GPU): ``MCMC(chain_inits=n,
    fitsurvey_samples=10000, sd_fitdistance=6.0)``'s survey (Framework.py:993-1012) — LHS
    draws through the priors, chi of each by the C restatement of the device integrator
    ('auto'; oracle/rk_ref.c), the samples whose chi beats the data shifted by 6 log sigmas,
    drawn with replacement by pandas — numpy's global RNG seeded as tools/demo_fit.py does.
    The CPU baseline and the device run then start their chains from the SAME parameters."""
    import numpy as np
    from oracle import rk_ref

    def survey(samples=1000, cpu_cores=1):
        ps = m._lhs_samples(samples)[m.get_pnames()]
        th = np.ascontiguousarray(ps.to_numpy(dtype=float).T)
        y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], th.shape[1], axis=1)
        out = ps.reset_index(drop=True)
        out["chi"] = rk_ref.integrate(m.fit_problem(), y0, th, trajectory=False)["chi"]
        return out
    np.random.seed(20261017 + n)
    saved, m.fit_survey = m.fit_survey, survey
    try:
        starts = m._survey_chain_starts(n, 10000, 6.0, 8)
    finally:
        m.fit_survey = saved
    return [starts.iloc[i][m.get_pnames()].to_dict() for i in range(n)]


_DEMO_ORACLE = None


def _cpu_demo_worker(args):
    chains, nits = args
    import numpy as np
    from oracle import cpu_ref
    t0 = time.perf_counter()
    for c, start in chains:
        for p, v in start.items():
            _DEMO_ORACLE.parameters[p].val = np.float64(v)
        _DEMO_ORACLE.random_seed = c
        cpu_ref.metropolis_hastings(_DEMO_ORACLE, nits=nits)
    return len(chains) * (nits - 1), time.perf_counter() - t0


def cpu_demo_fit_baseline(m, starts, nits=101, full_nits=DEMO_NITS):
    """The reference's MCMC loop (Samplers.py:53-174 via oracle/cpu_ref.py: scipy odeint =
    LSODA, the lognorm priors' pdf/rvs, chain i seeded i as Framework.py:1015) from the notebook
    fit's chain starts (demo_fit_starts), one chain per pool task (Framework.py:779) on the
    host cores; a bounded sample of the first ``nits`` iterations, scaled to ``full_nits``."""
    import multiprocessing as mp
    global _DEMO_ORACLE
    _DEMO_ORACLE = _oracle_mh_model(m)
    cores, _ = host_cores()
    idx = list(enumerate(starts))
    jobs = [([cs for cs in idx if cs[0] % cores == k], nits) for k in range(min(cores, len(starts)))]
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(len(jobs)) as pool:
        res = pool.map(_cpu_demo_worker, jobs)
    wall = time.perf_counter() - t0
    return {"wall_s_sample": wall, "chain_iterations_sample": sum(r[0] for r in res), "cores": len(jobs),
            "wall_s_scaled_to_full_run": wall * (full_nits - 1) / (nits - 1),
            "ms_per_iteration_scaled": wall / (nits - 1) * 1e3,
            "sample": f"the notebook fit's {len(starts)} chains (same LHS starts as the device leg) x {nits - 1} "
                      f"iterations of the reference MH loop (scipy odeint, lognorm priors' pdf/rvs, seed = chain), "
                      f"Pool({len(jobs)}); scaled to {full_nits - 1} iterations"}


def cpu_rk4_c(fp, y0, W, cores):
    """The same fixed-step RK4 + fused likelihood in C (oracle/rk_ref.c, OpenMP over
    64-walker groups, interval-major so rows are written as runs of walkers) on the
    full bench workload: the apples-to-apples CPU number for the GPU kernel (SURVEY
    §8d).  Runs in this process after the fork pool and before GPU initialisation."""
    import numpy as np
    os.environ["OMP_NUM_THREADS"] = str(cores)
    from oracle import rk_ref
    theta = synthetic_walkers(W, 5)
    Y0 = np.ascontiguousarray(np.repeat(y0[:, None], W, axis=1))
    rk_ref.integrate(fp, Y0[:, :64 * cores].copy(), theta[:, :64 * cores].copy())  # threads up, pages in
    best = None
    for _ in range(2):
        t0 = time.perf_counter()
        rk_ref.integrate(fp, Y0, theta, trajectory=True)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    T = len(fp.times)
    return {"value": W * (T - 1) / best, "unit": "walker-timesteps/s", "cores": cores, "kind": "port",
            "sample": f"{W} walkers x {T - 1} intervals, RK4 + trajectory store + chi in C "
                      f"(oracle/rk_ref.c, gcc -O2, OpenMP {cores} threads), best of 2: {best:.2f} s"}


def tolerance_of(model: str, method: str, substeps: int, rtol: float, atol: float) -> str:
    """The accuracy the bench's configuration is pinned to (the tests that pin it):
    RK4 is fixed-step, so its bar is what tests/test_gpu_parity.py checks against tight
    odeint for that model and substep count; the adaptive methods run at the problem's
    rtol/atol (odeint's defaults) and are checked within 1e-6 of tight odeint / Radau."""
    if method == "rk4":
        if model == "two_i" and substeps >= 1:
            return "vs tight odeint: rtol 1e-6, atol 1e-6 (test-pinned, rk4_substeps=%d)" % substeps
        if model == "chain20":
            return ("vs tight odeint: rtol 1e-6, atol 1e-4 (test-pinned)" if substeps < 3
                    else "vs tight odeint: rtol 1e-6, atol 1e-6 (test-pinned)")
        return "fixed step (rk4_substeps=%d); not pinned for this model" % substeps
    return "rtol=%g, atol=%g (%s; within 1e-6 of tight odeint, test-pinned)" % (
        rtol, atol, "odeint defaults" if rtol == atol == 1.49012e-8 else "user tolerances")


def write_ceiling(buf, stream, launches=20, warm_ms=60.0):
    """What this box's HBM sustains for a plain streaming write of the trajectory buffer:
    torch's fill kernel over the same bytes, back to back, after a warm-up (untimed by the
    metric).  The kernel's fraction of it separates the kernel from the box: the C1 kernel
    time varies 0.335-0.379 ms between boxes of the pool with the same code."""
    import torch
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < warm_ms:
        buf.zero_()
        torch.cuda.synchronize()
    e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    e[0].record(stream)
    for _ in range(launches):
        buf.zero_()
    e[1].record(stream)
    torch.cuda.synchronize()
    ms = e[0].elapsed_time(e[1]) / launches
    nbytes = buf.numel() * buf.element_size()
    return {"what": f"torch zero_() of the {nbytes / 1e9:.2f} GB trajectory buffer, {launches} back-to-back launches",
            "ms": ms, "GB/s": nbytes / (ms / 1e3) / 1e9}


# ------------------------------------------------------------------ GPU legs
class Ranks:
    """This rank's device and the collectives the timing needs (barrier, max)."""

    def __init__(self, world, rank, local_rank):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world, self.rank = world, rank
        # one process per GPU; ODELIB_BENCH_BACKEND=gloo lets several ranks share one GPU to
        # rehearse the multi-rank path (the driver's N>1 runs use nccl = RCCL over xGMI)
        self.backend = os.environ.get("ODELIB_BENCH_BACKEND", "nccl")
        ndev = torch.cuda.device_count()
        self.dev_index = local_rank % max(ndev, 1)
        torch.cuda.set_device(self.dev_index)
        self.dev = torch.device("cuda", self.dev_index)
        self.comm_timeout = float(os.environ.get("ODELIB_BENCH_COMM_TIMEOUT", "180"))
        if world > 1:
            from odelib_amd.distributed import watch
            with watch(f"init_process_group ({self.backend})", rank, self.comm_timeout):
                if self.backend == "nccl":
                    dist.init_process_group("nccl", device_id=self.dev)
                else:
                    dist.init_process_group(self.backend)
        self.red_dev = self.dev if self.backend == "nccl" else torch.device("cpu")

    def fence(self):
        """barrier + synchronize (both sides of every timed region); a barrier that has not
        returned after the communication timeout names itself and ends the rank (exit 87)."""
        if self.world > 1:
            from odelib_amd.distributed import watch
            with watch("barrier", self.rank, self.comm_timeout, log=False):
                self.dist.barrier()
        self.torch.cuda.synchronize(self.dev)

    def max(self, *vals):
        if self.world == 1:
            return vals if len(vals) > 1 else vals[0]
        t = self.torch.tensor(list(vals), dtype=self.torch.float64, device=self.red_dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        out = tuple(float(x) for x in t.cpu())
        return out if len(out) > 1 else out[0]

    def engine(self, model, method, T, rk4_substeps=1):
        m, y0h = build_problem(model, method, T, rk4_substeps)
        m.device = self.dev_index  # this rank's GPU (the model's default device is 0)
        eng = m.engine()
        assert eng.device == self.dev_index
        return eng, y0h


def warm(fn, min_s=0.06, first=1):
    """Untimed launches until at least ``min_s`` of wall time has passed (clocks settle)."""
    import torch
    n, t0 = 0, time.perf_counter()
    while n < first or time.perf_counter() - t0 < min_s:
        fn()
        n += 1
        if n % 5 == 0 or n == first:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return n


def mcmc_leg(args, R, eng, theta, y0, Wl, T, S, P, only=False):
    """Device Metropolis–Hastings (RK4, Philox) over the rank's walkers."""
    import numpy as np
    nits = args.mcmc_iters
    burn = nits // 2
    walk = np.ones(P, np.uint8)
    off = R.rank * Wl
    if only:  # PMC child pass: exactly the dispatches of one mh_run
        eng.mh_run(theta, y0, nits=nits, burnin=burn, walk_mask=walk, rng="philox", seed=1234, walker_offset=off)
        return None
    eng.mh_run(theta, y0, nits=2, burnin=0, walk_mask=walk, rng="philox", seed=1)  # load the kernel
    R.fence()
    tm0 = time.perf_counter()
    r = eng.mh_run(theta, y0, nits=nits, burnin=burn, walk_mask=walk, rng="philox", seed=1234, walker_offset=off)
    R.fence()
    t_mh = R.max(time.perf_counter() - tm0)
    mh_kernel_ms = eng.last_kernel_ms()
    # the same chains with the reference's numpy legacy streams generated on the device
    # (seed = global chain index, one lognorm prior draw per parameter)
    seeds = np.arange(off, off + Wl)
    eng.mh_run(theta, y0, nits=nits, burnin=burn, walk_mask=walk, rng="numpy", numpy_seeds=seeds, prior_draws=P)
    np_kernel_ms = eng.last_kernel_ms()
    # Fitting-report statistics of the pooled posterior (rawstats, Framework.py:11-17)
    # from two all-reduces of per-parameter sufficient statistics
    from odelib_amd.distributed import pooled_rawstats
    pooled_rawstats(r["samples"], P)  # untimed: first use loads torch's reduction kernels
    R.fence()
    tr0 = time.perf_counter()
    med, _ = pooled_rawstats(r["samples"], P)
    t_rs = time.perf_counter() - tr0
    mh_wts = R.world * Wl * (T - 1) * nits  # a-priori integrate + nits-1 proposals
    out = {"workload": f"two_i RK4 Metropolis-Hastings, {Wl} chains per GPU, Philox draws, chi only",
           "iterations": nits, "walker_timesteps_per_s": mh_wts / t_mh, "wall_s": t_mh,
           "kernel_ms": mh_kernel_ms, "kernel_ms_note": "events around the whole mh_run (k_mh + k_philox_draws)",
           "kernel_ms_numpy_rng": np_kernel_ms, "rawstats_allreduce_s": t_rs,
           "posterior_median": [float(x) for x in med], "rng": "philox"}
    return out


def mcmc_roofline(mh, flops_pmc, note, Wl, T, nits):
    """FP64-VALU roofline of the MCMC leg: PMC-counted fp64 flops of the k_mh dispatches
    ÷ the mh_run's kernel span."""
    if flops_pmc is None:
        return {"bound": "fp64-valu", "achieved": None, "peak": FP64_VALU_TFS, "unit": "TFLOP/s", "frac": None,
                "note": note}
    f = flops_pmc["flops"]
    ach = f / (mh["kernel_ms"] / 1e3) / 1e12
    return {"bound": "fp64-valu", "achieved": ach, "peak": FP64_VALU_TFS, "unit": "TFLOP/s",
            "frac": ach / FP64_VALU_TFS, "flops_per_mh_run": f,
            "flops_per_walker_timestep": f / (Wl * (T - 1) * nits),
            "k_mh_dispatches": flops_pmc["k_mh_dispatches"], "counters_sum": flops_pmc["counters_sum"],
            "source": note, "time": "kernel_ms (span includes the small k_philox_draws launches)"}


def c4_leg(args, R, T, P):
    """BASELINE.json configs[4]: 1 048 576 two_i walkers sharded over the ranks (contiguous
    global ids), RK4 trajectory integrate + MH (Philox keyed by global id) + the ONE
    posterior all-gather.  Every phase is timed between barriers, max over ranks."""
    import numpy as np
    import torch
    from odelib_amd.distributed import allgather_walkers, shard
    off, cnt = shard(C4_WALKERS, R.rank, R.world)
    eng, y0h = R.engine("two_i", "rk4", T)
    theta_all = synthetic_walkers(C4_WALKERS, P)
    theta = torch.as_tensor(np.ascontiguousarray(theta_all[:, off:off + cnt]), device=R.dev)
    y0 = torch.as_tensor(np.repeat(y0h[:, None], cnt, axis=1), device=R.dev).contiguous()
    S = len(y0h)
    res = {"workload": f"two_i RK4, {C4_WALKERS} walkers sharded over {R.world} GPU(s) "
                       f"({cnt} on rank {R.rank}): trajectory integrate, MH nits={C4_NITS}, posterior all-gather",
           "walkers_total": C4_WALKERS, "walkers_per_gpu": cnt, "n_gpus": R.world}
    # (1) trajectory-mode integrate, K back-to-back launches
    traj = eng.empty_traj(cnt)

    def step():
        return eng.integrate(y0, theta, trajectory=True, traj_out=traj, sync=False, timing=False,
                             kernel="half" if args.half_waves else args.kernel)
    warm(step)
    K = args.c4_steps
    R.fence()
    stream = torch.cuda.current_stream(R.dev)
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    ev[0].record(stream)
    for _ in range(K):
        out = step()
    ev[1].record(stream)
    R.fence()
    wall, kms = R.max(time.perf_counter() - t0, ev[0].elapsed_time(ev[1]) / K)
    res["integrate"] = {"steps": K, "ms_per_step": wall / K * 1e3, "kernel_ms_max_rank": kms,
                        "walker_timesteps_per_s": C4_WALKERS * (T - 1) * K / wall, "kernel": eng.last_variant(),
                        "hbm_frac_per_gpu": cnt * (T - 1) * 8 * S / (kms / 1e3) / 1e9 / HBM_PEAK_GBS,
                        "chi_finite": bool(torch.isfinite(out["chi"]).all().item())}
    del traj, out
    torch.cuda.empty_cache()
    # (2) MH over the shard, Philox keyed by the global walker id
    walk = np.ones(P, np.uint8)
    burn = C4_NITS // 2
    eng.mh_run(theta[:, :256], y0[:, :256], nits=2, burnin=0, walk_mask=walk, rng="philox", seed=1)
    R.fence()
    t0 = time.perf_counter()
    r = eng.mh_run(theta, y0, nits=C4_NITS, burnin=burn, walk_mask=walk, rng="philox", seed=4242, walker_offset=off)
    R.fence()
    t_mh = R.max(time.perf_counter() - t0)
    res["mh"] = {"iterations": C4_NITS, "burnin": burn, "wall_s": t_mh,
                 "walker_timesteps_per_s": C4_WALKERS * (T - 1) * C4_NITS / t_mh,
                 "kernel_ms_rank0": eng.last_kernel_ms()}
    # (3) the ONE posterior all-gather (Framework.py:1037 pd.concat analogue).  --pool cabi:
    # the C-ABI's own RCCL communicator (oe_comm + oe_allgather_samples: pad, ncclAllGather,
    # rank-major -> walker-minor re-layout), the path INTEGRATION.md gives ODElib; it needs
    # one GPU per rank (RCCL), so a gloo rehearsal with ranks sharing a GPU pools with torch.
    # At N = 1 the C-ABI path still runs (a 1-rank communicator) so its fields are reported.
    blk = r["samples"]
    res["posterior_block_bytes_per_rank"] = blk.numel() * 8
    pool = args.pool if (R.world == 1 or R.backend == "nccl") else "torch"
    cabi_error = None
    from odelib_amd.distributed import watch

    def w(what):  # every collective of the pooling, named in the log and bounded (no hang)
        return watch(f"C4 {what}", R.rank, args.comm_timeout, log=R.world > 1)
    if pool == "cabi":
        # Every rank takes the same path: an error RAISED by the communicator set-up or the
        # untimed first gather is agreed on by an all-reduce of an error flag before the timed
        # gather, and the timed gather's outcome after it — a rank that fell back alone would
        # enter a different collective than its peers.  A rank that never returns from one of
        # these calls is named and ended by watch() (a peer already inside the collective
        # cannot be released by a flag).
        from odelib_amd.distributed import native_allgather_walkers, native_comm
        comm, pooled = None, None
        try:
            try:
                with w("oe_comm_init (rank 0's id broadcast, ncclCommInitRank)"):
                    comm = native_comm(R.dev.index, None)
                src = blk.contiguous()
                with w("oe_allgather_samples, untimed first"):
                    native_allgather_walkers(src[:1], C4_WALKERS if R.world > 1 else cnt, comm)
                    torch.cuda.synchronize(R.dev)
                ok = 1.0
            except Exception as e:  # an error raised by the C-ABI path (not a hang)
                cabi_error, ok = f"{type(e).__name__}: {e}"[:300], 0.0
            with w("error-flag all-reduce"):
                agreed = -R.max(-ok) > 0.0  # min over ranks: every rank set up its communicator
            if agreed:
                with w("barrier before the timed gather"):
                    R.fence()
                t0 = time.perf_counter()
                try:
                    with w("oe_allgather_samples, timed"):
                        pooled = native_allgather_walkers(src, C4_WALKERS if R.world > 1 else cnt, comm)
                        torch.cuda.synchronize(R.dev)
                    ok = 1.0
                except Exception as e:
                    cabi_error, ok, pooled = f"{type(e).__name__}: {e}"[:300], 0.0, None
                with w("barrier after the timed gather"):
                    R.fence()
                t_ag = R.max(time.perf_counter() - t0)
                n_ranks = comm.n_ranks
                with w("error-flag all-reduce after the gather"):
                    if -R.max(-ok) == 0.0:
                        pooled = None
            if pooled is None:  # some rank failed: all pool with torch, and say so
                cabi_error = cabi_error or "another rank's C-ABI pooling failed"
                pool = "torch"
        finally:
            if comm is not None:
                with w("oe_comm_destroy"):
                    comm.close()
    if pool == "cabi":
        pass
    elif R.world > 1:
        src = blk.contiguous() if R.backend == "nccl" else blk.cpu()
        with w("torch all_gather, untimed first"):
            allgather_walkers(src[:1], C4_WALKERS)  # communicator / channel set-up
        with w("barrier before the timed gather"):
            R.fence()
        t0 = time.perf_counter()
        with w("torch all_gather, timed"):
            pooled = allgather_walkers(src, C4_WALKERS)
        with w("barrier after the timed gather"):
            R.fence()
        t_ag = R.max(time.perf_counter() - t0)
        n_ranks = R.world
    else:
        pooled = None
    if pooled is not None:
        assert pooled.shape[-1] == (C4_WALKERS if R.world > 1 else cnt)
        gathered = pooled.numel() * 8
        res["allgather"] = {"pool": pool, "backend": "rccl (oe_comm)" if pool == "cabi" else R.backend,
                            "comm_n_ranks": n_ranks, "world_size": R.world, "bytes_gathered": gathered,
                            "s": t_ag, "algbw_GBps": gathered / t_ag / 1e9,
                            "busbw_GBps": gathered * (R.world - 1) / R.world / t_ag / 1e9}
        if cabi_error:
            res["allgather"]["cabi_error"] = cabi_error
        del pooled
    else:
        res["allgather"] = {"pool": "torch", "comm_n_ranks": 1, "world_size": 1,
                            "note": "one GPU, torch pooling: nothing to gather"}
        if cabi_error:
            res["allgather"]["cabi_error"] = cabi_error
    del r, blk
    torch.cuda.empty_cache()
    return res


def extra_configs(args, R, T, P):
    """The other single-GPU configs of BASELINE.json (C2, C3), kernel time only."""
    import numpy as np
    import torch
    extra = {}
    # C2-stiffmix: the C2 draws with 0.1 % of the walkers made stiff (tau = 1e5, the I1
    # compartment relaxing 4e4x faster): 'dopri5' keeps them in the shared step, so their
    # waves crawl at the stability limit; 'auto' (the drop-in default, LSODA-like) hands
    # them to BDF at their eviction points, a step size and an order per walker.
    # C3 at rk4_substeps=1 is within rtol 1e-6 / atol 1e-4 of tight odeint (SURVEY §8c's
    # 20-state RK4 tolerance; tests/test_gpu_parity.py::test_c3_rk4_bench_accuracy);
    # rk4_substeps=3 is within rtol = atol = 1e-6 (2 is not: 1.09 of that budget).
    cfgs = (("C2", "two_i", "dopri5", 65536, 0.0, 1, "rtol=atol=1.49012e-8 (odeint defaults)"),
            # C2 on the store-wave kernel (4 compute + 4 store waves per workgroup, per-wave LDS
            # slot rings with produced/consumed counters, no phase barrier; bitwise the direct
            # kernel: tests/test_gpu_dopri5_piped.py)
            ("C2-storewaves", "two_i", "dopri5", 65536, 0.0, 1, "rtol=atol=1.49012e-8 (odeint defaults)"),
            ("C2-auto", "two_i", "auto", 65536, 0.0, 1, "rtol=atol=1.49012e-8 (odeint defaults)"),
            ("C2-stiffmix-dopri5", "two_i", "dopri5", 65536, 1e-3, 1, "rtol=atol=1.49012e-8"),
            ("C2-stiffmix-auto", "two_i", "auto", 65536, 1e-3, 1, "rtol=atol=1.49012e-8"),
            ("C3", "chain20", "rk4", 262144, 0.0, 1, "vs tight odeint: rtol 1e-6, atol 1e-4 (test-pinned)"),
            ("C3-rk4x3", "chain20", "rk4", 262144, 0.0, 3, "vs tight odeint: rtol 1e-6, atol 1e-6 (test-pinned)"),
            ("C3-dopri5", "chain20", "dopri5", 262144, 0.0, 1, "rtol=atol=1.49012e-8 (odeint defaults)"),
            # the same with one lane per walker (OE_NO_SPLIT): the round-2 kernel, for reference
            ("C3-dopri5-onelane", "chain20", "dopri5", 262144, 0.0, 1, "rtol=atol=1.49012e-8 (odeint defaults)"))
    for name, model, method, W, stiff, subs, tol in cfgs:
        split = not name.endswith("-onelane")
        kern = (("half" if args.half_waves else args.kernel) if method == "rk4"
                else "pipe2" if name.endswith("-storewaves") else None)
        ex, y0x = R.engine(model, method, T, subs)
        Sx = len(y0x)
        thh = synthetic_walkers(W, P)
        n_stiff = int(round(stiff * W))
        if n_stiff:
            thh[4, np.random.RandomState(7).choice(W, n_stiff, replace=False)] = 1e5
        thx = torch.as_tensor(thh, device=R.dev).contiguous()
        y0t = torch.as_tensor(np.repeat(y0x[:, None], W, axis=1), device=R.dev).contiguous()
        trx = ex.empty_traj(W)
        # as the headline: at least 60 ms of untimed launches first, so a compute-bound
        # kernel (DOPRI5) is timed at the clock it sustains (C2: 0.57 ms per launch over the
        # first 10 back-to-back launches, 0.49 over 50), then K back-to-back launches
        # without event markers, timed by two events on the stream
        K = 20 if not n_stiff else 3
        warm(lambda: ex.integrate(y0t, thx, trajectory=True, traj_out=trx, sync=False, timing=False,
                                  xcd_remap=XCD_ARG[args.xcd], split=split, kernel=kern))
        sx = torch.cuda.current_stream(R.dev)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record(sx)
        for _ in range(K):
            outx = ex.integrate(y0t, thx, trajectory=True, traj_out=trx, sync=False, timing=False,
                                xcd_remap=XCD_ARG[args.xcd], split=split, kernel=kern)
        ev[1].record(sx)
        torch.cuda.synchronize(R.dev)
        kms = ev[0].elapsed_time(ev[1]) / K
        byt = W * (T - 1) * 8 * Sx
        extra[name] = {"workload": f"{model} {method}, {W} walkers, trajectory mode"
                       + (f", {n_stiff} stiff walkers (tau=1e5)" if n_stiff else ""), "kernel_ms": kms,
                       "timing": f"{K} back-to-back launches, events around them",
                       "walker_timesteps_per_s": W * (T - 1) / (kms / 1e3),
                       "hbm_frac": byt / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, "tolerance": tol}
        if method == "rk4":
            extra[name]["rk4_substeps"] = subs
            extra[name]["kernel"] = ex.last_variant()
        if name.endswith("-storewaves"):
            extra[name]["kernel"] = "k_integrate_dopri5_piped (OE_PIPE)"
        if model == "chain20" and method == "dopri5":
            extra[name]["lanes_per_walker"] = 2 if split else 1
        if n_stiff:
            stx = outx["status"].cpu().numpy()
            extra[name]["walkers_flagged_stiff"] = int(((stx & 8) != 0).sum())
            extra[name]["walkers_maxstep"] = int(((stx & 4) != 0).sum())
        del trx, thx, y0t, ex
        torch.cuda.empty_cache()
    extra.update(small_mcmc(R, T, P))
    return extra


def small_mcmc(R, T, P, nits=1001):
    """The reference's own MCMC shape — few chains, 1000 iterations (the notebook: 32
    chains) — with one iteration per step and with speculative rounds:
    wall time of one mh_run each, Philox draws, same chains (parameters compared)."""
    import numpy as np
    import torch
    out = {}
    for method in ("rk4", "auto"):
        for W in (32, 1024):
            ex, y0x = R.engine("two_i", method, T)
            th = torch.as_tensor(synthetic_walkers(W, P), device=R.dev).contiguous()
            yy = torch.as_tensor(np.repeat(y0x[:, None], W, axis=1), device=R.dev).contiguous()
            walk = np.ones(P, np.uint8)
            row, runs = {}, {}
            for spec in (0, "auto"):
                ex.mh_run(th, yy, nits=3, burnin=0, walk_mask=walk, rng="philox", seed=1, speculate=spec)
                torch.cuda.synchronize(R.dev)
                t0 = time.perf_counter()
                runs[spec] = ex.mh_run(th, yy, nits=nits, burnin=nits // 2, walk_mask=walk, rng="philox", seed=5,
                                       speculate=spec)
                row[f"wall_s_speculate_{spec}"] = time.perf_counter() - t0
                row[f"depth_{spec}"] = ex.last_mh_depth()
            row["speedup"] = row["wall_s_speculate_0"] / row["wall_s_speculate_auto"]
            row["same_parameters"] = bool(torch.equal(runs[0]["samples"][:, :P], runs["auto"]["samples"][:, :P]))
            row["workload"] = f"two_i {method} MH, {W} chains x {nits - 1} iterations, Philox, chi only"
            out[f"MCMC-{W}chains-{method}"] = row
            del runs, th, yy, ex
            torch.cuda.empty_cache()
    return out


def demo_fit_leg(demo, cpu):
    """The notebook's fit on the device through the drop-in API: ``MCMC`` from the chain
    starts the CPU baseline used (demo_fit_starts), 32 chains x 1000 iterations, the default
    method ('auto'), the reference's numpy draws (rng='replay', chain i seeded i), with one
    iteration per step and with speculative rounds; beside it the synthetic 32-chain 'auto'
    MH (small_mcmc) for the per-iteration ratio."""
    import numpy as np
    import torch
    m, starts = demo["model"], demo["starts"]
    row = {"workload": f"the notebook fit: MCMC from {len(starts)} LHS chain starts (fitsurvey_samples=10000, "
                       f"sd_fitdistance=6), {DEMO_NITS - 1} iterations, method {m.method}, rng replay"}
    m.MCMC(chain_inits=starts[:2], iterations_per_chain=5, print_report=False, print_iterations=False)  # warm
    posts = {}
    for spec in (0, "auto"):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            posts[spec] = m.MCMC(chain_inits=starts, iterations_per_chain=DEMO_NITS - 1, print_report=False,
                                 print_iterations=False, speculate=spec)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        row[f"wall_s_speculate_{spec}"] = wall
        row[f"ms_per_iteration_speculate_{spec}"] = wall / (DEMO_NITS - 1) * 1e3
        row[f"depth_{spec}"] = m.engine().last_mh_depth()
    pn = m.get_pnames()
    row["same_parameters"] = bool(np.array_equal(posts[0][pn].to_numpy(), posts["auto"][pn].to_numpy()))
    row["posterior_q99_max"] = {p: [float(posts[0][p].quantile(0.99)), float(posts[0][p].max())]
                                for p in ("phi", "beta", "lam", "tau")}
    if cpu and "mcmc_demo_fit_32chains" in cpu:
        c = cpu["mcmc_demo_fit_32chains"]
        row["cpu_reference_ms_per_iteration"] = c["ms_per_iteration_scaled"]
        row["speedup_vs_cpu_speculate_auto"] = c["ms_per_iteration_scaled"] / row["ms_per_iteration_speculate_auto"]
    return row


# ------------------------------------------------------------------ main
def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and env_world is None:
        sys.exit(relaunch_under_torchrun(args.gpus))
    world = int(env_world or 1)
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; refusing to report a mismatched run",
              file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    P = 5

    # host-side problem set-up, then the CPU baseline and the PMC child passes (all
    # before this process touches the GPU)
    m, y0h = build_problem(args.model, args.method, args.times)
    fp_host = m.fit_problem()
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.mcmc_only:
        cpu = cpu_baseline(args.model, fp_host, y0h, args.cpu_seconds, P)
        if args.method == "rk4":
            cpu["rk4_c_openmp"] = cpu_rk4_c(fp_host, y0h, args.walkers, cpu["cores"])
        if args.model == "two_i" and not args.no_extra_configs:
            cpu["mcmc_32chains"] = cpu_mcmc_baseline(m)
    demo = None
    if args.model == "two_i" and not args.no_extra_configs and world == 1:
        dm = demo_model()
        demo = {"model": dm, "starts": demo_fit_starts(dm)}
        if cpu is not None:
            cpu["mcmc_demo_fit_32chains"] = cpu_demo_fit_baseline(dm, demo["starts"])
    traffic, traffic_note = None, "skipped (--no-pmc or N>1)"
    mh_flops, mh_flops_note = None, "skipped (--no-pmc, N>1 or no MCMC leg)"
    if world == 1 and not args.no_pmc and not args.mcmc_only:
        traffic, traffic_note = pmc_traffic(args)
        if args.mcmc_iters > 1 and args.model == "two_i":
            mh_flops, mh_flops_note = pmc_mh_flops(args)

    import numpy as np
    import torch

    os.environ.setdefault("ODELIB_BENCH_COMM_TIMEOUT", str(args.comm_timeout))
    R = Ranks(world, rank, local_rank)
    eng, _ = R.engine(args.model, args.method, args.times)
    dev = R.dev
    fp = eng.problem
    S, T = fp.n_states, fp.n_times
    Wl = args.walkers
    theta_all = synthetic_walkers(Wl * world, P)
    theta = torch.as_tensor(np.ascontiguousarray(theta_all[:, rank * Wl:(rank + 1) * Wl]), device=dev)
    y0 = torch.as_tensor(np.repeat(y0h[:, None], Wl, axis=1), device=dev).contiguous()

    if args.mcmc_only:
        mcmc_leg(args, R, eng, theta, y0, Wl, T, S, P, only=True)
        torch.cuda.synchronize(dev)
        if world > 1:
            R.dist.destroy_process_group()
        return

    traj = eng.empty_traj(Wl)
    kernel = "half" if args.half_waves else args.kernel

    def step():
        # no timing-event markers between the timed launches (measured: markers between
        # back-to-back launches cost ~4 % of the C1 wall time, tools/launch_gaps.py)
        return eng.integrate(y0, theta, trajectory=True, traj_out=traj, nt_stores=not args.cached_stores,
                             sync=False, timing=False, kernel=kernel,
                             xcd_remap=XCD_ARG[args.xcd], split=not args.no_split)

    # W untimed warm-up steps, continued (in batches of 5, untimed) until at least
    # --warmup-ms of launches have run: under a kernel trace the C1 kernel runs 0.33-0.38 ms
    # for its first ~8 launches, 0.42-0.45 ms over launches ~10-20 (the chip's power
    # management settling) and 0.37 +- 0.02 ms from ~40 ms on (profiles/r02w3_launch_series.txt), so 20
    # steps timed right after 5 warm-ups report the transient, not the sustained rate
    n_warm = 0
    tw = time.perf_counter()
    while n_warm < args.warmup or (time.perf_counter() - tw) * 1e3 < args.warmup_ms:
        for _ in range(args.warmup if n_warm < args.warmup else 5):
            step()
            n_warm += 1
        torch.cuda.synchronize(dev)
    R.fence()
    stream = torch.cuda.current_stream(dev)  # the stream the engine launches on
    span = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    span[0].record(stream)
    for k in range(args.steps):
        out = step()
    span[1].record(stream)
    R.fence()
    elapsed = R.max(time.perf_counter() - t0)
    # average launch duration over the timed region: HIP events bracketing the K
    # back-to-back launches on the launch stream
    kern_avg_s = span[0].elapsed_time(span[1]) / args.steps / 1e3
    # per-dispatch durations (event pair around each launch; the rocprofv3 view), in an
    # untimed pass of the same launches after the timed region
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    kern_dispatch_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    ran = eng.last_variant()
    tune = eng.tune_times() if kernel == "auto" else None
    ceiling = write_ceiling(traj, stream)
    wts = world * Wl * (T - 1) * args.steps  # walkers every rank actually ran
    value = wts / elapsed
    bytes_launch = Wl * (T - 1) * 8 * S + Wl * 8 * (S + P + 2)  # traj + y0/θ/chi/ssres
    achieved = bytes_launch / kern_avg_s / 1e9
    chi_ok = bool(torch.isfinite(out["chi"]).all().item())
    del traj, out
    torch.cuda.empty_cache()

    mcmc = None
    if args.mcmc_iters > 1:
        mcmc = mcmc_leg(args, R, eng, theta, y0, Wl, T, S, P)
        if args.model == "two_i":
            mcmc["roofline"] = mcmc_roofline(mcmc, mh_flops, mh_flops_note, Wl, T, args.mcmc_iters)

    extra = {}
    if not args.no_c4 and args.model == "two_i":
        extra["C4"] = c4_leg(args, R, T, P)
    if world == 1 and not args.no_extra_configs:
        extra.update(extra_configs(args, R, T, P))
        if demo is not None:
            extra["MCMC-demo-fit-32chains"] = demo_fit_leg(demo, cpu)

    if rank == 0:
        line = {
            "metric": "walker-timesteps/sec, 4-state infection ODE, 65536 walkers, 1/2/4/8 MI355X"
            if args.model == "two_i" else f"walker-timesteps/sec, {S}-state chain ODE",
            "value": value, "unit": "walker-timesteps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "warmup_launches": n_warm, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"{args.model} {args.method} trajectory-mode integrate + fused chi",
                       "walkers_per_gpu": Wl, "walkers_total": Wl * world, "states": S, "times": T,
                       "method": args.method, "rk4_substeps": 1,
                       "tolerance": tolerance_of(args.model, args.method, 1, fp.rtol, fp.atol),
                       "stores": "cached" if args.cached_stores else "nontemporal",
                       "kernel": ran, "kernel_choice": kernel, "kernel_tune_ms": tune, "xcd": args.xcd,
                       "parallelism": f"walker-shard x{world}",
                       "launch": "torchrun, one rank per GPU" if world > 1 else "single process"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "frac_wall": bytes_launch / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS,
                         "frac_note": "frac: the timed region's event span per launch (kernel time); frac_wall: "
                                      "ms_per_step, the wall time value is computed from (host launch gaps included)",
                         "traffic": traffic_of(traffic, ran, args.method),
                         "traffic_note": traffic_note,
                         "kernel_ms": kern_avg_s * 1e3, "kernel_ms_note": "timed-region event span / steps",
                         "kernel_ms_per_dispatch": kern_dispatch_ms, "bytes_per_launch": bytes_launch,
                         "box_write_ceiling": dict(ceiling, frac_of_ceiling=achieved / ceiling["GB/s"])},
            "cpu_baseline": cpu,
            "mcmc": mcmc,
            "other_configs": extra or None,
            "chi_finite": chi_ok,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        R.dist.destroy_process_group()


if __name__ == "__main__":
    main()
