"""The reference notebook's fit, end to end through the drop-in API (run on the GPU box).

    python tools/demo_fit.py --chains 32 1024 8192

Builds the 4-state model exactly as `demo/Demo_InfectionStates.ipynb` does (a plain Python
ODE, lognorm priors, `demodata.csv`, H = S + I1 + I2) with `import odelib_amd as ODElib`
and runs the notebook's call `MCMC(chain_inits=N, cpu_cores=8, fitsurvey_samples=10000,
sd_fitdistance=6.0)` (1000 iterations per chain, the reference default), timing the whole
call — LHS fit survey, chain start selection, the device Metropolis–Hastings chains and
the posterior DataFrame — and printing one JSON line per chain count with the posterior
medians (`rawstats`, Framework.py:11-17).  The reference runs each chain on a CPU core with
scipy odeint; bench.py's cpu_baseline times that path on the same host.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def two_i(y, t, ps):
    """The notebook's two-infection-state model (Demo_InfectionStates.ipynb:60-75)."""
    mu, phi, beta, lam, tau = ps[0], ps[1], ps[2], ps[3], ps[4]
    S, I1, I2, V = y[0], y[1], y[2], y[3]
    dSdt = mu * S - phi * S * V
    dI1dt = phi * S * V - tau * I1
    dI2dt = tau * I1 - lam * I2
    dVdt = beta * lam * I2 - phi * S * V
    return [dSdt, dI1dt, dI2dt, dVdt]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", nargs="+", type=int, default=[32, 1024, 8192])
    ap.add_argument("--iterations", type=int, default=1000)
    ap.add_argument("--method", default=None, help="engine method (default: the drop-in default, 'auto')")
    ap.add_argument("--speculate", nargs="+", default=["auto"], help="MCMC speculate values to time (auto, 0, d)")
    args = ap.parse_args()
    import pandas as pd
    import scipy.stats
    import torch
    import odelib_amd as ODElib
    from odelib_amd.Framework import rawstats

    df = pd.read_csv(os.path.join(ROOT, "tests", "golden", "demodata.csv")).replace({"virus": "V", "host": "H"})
    priors = {"mu": {"s": 3, "scale": 1e-8}, "phi": {"s": 3, "scale": 1e-8}, "beta": {"s": 1, "scale": 20},
              "lam": {"s": 2, "scale": .1}, "tau": {"s": 2, "scale": 1}}
    init = {"mu": 7.475e-9, "phi": 1.069e-7, "beta": 19.73, "lam": 1.934, "tau": 2.799}
    pars = {k: ODElib.parameter(stats_gen=scipy.stats.lognorm, hyperparameters=dict(priors[k]), init_value=init[k])
            for k in priors}
    kw = {"method": args.method} if args.method else {}
    m = ODElib.ModelFramework(ODE=two_i, parameter_names=list(priors), state_names=["S", "I1", "I2", "V"],
                              dataframe=df, state_summations={"H": ["S", "I1", "I2"]}, S=5236900, **pars, **kw)
    # wall-time split of one MCMC call: fit survey, device chains (kernel time from the
    # engine's events), everything else on the host (chain copies, posterior DataFrame)
    from odelib_amd.Statistics import Samplers
    split = {}

    def timed(name, fn):
        def w(*a, **k):
            t = time.perf_counter()
            r = fn(*a, **k)
            torch.cuda.synchronize()
            split[name] = split.get(name, 0.0) + time.perf_counter() - t
            return r
        return w
    m.fit_survey = timed("fit_survey_s", m.fit_survey)
    eng = m.engine()
    mh = eng.mh_run

    def mh_timed(*a, **k):
        r = timed("mh_run_s", mh)(*a, **k)
        split["mh_kernel_s"] = split.get("mh_kernel_s", 0.0) + eng.last_kernel_ms() / 1e3
        return r
    eng.mh_run = mh_timed
    # first call: kernel loads, LHS code paths, pandas warm-up (untimed)
    m.MCMC(chain_inits=2, iterations_per_chain=10, print_report=False, fitsurvey_samples=200, sd_fitdistance=6.0,
           print_iterations=False)
    torch.cuda.synchronize()
    import numpy as np
    posts = {}
    for n, spec in ((n, s) for n in args.chains for s in args.speculate):
        spec = spec if spec == "auto" else int(spec)
        split.clear()
        # the chain starts come from the LHS survey and pandas' sample (numpy's global RNG):
        # seeded alike for every call, so the calls for one chain count run the same chains
        np.random.seed(20261017 + n)
        t0 = time.perf_counter()
        post = m.MCMC(chain_inits=n, iterations_per_chain=args.iterations, cpu_cores=8, print_report=False,
                      fitsurvey_samples=10000, sd_fitdistance=6.0, print_iterations=False, speculate=spec)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        med = {p: float(rawstats(post[p])[0]) for p in priors}
        posts[(n, spec)] = post
        same = None
        if spec != 0 and (n, 0) in posts:  # the same chains as one iteration per step?
            ref = posts[(n, 0)]
            same = bool(np.array_equal(ref[list(priors)].to_numpy(), post[list(priors)].to_numpy()))
        print(json.dumps({"chains": n, "speculate": spec, "depth": eng.last_mh_depth(),
                          "same_parameters_as_speculate_0": same,
                          "iterations_per_chain": args.iterations, "wall_s": round(wall, 3),
                          "posterior_rows": int(len(post)), "chains_in_posterior": int(post["chain#"].nunique()),
                          "acceptance_ratio_mean": float(post.groupby("chain#")["acceptance_ratio"].last().mean()),
                          "method": m.method, "split": {k: round(v, 3) for k, v in split.items()},
                          "posterior_median": med,
                          "posterior_q99_max": {p: [float(post[p].quantile(0.99)), float(post[p].max())]
                                                for p in ("beta", "lam", "tau")}}), flush=True)


if __name__ == "__main__":
    main()
