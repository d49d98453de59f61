"""A/B timing of library builds on the bench workload (run on the GPU box).

    python tools/ab_bench.py --libs base=alt_lib/base/libodelib_amd.so new=odelib_amd/csrc/libodelib_amd.so \
        --reps 2 -- --method dopri5

Each repetition runs ``bench.py`` once per library, interleaved (A B A B ...), as a child
process with ODELIB_AMD_LIB pointing at that build; the bench's own timing (K back-to-back
launches between two events after its warm-up) is collected from its JSON line.  Extra
arguments after ``--`` go to bench.py (defaults: no CPU baseline, no PMC, no MCMC leg, no
extra configs, 50 timed steps).
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    argv = sys.argv[1:]
    extra = []
    if "--" in argv:
        k = argv.index("--")
        argv, extra = argv[:k], argv[k + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True, help="name=path pairs")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--timeout", type=int, default=120)
    args = ap.parse_args(argv)
    libs = [s.split("=", 1) for s in args.libs]
    base = [sys.executable, "bench.py", "--no-cpu-baseline", "--no-pmc", "--mcmc-iters", "0",
            "--no-extra-configs", "--steps", "50"]
    res = {name: [] for name, _ in libs}
    for rep in range(args.reps):
        for name, path in libs:
            env = dict(os.environ, ODELIB_AMD_LIB=os.path.abspath(os.path.join(ROOT, path)))
            r = subprocess.run(base + extra, cwd=ROOT, env=env, capture_output=True, text=True,
                               timeout=args.timeout)
            if r.returncode != 0:
                print(r.stdout[-2000:], r.stderr[-2000:])
                raise SystemExit(f"bench failed for {name} ({r.returncode})")
            line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
            d = json.loads(line)
            ms = d["roofline"]["kernel_ms"]
            res[name].append(ms)
            print(json.dumps({"rep": rep, "lib": name, "kernel_ms": ms, "frac": d["roofline"]["frac"],
                              "workload": d["config"]["workload"]}), flush=True)
    print(json.dumps({"summary": {k: {"min": min(v), "mean": sum(v) / len(v), "all": v} for k, v in res.items()},
                      "bench_args": extra}))


if __name__ == "__main__":
    main()
