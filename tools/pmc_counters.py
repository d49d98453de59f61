"""Per-dispatch means of SQ/TCC counters for one bench configuration (GPU box).

    python tools/pmc_counters.py --kernel-regex 'k_integrate' --counters SQ_WAVES SQ_BUSY_CYCLES -- --method dopri5

One rocprofv3 --pmc pass per counter (no tracing domains), each running bench.py with
the C2/C3 extras, MCMC leg, CPU baseline and its own PMC passes switched off.  Prints a
JSON object {counter: mean per dispatch} and writes it to gpurun_out/pmc_<tag>.json.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="counters")
    ap.add_argument("--kernel-regex", default="k_integrate")
    ap.add_argument("--counters", nargs="+", required=True)
    ap.add_argument("--timeout", type=int, default=240)
    ap.add_argument("--one-pass", action="store_true",
                    help="all counters in ONE pass (the caller keeps them within one pass's block limits)")
    args, bench_args = ap.parse_known_args()
    bench_args = [a for a in bench_args if a != "--"]
    from tools.profile import pmc_counts, pmc_pass
    out = os.path.join(ROOT, "gpurun_out", f"pmc_{args.tag}")
    os.makedirs(out, exist_ok=True)
    res = {}
    if args.one_pass:
        r = pmc_counts(out, args.counters, bench_args + ["--no-pmc"], args.kernel_regex, args.timeout)
        res = {c: r[c]["mean"] for c in args.counters}
        res["dispatches"] = r[args.counters[0]]["dispatches"]
    for c in ([] if args.one_pass else args.counters):
        try:
            r = pmc_pass(out, c, bench_args + ["--no-pmc"], args.kernel_regex, args.timeout)
            res[c] = r["mean"]
        except SystemExit as e:  # an unknown counter fails its own pass only
            res[c] = f"failed: {e}"
        print(c, res[c], flush=True)
    with open(os.path.join(ROOT, "gpurun_out", f"pmc_{args.tag}.json"), "w") as f:
        json.dump({"bench_args": bench_args, "kernel_regex": args.kernel_regex, "per_dispatch_mean": res}, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
