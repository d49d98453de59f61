"""Profile the bench workload with rocprofv3 (run on the GPU box).

    python tools/profile.py --tag r01 [bench args...]

1. kernel trace + stats      rocprofv3 --kernel-trace --stats
2. PMC pass FETCH_SIZE       rocprofv3 --pmc FETCH_SIZE   (own pass: 3 TCC slots)
3. PMC pass WRITE_SIZE       rocprofv3 --pmc WRITE_SIZE   (own pass: 2 TCC slots)

Each pass runs ``python3 bench.py`` directly after ``--`` (no launcher hops).  Outputs
go to gpurun_out/prof_<tag>/; the summary (per-kernel mean duration, HBM bytes per
dispatch with the gfx950 FETCH_SIZE ×2 correction of MI355X_MICROARCH.md §HBM) is
written to gpurun_out/prof_<tag>/<tag>_summary.json with the stats CSV; copy both into
profiles/ (tracked) to commit them.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rocprof():
    """rocprofv3 is a `#!/usr/bin/env python3` script: run it with this interpreter so no
    env -> python3 exec hop happens in the process tree."""
    path = shutil.which("rocprofv3")
    if path is None:
        raise SystemExit("rocprofv3 not found")
    return [sys.executable, path]


def run(cmd, timeout):
    print("+", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, cwd=ROOT, timeout=timeout, capture_output=True, text=True)
    tail = (r.stdout[-2000:] + r.stderr[-2000:])
    if r.returncode != 0:
        print(tail)
        raise SystemExit(f"command failed ({r.returncode})")
    return r.stdout


def find(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    return hits[0] if hits else None


def read_csv(path):
    with open(path) as f:
        return list(csv.DictReader(f))


TRAJ_ONLY = ["--no-cpu-baseline", "--mcmc-iters", "0", "--no-extra-configs", "--no-c4", "--steps", "5", "--warmup", "1"]


def pmc_counts(out, counters, bench_args, kernel_regex, timeout, base=None, tag=None):
    """One rocprofv3 --pmc pass over ``bench.py <base> <bench_args>`` collecting
    ``counters`` (all in ONE pass: the caller keeps them within one pass's block limits)
    for the dispatches matching ``kernel_regex``.  Returns {counter: {dispatches, mean,
    sum, csv}}, values summed over XCD / SE instances of each dispatch."""
    counters = [counters] if isinstance(counters, str) else list(counters)
    d = os.path.join(out, f"pmc_{(tag or '_'.join(counters)).lower()}")
    run(rocprof() + ["--pmc", *counters, "--kernel-include-regex", kernel_regex, "--output-format", "csv",
         "-d", d, "-o", "run", "--", sys.executable, "bench.py", *(TRAJ_ONLY if base is None else base),
         *bench_args], timeout)
    path = find(os.path.join(d, "**", "*counter_collection.csv"))
    rows = read_csv(path)
    res = {}
    for c in counters:
        vals = {}
        for r in rows:
            if r.get("Counter_Name") != c:
                continue
            key = (r.get("Dispatch_Id"), r.get("Kernel_Name"))
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])  # sum over XCD / instances
        per = list(vals.values())
        by = {}
        for (_, name), v in vals.items():
            by.setdefault(name, []).append(v)
        res[c] = {"dispatches": len(per), "mean": sum(per) / max(len(per), 1), "sum": sum(per),
                  "by_kernel": {n: {"dispatches": len(v), "mean": sum(v) / len(v)} for n, v in by.items()},
                  "csv": os.path.relpath(path, ROOT)}
    return res


def pmc_pass(out, counter, bench_args, kernel_regex, timeout, base=None):
    return pmc_counts(out, [counter], bench_args, kernel_regex, timeout, base=base)[counter]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--kernel-regex", default="k_integrate")
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("--skip-pmc", action="store_true")
    args, bench_args = ap.parse_known_args()
    out = os.path.join(ROOT, "gpurun_out", f"prof_{args.tag}")
    os.makedirs(out, exist_ok=True)

    # 1. kernel trace + stats (same command line as the bench run, minus the CPU leg)
    d = os.path.join(out, "trace")
    stdout = run(rocprof() + ["--kernel-trace", "--stats", "--output-format", "csv", "-d", d, "-o", "run", "--",
                  sys.executable, "bench.py", "--no-cpu-baseline", "--no-extra-configs", "--no-c4", "--no-pmc",
                  *bench_args],
                 args.timeout)
    bench_line = [l for l in stdout.splitlines() if l.startswith("{")]
    stats_csv = find(os.path.join(d, "**", "*kernel_stats.csv"))
    stats = read_csv(stats_csv)
    shutil.copyfile(stats_csv, os.path.join(out, f"{args.tag}_kernel_stats.csv"))
    summary = {"tag": args.tag, "bench_args": bench_args, "kernels": []}
    for r in stats:
        summary["kernels"].append({k: r[k] for k in r})
    summary["bench_line_under_profiler"] = json.loads(bench_line[-1]) if bench_line else None
    # the bench's timed region alone, from the kernel trace: the K dispatches of the kernel
    # the bench ran (config.kernel; kernel="auto" tunes among several during the warm-up)
    # right before the K of the per-dispatch (event-marked) pass, which are the last ones
    bl = summary["bench_line_under_profiler"]
    trace_csv = find(os.path.join(d, "**", "*kernel_trace.csv"))
    if bl and trace_csv:
        meth = {"rk4": 0, "dopri5": 1}[bl["config"]["method"]]
        kern = bl["config"].get("kernel", "direct")
        name = (f"k_integrate_rk4_piped<oe::TwoI, true, {kern[4:].rstrip('x')}>" if kern.startswith("pipe")
                else f"k_integrate<oe::TwoI, {meth}, true, true>")
        hot = [r for r in read_csv(trace_csv) if name in r["Kernel_Name"]]
        hot.sort(key=lambda r: int(r["Start_Timestamp"]))
        k = bl["steps"]
        timed = hot[-2 * k:-k]
        if len(timed) == k:
            durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in timed]
            span = (int(timed[-1]["End_Timestamp"]) - int(timed[0]["Start_Timestamp"])) / 1e6
            summary["timed_region"] = {"kernel": name, "dispatches": k, "mean_dispatch_ms": sum(durs) / k,
                                       "span_ms_per_dispatch": span / k,
                                       "bench_event_kernel_ms": bl["roofline"]["kernel_ms"]}

    # 2./3. HBM traffic per dispatch of the hot kernel, separate PMC passes
    if not args.skip_pmc:
        fetch = pmc_pass(out, "FETCH_SIZE", bench_args, args.kernel_regex, args.timeout)
        write = pmc_pass(out, "WRITE_SIZE", bench_args, args.kernel_regex, args.timeout)
        # units: kilobytes; gfx950 FETCH_SIZE reads half the bytes of a wide coalesced
        # stream (MI355X_MICROARCH.md §HBM) -> x2
        fetch_b = fetch["mean"] * 1024 * 2
        write_b = write["mean"] * 1024
        summary["pmc"] = {"kernel_regex": args.kernel_regex, "FETCH_SIZE_kB_raw": fetch["mean"],
                          "WRITE_SIZE_kB": write["mean"], "fetch_bytes_corrected": fetch_b,
                          "write_bytes": write_b, "hbm_bytes_per_dispatch": fetch_b + write_b,
                          "dispatches": [fetch["dispatches"], write["dispatches"]],
                          "csv": [fetch["csv"], write["csv"]]}
    # written under gpurun_out/ (merged back by gpurun); copy into profiles/ to commit
    with open(os.path.join(out, f"{args.tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary.get("pmc"), indent=1))
    print(json.dumps(summary.get("timed_region"), indent=1))
    for k in summary["kernels"]:
        print({kk: k[kk] for kk in k if kk in ("Name", "Calls", "AverageNs", "TotalDurationNs", "Percentage")})


if __name__ == "__main__":
    main()
