#!/bin/bash
# C1 under each walker-block order (bench.py --xcd), back-to-back bench runs on one box,
# with the box's write ceiling beside each (GPU box):  bash tools/ab_xcd.sh <tag>
tag=$1
for x in runs ranges off runs; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --mcmc-iters 0 --no-extra-configs --no-c4 --no-pmc \
    --steps 20 --xcd $x > gpurun_out/${tag}_xcd_$x.log 2>&1 || exit 1
  python - "$x" "gpurun_out/${tag}_xcd_$x.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
r = d["roofline"]
print(sys.argv[1], round(r["kernel_ms"], 4), round(r["frac"], 3), "fill", round(r["box_write_ceiling"]["ms"], 4), flush=True)
PY
done
