# A/B of library builds on the stiff MH workloads, interleaved: the lone-lane BDF step
# (tools/bdf_one.py), C2 + 0.1 % stiff (tools/stiff_bench.py) and the notebook fit speculative
# and sequential (tools/demo_fit.py).   bash tools/ab_mh.sh OUTDIR name=lib.so ...
set -euo pipefail
out=$1; shift
mkdir -p "$out"
pick() { python -c "
import json, sys
keys = sys.argv[1].split(',')
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(json.dumps({k: d.get(k) for k in keys}))" "$1"; }
for rep in 1 2; do
  for pair in "$@"; do
    name=${pair%%=*}; export ODELIB_AMD_LIB=$(realpath "${pair#*=}")
    {
      echo "== $name rep $rep"
      timeout -k 10 60 python -u tools/bdf_one.py --case tau1e5 2>&1 | pick case,kernel_ms_min,us_per_step
      timeout -k 10 120 python -u tools/stiff_bench.py --fracs 0.001 --taus 1e5 --methods auto 2>&1 | pick stiff_frac,kernel_ms
      timeout -k 10 200 python -u tools/demo_fit.py --chains 32 --speculate auto 0 2>&1 | pick chains,speculate,wall_s
    } >> "$out/ab_mh.log"
  done
done
