#!/bin/bash
# A/B of a measurement build (alt_lib/<name>) against the in-tree library on one box:
# lone-lane BDF step cost (tools/bdf_one.py), C2 + 0.1 % stiff (tools/stiff_bench.py), the
# notebook fit (tools/demo_fit.py); two rounds each.   bash tools/ab_bdf.sh <name>
set -e
ALT=$PWD/alt_lib/$1/odelib_amd/csrc/libodelib_amd.so
pick() { python -c "
import json, sys
keys = sys.argv[1].split(',')
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(json.dumps({k: d.get(k) for k in keys}))" "$1"; }
for rep in 1 2; do
for lib in tree $1; do
  if [ $lib = tree ]; then unset ODELIB_AMD_LIB; else export ODELIB_AMD_LIB=$ALT; fi
  echo "== $lib rep $rep"
  timeout -k 10 60 python -u tools/bdf_one.py --case tau1e5 2>&1 | pick case,kernel_ms_min,us_per_step
  timeout -k 10 120 python -u tools/stiff_bench.py --fracs 0.001 --taus 1e5 --methods auto 2>&1 | pick stiff_frac,kernel_ms
  timeout -k 10 120 python -u tools/demo_fit.py --chains 32 --speculate auto 0 2>&1 | pick chains,speculate,wall_s
done
done
