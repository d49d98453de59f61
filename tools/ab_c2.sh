set -euo pipefail
out=$1; shift
mkdir -p "$out"
for rep in 1 2 3; do
  for pair in "$@"; do
    name=${pair%%=*}; lib=${pair#*=}
    ODELIB_AMD_LIB=$(realpath "$lib") timeout -k 10 200 python -u tools/stiff_bench.py --fracs 0 0.001 \
      --taus 1e5 --methods dopri5 auto --reps 5 2>&1 | grep '^{' | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l)
    if d['method']=='dopri5' and d['stiff_frac']>0: continue
    print('$name', d['method'], d['stiff_frac'], d['kernel_ms'])" >> "$out/ab_c2.log"
  done
done
