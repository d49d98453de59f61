# One workgroup (256 walkers) with 1 / 2 / 4 stiff walkers (tau = 1e5), 'auto' with trajectories:
# the kernel time is the stiff walkers' hand-over + BDF pass (tools/stiff_bench.py), per build.
#   bash tools/ab_lone_stiff.sh OUTDIR name=lib.so [name=lib.so ...]
set -euo pipefail
out=$1; shift
mkdir -p "$out"
for pair in "$@"; do
  name=${pair%%=*}; lib=${pair#*=}
  for n in 1 2 4; do
    ODELIB_AMD_LIB=$(realpath "$lib") timeout -k 10 120 python -u tools/stiff_bench.py --walkers 256 \
      --fracs $(python3 -c "print($n/256)") --taus 1e5 --methods auto --reps 5 --contiguous >> "$out/${name}_lone.log" 2>&1
  done
done
