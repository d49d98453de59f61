# A/B of the 'auto' integrate kernels on C2 + stiff walkers (tools/stiff_bench.py), interleaved
# over library builds: bash tools/ab_stiffmix.sh OUTDIR name=lib.so ...  LONE=1 adds one workgroup
# (256 walkers) with 1 / 2 / 4 contiguous stiff walkers.
set -euo pipefail
out=$1; shift
mkdir -p "$out"
for rep in 1 2; do
  for pair in "$@"; do
    name=${pair%%=*}; lib=${pair#*=}
    ODELIB_AMD_LIB=$(realpath "$lib") timeout -k 10 300 python -u tools/stiff_bench.py --fracs 0 0.001 0.01 \
      --taus 1e5 --methods auto --reps 5 > "$out/${name}_${rep}.log" 2>&1
    if [[ ${LONE:-0} == 1 && $rep == 1 ]]; then
      for n in 1 2 4; do
        ODELIB_AMD_LIB=$(realpath "$lib") timeout -k 10 120 python -u tools/stiff_bench.py --walkers 256 \
          --fracs $(python3 -c "print($n/256)") --taus 1e5 --methods auto --reps 5 --contiguous \
          >> "$out/${name}_lone.log" 2>&1
      done
    fi
  done
done
