# The hand-over queue against the in-wave BDF pass over ensemble sizes (one library, OE_NO_HANDQ
# for the in-wave runs): bash tools/ab_handq_w.sh OUTDIR lib.so
set -euo pipefail
out=$1; lib=$(realpath "$2")
mkdir -p "$out"
for W in 1024 4096 16384 65536; do
  for hq in 1 0; do
    ODELIB_AMD_LIB=$lib timeout -k 10 200 python -u tools/stiff_bench.py --walkers $W --fracs 0 0.001 0.01 \
      --taus 1e5 --methods auto --reps 5 --handq $hq >> "$out/handq_w.log" 2>&1
  done
done
