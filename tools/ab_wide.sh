# A/B of two library builds on the wide-model DOPRI5 kernels (C3-dopri5 trajectory,
# no-trajectory integrate and MH per iteration): bash tools/ab_wide.sh <tag> [base_lib]
set -o pipefail
tag=$1; base=${2:-alt_lib/base/libodelib_amd.so}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_bench.py --libs base=$base new=odelib_amd/csrc/libodelib_amd.so --reps 3 \
  -- --model chain20 --method dopri5 --walkers 262144 --steps 20 > gpurun_out/${tag}_ab_c3dopri5.log 2>&1 || exit 1
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then L=$base; else L=odelib_amd/csrc/libodelib_amd.so; fi
    ODELIB_AMD_LIB=$L timeout -k 10 200 python -u tools/mh_scaling.py --cases chain20:dopri5 chain10:dopri5 --walkers 262144 --nits 6 \
      | sed "s/^/{\"lib\": \"$lib\", \"rep\": $r} /" >> gpurun_out/${tag}_mh_wide.log 2>&1 || exit 1
  done
done
