set -e
OLD=$PWD/alt_lib/r05mh/odelib_amd/csrc/libodelib_amd.so
for rep in 1 2; do
for lib in new old; do
  if [ $lib = old ]; then export ODELIB_AMD_LIB=$OLD; else unset ODELIB_AMD_LIB; fi
  echo "== $lib rep $rep" >> gpurun_out/r05f_ab.log
  timeout -k 10 120 python -u tools/demo_fit.py --chains 32 --speculate auto 0 2>&1 | grep "{" >> gpurun_out/r05f_ab.log
  timeout -k 10 120 python -u tools/stiff_bench.py --fracs 0.001 --taus 1e5 --methods auto bdf >> gpurun_out/r05f_ab.log 2>&1
  timeout -k 10 60 python -u tools/bdf_one.py --case tau1e5 >> gpurun_out/r05f_ab.log 2>&1
done
done
