# A/B of the integrate kernels' workgroup-level BDF hand-over (in-tree library) against the
# previous build (alt_lib/head): C2 + 0.1 % / 1 % stiff, and 2 / 4 / 8 stiff walkers
# sharing one wave of a 256-walker workgroup.   bash tools/ab_handover.sh
set -e
ALT=$PWD/alt_lib/head/odelib_amd/csrc/libodelib_amd.so
for rep in 1 2; do
for lib in tree head; do
  if [ $lib = tree ]; then unset ODELIB_AMD_LIB; else export ODELIB_AMD_LIB=$ALT; fi
  echo "== $lib rep $rep"
  timeout -k 10 120 python -u tools/stiff_bench.py --fracs 0.001 0.01 --taus 1e5 --methods auto 2>&1 | grep "{" | cut -c40-200
  timeout -k 10 120 python -u tools/stiff_bench.py --walkers 256 --contiguous --fracs 0.0078125 0.015625 0.03125 --taus 1e5 --methods auto 2>&1 | grep "{" | cut -c20-200
done
done
