#!/bin/bash
# two_i DOPRI5 MH: one lane per chain (product, per-lane steps) vs the chain over 4 lanes
# (split.cuh, OE_SPLIT_TWOI=4 measurement build: one state per lane, 16 chains per step size)
set -e
ALT=$PWD/alt_lib/split4/odelib_amd/csrc/libodelib_amd.so
ODELIB_AMD_LIB=$ALT timeout -k 10 120 python -u tools/check_split_twoi.py 4
for lib in one split4; do
  if [ $lib = split4 ]; then export ODELIB_AMD_LIB=$ALT; else unset ODELIB_AMD_LIB; fi
  echo "== $lib"
  timeout -k 10 200 python -u tools/lane_cost.py 2>&1 | grep '"dopri5"'
  timeout -k 10 200 python -u tools/demo_fit.py --chains 32 1024 --method dopri5 --speculate auto 0 2>&1 | grep "{" | cut -c1-160
done
