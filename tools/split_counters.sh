#!/bin/bash
# SQ counters of the DOPRI5 kernels, one lane vs split, one rocprofv3
# --pmc pass per case (GPU box):  bash tools/split_counters.sh <tag>
# C2: two_i 65 536 walkers, the product library (one lane) and the OE_SPLIT_TWOI
# measurement library (alt_lib/split2, two lanes); C3-dopri5: chain20 262 144 walkers,
# split (product) and --no-split.  (alt_lib/ is gpurun-ignored: drop that line to rerun.)
set -e
tag=$1
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
run() { timeout -k 10 200 python -u tools/pmc_counters.py --one-pass --counters $C --kernel-regex 'k_integrate' "$@"; }
run --tag ${tag}_c2_onelane -- --method dopri5 --steps 5 --warmup 1
ODELIB_AMD_LIB=alt_lib/split2/odelib_amd/csrc/libodelib_amd.so run --tag ${tag}_c2_split -- --method dopri5 --steps 5 --warmup 1
run --tag ${tag}_c3_split -- --model chain20 --walkers 262144 --method dopri5 --steps 3 --warmup 1
run --tag ${tag}_c3_onelane -- --model chain20 --walkers 262144 --method dopri5 --steps 3 --warmup 1 --no-split
