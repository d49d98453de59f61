#!/bin/bash
# SQ counters of the C2 DOPRI5 trajectory kernel, direct (one wave per 64 walkers) vs the
# store-wave kernel (k_integrate_dopri5_piped, OE_PIPE), one rocprofv3 --pmc pass each
# (GPU box):  bash tools/c2_counters.sh <tag>
set -e
tag=$1
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
run() { timeout -k 10 200 python -u tools/pmc_counters.py --one-pass --counters $C --kernel-regex 'k_integrate' "$@"; }
run --tag ${tag}_c2_direct -- --method dopri5 --kernel direct --steps 5 --warmup 1
run --tag ${tag}_c2_storewaves -- --method dopri5 --kernel pipe2 --steps 5 --warmup 1
