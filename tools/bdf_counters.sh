#!/bin/bash
# SQ counters of the BDF trajectory kernel (two_i, 65 536 demo walkers, every walker BDF),
# one rocprofv3 --pmc pass (GPU box):  bash tools/bdf_counters.sh <tag>
set -e
tag=$1
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
run() { timeout -k 10 200 python -u tools/pmc_counters.py --one-pass --counters $C --kernel-regex 'k_integrate' "$@"; }
run --tag ${tag}_bdf -- --method bdf --kernel direct --steps 3 --warmup 1
run --tag ${tag}_dopri5 -- --method dopri5 --kernel direct --steps 3 --warmup 1
