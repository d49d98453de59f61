#!/bin/bash
# SQ counters of the C2 trajectory kernels (two_i, 65 536 walkers): DOPRI5 (k_integrate<.., 1>) and
# 'auto' without stiff walkers (k_integrate_hq), one rocprofv3 PMC pass each (GPU box):
#   bash tools/c2_counters_r06.sh <tag>
# Per lockstep step: SQ_INSTS_* / SQ_WAVES / steps per wave (tools/lane_steps.py, NOTES round 6).
set -e
tag=$1
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM"
for m in dopri5 auto; do
  timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex 'k_integrate' --output-format csv \
    -d gpurun_out/pmc_c2_${m}_$tag -o run -- python3 tools/stiff_bench.py --fracs 0 --methods $m --reps 2
done
