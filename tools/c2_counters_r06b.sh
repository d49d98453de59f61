#!/bin/bash
# Where C2's DOPRI5 wave cycles go (GPU box): one rocprofv3 PMC pass of 8 SQ counters on
# k_integrate<TwoI, dopri5> at 65 536 walkers (issue by instruction type, waits):
#   bash tools/c2_counters_r06b.sh <tag>
set -e
tag=$1
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC"
timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex 'k_integrate' --output-format csv \
  -d gpurun_out/pmc_c2_cycles_$tag -o run -- python3 tools/stiff_bench.py --fracs 0 --methods dopri5 --reps 2
