#!/bin/bash
# Instruction-fetch counters of the notebook fit's speculative rounds (k_mh_tree, tools/demo_fit.py)
# and of C2 + 0.1 % stiff (k_integrate, tools/stiff_bench.py): is the instruction cache a limit
# when several waves of one CU run the large per-lane DOPRI5 + BDF code at different places?
#   bash tools/fit_fetch.sh <tag>      (GPU box; one rocprofv3 PMC pass per counter set)
set -e
tag=$1
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
C2="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex k_mh_tree --output-format csv -d gpurun_out/pmc_fit_sq_$tag -o run -- python3 tools/demo_fit.py --chains 32 --speculate auto
timeout -s KILL 150 rocprofv3 --pmc $C2 --kernel-include-regex k_mh_tree --output-format csv -d gpurun_out/pmc_fit_ic_$tag -o run -- python3 tools/demo_fit.py --chains 32 --speculate auto
timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex k_integrate --output-format csv -d gpurun_out/pmc_smix_sq_$tag -o run -- python3 tools/stiff_bench.py --fracs 0.001 --taus 1e5 --methods auto --reps 1
timeout -s KILL 150 rocprofv3 --pmc $C2 --kernel-include-regex k_integrate --output-format csv -d gpurun_out/pmc_smix_ic_$tag -o run -- python3 tools/stiff_bench.py --fracs 0.001 --taus 1e5 --methods auto --reps 1
