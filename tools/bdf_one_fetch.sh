#!/bin/bash
# instruction-fetch counters of a lone stiff lane's per-lane BDF pass (tools/bdf_one.py, k_mh)
set -e
tag=$1
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_WAIT_ANY SQ_INSTS_VALU"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex k_mh --output-format csv -d gpurun_out/pmc_bdf_fetch_$tag -o run -- python3 tools/bdf_one.py --reps 3
C2="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
timeout -s KILL 120 rocprofv3 --pmc $C2 --kernel-include-regex k_mh --output-format csv -d gpurun_out/pmc_bdf_icache_$tag -o run -- python3 tools/bdf_one.py --reps 3
