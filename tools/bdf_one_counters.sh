#!/bin/bash
# SQ counters of a lone stiff lane's per-lane BDF pass (tools/bdf_one.py, k_mh), one rocprofv3 --pmc pass
# per library build:  bash tools/bdf_one_counters.sh <tag> [lib.so]   (GPU box)
set -e
tag=$1
lib=${2:-}
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD"
out=gpurun_out/pmc_bdf_one_$tag
if [ -n "$lib" ]; then export ODELIB_AMD_LIB=$lib; fi
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex k_mh --output-format csv -d $out -o run -- python3 tools/bdf_one.py --reps 3
