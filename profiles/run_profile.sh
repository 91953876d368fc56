#!/bin/bash
# Profiling recipe (GPU box): kernel-trace stats + separate PMC passes (MI355X_MICROARCH.md §rocprofv3).
# usage: bash scripts_prof.sh <tag> [bench args...]
set -e
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py "$@" > $OUT/trace.log 2>&1
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  N=$(echo $P | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_$N -o run -- python3 bench.py "$@" > $OUT/pmc_$N.log 2>&1
done
echo done
