#!/bin/bash
# SQ counters of one row-stripe tile's kernels (GPU box), one rocprofv3 --pmc pass per counter set.
# usage: bash profiles/pmc_tile.sh <tag> [render_tile.py args...]  -> gpurun_out/<tag>/pmc_<n>/
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
n=0
for P in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD"; do
  n=$((n + 1))
  timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_$n -o run -- python3 profiles/render_tile.py "$@" > $OUT/pmc_$n.log 2>&1
done
python3 profiles/pmc_tile_summary.py $OUT > $OUT/pmc_summary.txt
