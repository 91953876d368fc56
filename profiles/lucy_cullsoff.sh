#!/bin/bash
# The Lucy-class configuration (BASELINE configs[4]: 28,055,742 triangles, 4096x4096, sampleRate 4) with
# both host-build culls off (RT_DET_CULL=0, RT_CULL_UNHITTABLE=0: all 28M triangles in the tree, the same
# bits — test_tree_cull_knobs_change_no_bits), so the frame traverses the whole mesh: the bench line,
# a kernel-trace pass and the HBM counter passes (each its own rocprofv3 --pmc run).  GPU box.
# usage: bash profiles/lucy_cullsoff.sh <tag>
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT/prof
export TMPDIR=/tmp
export RT_DET_CULL=0 RT_CULL_UNHITTABLE=0
ARGS="--config lucy --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 python3 -u bench.py $ARGS > $OUT/bench_lucy_cullsoff.json 2> $OUT/bench_lucy_cullsoff.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof/trace -o run -- \
    python3 bench.py $ARGS > $OUT/prof/trace.log 2>&1
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  N=$(echo $P | cut -d' ' -f1)
  timeout -k 10 600 rocprofv3 --pmc $P --output-format csv -d $OUT/prof/pmc_$N -o run -- \
      python3 bench.py $ARGS > $OUT/prof/pmc_$N.log 2>&1
done
echo done
