#!/bin/bash
# Env-knob sweep on the GPU box: bash profiles/sweep.sh VAR "v1 v2 ..." [bench args...]
VAR=$1; VALS=$2; shift 2
mkdir -p gpurun_out
for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/sweep.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/sweep.log').read().strip().splitlines()[-1]); print('$VAR=$v', d['value'], d['ms_per_step'], d['roofline'].get('simd_efficiency'))"
done
