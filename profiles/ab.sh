#!/bin/bash
# A/B timing of two in-tree builds of librtmi.so on the GPU box (alternating runs).
# usage: bash profiles/ab.sh <libA> <libB> <rounds> [bench args...]
A=$1; B=$2; R=$3; shift 3
for i in $(seq 1 $R); do
  for L in $A $B; do
    RTMI_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$(basename $L)', d['value'], d['ms_per_step'])"
  done
done
