#!/bin/bash
# A/B/n timing on the GPU box: each argument "LABEL:ENV=V,ENV=V:LIB" (ENV part may be empty,
# LIB empty = the in-tree build); ROUNDS alternating passes; bench args via BENCH_ARGS.
R=${ROUNDS:-2}
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for spec in "$@"; do
    IFS=: read -r LABEL ENVS LIB <<< "$spec"
    E=""; [ -n "$ENVS" ] && E=$(echo $ENVS | tr ',' ' ')
    [ -n "$LIB" ] && E="$E RTMI_LIB=$LIB"
    env $E timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:---steps 3} > gpurun_out/abn.log 2>&1 || { tail -5 gpurun_out/abn.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abn.log').read().strip().splitlines()[-1]); print('$LABEL', d['value'], d['ms_per_step'])"
  done
done
