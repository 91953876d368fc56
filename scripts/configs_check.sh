#!/bin/bash
# GPU box: the bench's other configurations at N=1, and the N>1 code path rehearsed with
# two ranks on the one GPU over gloo (strong-scaling row stripes, the default; weak-scaling frames).
# usage: bash scripts/configs_check.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-cfg}
mkdir -p $OUT
for c in bunny spheres lucy; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 3 > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
done
export BENCH_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --scaling weak > $OUT/rehearse_weak.json 2> $OUT/rehearse_weak.err || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --scaling strong > $OUT/rehearse_strong.json 2> $OUT/rehearse_strong.err || exit 1
echo ok
