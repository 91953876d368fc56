# the other BASELINE configurations with the final build (each line with its CPU baseline and bit-exact flag)
set -o pipefail
O=gpurun_out/r03zd; mkdir -p $O
timeout -k 10 300 python bench.py --config bunny > $O/bench_bunny.json 2> $O/bench_bunny.err && \
timeout -k 10 300 python bench.py --config spheres > $O/bench_spheres.json 2> $O/bench_spheres.err
