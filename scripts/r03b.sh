set -o pipefail
O=gpurun_out/r03b
mkdir -p $O
# 1) a pixel's chain with the megakernel to itself (diagnostics build)
RTMI_LIB=build_ab/diag1.so timeout -k 10 300 python profiles/chain_alone.py > $O/chain_alone.jsonl 2> $O/chain_alone.err || exit $?
# 2) the other BASELINE configurations with their CPU baseline (bit-exact flags)
timeout -k 10 300 python bench.py --config spheres --steps 20 --warmup 3 > $O/bench_spheres.json 2> $O/bench_spheres.err || exit $?
timeout -k 10 300 python bench.py --config bunny --steps 20 --warmup 3 > $O/bench_bunny.json 2> $O/bench_bunny.err || exit $?
# 3) kernel statistics of the headline bench command
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
