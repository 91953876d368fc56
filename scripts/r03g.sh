set -o pipefail
O=gpurun_out/r03g
mkdir -p $O
export BENCH_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --comm torch --steps 3 --warmup 1 > $O/rehearse_strong.json 2> $O/rehearse_strong.err || exit $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --scaling weak --steps 3 --warmup 1 > $O/rehearse_weak.json 2> $O/rehearse_weak.err || exit $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --comm torch --config spheres --steps 10 --warmup 2 > $O/rehearse_spheres.json 2> $O/rehearse_spheres.err || exit $?
unset BENCH_DIST_BACKEND
timeout -k 10 300 python bench.py --config spheres --steps 20 --warmup 3 > $O/bench_spheres.json 2> $O/bench_spheres.err || exit $?
timeout -k 10 300 python bench.py --config bunny --steps 20 --warmup 3 > $O/bench_bunny.json 2> $O/bench_bunny.err || exit $?
timeout -k 10 400 python bench.py --config lucy --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_lucy.json 2> $O/bench_lucy.err || exit $?
