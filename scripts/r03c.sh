set -o pipefail
O=gpurun_out/r03c
mkdir -p $O
RTMI_LIB=build_ab/diag1.so timeout -k 10 400 python profiles/chain_alone.py --pixels 1844,198 1807,633 --k 1 2 4 8 16 32 64 > $O/chain_k.jsonl 2> $O/chain_k.err || exit $?
for s in 1 0; do RT_SCHEDULE=$s timeout -k 10 200 python bench.py --config bunny --steps 20 --warmup 3 --no-cpu-baseline > $O/bunny_sched$s.json 2>> $O/bunny.err || exit $?; done
bash profiles/run_profile.sh r03c --steps 3 --no-cpu-baseline || exit $?
bash profiles/pmc_extra.sh r03c --steps 3 --no-cpu-baseline || exit $?
