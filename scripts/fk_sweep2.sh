# fetch_k x fetch_k_box grid on the dragon frame (GPU box)
set -o pipefail
for p in "24 16" "32 16" "40 16" "24 24" "32 32" "24 8" "24 16" "32 16"; do
  set -- $p
  RT_FETCH_K=$1 RT_FETCH_K_BOX=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/sweep.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/sweep.log').read().strip().splitlines()[-1]); print('fk=$1 fkbox=$2', d['value'], d['ms_per_step'])"
done
