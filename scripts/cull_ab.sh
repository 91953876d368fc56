set -o pipefail
O=gpurun_out/cull
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for r in 1 2; do
  for c in 0 1; do
    RT_CULL_UNHITTABLE=$c timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 > $O/dragon_c${c}_r${r}.json 2> $O/err.log || exit 1
  done
done
timeout -k 10 300 python bench.py --config lucy --no-cpu-baseline --steps 2 > $O/lucy_c1.json 2> $O/err_lucy.log || exit 1
echo ok
