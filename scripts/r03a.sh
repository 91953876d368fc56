set -o pipefail
mkdir -p gpurun_out/r03a
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03a/pytest.log 2>&1
rc=$?
echo "pytest rc $rc" >> gpurun_out/r03a/pytest.log
# test failures (1) still leave a healthy GPU; anything else (timeout, abort, fault) ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err
