set -o pipefail
mkdir -p gpurun_out/s1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s1/pytest.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s1/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/s1/bench.json 2> gpurun_out/s1/bench.err
