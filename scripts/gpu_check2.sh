set -o pipefail
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s2/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s2/bench.json 2> gpurun_out/s2/bench.err && \
timeout -k 10 300 python profiles/tile_scaling.py > gpurun_out/s2/tiles.json 2> gpurun_out/s2/tiles.err
