# last check of the round's final build: GPU tests, smoke, bench (with the CPU baseline), tiles
set -o pipefail
O=gpurun_out/r03zd; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles.json 2> $O/tiles.err
