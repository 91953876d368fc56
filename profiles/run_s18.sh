# final round check of the build with the hit normal in LDS (stack 20): tests, smoke, bench, PMC, tiles
set -o pipefail
bash scripts/round_check.sh r03zc && \
timeout -k 10 200 python -u profiles/tile_scaling.py > gpurun_out/r03zc/tiles.json 2> gpurun_out/r03zc/tiles.err
