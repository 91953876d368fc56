set -o pipefail
mkdir -p gpurun_out/s2
timeout -k 10 300 python -u profiles/ab_inproc.py base=ab/base.so new= --rounds 6 > gpurun_out/s2/ab.txt 2>&1 && \
timeout -k 10 200 python -u profiles/tile_scaling.py > gpurun_out/s2/tiles_new.json 2> gpurun_out/s2/tiles_new.err && \
RTMI_LIB=ab/base.so timeout -k 10 200 python -u profiles/tile_scaling.py > gpurun_out/s2/tiles_base.json 2> gpurun_out/s2/tiles_base.err && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s2/pytest.log 2>&1
