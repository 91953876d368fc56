# r03 session 2: list word per pixel (lpack) + 4-item cooperative seed rounds, A/B against HEAD
set -o pipefail
O=gpurun_out/s3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "split or list or golden or oracle" > $O/pytest_quick.log 2>&1 && \
timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_multi.json 2> $O/tiles_multi.err && \
RTMI_LIB=ab/single.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_single.json 2> $O/tiles_single.err && \
RTMI_LIB=ab/base.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_base.json 2> $O/tiles_base.err && \
timeout -k 10 300 python -u profiles/ab_inproc.py base=ab/base.so new= --rounds 6 > $O/ab.txt 2>&1
