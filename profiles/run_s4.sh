# A/B: HEAD vs coop_round + per-pixel list word in the seed pass (k_tris unchanged); seed-pass unroll 2/4/6
set -o pipefail
O=gpurun_out/s4; mkdir -p $O
timeout -k 10 300 python -u profiles/ab_inproc.py base=ab/base.so new= --rounds 6 > $O/ab.txt 2>&1 && \
timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_new.json 2> $O/tiles_new.err && \
RTMI_LIB=ab/u2.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_u2.json 2> $O/tiles_u2.err && \
RTMI_LIB=ab/u6.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_u6.json 2> $O/tiles_u6.err && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
