# seed pass without VGPR spills (partly taken leaf written back early): split parity + tiles A/B
set -o pipefail
O=gpurun_out/s20; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "split" > $O/pytest_split.log 2>&1 && \
timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_new.json 2> $O/tiles_new.err && \
RTMI_LIB=ab/head.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_head.json 2> $O/tiles_head.err && \
timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_new2.json 2> $O/tiles_new2.err && \
RTMI_LIB=ab/head.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_head2.json 2> $O/tiles_head2.err
