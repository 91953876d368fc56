# coop_round item assignment branch-free (seed pass -6 % static instructions): tiles A/B + split parity
set -o pipefail
O=gpurun_out/s15; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "split" > $O/pytest_split.log 2>&1 && \
timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_new.json 2> $O/tiles_new.err && \
RTMI_LIB=ab/prev.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_prev.json 2> $O/tiles_prev.err && \
timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_new2.json 2> $O/tiles_new2.err && \
RTMI_LIB=ab/prev.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_prev2.json 2> $O/tiles_prev2.err
