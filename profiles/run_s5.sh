# paired leaf steps in the one-lane seed pass (A/B on tiles) + kernel traces of the 8-way tile
set -o pipefail
O=gpurun_out/s5; mkdir -p $O
export TMPDIR=/tmp
RTMI_LIB=ab/pair.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_pair.json 2> $O/tiles_pair.err && \
timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_new.json 2> $O/tiles_new.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t8 -o run -- python3 profiles/render_tile.py --tile 8,8,0 --reps 3 > $O/t8.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t8p -o run -- python3 profiles/render_tile.py --tile 8,8,0 --reps 3 --lib ab/pair.so > $O/t8p.log 2>&1
