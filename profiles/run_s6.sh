# seed-pass queries end at the first accepted triangle (existence) vs closest hit; + paired steps
set -o pipefail
O=gpurun_out/s6; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "split" > $O/pytest_split.log 2>&1 && \
timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_new.json 2> $O/tiles_new.err && \
RTMI_LIB=ab/noexists.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_noexists.json 2> $O/tiles_noexists.err && \
RTMI_LIB=ab/pair.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_pair.json 2> $O/tiles_pair.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t8 -o run -- python3 profiles/render_tile.py --tile 8,8,0 --reps 3 > $O/t8.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t8p -o run -- python3 profiles/render_tile.py --tile 8,8,0 --reps 3 --lib ab/pair.so > $O/t8p.log 2>&1
