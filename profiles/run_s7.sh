# long-chain seed pass: chains per wave 16 (default) / 8 / 4 on the 8-way tile; seed-pass chain stats
set -o pipefail
O=gpurun_out/s7; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_new.json 2> $O/tiles_new.err && \
RTMI_LIB=ab/gpw8.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_gpw8.json 2> $O/tiles_gpw8.err && \
RTMI_LIB=ab/gpw4.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_gpw4.json 2> $O/tiles_gpw4.err && \
timeout -k 10 200 python -u profiles/seed_stats.py --tile 8,8,0 > $O/seed_stats.json 2> $O/seed_stats.err
