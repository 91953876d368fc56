# k_tris list word in LDS + 23-entry stack: longer A/B, and the tiles
set -o pipefail
O=gpurun_out/s12; mkdir -p $O
timeout -k 10 500 python -u profiles/ab_inproc.py base= d23lw=ab/d23lw.so --rounds 14 > $O/ab.txt 2>&1 && \
RTMI_LIB=ab/d23lw.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_d23lw.json 2> $O/tiles_d23lw.err
