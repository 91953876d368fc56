# experiment: k_tris list word in LDS, with the stack one entry shorter so that LDS stays 31232 B/block
set -o pipefail
O=gpurun_out/s11; mkdir -p $O
timeout -k 10 400 python -u profiles/ab_inproc.py base= d23=ab/d23.so d23lw=ab/d23lw.so --rounds 6 > $O/ab.txt 2>&1
