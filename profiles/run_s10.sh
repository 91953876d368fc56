# experiment: shadow rays pass over their origin triangle (timing only)
set -o pipefail
O=gpurun_out/s10; mkdir -p $O
timeout -k 10 300 python -u profiles/ab_inproc.py base= skipown=ab/skipown.so --rounds 6 > $O/ab.txt 2>&1
