# experiment: the closest hit's normal formed at its accept and kept in LDS (stack 20 entries to fit)
set -o pipefail
O=gpurun_out/s16; mkdir -p $O
timeout -k 10 500 python -u profiles/ab_inproc.py base= d20=ab/d20.so d20hn=ab/d20hn.so --rounds 10 > $O/ab.txt 2>&1
