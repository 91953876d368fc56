# re-tune after the LDS changes: completed queries per stepping round 16/24/32, steps per exit check 4/6/8
set -o pipefail
O=gpurun_out/s23; mkdir -p $O
timeout -k 10 600 python -u profiles/ab_inproc.py base= fk16=ab/fk16.so fk32=ab/fk32.so su4=ab/su4.so su8=ab/su8.so --rounds 6 > $O/ab.txt 2>&1
