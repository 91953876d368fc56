set -o pipefail
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 400 python -u profiles/ab_inproc.py base= batch=build_ab/batch.so --rounds 6 > $O/ab_dragon.txt 2>&1 || exit $?
timeout -k 10 200 python -u profiles/ab_inproc.py base= batch=build_ab/batch.so --rounds 20 --config bunny > $O/ab_bunny.txt 2>&1 || exit $?
