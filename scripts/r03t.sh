set -o pipefail
O=gpurun_out/r03t
mkdir -p $O
export TMPDIR=/tmp
RT_LIST_STATS=1 timeout -k 10 200 python3 profiles/render_tile.py --tile 8,8,0 --reps 1 > $O/stats32.log 2>&1 || exit $?
RT_LIST_STATS=1 timeout -k 10 200 python3 profiles/render_tile.py --tile 8,8,0 --reps 1 --lib build_ab/list64.so > $O/stats64.log 2>&1 || exit $?
timeout -k 10 400 python -u profiles/ab_inproc.py base= list64=build_ab/list64.so --rounds 5 > $O/ab_dragon.txt 2>&1 || exit $?
timeout -k 10 200 python3 profiles/render_tile.py --tile 8,8,0 --reps 3 > $O/tile8_32.log 2>&1 || exit $?
timeout -k 10 200 python3 profiles/render_tile.py --tile 8,8,0 --reps 3 --lib build_ab/list64.so > $O/tile8_64.log 2>&1 || exit $?
