set -o pipefail
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 240 python -u profiles/occupancy.py --tile 8,8,0 > $O/occ_n8.txt 2>&1 || exit $?
