set -o pipefail
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 240 python -u profiles/occupancy.py --config bunny > $O/occ_bunny.txt 2>&1 || exit $?
timeout -k 10 240 python -u profiles/occupancy.py --config bunny > $O/occ_bunny2.txt 2>&1 || exit $?
