set -o pipefail
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 300 python profiles/occupancy.py --config dragon > $O/occupancy_full.json 2> $O/occ.err || exit $?
timeout -k 10 300 python profiles/occupancy.py --config dragon --tile 8,8,0 > $O/occupancy_n8.json 2>> $O/occ.err || exit $?
timeout -k 10 300 python profiles/occupancy.py --config dragon --tile 8,2,0 > $O/occupancy_n2.json 2>> $O/occ.err || exit $?
