set -o pipefail
O=gpurun_out/r03x
mkdir -p $O
export TMPDIR=/tmp
for V in seedu4 seedu6 seedu8; do
L=""; if [ $V != base ]; then L="--lib build_ab/$V.so"; fi
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$V -o run -- python3 profiles/render_tile.py --tile 8,8,0 --reps 3 $L > $O/$V.log 2>&1 || exit $?
done
