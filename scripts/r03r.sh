set -o pipefail
O=gpurun_out/r03r
mkdir -p $O
export TMPDIR=/tmp
for G in 16 4 1; do
RT_SPLIT=1 RT_SPLIT_SERIAL=1 RT_SPLIT_GPW=$G timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/serial_g$G -o run -- python3 profiles/render_tile.py --tile 8,8,0 --reps 2 > $O/serial_g$G.log 2>&1 || exit $?
done
