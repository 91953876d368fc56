set -o pipefail
O=gpurun_out/r03m
mkdir -p $O
export TMPDIR=/tmp
RT_SPLIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/split8 -o run -- python3 profiles/render_tile.py --tile 8,8,0 > $O/split8.log 2>&1 || exit $?
RT_SPLIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/split1 -o run -- python3 profiles/render_tile.py --reps 2 > $O/split1.log 2>&1 || exit $?
