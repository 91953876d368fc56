set -o pipefail
O=gpurun_out/r03s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "sample_split" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
RT_SPLIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/split8 -o run -- python3 profiles/render_tile.py --tile 8,8,0 --reps 2 > $O/split8.log 2>&1 || exit $?
RT_SPLIT=1 timeout -k 10 300 python -u profiles/tile_scaling.py > $O/tiles_split.json 2> $O/tiles_split.err || exit $?
