set -o pipefail
O=gpurun_out/r03y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "sample_split or schedule_changes or traversal_switch" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t8 -o run -- python3 profiles/render_tile.py --tile 8,8,0 --reps 3 > $O/t8.log 2>&1 || exit $?
timeout -k 10 300 python -u profiles/tile_scaling.py > $O/tiles.json 2> $O/tiles.err || exit $?
