set -o pipefail
O=gpurun_out/r03q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "sample_split" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
RT_SPLIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/split8 -o run -- python3 profiles/render_tile.py --tile 8,8,0 > $O/split8.log 2>&1 || exit $?
RT_SPLIT=1 RT_SPLIT_PROBE=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/split8_lane -o run -- python3 profiles/render_tile.py --tile 8,8,0 > $O/split8_lane.log 2>&1 || exit $?
