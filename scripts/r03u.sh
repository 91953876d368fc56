set -o pipefail
O=gpurun_out/r03u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "sample_split" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for F in 3 1 0; do
RT_SPLIT=1 RT_SPLIT_FUSED=$F timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/f$F -o run -- python3 profiles/render_tile.py --tile 8,8,0 --reps 3 > $O/f$F.log 2>&1 || exit $?
done
