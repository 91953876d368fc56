set -o pipefail
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python profiles/ab_inproc.py aligned= r02=build_ab/r02zz.so --rounds 8 > $O/ab_aligned.txt 2>&1 || exit $?
export TMPDIR=/tmp
for P in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  N=$(echo $P | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $O/aligned_pmc_$N -o run -- python3 bench.py --steps 3 --no-cpu-baseline > $O/aligned_pmc_$N.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err
