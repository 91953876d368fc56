set -o pipefail
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 400 python profiles/ab_inproc.py tile16= fixed=build_ab/fixed_lists.so r02=build_ab/r02zz.so --rounds 8 > $O/ab_lists.txt 2>&1 || exit $?
export TMPDIR=/tmp
for P in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  N=$(echo $P | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $O/tile16_pmc_$N -o run -- python3 bench.py --steps 3 --no-cpu-baseline > $O/tile16_pmc_$N.log 2>&1 || exit $?
  RTMI_LIB=build_ab/fixed_lists.so timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $O/fixed_pmc_$N -o run -- python3 bench.py --steps 3 --no-cpu-baseline > $O/fixed_pmc_$N.log 2>&1 || exit $?
  RTMI_LIB=build_ab/r02zz.so timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $O/r02_pmc_$N -o run -- python3 bench.py --steps 3 --no-cpu-baseline > $O/r02_pmc_$N.log 2>&1 || exit $?
done
