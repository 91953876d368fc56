# same-box check: stack 23 without the hit normal in LDS (f04fd2f) vs the current build (stack 20 + normal in LDS)
set -o pipefail
O=gpurun_out/s19; mkdir -p $O
timeout -k 10 500 python -u profiles/ab_inproc.py cur= s23=ab/s23.so --rounds 10 > $O/ab.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_cur.json 2> $O/bench_cur.err && \
RTMI_LIB=ab/s23.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_s23.json 2> $O/bench_s23.err
