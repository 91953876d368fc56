# experiment: throughput from depth + the hit normal in LDS (stack 23): parity subset and A/B
set -o pipefail
O=gpurun_out/s17; mkdir -p $O
RTMI_LIB=ab/hn23.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dragon or golden or tris or split" > $O/pytest_hn23.log 2>&1 && \
timeout -k 10 500 python -u profiles/ab_inproc.py base= hn23=ab/hn23.so d20hn=ab/d20hn.so --rounds 10 > $O/ab.txt 2>&1
