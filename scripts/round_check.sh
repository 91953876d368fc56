#!/bin/bash
# Round-end style check on the GPU box: GPU parity tests, smoke, default bench (with CPU
# baseline), then the rocprofv3 kernel-trace + PMC passes of the same bench command.
# usage: bash scripts/round_check.sh <tag>
set -o pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
bash profiles/run_profile.sh $TAG --steps 3 --no-cpu-baseline && \
bash profiles/pmc_extra.sh $TAG --steps 3 --no-cpu-baseline
