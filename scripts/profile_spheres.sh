#!/bin/bash
# Kernel-trace + PMC passes of the sphere configuration (bench.py --config spheres): the VALU /
# transcendental-bound raytrace kernel.  usage (GPU box): bash scripts/profile_spheres.sh <tag>
set -o pipefail
TAG=${1:-spheres}
timeout -k 10 120 python bench.py --config spheres --steps 50 --warmup 5 --no-cpu-baseline \
    > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err && \
bash profiles/run_profile.sh $TAG --config spheres --steps 50 --warmup 5 --no-cpu-baseline && \
bash profiles/pmc_extra.sh $TAG --config spheres --steps 50 --warmup 5 --no-cpu-baseline
