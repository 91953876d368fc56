#!/bin/bash
# Build librtmi.so with extra compile definitions into OUT (A/B experiments, container side).
# usage: bash profiles/build_variant.sh OUT.so -DNAME=VALUE ...
set -e
OUT=$(realpath -m $1); shift
SRC=${SRC_DIR:-$(dirname $(realpath $0))/../pathtracer.cl_amd/csrc}
B=$(mktemp -d)
cd $SRC
FL="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wno-unused-function -I../../include -I. $@"
DEV="--offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics"
/opt/rocm/bin/hipcc $FL $DEV -c -o $B/k.o rt_kernels.hip &
/opt/rocm/bin/hipcc $FL -c -o $B/h.o rt_host.cpp &
/opt/rocm/bin/hipcc $FL -c -o $B/b.o rt_bvh.cpp &
/opt/rocm/bin/hipcc $FL -c -o $B/p.o rt_ply.cpp &
/opt/rocm/bin/hipcc $FL $DEV -c -o $B/g.o rt_build_gpu.hip &
/opt/rocm/bin/hipcc $FL $DEV -c -o $B/c.o rt_comm.hip &
/opt/rocm/bin/hipcc $FL $DEV -c -o $B/s.o rt_sched.hip &
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT $B/k.o $B/h.o $B/b.o $B/p.o $B/g.o $B/c.o $B/s.o -lpthread \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf $B
echo built $OUT
