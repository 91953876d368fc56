#!/bin/bash
# gather microbenchmark sweep (GPU box)
set -e
for MB in 4 16 64; do for G in 64 16 4; do
  timeout -k 10 60 ./profiles/gather_microbench $MB 2000 $G
done; done
