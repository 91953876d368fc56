#!/bin/bash
# usage (GPU box): bash profiles/fetch_ab.sh <outdir> "ENV=.. ENV=.." ...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
i=0
for cfg in "$@"; do
  env $cfg timeout -k 10 240 python -u profiles/fetch_ab.py >> $OUT/ab.jsonl 2>> $OUT/ab.err || exit 1
  i=$((i+1))
done
echo done
