# tree top levels in LDS for the long-chain seed pass (0 / 85 / 341 nodes), then the round check
set -o pipefail
O=gpurun_out/s8; mkdir -p $O
for v in top0 top85 top341; do
  RTMI_LIB=ab/$v.so timeout -k 10 200 python -u profiles/tile_scaling.py > $O/tiles_$v.json 2> $O/tiles_$v.err || exit 1
done
bash scripts/round_check.sh r03z
