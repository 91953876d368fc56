set -o pipefail
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 600 python profiles/tile_scaling.py --config dragon > $O/tile_scaling_dragon.json 2> $O/tile_scaling_dragon.err || exit $?
timeout -k 10 600 python profiles/tile_scaling.py --config lucy > $O/tile_scaling_lucy.json 2> $O/tile_scaling_lucy.err || exit $?
bash profiles/run_profile.sh r03f --steps 3 --no-cpu-baseline || exit $?
bash profiles/pmc_extra.sh r03f --steps 3 --no-cpu-baseline || exit $?
