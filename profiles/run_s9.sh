# full frame: all pixels / mesh pixels only / box pixels only (diagnostics builds; wrong frames, times only)
set -o pipefail
O=gpurun_out/s9; mkdir -p $O
timeout -k 10 200 python -u profiles/render_tile.py --reps 4 > $O/full.txt 2>&1 && \
timeout -k 10 200 python -u profiles/render_tile.py --reps 4 --lib ab/skipbox.so > $O/meshonly.txt 2>&1 && \
timeout -k 10 200 python -u profiles/render_tile.py --reps 4 --lib ab/skipmesh.so > $O/boxonly.txt 2>&1
