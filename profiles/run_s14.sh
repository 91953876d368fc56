# PMC of the 8-way tile's kernels (the long-chain seed pass): instructions and wave cycles
set -o pipefail
O=gpurun_out/s14; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --output-format csv -d $O/pmc1 -o run -- python3 profiles/render_tile.py --tile 8,8,0 --reps 2 > $O/pmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2 -o run -- python3 profiles/render_tile.py --tile 8,8,0 --reps 2 > $O/pmc2.log 2>&1
