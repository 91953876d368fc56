#!/bin/bash
# Steady-state profile of the headline kernel (GPU box): profiles/steady_state.py under rocprofv3 —
# one kernel-trace + stats pass, then every counter group in its own --pmc pass (MI355X_MICROARCH.md
# §rocprofv3: no --pmc together with the trace domains).  summarize with
#   python profiles/summarize_pmc.py <tag> gpurun_out/prof_<tag> "<workload>" --last <frames>
# usage: bash profiles/profile_steady.sh <tag> [frames]
set -e
TAG=$1
FR=${2:-8}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 profiles/steady_state.py --frames $FR > $OUT/driver.json 2> $OUT/trace.log
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
         "GRBM_GUI_ACTIVE GRBM_COUNT" "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
         "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES"; do
  N=$(echo $P | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_$N -o run -- \
      python3 profiles/steady_state.py --frames $FR > $OUT/pmc_$N.log 2>&1
done
echo done
