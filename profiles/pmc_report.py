"""Print the per-launch PMC counters of the triangle kernel from profiles/pmc_extra.sh output.

    python profiles/pmc_report.py gpurun_out/prof_<tag> [kernel substring]
"""
import glob
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from summarize_pmc import counters  # full-size dispatches only (the bench's 1-row tile launches excluded)

src = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "k_tris<4, false, false>"
c = counters(sorted(glob.glob(f"{src}/pmcx_*/run_counter_collection.csv")), kname)
for k in sorted(c):
    print(f"{k:40s} {c[k]:.4g}")
cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
if cyc:
    print(f"kernel cycles (per XCD)                  {cyc:.4g}")
    if "TA_BUSY_avr" in c:
        print(f"TA busy fraction                         {c['TA_BUSY_avr'] / cyc:.3f}")
    if "SQ_INSTS_VALU" in c:
        print(f"VALU issue fraction (2 cyc/inst, 4 SIMD) {c['SQ_INSTS_VALU'] / 256 * 2 / 4 / cyc:.3f}")
    if "SQ_INSTS_VMEM_RD" in c:
        print(f"TA cycles per VMEM read instruction      {c.get('TA_BUSY_avr', 0) / (c['SQ_INSTS_VMEM_RD'] / 256):.2f}")
if "SQ_WAVE_CYCLES" in c:
    for k in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY"):
        if k in c:
            print(f"{k + ' / SQ_WAVE_CYCLES':40s} {c[k] / c['SQ_WAVE_CYCLES']:.3f}")
