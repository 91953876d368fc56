"""Summarise a profiles/run_profile.sh run into profiles/<tag>/pmc_summary.json.

Per launch of the timed triangle kernel (k_tris<false, false>):
  - HBM traffic: FETCH_SIZE and WRITE_SIZE (KB, rocprofv3 derived counters) from their own
    --pmc passes; gfx950 correction per MI355X_MICROARCH.md §HBM: FETCH_SIZE counts 64 B per
    128-B request (½ of the bytes of wide reads), so read bytes = 2 x FETCH_SIZE x 1024
    (an upper bound for this kernel's 16-B/lane gathers, whose width is uncalibrated);
    WRITE_SIZE x 1024 is exact for 16-B/lane stores.
  - L2 hit rate, SQ wave-cycle breakdown, VALU instruction count, effective clock.
Also refreshes profiles/pmc_traffic.json, which bench.py reads for its roofline.traffic.

    python profiles/summarize_pmc.py <tag> [gpurun_out/prof_<tag>] [workload]
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KERNEL = "k_tris<4, false>"


def counters(path: Path):
    out = defaultdict(dict)
    if not path.exists():
        return out
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"]:
            out[int(r["Dispatch_Id"])][r["Counter_Name"]] = out[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(
                r["Counter_Value"])
    return out


def mean_counter(d, name):
    vals = [v[name] for v in d.values() if name in v]
    return sum(vals) / len(vals) if vals else None


def main():
    tag = sys.argv[1]
    src = Path(sys.argv[2]) if len(sys.argv) > 2 else ROOT / "gpurun_out" / f"prof_{tag}"
    workload = sys.argv[3] if len(sys.argv) > 3 else None
    c = {}
    for sub in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"):
        d = counters(src / f"pmc_{sub}" / "run_counter_collection.csv")
        for name in {k for v in d.values() for k in v}:
            c[name] = mean_counter(d, name)
    stats = list(csv.DictReader(open(src / "trace" / "run_kernel_stats.csv")))
    k = next(r for r in stats if KERNEL in r["Name"])
    avg_ns = float(k["AverageNs"])
    fetch_b = 2 * c["FETCH_SIZE"] * 1024 if c.get("FETCH_SIZE") else None
    write_b = c["WRITE_SIZE"] * 1024 if c.get("WRITE_SIZE") else None
    summ = {
        "kernel": KERNEL,
        "avg_kernel_ms_rocprof": avg_ns / 1e6,
        "fetch_size_kb": c.get("FETCH_SIZE"),
        "write_size_kb": c.get("WRITE_SIZE"),
        "hbm_read_bytes_corrected": fetch_b,
        "hbm_write_bytes": write_b,
        "hbm_bytes_per_launch": (fetch_b or 0) + (write_b or 0),
        "hbm_gbps": ((fetch_b or 0) + (write_b or 0)) / (avg_ns * 1e-9) / 1e9,
        "l2_hit_rate": c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]) if c.get("TCC_HIT_sum") else None,
        "sq_wait_any_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None,
        "sq_active_inst_frac": c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None,
        "sq_insts_valu": c.get("SQ_INSTS_VALU"),
        "effective_clock_ghz": c["GRBM_GUI_ACTIVE"] / 8 / (avg_ns * 1e-9) / 1e9 if c.get("GRBM_GUI_ACTIVE") else None,
    }
    out = ROOT / "profiles" / tag
    out.mkdir(parents=True, exist_ok=True)
    (out / "pmc_summary.json").write_text(json.dumps(summ, indent=1) + "\n")
    if workload:
        (ROOT / "profiles" / "pmc_traffic.json").write_text(json.dumps(
            {"tag": tag, "workload": workload, "kernel": KERNEL,
             "hbm_bytes_per_launch": summ["hbm_bytes_per_launch"],
             "source": f"profiles/{tag}/pmc_summary.json"}, indent=1) + "\n")
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
