"""Summarise the rocprofv3 passes of one bench command into profiles/<tag>/pmc_summary.json and
refresh the workload's entry in profiles/pmc_roofline.json (read by bench.py's roofline).

Input: gpurun_out/prof_<tag>/ from profiles/run_profile.sh (kernel trace + pmc_* passes) and
profiles/pmc_extra.sh (pmcx_* passes), every pass its own `rocprofv3 --pmc` run.

Per launch of the timed kernel (default k_tris<4, false>; k_spheres<false> for the sphere
config), with the gfx950 rules of MI355X_MICROARCH.md §HBM:
  - HBM traffic: read bytes = 2 x FETCH_SIZE x 1024 (FETCH_SIZE counts 64 B per 128-B request:
    an upper bound for 16-B/lane gathers), write bytes = WRITE_SIZE x 1024;
  - VALU issue: SQ_INSTS_VALU wave-instructions, 2 cycles each on a SIMD-32 (wave64), over
    1024 SIMDs x kernel cycles (GRBM_GUI_ACTIVE / 8 XCDs);
  - SALU issue: SQ_INSTS_SALU over 256 scalar units x kernel cycles;
  - vector-memory address path: TA_BUSY_avr / kernel cycles;
  - L2 hit rate, wave-cycle breakdown, effective clock.

    python profiles/summarize_pmc.py <tag> [gpurun_out/prof_<tag>] [workload] [kernel] [--last N]

--last N: only the kernel's last N full-size dispatches of every pass (the steady-state frames of
profiles/steady_state.py, whose earlier dispatches are a view's pilot and first frames).
"""
from __future__ import annotations

import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
N_CU, N_SIMD, N_XCD = 256, 1024, 8


def counters(paths, kernel, last=0):
    """mean over the kernel's full-size dispatches (the largest grid: bench.py also launches the
    kernel on 1-row tiles for its critical-path figure) — the last `last` of them if > 0 — per
    counter, over the collection files"""
    tot = defaultdict(list)
    for path in paths:
        per = defaultdict(lambda: defaultdict(float))
        grid = {}
        for r in csv.DictReader(open(path)):
            if kernel in r["Kernel_Name"]:
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                grid[r["Dispatch_Id"]] = int(r["Grid_Size"])
        gmax = max(grid.values()) if grid else 0
        ids = sorted((did for did in per if grid[did] == gmax), key=int)
        for did in ids[-last:] if last else ids:
            for k, v in per[did].items():
                tot[k].append(v)
    return {k: sum(v) / len(v) for k, v in tot.items()}


def kernel_ns(src, kernel, last=0):
    """mean duration and count of the kernel's full-size dispatches in the kernel trace (the last
    `last` of them if > 0, in start order)"""
    rows = [r for r in csv.DictReader(open(src / "trace" / "run_kernel_trace.csv")) if kernel in r["Kernel_Name"]]
    size = lambda r: int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    gmax = max(size(r) for r in rows)
    full = sorted((r for r in rows if size(r) == gmax), key=lambda r: int(r["Start_Timestamp"]))
    if last:
        full = full[-last:]
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in full]
    return sum(d) / len(d), len(d)


def main():
    argv = list(sys.argv[1:])
    last = 0
    if "--last" in argv:
        i = argv.index("--last")
        last = int(argv[i + 1])
        del argv[i:i + 2]
    tag = argv[0]
    src = Path(argv[1]) if len(argv) > 1 else ROOT / "gpurun_out" / f"prof_{tag}"
    workload = argv[2] if len(argv) > 2 else None
    kernel = argv[3] if len(argv) > 3 else "k_tris<4, false, false, true>"
    files = sorted(glob.glob(f"{src}/pmc_*/run_counter_collection.csv")) + sorted(
        glob.glob(f"{src}/pmcx_*/run_counter_collection.csv"))
    c = counters(files, kernel, last)
    avg_ns, n_disp = kernel_ns(src, kernel, last)
    cyc = c["GRBM_GUI_ACTIVE"] / N_XCD if c.get("GRBM_GUI_ACTIVE") else None
    fetch_b = 2 * c["FETCH_SIZE"] * 1024 if c.get("FETCH_SIZE") else None
    write_b = c["WRITE_SIZE"] * 1024 if c.get("WRITE_SIZE") else None

    def frac(num, den):
        return num / den if (num is not None and den) else None

    summ = {
        "kernel": kernel,
        "avg_kernel_ms_rocprof": avg_ns / 1e6,
        "dispatches": n_disp,
        "dispatch_selection": f"the last {last} full-grid dispatches (steady state)" if last else "every full-grid dispatch",
        "fetch_size_kb": c.get("FETCH_SIZE"),
        "write_size_kb": c.get("WRITE_SIZE"),
        "hbm_read_bytes_corrected": fetch_b,
        "hbm_write_bytes": write_b,
        "hbm_bytes_per_launch": (fetch_b or 0) + (write_b or 0),
        "hbm_gbps": ((fetch_b or 0) + (write_b or 0)) / (avg_ns * 1e-9) / 1e9,
        "l2_hit_rate": frac(c.get("TCC_HIT_sum"), (c.get("TCC_HIT_sum") or 0) + (c.get("TCC_MISS_sum") or 0)),
        "kernel_cycles_per_xcd": cyc,
        "effective_clock_ghz": cyc / (avg_ns * 1e-9) / 1e9 if cyc else None,
        "sq_insts_valu": c.get("SQ_INSTS_VALU"),
        "sq_insts_salu": c.get("SQ_INSTS_SALU"),
        "sq_insts_vmem_rd": c.get("SQ_INSTS_VMEM_RD"),
        "sq_insts_lds": c.get("SQ_INSTS_LDS"),
        "ta_busy_avr": c.get("TA_BUSY_avr"),
        "valu_issue_frac": frac(c["SQ_INSTS_VALU"] / N_SIMD * 2, cyc) if c.get("SQ_INSTS_VALU") else None,
        "salu_issue_frac": frac(c["SQ_INSTS_SALU"] / N_CU, cyc) if c.get("SQ_INSTS_SALU") else None,
        "ta_busy_frac": frac(c.get("TA_BUSY_avr"), cyc),
        "sq_wait_any_frac": frac(c.get("SQ_WAIT_ANY"), c.get("SQ_WAVE_CYCLES")),
        "sq_active_inst_frac": frac(c.get("SQ_ACTIVE_INST_ANY"), c.get("SQ_WAVE_CYCLES")),
        "counters": c,
    }
    drv = src / "driver.json"  # profiles/steady_state.py's line: the counting launch's algorithmic bytes
    if drv.exists() and drv.read_text().strip():
        d = json.loads(drv.read_text().strip().splitlines()[-1])
        summ["algorithmic_bytes_per_launch"] = d["algorithmic_bytes_per_launch"]
        summ["algorithmic_gbps"] = d["algorithmic_bytes_per_launch"] / (avg_ns * 1e-9) / 1e9
        summ["algorithmic_frac_of_hbm_peak"] = summ["algorithmic_gbps"] / 8000.0
        summ["driver"] = d
    out = ROOT / "profiles" / tag
    out.mkdir(parents=True, exist_ok=True)
    (out / "pmc_summary.json").write_text(json.dumps(summ, indent=1) + "\n")
    if workload:
        p = ROOT / "profiles" / "pmc_roofline.json"
        allw = json.loads(p.read_text()) if p.exists() else {}
        allw[workload] = {key: summ[key] for key in (
            "kernel", "avg_kernel_ms_rocprof", "hbm_bytes_per_launch", "effective_clock_ghz", "sq_insts_valu",
            "sq_insts_salu", "ta_busy_avr", "kernel_cycles_per_xcd", "valu_issue_frac", "salu_issue_frac",
            "ta_busy_frac", "l2_hit_rate", "dispatches", "dispatch_selection")}
        for key in ("algorithmic_bytes_per_launch", "algorithmic_frac_of_hbm_peak"):
            if key in summ:
                allw[workload][key] = summ[key]
        allw[workload]["source"] = f"profiles/{tag}/pmc_summary.json"
        p.write_text(json.dumps(allw, indent=1) + "\n")
    print(json.dumps({k: v for k, v in summ.items() if k != "counters"}, indent=1))


if __name__ == "__main__":
    main()
