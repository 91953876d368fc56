"""Per-kernel SQ counters of the last render in profiles/pmc_tile.sh passes: for each kernel of the
render (matched by name and order) the counters of its dispatch, and per wave.

    python profiles/pmc_tile_summary.py gpurun_out/<tag>
"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    table = defaultdict(dict)
    for path in sorted(glob.glob(f"{root}/pmc_*/**/*counter_collection.csv", recursive=True)):
        rows = list(csv.DictReader(open(path)))
        by_disp = defaultdict(dict)
        names = {}
        for r in rows:
            d = int(r["Dispatch_Id"])
            by_disp[d][r["Counter_Name"]] = by_disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
        disp = sorted(by_disp)
        # the last render: its dispatches after the second-to-last k_split_finish
        fin = [d for d in disp if "k_split_finish" in names[d]]
        start = fin[-2] if len(fin) >= 2 else -1
        k = 0
        for d in disp:
            if d <= start or not any(n in names[d] for n in ("k_chain", "k_tris", "k_split")):
                continue
            nm = names[d]
            nm = nm[nm.find("k_"):nm.find("(")] if "(" in nm else nm
            table[(k, nm)].update(by_disp[d])
            k += 1
    for (k, nm), c in sorted(table.items()):
        w = c.get("SQ_WAVES", 0) or 1
        line = " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items()))
        per = {n: c[n] / w for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES") if n in c}
        print(f"{k} {nm}: {line}\n    per wave: " + " ".join(f"{n}={v:.4g}" for n, v in per.items()))


if __name__ == "__main__":
    main()
