"""Measured ceiling for the roofline's record_gather fraction (bench.py): random 64-B records
fetched as 4 x dwordx4 per lane in dependent chains (profiles/gather_microbench.hip, `direct`),
5 waves/SIMD, every lane its own record (G = 64) or lanes sharing records (G = 32), from an
L2-resident table (4 MB: the dragon traversal's PMC L2 hit rate is 98.8 %, and its wave-loads
touch ~39 distinct lines: TCP_TOTAL_CACHE_ACCESSES / SQ_INSTS_VMEM_RD) and from a table the size
of the dragon scene's records (56 MB: nodes 13.9 MB + triangles 41.8 MB).  The ceiling used is
the best of these rates.  Writes profiles/gather_ceiling.json.

    python profiles/gather_ceiling.py   (GPU box; needs profiles/gather_microbench built)
"""
import json
import re
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def main():
    exe = ROOT / "profiles" / "gather_microbench"
    runs = []
    for mb, g in ((4, 64), (4, 32), (56, 64), (56, 32)):
        txt = subprocess.run(["timeout", "-k", "5", "60", str(exe), str(mb), "2000", str(g)], check=True,
                             capture_output=True, text=True).stdout
        for ln in txt.splitlines():
            m = re.search(r"table (\d+) MB G=(\d+) (.+?)\s+([\d.]+) ms\s+([\d.]+) Grec/s", ln)
            if m and m.group(3).startswith("direct"):
                runs.append({"table_mb": int(m.group(1)), "G": int(m.group(2)), "grec_per_s": float(m.group(5))})
    best = max(runs, key=lambda r: r["grec_per_s"])
    out = {"best_grec_per_s": best["grec_per_s"], "best": best, "runs": runs,
           "source": "profiles/gather_microbench.hip k_direct (4 x dwordx4 per lane, dependent chains, 5 waves/SIMD)"}
    (ROOT / "profiles" / "gather_ceiling.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
