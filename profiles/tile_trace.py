"""Per-kernel spans of the last render in a rocprofv3 kernel trace of profiles/render_tile.py:
each path-tracer kernel's start and end (ms, from the render's first kernel) and duration, so the
streams of a sample-split tile (the long chains' seed pass, chunks and sums beside the mesh
pixels' chunks, the repair pass and the sums) can be read apart.

    python profiles/tile_trace.py <rocprofv3 output dir>
"""
import csv
import glob
import sys

NAMES = ("k_tris", "k_split_seeds", "k_chain_seeds", "k_chain_wave", "k_split_finish", "k_pixel_lists", "k_probe_cost")


def short(name):
    for n in NAMES:
        if n in name:
            i = name.find(n)
            return name[i:name.find("(", i)] if "(" in name[i:] else name[i:]
    return None


def main():
    path = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(path)) if short(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # renders are separated by idle gaps of the device (the host synchronises between them): a
    # kernel starting 0.1 ms or more after every earlier kernel has ended opens a new render
    groups, cur, busy_to = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur and busy_to is not None and s - busy_to >= 100_000:
            groups.append(cur)
            cur = []
        cur.append(r)
        busy_to = e if busy_to is None else max(busy_to, e)
    if cur:
        groups.append(cur)
    last = groups[-1]
    t0 = min(int(r["Start_Timestamp"]) for r in last)
    t1 = max(int(r["End_Timestamp"]) for r in last)
    print(f"renders found: {len(groups)}; last render span {(t1 - t0) / 1e6:.3f} ms")
    for r in last:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"  {short(r['Kernel_Name']):34s} grid {int(r['Grid_Size_X']):8d}  start {(s - t0) / 1e6:8.3f}  end "
              f"{(e - t0) / 1e6:8.3f}  dur {(e - s) / 1e6:8.3f} ms  stream {r.get('Stream_Id', '?')}")


if __name__ == "__main__":
    main()
