"""Data for the rank partition of a tile-parallel frame: where the long chains and
the traversal work lie in the frame.

For N ranks (row-stripe tiles, the library's current partition) every rank's tile is rendered and
its long chains (rt_last_long_chains, tile-local y * W + x) mapped back to frame rows; a counting
launch of the whole frame with per-pixel stats (RT_PIXEL_STATS) gives every pixel's queries and
traversal steps.  Writes an .npz with
    long_rows[H]    long chains per frame row (from the N-way tiles)
    steps_rows[H]   traversal steps per frame row (whole frame, whole-pixel launch)
    queries_rows[H] queries per frame row
    rank_ms[N]      each rank's tile time (best of --reps)
and prints a JSON summary.

    python profiles/partition_data.py [--n 8] [--stripe 8] [--out gpurun_out/partition.npz]
"""
import argparse
import json
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--stripe", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--out", default="gpurun_out/partition.npz")
    args = ap.parse_args()
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    ptdist = ptload.submodule("dist")
    W, H, sr = 1920, 1080, 16
    rt = pt.RayTracer(0)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS["dragon"]))
    long_rows = np.zeros(H, np.int64)
    rank_ms = []
    for r in range(args.n):
        tile = (args.stripe, args.n, r)
        rows = ptdist.tile_rows(H, args.stripe, args.n, r)
        buf = torch.zeros(len(rows) * W * 4, dtype=torch.float32, device="cuda:0")
        best = 1e9
        for _ in range(args.reps):
            rt.rayTrace(buf, W, H, 0, kernel=2, tile=tile)
            best = min(best, rt.lastKernelMs())
        rank_ms.append(best)
        lc = rt.longChains().astype(np.int64)
        np.add.at(long_rows, rows[lc // W], 1)
        print(f"rank {r}: {best:.3f} ms, {len(lc)} long chains", file=sys.stderr, flush=True)
    path = os.path.join(tempfile.gettempdir(), f"partition_stats_{os.getpid()}.bin")
    os.environ["RT_PIXEL_STATS"] = path
    rt.setCounting(True)
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    rt.rayTrace(out, W, H, 0, kernel=2)
    rt.setCounting(False)
    os.environ.pop("RT_PIXEL_STATS")
    st = np.fromfile(path, np.uint32).reshape(H, W, 8).astype(np.int64)
    os.remove(path)
    steps_rows = st[..., 3].sum(axis=1)
    queries_rows = st[..., 2].sum(axis=1)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(args.out, long_rows=long_rows, steps_rows=steps_rows, queries_rows=queries_rows,
                        rank_ms=np.array(rank_ms), steps_px=st[..., 3].astype(np.uint32))
    print(json.dumps({"n": args.n, "stripe": args.stripe, "rank_ms": [round(x, 3) for x in rank_ms],
                      "long_total": int(long_rows.sum()), "steps_total": int(steps_rows.sum())}))


if __name__ == "__main__":
    main()
