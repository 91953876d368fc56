"""Costliest pixels of the dragon frame and of its row-stripe tiles (counting launches with
RT_PIXEL_STATS: per-pixel wall clocks, queries, traversal steps).  One JSON line per launch.

    python profiles/chain_tiles.py
"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch
    import ptload

    dump = "/tmp/rt_pixel_stats_tiles.bin"
    os.environ["RT_PIXEL_STATS"] = dump
    os.environ["RT_SPLIT"] = "0"  # whole-pixel tasks: the per-pixel chains these clocks describe
    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = 1920, 1080, 16
    rt = pt.RayTracer(0)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS["dragon"]))
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    rt.rayTrace(out, W, H, 0, kernel=2)
    for name, tile in (("full", None), ("n8_r0", (8, 8, 0)), ("n4_r2", (8, 4, 2)), ("row81", (1, H, 81))):
        rows = H if tile is None else len([y for y in range(H) if (y // tile[0]) % tile[1] == tile[2]])
        rt.setCounting(True)
        rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
        ms = rt.lastKernelMs()
        cn = rt.counters()
        rt.setCounting(False)
        if name == "full":
            print(json.dumps(cn), flush=True)
        s = np.fromfile(dump, np.uint32).reshape(rows * W, 8).astype(np.int64)
        dur = ((s[:, 1] - s[:, 0]) & 0xFFFFFFFF) / 1e5
        top = np.argsort(dur)[-4:][::-1]
        t0 = s[:, 0].min()
        end = ((s[:, 1] - t0) & 0xFFFFFFFF) / 1e5  # ms after the first pixel started
        start = ((s[:, 0] - t0) & 0xFFFFFFFF) / 1e5
        timeline = {f"end_p{q}": round(float(np.percentile(end, q)), 2) for q in (50, 90, 99, 99.9, 100)}
        timeline["costliest_start_ms"] = [round(float(start[i]), 2) for i in top]
        print(json.dumps({name: {"kernel_ms": round(ms, 2), "pixels_long": cn["pixels_long"],
                                 "steps_per_query": round((cn["nodes_visited"] + cn["leaves_visited"]) /
                                                          max(cn["rays_closest"] + cn["rays_shadow"], 1), 2),
                                 "timeline": timeline,
                                 "costliest": [{"px": [int(i % W), int(i // W)], "wall_ms": round(float(dur[i]), 2),
                                                "queries": int(s[i, 2]), "steps": int(s[i, 3]),
                                                "shade_refill_step": [round(float(s[i, k]) / max(float(s[i, 4] + s[i, 5] + s[i, 6]), 1.0), 3) for k in (4, 5, 6)],
                                                "iterations": int(s[i, 7])} for i in top]}}),
              flush=True)


if __name__ == "__main__":
    main()
