"""Where a long pixel chain spends its wall time: counting launches with RT_PIXEL_STATS record, per
pixel, the clocks of the loop phases while the pixel was live (D path advance, A/B refill + camera
ray, C stepping rounds), its loop iterations, queries and traversal steps.  Prints the costliest
pixels of (a) row 81 rendered alone and (b) the full dragon frame.

    python profiles/chain_phases.py
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

    dump = "/tmp/rt_pixel_stats_phases.bin"
    os.environ["RT_PIXEL_STATS"] = dump
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
    res = {"env": {k: v for k, v in os.environ.items() if k.startswith("RT_")}}
    for name, tile, rows in (("row81_alone", (1, H, 81), 1), ("full_frame", None, H)):
        rt.setCounting(True)
        rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
        ms = rt.lastKernelMs()
        rt.setCounting(False)
        s = np.fromfile(dump, np.uint32).reshape(rows, W, 8).astype(np.int64).reshape(-1, 8)
        dur = (s[:, 1] - s[:, 0]) / 1e5  # ms
        top = np.argsort(dur)[-5:][::-1]
        res[name] = {"kernel_ms": round(ms, 2), "costliest": [
            {"px": int(i), "wall_ms": round(float(dur[i]), 2), "queries": int(s[i, 2]), "steps": int(s[i, 3]),
             "iters": int(s[i, 7]), "D_ms": round(s[i, 4] * 64 / 2.4e6, 2), "AB_ms": round(s[i, 5] * 64 / 2.4e6, 2),
             "C_ms": round(s[i, 6] * 64 / 2.4e6, 2),
             "us_per_step_in_C": round(s[i, 6] * 64 / 2.4e3 / max(s[i, 3], 1), 3)} for i in top]}
        print(json.dumps({name: res[name]}), flush=True)


if __name__ == "__main__":
    main()
