"""Intrinsic latency of a pixel's serial sample chain on an idle chip.

Renders single rows of the dragon bench frame alone (tile = one row: stripe 1, n_ranks = H),
so the launch holds 30 waves on a 256-CU chip and its time is the row's longest pixel chain.
A counting launch of the same row gives that chain's traversal steps and queries, so
kernel_ms / steps is the per-step latency of a chain with the chip to itself — against the
≈2 µs per step the chains run at under full load.

    python profiles/chain_latency.py [--rows 0:1080:27]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="0:1080:27")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch
    import ptload

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
    out = torch.zeros(W * 4, dtype=torch.float32, device="cuda:0")
    a, b, s = (int(v) for v in args.rows.split(":"))
    res = []
    for r in range(a, b, s):
        tile = (1, H, r)
        best = 1e9
        for _ in range(args.reps):
            rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
            best = min(best, rt.lastKernelMs())
        rt.setCounting(True)
        rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
        cnt = rt.counters()
        rt.setCounting(False)
        steps, q = cnt["pixel_steps_max"], cnt["pixel_rays_max"]
        res.append({"row": r, "kernel_ms": round(best, 3), "max_steps": steps, "max_queries": q,
                    "us_per_step": round(best * 1e3 / max(steps, 1), 3),
                    "us_per_query": round(best * 1e3 / max(q, 1), 3)})
        print(json.dumps(res[-1]), flush=True)
    worst = max(res, key=lambda d: d["kernel_ms"])
    print(json.dumps({"summary": "slowest row alone", **worst}))


if __name__ == "__main__":
    main()
