"""Single-GPU rehearsal of strong scaling: time one rank's row-stripe tile of the bench
frame for N = 1, 2, 4, 8 ranks (rank 0 and the slowest rank) against 1/N of the full frame.

    python profiles/tile_scaling.py [--config dragon] [--stripe 8]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="dragon")
    ap.add_argument("--stripe", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = {"dragon": (1920, 1080, 16), "lucy": (4096, 4096, 4), "bunny": (1024, 1024, 1)}[args.config]
    rt = pt.RayTracer(0)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS[args.config]))
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    res = {}
    for n in (1, 2, 4, 8):
        times = []
        for r in range(n):
            tile = (args.stripe, n, r) if n > 1 else None
            best = 1e9
            for _ in range(args.reps):
                rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
                best = min(best, rt.lastKernelMs())
            times.append(best)
            if n > 1 and r >= 1 and n == 8 and r >= 3:
                break  # a few ranks suffice to see the spread
        res[n] = {"max_ms": max(times), "min_ms": min(times), "ranks_timed": len(times)}
    # the costliest pixel (counting launch): clocks, queries, traversal steps
    for n, r in ((1, 0), (8, 0), (8, 1)):
        rt.setCounting(True)
        rt.rayTrace(out, W, H, 0, kernel=2, tile=(args.stripe, n, r) if n > 1 else None)
        c = rt.counters()
        rt.setCounting(False)
        px = W * (H if n == 1 else len(range(0, H)) // n)
        res.setdefault("pixel", {})[f"{n}:{r}"] = {
            "kernel_ms": rt.lastKernelMs(), "max_pixel_ms_at_2.4GHz": c["pixel_clocks_max"] / 2.4e6,
            "max_pixel_rays": c["pixel_rays_max"], "max_pixel_steps": c["pixel_steps_max"],
            "mean_pixel_rays": (c["rays_closest"] + c["rays_shadow"]) / px}
    full = res[1]["max_ms"]
    for n in (2, 4, 8):
        res[n]["ideal_ms"] = full / n
        res[n]["efficiency_vs_full"] = round(full / n / res[n]["max_ms"], 3)
    print(json.dumps({"config": args.config, "W": W, "H": H, "spp": sr * sr, "tiles": res}))


if __name__ == "__main__":
    main()
