"""Is the slowest 8-way rank its content or its place in the render order?  Renders every rank's
dragon tile in ascending, then descending rank order (best of --reps each) and prints both.

    python profiles/rank_order.py [--stripe 8] [--reps 3]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripe", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
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
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    res = {}
    for name, order in (("ascending", range(8)), ("descending", range(7, -1, -1)), ("ascending2", range(8))):
        t = {}
        for r in order:
            best, all_ms = 1e9, []
            for _ in range(args.reps):
                rt.rayTrace(out, W, H, 0, kernel=2, tile=(args.stripe, 8, r))
                all_ms.append(round(rt.lastKernelMs(), 3))
            info = rt.renderInfo()
            t[r] = {"min": min(all_ms), "all": all_ms, "long": int(info["pixels_long"]),
                    "repaired": int(info["split_repaired"])}
        res[name] = t
        print(name, {r: t[r]["min"] for r in sorted(t)}, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
