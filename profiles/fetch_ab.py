"""A/B of the stepping-round exit rule (RT_FETCH_FRAC, RT_BOX_EXIT env knobs, read at rt_create):
full dragon frame (N = 1), one row alone (row 81: the costliest chain), and the row-stripe tiles
of N = 2 / 4 / 8 ranks (every rank timed: the slowest sets the frame).  One JSON line.

    RT_FETCH_FRAC=24 RT_BOX_EXIT=1 python profiles/fetch_ab.py
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
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
    ref = torch.zeros_like(out)

    def best(tile, reps=2):
        b = 1e9
        for _ in range(reps):
            rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
            b = min(b, rt.lastKernelMs())
        return b

    res = {"env": {k: os.environ.get(k) for k in ("RT_FETCH_FRAC", "RT_BOX_EXIT", "RT_FETCH_K", "RT_FETCH_K_BOX", "RT_DEFER", "RT_SPREAD", "RT_PIXEL_LISTS", "RT_GRID_PCT")}}
    seeds0 = None
    rt.rayTrace(out, W, H, 0, kernel=2)
    seeds0 = rt.getSeeds()
    Wp, Hp = sc.padded_dims(W, H)
    pre = []
    for _ in range(5):
        rt.rayTrace(out, W, H, 0, kernel=2)
        pre.append(rt.lastKernelSplitMs()[0])
    res["full_prepass_ms"] = round(sorted(pre)[2], 3)
    res["full_ms"] = round(best(None, 3), 2)
    res["row81_ms"] = round(best((1, H, 81)), 2)
    for n in (2, 4, 8):
        res[f"n{n}_ms"] = [round(best((8, n, r)), 2) for r in range(n)]
        res[f"n{n}_eff"] = round(res["full_ms"] / n / max(res[f"n{n}_ms"]), 3)
    # frames are independent of the schedule: the full frame from seeds0 hashed for cross-run checks
    rt.setSeeds(Wp, Hp, seeds0)
    rt.rayTrace(out, W, H, 0, kernel=2)
    res["frame_hash"] = int(out.view(torch.int32).to(torch.int64).sum().item())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
