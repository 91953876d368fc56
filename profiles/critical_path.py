"""How much of the dragon frame time is the longest pixel's serial chain?  Renders the bench
scene at 1920 x H for shrinking H (fewer pixels, same per-pixel work) and prints kernel ms:
once the frame is bound by its slowest pixels, time stops falling with the pixel count.

    python profiles/critical_path.py
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    rt = pt.RayTracer(0)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS["dragon"]))
    out = torch.zeros(1920 * 1080 * 4, dtype=torch.float32, device="cuda:0")
    res = []
    for sr in (16, 4):
        rt.setSampleRate(sr)
        for H in (1080, 540, 270, 135, 64, 16):
            best = 1e9
            for _ in range(2):
                rt.rayTrace(out, 1920, H, 0, kernel=2)
                best = min(best, rt.lastKernelMs())
            cnt = rt.counters()
            res.append({"spp": sr * sr, "H": H, "kernel_ms": round(best, 2),
                        "rays": cnt["rays_closest"] + cnt["rays_shadow"]})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
