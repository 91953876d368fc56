"""A/B of a view's first frame: the dragon frame right after a 3-degree camera move
(lists, probe and schedule rebuilt) under the probe's order (RT_PILOT=0) and under the order of a
pilot render of RT_PILOT^2 samples per pixel; one fresh context per setting, settings alternating
round after round.  Reports the cold frame's wall time (the bench's cold_frame_ms), its pre-pass
(candidate lists + pilot) and main-kernel times, and the view's next frame.

    python profiles/cold_ab.py [--pilots 0,2,3] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pilots", default="0,2,3")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = 1920, 1080, 16
    mesh = sc.make_mesh(sc.MESH_CONFIGS["dragon"])
    c = sc.PLY_CAMERA
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    pilots = [v for v in args.pilots.replace(":", ",").split(",")]  # RT_PILOT values
    tracers = {}
    for p in pilots:
        os.environ["RT_PILOT"] = p
        rt = pt.RayTracer(0)
        rt.setSpheres(sc.ply_scene())
        rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
        rt.setFoVAngle(sc.DEFAULT_FOV)
        rt.setSampleRate(sr)
        rt.setMaxPathDepth(6)
        rt.setMesh(*mesh)
        for _ in range(2):
            rt.rayTrace(out, W, H, 0, kernel=2)
        tracers[p] = rt
    os.environ.pop("RT_PILOT", None)
    res = {p: {"cold_ms": [], "cold_pre_ms": [], "cold_main_ms": [], "next_ms": [], "pilot": []} for p in pilots}
    for r in range(args.rounds):
        for p in pilots:
            rt = tracers[p]
            az = c["azimuth"] + (3.0 if r % 2 == 0 else -3.0)
            rt.setCameraSpherical(c["target"], c["elevation"], az, c["distance"])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rt.rayTrace(out, W, H, 0, kernel=2)
            torch.cuda.synchronize()
            res[p]["cold_ms"].append((time.perf_counter() - t0) * 1e3)
            pre, main = rt.lastKernelSplitMs()
            res[p]["cold_pre_ms"].append(pre)
            res[p]["cold_main_ms"].append(main)
            res[p]["pilot"].append(rt.renderInfo()["schedule_pilot"])
            rt.rayTrace(out, W, H, 0, kernel=2)
            res[p]["next_ms"].append(rt.lastKernelMs())
        print(f"round {r}: " + " ".join(f"pilot {p}: cold {res[p]['cold_ms'][-1]:.2f} ms" for p in pilots),
              file=sys.stderr, flush=True)
    summary = {str(p): {k: (round(statistics.median(v), 3) if k != "pilot" else v) for k, v in d.items()}
               for p, d in res.items()}
    print(json.dumps({"frame": "dragon 1920x1080 sr16, first frame after a 3-degree camera move", "median": summary,
                      "raw": {str(p): d for p, d in res.items()}}))


if __name__ == "__main__":
    main()
