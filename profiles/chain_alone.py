"""A pixel's serial sample chain with the megakernel to itself (diagnostics build).

With librtmi built -DRT_DIAG_ONE_PIXEL=1 (profiles/build_variant.sh), k_tris renders only the
pixel RT_DIAG_PIXEL=x,y names: its lane is the only live lane of its wave and of the chip, so
the main kernel's time is that pixel's chain at the megakernel's best (no other lane holds a
stepping round open, no other wave competes).  Printed per pixel: main-kernel ms, queries,
traversal steps, us per query and step.  (Until r03 the chains were also timed with their
shadow rays deferred — profiles/r03c; deferral was replaced by sample-split tiles.)

    RTMI_LIB=build_ab/diag1.so python profiles/chain_alone.py [--pixels 1844,198 1807,633]
"""
import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pixels", nargs="+", default=["1844,198", "1807,633", "1844,31", "960,540"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--k", nargs="+", type=int, default=[1],
                    help="pixels of the target's 8x8 tile rendered with it (one wave): 1 = the chain alone")
    args = ap.parse_args()
    import numpy as np
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = 1920, 1080, 16
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS["dragon"])
    seeds = sc.default_seeds(Wp, Hp)
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    for defer in ("0",):
        rt = pt.RayTracer(0)
        rt.setSpheres(sc.ply_scene())
        c = sc.PLY_CAMERA
        rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
        rt.setSampleRate(sr)
        rt.setMaxPathDepth(6)
        rt.setMesh(verts, idx)
        for px, k in [(p_, k_) for p_ in args.pixels for k_ in args.k]:
            os.environ["RT_DIAG_PIXEL"] = f"{px},{k}"
            rt.setCounting(True)
            rt.setSeeds(Wp, Hp, seeds)
            rt.rayTrace(out, W, H, 0, kernel=2)
            cnt = rt.counters()
            rt.setCounting(False)
            best = 1e9
            for _ in range(args.reps):
                rt.setSeeds(Wp, Hp, seeds)
                rt.rayTrace(out, W, H, 0, kernel=2)
                best = min(best, rt.lastKernelSplitMs()[1])
            q = cnt["rays_closest"] + cnt["rays_shadow"]
            steps = cnt["nodes_visited"] + cnt["leaves_visited"]
            print(json.dumps({"pixel": px, "k": k, "defer": defer, "max_pixel_queries": int(cnt["pixel_rays_max"]),
                              "max_pixel_steps": int(cnt["pixel_steps_max"]), "main_ms": round(best, 3), "queries": int(q),
                              "closest": int(cnt["rays_closest"]), "skipped": int(cnt["rays_skipped"]),
                              "steps": int(steps), "us_per_query": round(best * 1e3 / max(q, 1), 3),
                              "us_per_step": round(best * 1e3 / max(steps, 1), 3)}), flush=True)
        rt.close()


if __name__ == "__main__":
    main()
