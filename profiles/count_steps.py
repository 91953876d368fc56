"""Counting launch of the dragon frame (BASELINE configs[3]) with a given librtmi build: the traversal
counters (node visits, triangle tests, leaf steps, lane slots = lanes x stepping-loop wave-steps) and
the frame's ray counts, as one JSON line — for comparing traversal step forms.

    python profiles/count_steps.py [--lib build.so]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    args = ap.parse_args()
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = 1920, 1080, 16
    rt = pt.RayTracer(0, lib_path=args.lib or None)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS["dragon"]))
    Wp, Hp = sc.padded_dims(W, H)
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    rt.setSeeds(Wp, Hp, sc.default_seeds(Wp, Hp))
    rt.rayTrace(out, W, H, 0, kernel=2)
    rt.setSeeds(Wp, Hp, sc.default_seeds(Wp, Hp))
    rt.setCounting(True)
    rt.rayTrace(out, W, H, 0, kernel=2)
    cnt = rt.counters()
    rays = cnt["rays_closest"] + cnt["rays_shadow"]
    print(json.dumps({"lib": args.lib or "in-tree", "kernel_ms_counting": rt.lastKernelMs(), **cnt,
                      "wave_steps": cnt["lane_slots"] / 64, "lane_slots_per_ray": cnt["lane_slots"] / rays,
                      "records_per_lane_slot": (cnt["nodes_visited"] + cnt["leaves_visited"]) / cnt["lane_slots"]}))


if __name__ == "__main__":
    main()
