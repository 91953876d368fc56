"""Wave-step mix of k_tris's stepping rounds (diagnostics build -DRT_DIAG_MIX=1, GPU box): how many
wave-steps hold both node and leaf lanes (both blocks of trav_step_q execute), nodes only, leaves
only, on the bench frame (counting launch).

    python profiles/step_mix.py --lib build_ab/mix.so [--config dragon] [--tile 8,8,0]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--config", default="dragon")
    ap.add_argument("--tile", default=None)
    args = ap.parse_args()
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = {"dragon": (1920, 1080, 16), "bunny": (1024, 1024, 1)}[args.config]
    tile = tuple(int(v) for v in args.tile.replace(":", ",").split(",")) if args.tile else None
    rt = pt.RayTracer(0, lib_path=args.lib)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS[args.config]))
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
    rt.setCounting(True)
    rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
    cn = rt.counters()
    both, nodes, leaves = cn["pixel_clocks_max"], cn["pixel_rays_max"], cn["pixel_steps_max"]
    tot = both + nodes + leaves
    print(json.dumps({"config": args.config, "tile": tile, "wave_steps": tot, "both": both, "nodes_only": nodes,
                      "leaves_only": leaves, "frac_both": both / max(tot, 1), "lane_steps": cn["nodes_visited"] +
                      cn["leaves_visited"], "lane_slots": cn["lane_slots"], "nodes": cn["nodes_visited"],
                      "tests": cn["tris_tested"], "leaves": cn["leaves_visited"]}))


if __name__ == "__main__":
    main()
