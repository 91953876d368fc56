"""Seed-pass width A/B on the 8-way (or N-way) row-stripe tiles of a bench configuration: for each
RT_SEED_WIDTH (lanes per long chain: 8-64 subtree-parallel k_chain_seeds, 3 coop_round) a fresh
context renders every rank's tile (best of --reps) and the slowest rank is reported, with the
tile's frame bits checked equal across widths.

    python profiles/seed_width_ab.py [--config dragon] [--n 8] [--widths 16,4,8,32] [--reps 2] [--balanced]
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
    ap.add_argument("--config", default="dragon")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--widths", default="16,4,8,32")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--stripe", type=int, default=8)
    ap.add_argument("--balanced", action="store_true", help="the tiles under rt_partition_stripes' owner map")
    args = ap.parse_args()
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = {"dragon": (1920, 1080, 16), "lucy": (4096, 4096, 4), "bunny": (1024, 1024, 1)}[args.config]
    mesh = sc.make_mesh(sc.MESH_CONFIGS[args.config])
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    ref = {}
    res = {}
    for spec in args.widths.replace(":", ",").split(","):
        os.environ["RT_SEED_WIDTH"] = spec
        wd = spec
        rt = pt.RayTracer(0)
        rt.setSpheres(sc.ply_scene())
        c = sc.PLY_CAMERA
        rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
        rt.setSampleRate(sr)
        rt.setMaxPathDepth(6)
        rt.setMesh(*mesh)
        times, same = [], True
        owner = rt.partitionStripes(W, H, args.stripe, args.n) if args.balanced else None
        for r in range(args.n):
            tile = (args.stripe, args.n, r) + ((owner,) if owner is not None else ())
            best = 1e9
            for _ in range(args.reps):
                rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
                best = min(best, rt.lastKernelMs())
            info = rt.renderInfo()
            assert info.get("split_guard", 0) == 0, info
            h = hash(out.cpu().numpy().tobytes())
            if r in ref:
                same &= ref[r] == h
            else:
                ref[r] = h
            times.append(round(best, 3))
        res[wd] = {"max_ms": max(times), "rank_ms": times, "split_coop": info.get("split_coop"),
                   "bits_equal_first_width": same}
        print(wd, json.dumps(res[wd]), flush=True)
        rt.close()
    print(json.dumps({"config": args.config, "n": args.n, "widths": res}))


if __name__ == "__main__":
    main()
