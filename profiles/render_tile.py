"""Render one row-stripe tile (or the whole frame) of a bench configuration a few times, for
kernel traces (rocprofv3 --kernel-trace --stats) of one launch form; RT_* knobs from the env.

    python profiles/render_tile.py [--config dragon] [--tile 8,8,0] [--reps 3] [--lib build.so]
"""
import argparse
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="dragon")
    ap.add_argument("--tile", default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--balanced", action="store_true", help="the tile under rt_partition_stripes' owner map")
    ap.add_argument("--lib", default=None, help="another build of librtmi.so (A/B)")
    ap.add_argument("--env", action="append", default=[], help="NAME=VALUE set before the context is created")
    args = ap.parse_args()
    for kv in args.env:
        k, _, v = kv.partition("=")
        os.environ[k] = v
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = {"dragon": (1920, 1080, 16), "lucy": (4096, 4096, 4), "bunny": (1024, 1024, 1)}[args.config]
    rt = pt.RayTracer(0, lib_path=args.lib)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS[args.config]))
    tile = tuple(int(v) for v in args.tile.replace(":", ",").split(",")) if args.tile else None
    if tile and args.balanced:
        tile = tile + (rt.partitionStripes(W, H, tile[0], tile[1]),)
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    for _ in range(args.reps):
        rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
        print(f"{rt.lastKernelMs():.2f} ms", rt.renderInfo(), flush=True)


if __name__ == "__main__":
    main()
