"""In-process A/B of librtmi.so builds on the dragon frame (GPU box).

Every library gets its own RayTracer context (same mesh, camera, seeds); launches
alternate between the libraries round after round, so clock and neighbour drift
hit all variants alike.  Prints per-variant median / min kernel ms.

    python profiles/ab_inproc.py LABEL=path.so LABEL=path.so ... [--rounds 8] [--config dragon] [--tile 8,8,0]
                                 [--env NAME=VALUE ...]
    (LABEL= with an empty path: the in-tree build)
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--config", default="dragon", choices=["dragon", "bunny", "lucy"])
    ap.add_argument("--tile", default=None, help="stripe,n_ranks,rank: time one rank's row-stripe tile")
    ap.add_argument("--env", action="append", default=[], help="NAME=VALUE set before the contexts are created")
    args = ap.parse_args()
    for kv in args.env:
        k, _, v = kv.partition("=")
        os.environ[k] = v
    tile = tuple(int(v) for v in args.tile.replace(":", ",").split(",")) if args.tile else None
    import numpy as np
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H = (1920, 1080) if args.config == "dragon" else ((1024, 1024) if args.config == "bunny" else (4096, 4096))
    sr = 16 if args.config == "dragon" else (1 if args.config == "bunny" else 4)
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS[args.config])
    Wp, Hp = sc.padded_dims(W, H)
    seeds = sc.default_seeds(Wp, Hp)
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    variants = []
    for spec in args.libs:
        label, _, path = spec.partition("=")
        rt = pt.RayTracer(0, lib_path=path or None)
        rt.setSpheres(sc.ply_scene())
        c = sc.PLY_CAMERA
        rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
        rt.setFoVAngle(sc.DEFAULT_FOV)
        rt.setSampleRate(sr)
        rt.setMaxPathDepth(6)
        rt.setMesh(verts, idx)
        variants.append((label, rt, []))
    ref = None
    for r in range(args.rounds + 1):
        k = r % len(variants)  # rotate the order every round (no variant always first)
        for label, rt, ms in variants[k:] + variants[:k]:
            rt.setSeeds(Wp, Hp, seeds)
            rt.rayTrace(out, W, H, 0, kernel=pt.RayTracer.KERNEL_TRIS, tile=tile)
            torch.cuda.synchronize()
            if r == 0:  # warmup round; every variant's frame must be the same bits
                img = out.cpu().numpy().view(np.uint32).copy()
                if ref is None:
                    ref = img
                elif not np.array_equal(ref, img):
                    print(f"{label}: frame differs from {variants[0][0]}", flush=True)
            else:
                # the main kernel alone (k_tris + deferred-shadow kernels): builds that reuse the
                # candidate lists of an unchanged view skip the pre-pass, older builds do not
                try:
                    ms.append(rt.lastKernelSplitMs()[1] if tile is None else rt.lastKernelMs())
                except Exception:
                    ms.append(rt.lastKernelMs())
        if r > 0:
            print("round", r, " ".join(f"{l}={m[-1]:.2f}" for l, _, m in variants), flush=True)
    for label, _, ms in variants:
        print(f"{label:12s} median {statistics.median(ms):8.2f} ms  min {min(ms):8.2f} ms", flush=True)


if __name__ == "__main__":
    main()
