"""Sweep k_tris's stepping knobs on one context (GPU box): for each setting the frame's kernel
time (median of --reps renders) with RTMI_FETCH_K / RTMI_FETCH_FRAC / RTMI_GRID_BLOCKS set
(rt_host.cpp reads them at every render).  Settings alternate round after round.

    python profiles/bunny_sweep.py [--config bunny] [--reps 5] [--rounds 3] [--lib build.so] 24:24:0 16:24:0 ...
    (K:FRAC:GRID; GRID 0 = the host's grid)
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("settings", nargs="+")
    ap.add_argument("--config", default="bunny", choices=["bunny", "dragon"])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--lib", default=None, help="another build of librtmi.so")
    args = ap.parse_args()
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = (1024, 1024, 1) if args.config == "bunny" else (1920, 1080, 16)
    rt = pt.RayTracer(0, lib_path=args.lib)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setFoVAngle(sc.DEFAULT_FOV)
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS[args.config]))
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    for _ in range(3):
        rt.rayTrace(out, W, H, 0, kernel=pt.RayTracer.KERNEL_TRIS)
    res = {s: [] for s in args.settings}
    wall = {s: [] for s in args.settings}
    for r in range(args.rounds):
        for s in args.settings:
            k, f, g = (s.split(":") + ["0"] * 2)[:3]
            os.environ["RTMI_FETCH_K"] = k
            os.environ["RTMI_FETCH_FRAC"] = f
            os.environ["RTMI_GRID_BLOCKS"] = g
            rt.rayTrace(out, W, H, 0, kernel=pt.RayTracer.KERNEL_TRIS)  # settle
            for _ in range(args.reps):
                t0 = time.perf_counter()
                rt.rayTrace(out, W, H, 0, kernel=pt.RayTracer.KERNEL_TRIS)
                wall[s].append((time.perf_counter() - t0) * 1e3)
                res[s].append(rt.lastKernelMs())
        print("round", r, " ".join(f"{s}={statistics.median(res[s][-args.reps:]):.3f}" for s in args.settings), flush=True)
    for s in args.settings:
        print(f"{s:12s} kernel median {statistics.median(res[s]):.3f} ms  min {min(res[s]):.3f}  "
              f"wall median {statistics.median(wall[s]):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
