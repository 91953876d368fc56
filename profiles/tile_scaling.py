"""Single-GPU rehearsal of strong scaling: time every rank's row-stripe tile of the bench frame
for N = 1, 2, 4, 8 ranks against the full frame, plus the root's assembly (the staging copy of
the other ranks' tiles and k_assemble, HIP events) and a one-link xGMI model of the transfer.

    python profiles/tile_scaling.py [--config dragon] [--stripe 8]
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="dragon")
    ap.add_argument("--stripe", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--ns", default="1,2,4,8", help="rank counts to rehearse (1 is always timed: the reference)")
    ap.add_argument("--partition", default="balanced", choices=["balanced", "interleaved"],
                    help="the stripes' owners: rt_partition_stripes (probed cost, LPT; bench.py's default) or round-robin")
    args = ap.parse_args()
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = {"dragon": (1920, 1080, 16), "lucy": (4096, 4096, 4), "bunny": (1024, 1024, 1)}[args.config]
    rt = pt.RayTracer(0)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS[args.config]))
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    res = {}
    ptdist = ptload.submodule("dist")
    frame = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    ns = sorted({1} | {int(v) for v in args.ns.replace(":", ",").split(",")})
    owners = {}
    for n in ns:
        times, repaired, longc, tiles = [], [], [], []
        owner = rt.partitionStripes(W, H, args.stripe, n) if (n > 1 and args.partition == "balanced") else None
        owners[n] = owner
        for r in range(n):  # every rank's tile: the slowest sets the N-GPU frame time
            tile = (args.stripe, n, r, owner) if n > 1 else None
            rows = len(ptdist.tile_rows(H, args.stripe, n, r, owner)) if n > 1 else H
            buf = torch.zeros(rows * W * 4, dtype=torch.float32, device="cuda:0")
            best = 1e9
            for _ in range(args.reps):
                rt.rayTrace(buf, W, H, 0, kernel=2, tile=tile)
                best = min(best, rt.lastKernelMs())
            times.append(best)
            tiles.append(buf)
            info = rt.renderInfo()
            repaired.append(int(info.get("split_repaired", 0)))
            longc.append(int(info.get("pixels_long", 0)))
        info = rt.renderInfo()
        res[n] = {"max_ms": max(times), "min_ms": min(times), "ranks_timed": len(times),
                  "partition": args.partition if n > 1 else None,
                  "rows": [len(ptdist.tile_rows(H, args.stripe, n, r, owner)) for r in range(n)] if n > 1 else [H],
                  "rank_ms": [round(t, 3) for t in times], "split_chunks": info.get("split_chunks", 0),
                  "split_spec": info.get("split_spec", 0), "long_chains": longc, "repaired": repaired}
        if n > 1:
            # the root's side of the gather (rt_comm_gather_frame): the other ranks' tiles land in a
            # staging buffer (here a device copy; over xGMI each peer's tile crosses its own link
            # into the root's HBM) and k_assemble scatters every tile's stripes into the frame
            stage = torch.empty(sum(t.numel() for t in tiles[1:]), dtype=torch.float32, device="cuda:0")
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = 1e9
            for _ in range(5):
                torch.cuda.synchronize()
                ev0.record()
                off, views = 0, [tiles[0]]
                for t in tiles[1:]:
                    stage[off:off + t.numel()].copy_(t)
                    views.append(stage[off:off + t.numel()])
                    off += t.numel()
                ptdist.assemble_native(views, H, W, args.stripe, frame, owner=owner)
                ev1.record()
                torch.cuda.synchronize()
                best = min(best, ev0.elapsed_time(ev1))
            link_ms = max(t.numel() * 4 for t in tiles[1:]) / 153e9 * 1e3  # one 153 GB/s xGMI link per peer
            res[n]["assembly_ms"] = round(best, 4)
            res[n]["xgmi_link_ms_model"] = round(link_ms, 4)
            res[n]["max_plus_assembly_ms"] = round(max(times) + best + link_ms, 3)
        del tiles
    # the costliest pixel (counting launch with per-pixel stats, RT_PIXEL_STATS): queries and traversal
    # steps; in a sample-split tile a pixel's samples run as chunk tasks, whose counts add up per pixel
    # (the seed pass's rounds are reported apart)
    path = os.path.join(tempfile.gettempdir(), f"tile_stats_{os.getpid()}.bin")
    for n, r in ((1, 0), (8, 0), (8, 1)) if 8 in ns else ((1, 0),):
        tile = (args.stripe, n, r, owners.get(n)) if n > 1 else None
        os.environ["RT_PIXEL_STATS"] = path
        rt.setCounting(True)
        rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
        c = rt.counters()
        info = rt.renderInfo()
        rt.setCounting(False)
        os.environ.pop("RT_PIXEL_STATS")
        t, _keep = pt._abi.tile_struct(tile)
        rows = rt._lib.rt_tile_rows(H, ctypes.byref(t) if t else None)
        st = np.fromfile(path, np.uint32).reshape(rows * W, 8).astype(np.int64)
        os.remove(path)
        split = info.get("split_chunks", 0) > 0
        q, steps = (st[:, 5], st[:, 6]) if split else (st[:, 2], st[:, 3])
        px = rows * W
        e = {"kernel_ms": rt.lastKernelMs(), "split": split, "max_pixel_rays": int(q.max()),
             "max_pixel_steps": int(steps.max()), "mean_pixel_rays": (c["rays_closest"] + c["rays_shadow"]) / px}
        if split:
            e["max_seed_pass_rounds"] = int(st[:, 2].max())
            e["long_chains"] = int(info.get("pixels_long", 0))
        else:
            e["max_pixel_ms_at_2.4GHz"] = c["pixel_clocks_max"] / 2.4e6
        res.setdefault("pixel", {})[f"{n}:{r}"] = e
    full = res[1]["max_ms"]
    for n in ns[1:]:
        res[n]["ideal_ms"] = full / n
        res[n]["efficiency_vs_full"] = round(full / n / res[n]["max_ms"], 3)
        res[n]["speedup_with_assembly"] = round(full / res[n]["max_plus_assembly_ms"], 3)
    print(json.dumps({"config": args.config, "W": W, "H": H, "spp": sr * sr, "stripe": args.stripe, "tiles": res}))


if __name__ == "__main__":
    main()
