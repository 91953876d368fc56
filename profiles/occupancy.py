"""Lane occupancy over a triangle launch: how much of the frame is the tail.

A counting launch with RT_PIXEL_STATS records each pixel's start and finish clock (s_memrealtime,
100 MHz).  The live pixels at time t (started, not finished) against the resident lanes give the
occupancy curve; printed: kernel ms, the times at which live pixels fall below 90 / 50 / 10 % of
the lanes, the idle lane fraction over the launch, and a 20-bin histogram of live pixels.

    python profiles/occupancy.py [--config dragon] [--tile STRIPE,N,R]
"""
import argparse
import json
import os
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="dragon")
    ap.add_argument("--tile", default=None)
    args = ap.parse_args()
    import numpy as np
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = {"dragon": (1920, 1080, 16), "lucy": (4096, 4096, 4), "bunny": (1024, 1024, 1)}[args.config]
    Wp, Hp = sc.padded_dims(W, H)
    rt = pt.RayTracer(0)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS[args.config]))
    tile = tuple(int(v) for v in args.tile.split(",")) if args.tile else None
    rows = H if tile is None else len(np.arange(H)[(np.arange(H) // tile[0]) % tile[1] == tile[2]])
    seeds = sc.default_seeds(Wp, Hp)
    out = np.zeros(W * rows * 4, np.float32)
    rt.setSeeds(Wp, Hp, seeds)
    rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)  # schedule + lists
    path = os.path.join(tempfile.gettempdir(), f"occ_{os.getpid()}.bin")
    os.environ["RT_PIXEL_STATS"] = path
    rt.setCounting(True)
    rt.setSeeds(Wp, Hp, seeds)
    rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
    ms = rt.lastKernelSplitMs()[1]
    info = rt.renderInfo()
    rt.setCounting(False)
    os.environ.pop("RT_PIXEL_STATS")
    st = np.fromfile(path, np.uint32).reshape(-1, 8).astype(np.int64)
    os.remove(path)
    t0 = st[:, 0].min()
    start = (st[:, 0] - t0) / 1e5  # ms
    end = (st[:, 1] - t0) / 1e5
    span = end.max()
    lanes = info["grid_blocks"] * 256
    grid = np.linspace(0, span, 2001)
    live = np.searchsorted(np.sort(start), grid, side="right") - np.searchsorted(np.sort(end), grid, side="right")
    occ = np.minimum(live / lanes, 1.0)
    def first_below(f):
        idx = np.nonzero((occ < f) & (grid > span * 0.05))[0]
        return round(float(grid[idx[0]]), 2) if len(idx) else None
    res = {"config": args.config, "tile": tile, "kernel_ms_counting": round(ms, 2), "span_ms": round(float(span), 2),
           "lanes": int(lanes), "pixels": int(len(st)),
           "below_90pct_ms": first_below(0.9), "below_50pct_ms": first_below(0.5), "below_10pct_ms": first_below(0.1),
           "idle_lane_fraction": round(float(1.0 - occ.mean()), 4),
           "end_quantiles_ms": {q: round(float(np.quantile(end, q / 100)), 2) for q in (50, 90, 99, 100)},
           "live_hist": [round(float(x), 3) for x in occ[::100]]}
    # pixels by their query count (a mesh pixel: ~2 per sample; a box pixel: ~2 x (maxDepth + 1) per sample)
    q = st[:, 2]
    spp = sr * sr
    classes = {}
    for name, lo, hi in (("q<=3spp", 0, 3 * spp), ("3spp<q<=6spp", 3 * spp, 6 * spp), ("q>6spp", 6 * spp, 1 << 62)):
        m = (q > lo) & (q <= hi) if lo else q <= hi
        if m.any():
            classes[name] = {"pixels": int(m.sum()), "start_max_ms": round(float(start[m].max()), 2),
                             "end_ms": {k: round(float(np.quantile(end[m], k / 100)), 2) for k in (50, 90, 99, 100)}}
    res["by_queries"] = classes
    print(json.dumps(res))


if __name__ == "__main__":
    main()
