"""Where does the dragon frame's time go, pixel by pixel?  A plain launch with
RT_PIXEL_STATS (per-pixel start / finish clocks) and a counting one (queries, traversal
steps per pixel), then: the finish
time distribution, the last pixels to finish and what they are (probe: box or mesh pixel),
and how the frame's last milliseconds are spent.  GPU box.

    python profiles/pixel_stats.py [out.json] [--config dragon|bunny] [--lib build.so] [--tile N:R]

`--tile N:R`: rank R's row-stripe tile (stripe 8) of an N-way split of the frame instead.

The plain launch records clocks only in a diagnostics build of the library
(`bash profiles/build_variant.sh ab/stats.so -DRT_PLAIN_PIXEL_STATS=1`, run with
RTMI_LIB=ab/stats.so); otherwise the clocks are the counting launch's (slower, distorted).
"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch
    import ptload

    dump = "/tmp/rt_pixel_stats.bin"
    os.environ["RT_PIXEL_STATS"] = dump
    argv = sys.argv[1:]
    cfg = "dragon"
    if "--config" in argv:
        i = argv.index("--config")
        cfg = argv[i + 1]
        del argv[i:i + 2]
    if "--lib" in argv:  # a diagnostics build (RT_PLAIN_PIXEL_STATS)
        i = argv.index("--lib")
        os.environ["RTMI_LIB"] = str(Path(argv[i + 1]).resolve())
        del argv[i:i + 2]
    tile = None
    if "--tile" in argv:  # rank R's row-stripe tile of N (stripe 8)
        i = argv.index("--tile")
        n, r = (int(v) for v in argv[i + 1].split(":"))
        tile = (8, n, r)
        del argv[i:i + 2]
    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = (1920, 1080, 16) if cfg == "dragon" else (1024, 1024, 1)
    rt = pt.RayTracer(0)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS[cfg]))
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    if tile:
        H = len(ptload.submodule("dist").tile_rows(H, *tile))  # the dump holds the tile's rows
    H_frame = H if not tile else {"dragon": 1080, "bunny": 1024}[cfg]
    rt.rayTrace(out, W, H_frame, 0, kernel=2, tile=tile)  # probe + warm
    rt.rayTrace(out, W, H_frame, 0, kernel=2, tile=tile)
    plain_ms = rt.lastKernelMs()
    s = np.fromfile(dump, np.uint32).reshape(H, W, 8).astype(np.int64)  # timing: the plain launch
    if not s[..., 1].any():  # the library records clocks in counting launches only
        s = None
    rt.setCounting(True)
    rt.rayTrace(out, W, H_frame, 0, kernel=2, tile=tile)
    count_ms = rt.lastKernelMs()
    sc_ = np.fromfile(dump, np.uint32).reshape(H, W, 8).astype(np.int64)  # queries / steps
    if s is None:
        s = sc_
    t0 = s[..., 0].min()
    start = (s[..., 0] - t0) / 1e5  # ms (100 MHz)
    fin = (s[..., 1] - t0) / 1e5
    q = sc_[..., 2]
    steps = sc_[..., 3]
    dur = fin - start
    end = fin.max()
    res = {"plain_ms": plain_ms, "counting_ms": count_ms, "span_ms": float(end),
           "finish_pct": {p: float(np.percentile(fin, p)) for p in (50, 90, 99, 99.9, 100)},
           "dur_pct": {p: float(np.percentile(dur, p)) for p in (50, 90, 99, 99.9, 100)},
           "queries_pct": {p: float(np.percentile(q, p)) for p in (50, 90, 99, 100)},
           "pixels_running_at_pct_of_span": {}}
    for f in (0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9, 0.95, 0.99):
        t = f * end
        res["pixels_running_at_pct_of_span"][f] = int(((start <= t) & (fin > t)).sum())
    res["started_pct"] = {p: float(np.percentile(start, p)) for p in (50, 90, 99, 100)}
    # loop iterations and phase clocks: the plain launch's in a RT_PLAIN_PIXEL_STATS build, else the
    # counting launch's
    ph = s if s[..., 4:8].any() else sc_
    res["phase_source"] = "plain" if ph is s and s is not sc_ else "counting"
    # the 20 last finishers
    idx = np.argsort(fin.ravel())[-20:]
    res["last"] = [{"x": int(i % W), "y": int(i // W), "start": round(float(start.ravel()[i]), 2),
                    "finish": round(float(fin.ravel()[i]), 2), "queries": int(q.ravel()[i]),
                    "steps": int(steps.ravel()[i]),
                    # counting launch: loop iterations and wave clocks (x 64) in the path advance (D),
                    # the refill + camera ray (A/B) and the stepping rounds (C) while the pixel ran
                    "plain_q": int(ph[..., 2].ravel()[i]), "plain_steps": int(ph[..., 3].ravel()[i]),
                    "iters": int(ph[..., 7].ravel()[i]), "d_kclk": int(ph[..., 4].ravel()[i]) * 64 // 1000,
                    "ab_kclk": int(ph[..., 5].ravel()[i]) * 64 // 1000,
                    "c_kclk": int(ph[..., 6].ravel()[i]) * 64 // 1000} for i in idx]
    # costly pixels: many queries
    heavy = q > 2 * np.median(q)
    res["heavy_pixels"] = int(heavy.sum())
    res["heavy_start_pct"] = {p: float(np.percentile(start[heavy], p)) for p in (50, 90, 100)}
    res["heavy_dur_pct"] = {p: float(np.percentile(dur[heavy], p)) for p in (10, 50, 90, 100)}
    res["light_dur_pct"] = {p: float(np.percentile(dur[~heavy], p)) for p in (10, 50, 90, 100)}
    it = ph[..., 7]
    res["iters_pct"] = {p: float(np.percentile(it, p)) for p in (50, 90, 99, 100)}
    res["heavy_iters_pct"] = {p: float(np.percentile(it[heavy], p)) for p in (50, 90, 100)}
    # iterations beyond a pixel's own need (one per query, plus its steps over 6 per stepping round)
    need = ph[..., 2] + (ph[..., 3] + 5) // 6
    res["excess_iters_pct"] = {p: float(np.percentile(it - need, p)) for p in (10, 50, 90, 99, 100)}
    res["excess_iters_heavy_pct"] = {p: float(np.percentile((it - need)[heavy], p)) for p in (10, 50, 90, 99, 100)}
    tot = ph[..., 4:7].sum(axis=(0, 1)).astype(np.float64)
    res["phase_share"] = {"D": tot[0] / tot.sum(), "AB": tot[1] / tot.sum(), "C": tot[2] / tot.sum()}
    txt = json.dumps(res, indent=1)
    print(txt)
    if argv:
        Path(argv[0]).write_text(txt + "\n")


if __name__ == "__main__":
    main()
