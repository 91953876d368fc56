"""Seed-pass chains of a sample-split tile, per pixel (diagnostics; RT_SPLIT=1 + RT_PIXEL_STATS):
duration, traversal steps and camera rays that missed the mesh, for the mesh-class and the
box-class pixels (the probe's classes).

    python profiles/seed_stats.py [--tile 8,8,0]
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
    ap.add_argument("--tile", default="8,8,0")
    ap.add_argument("--lib", default=None, help="a build with -DRT_SEED_STATS=1 adds queries / immediate answers / iterations")
    args = ap.parse_args()
    os.environ["RT_SPLIT"] = "1"
    import numpy as np
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = 1920, 1080, 16
    Wp, Hp = sc.padded_dims(W, H)
    rt = pt.RayTracer(0, lib_path=args.lib)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS["dragon"]))
    tile = tuple(int(v) for v in args.tile.replace(":", ",").split(","))
    rows = len(np.arange(H)[(np.arange(H) // tile[0]) % tile[1] == tile[2]])
    out = np.zeros(W * rows * 4, np.float32)
    rt.setSeeds(Wp, Hp, sc.default_seeds(Wp, Hp))
    rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
    path = os.path.join(tempfile.gettempdir(), f"seed_{os.getpid()}.bin")
    os.environ["RT_PIXEL_STATS"] = path
    rt.setSeeds(Wp, Hp, sc.default_seeds(Wp, Hp))
    rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
    os.environ.pop("RT_PIXEL_STATS")
    st = np.fromfile(path, np.uint32).reshape(-1, 8).astype(np.int64)
    os.remove(path)
    kind, iters = st[:, 4] & 15, st[:, 4] >> 4
    t0 = st[kind > 0, 0].min()
    res = {"tile": tile, "pixels": int(len(st))}
    for name, k in (("mesh", 2), ("box", 3)):
        m = kind == k
        if not m.any():
            continue
        dur = (st[m, 1] - st[m, 0]) / 1e5
        end = (st[m, 1] - t0) / 1e5
        steps, box = st[m, 2], st[m, 3]
        order = np.argsort(-dur)[:12]
        res[name] = {"pixels": int(m.sum()), "end_ms_max": round(float(end.max()), 2),
                     "end_ms": {q: round(float(np.quantile(end, q / 100)), 2) for q in (50, 70, 80, 90, 95, 99, 100)},
                     "dur_ms": {q: round(float(np.quantile(dur, q / 100)), 2) for q in (50, 90, 99, 100)},
                     "steps": {q: int(np.quantile(steps, q / 100)) for q in (50, 90, 99, 100)},
                     "missed_camera_rays": {q: int(np.quantile(box, q / 100)) for q in (50, 90, 99, 100)},
                     "pixels_with_misses": int((box > 0).sum()),
                     "longest": [[round(float(dur[i]), 2), int(steps[i]), int(box[i])] for i in order]}
        q, imm, it = st[m, 7] >> 16, st[m, 7] & 0xffff, iters[m]
        if it.max() > 0:  # an RT_SEED_STATS build
            res[name]["queries_with_rounds"] = {p: int(np.quantile(q, p / 100)) for p in (50, 90, 100)}
            res[name]["answered_in_advance"] = {p: int(np.quantile(imm, p / 100)) for p in (50, 90, 100)}
            res[name]["iterations"] = {p: int(np.quantile(it, p / 100)) for p in (50, 90, 100)}
            res[name]["us_per_iteration_longest"] = [round(float(dur[i]) * 1e3 / max(1, int(it[i])), 2) for i in order[:4]]
            res[name]["longest_q_imm_it"] = [[int(q[i]), int(imm[i]), int(it[i])] for i in order[:6]]
            adv, rnd = st[m, 5] * 64.0, st[m, 6] * 64.0  # shader clocks in the path advance / the rounds
            res[name]["advance_share_longest"] = [round(float(adv[i] / max(1.0, adv[i] + rnd[i])), 3) for i in order[:6]]
            res[name]["clocks_per_iteration_longest"] = [int((adv[i] + rnd[i]) / max(1, int(it[i]))) for i in order[:6]]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
