"""Diagnose context-to-context speed variance: K RayTracer contexts of the same library and
scene in one process, each timed over a few frames, plus one counting launch each
(traversal counts and s_memtime clocks).  GPU box.

    python profiles/ctx_variance.py [K] [lib.so]
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    lib = sys.argv[2] if len(sys.argv) > 2 else None
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = 1920, 1080, 16
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS["dragon"])
    Wp, Hp = sc.padded_dims(W, H)
    seeds = sc.default_seeds(Wp, Hp)
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    ctxs = []
    for k in range(K):
        rt = pt.RayTracer(0, lib_path=lib)
        rt.setSpheres(sc.ply_scene())
        c = sc.PLY_CAMERA
        rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
        rt.setSampleRate(sr)
        rt.setMaxPathDepth(6)
        rt.setMesh(verts, idx)
        ctxs.append(rt)
    for r in range(3):
        line = []
        for k, rt in enumerate(ctxs):
            rt.setSeeds(Wp, Hp, seeds)
            rt.rayTrace(out, W, H, 0, kernel=2)
            line.append(f"{rt.lastKernelMs():9.2f}")
        print("round", r, " ".join(line), flush=True)
    for k, rt in enumerate(ctxs):
        rt.setCounting(True)
        rt.setSeeds(Wp, Hp, seeds)
        rt.rayTrace(out, W, H, 0, kernel=2)
        c = rt.counters()
        rt.setCounting(False)
        print(k, f"{rt.lastKernelMs():9.2f} ms", {f: c[f] for f in ("nodes_visited", "lane_slots", "clocks_traversal",
                                                                      "clocks_total", "pixel_clocks_max")}, flush=True)


if __name__ == "__main__":
    main()
