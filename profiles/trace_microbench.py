"""Traversal micro-benchmark (GPU): closest-hit / any-hit throughput of the BVH and linear
traversal in isolation (k_trace_rays, one ray per lane, no path state machine), on the
dragon-class mesh, for coherent primary rays and incoherent random rays.

    python profiles/trace_microbench.py [n_tris]
"""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import ptload  # noqa: E402

pt = ptload.load()
sc = pt.scenes
n_tris = int(sys.argv[1]) if len(sys.argv) > 1 else sc.MESH_CONFIGS["dragon"]
verts, idx = sc.make_mesh(n_tris)
rt = pt.RayTracer(0)
rt.setMesh(verts, idx)
cam = sc.camera_spherical(1920, **sc.PLY_CAMERA)
prim = sc.camera_rays(cam, 1920, 1080)
rng = np.random.default_rng(1)
n = 2_000_000
rr = np.zeros(n, pt._abi.RAY_DTYPE)
rr["o"] = rng.uniform([-5.9, -4.9, -5.9], [5.9, 4.9, 5.9], (n, 3)).astype(np.float32)
d = rng.normal(size=(n, 3)).astype(np.float32)
rr["d"] = d / np.linalg.norm(d, axis=1, keepdims=True)
rr["tmin"] = np.float32(1e-4)
rr["tmax"] = np.float32(np.inf)
sh = rr.copy()
sh["tmax"] = rng.uniform(0, 10, n).astype(np.float32)
res = {}
for trav in ("bvh", "bvh2", "packet"):
    rt.setTraversal(trav)
    for name, rays, anyhit in [("primary_closest", prim, False), ("random_closest", rr, False),
                               ("random_anyhit", sh, True)]:
        rt.traceRays(rays[:1024], anyhit)
        best = None
        for _ in range(3):
            hit, _t = rt.traceRays(rays, anyhit)
            ms = rt.lastKernelMs()
            best = ms if best is None else min(best, ms)
        res[f"{trav}/{name}"] = {"rays": len(rays), "kernel_ms": round(best, 3),
                                 "mrays_per_s": round(len(rays) / best / 1e3, 1),
                                 "hit_frac": round(float((hit > 0).mean() if anyhit else (hit >= 0).mean()), 4)}
print(json.dumps({"n_tris": n_tris, "bvh": rt.meshInfo(), "results": res}))
