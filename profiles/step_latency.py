"""Per-step latency of ONE traversal on an idle chip (rt_trace_rays, one ray per launch).

For ray sets drawn like the dragon frame's queries — camera rays onto the mesh, shadow rays
from the mesh toward the light, and box-path rays (Lambert bounces and shadow rays from the
floor beside the mesh) — each ray is traced alone (one lane, one wave on the chip) and in a
wave of 64 copies, with a counting call giving its steps (nodes + leaf triangles).
kernel µs / steps = what one dependent traversal step costs a chain with the chip to itself.

    python profiles/step_latency.py [--n 48]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def unit(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def rays_for(kind, n, rng, pt):
    R = np.zeros(n, pt._abi.RAY_DTYPE)
    light = np.array([0.0, 4.0, 2.0])
    if kind == "primary":
        cam = np.array([3.0, -0.8, 2.0])
        tgt = np.stack([rng.uniform(-2.5, 2.5, n), -2.2 + rng.uniform(-2.5, 2.5, n), rng.uniform(-2.5, 2.5, n)], 1)
        o = np.tile(cam, (n, 1))
        d = unit(tgt - cam)
        tmax = np.full(n, np.inf)
    else:
        ang = rng.uniform(0, 2 * np.pi, n)
        rad = rng.uniform(2.4, 4.4, n)
        o = np.stack([rad * np.cos(ang), np.full(n, -5.0 + 1e-4), rad * np.sin(ang)], 1)
        if kind == "box_shadow":
            l = light - o
            ll = np.linalg.norm(l, axis=1)
            d = l / ll[:, None]
            tmax = ll - 0.5 - 1e-4
        else:  # box_bounce: cosine-weighted about +y
            r1, r2 = rng.uniform(0, 1, n), rng.uniform(0, 1, n)
            ct = np.sqrt(1 - r1)
            st = np.sqrt(1 - ct * ct)
            ph = 2 * np.pi * r2
            d = np.stack([np.cos(ph) * st, ct, np.sin(ph) * st], 1)
            tmax = np.full(n, np.inf)
    R["o"] = o.astype(np.float32)
    R["d"] = d.astype(np.float32)
    R["tmin"] = 1e-4
    R["tmax"] = tmax.astype(np.float32)
    return R


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=48)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    rt = pt.RayTracer(0)
    rt.setSpheres(sc.ply_scene())
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS["dragon"]))
    rng = np.random.default_rng(3)
    out = {}
    for kind in ("primary", "box_bounce", "box_shadow"):
        R = rays_for(kind, args.n, rng, pt)
        any_hit = kind == "box_shadow"
        rows = []
        for i in range(args.n):
            one = R[i:i + 1]
            rt.setCounting(True)
            rt.traceRays(one, any_hit)
            c = rt.counters()
            rt.setCounting(False)
            steps = c["nodes_visited"] + c["leaves_visited"]
            t1 = min(rt.traceRays(one, any_hit) and rt.lastKernelMs() for _ in range(args.reps))
            wave = np.repeat(one, 64)
            t64 = min(rt.traceRays(wave, any_hit) and rt.lastKernelMs() for _ in range(args.reps))
            rows.append((steps, t1 * 1e3, t64 * 1e3))
        a = np.array(rows, float)
        # least-squares fit: time = fixed + per_step * steps
        A = np.stack([np.ones(len(a)), a[:, 0]], 1)
        f1 = np.linalg.lstsq(A, a[:, 1], rcond=None)[0]
        f64 = np.linalg.lstsq(A, a[:, 2], rcond=None)[0]
        out[kind] = {"mean_steps": round(a[:, 0].mean(), 2), "mean_us_1lane": round(a[:, 1].mean(), 2),
                     "us_per_step_1lane": round(f1[1], 4), "fixed_us_1lane": round(f1[0], 2),
                     "us_per_step_wave": round(f64[1], 4), "fixed_us_wave": round(f64[0], 2)}
        print(json.dumps({kind: out[kind]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
