"""Profiling driver for the headline kernel's steady state (bench.py's timed frames, without the
bench's other legs): the dragon-class frame (BASELINE configs[3]: 871,414 triangles, 1920x1080,
sampleRate 16, maxDepth 6), one counting launch for the algorithmic bytes (k_tris<..., COUNT>, a
different kernel symbol; it builds the view's lists and schedule and records its pixels' costs, so
no pilot runs), two plain frames (the measured-cost order), and --frames steady-state frames
enqueued back to back as bench.py's timed loop does.  Under rocprofv3 the main kernel
k_tris<4, false, false, true> appears as 2 + --frames full-grid dispatches;
profiles/summarize_pmc.py --last <frames> averages the steady ones only.  Prints one JSON line: the steady frames' live kernel times (HIP events, a
synchronous pass after the pipelined one), their measured ray totals, and the counting launch's
algorithmic bytes (nodes x 64 B + triangle tests x 36 B + pixels x 32 B).

    python profiles/steady_state.py [--frames 8]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    args = ap.parse_args()
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = 1920, 1080, 16
    rt = pt.RayTracer(0)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setFoVAngle(sc.DEFAULT_FOV)
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS["dragon"]))
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    Wp, Hp = sc.padded_dims(W, H)
    rt.setSeeds(Wp, Hp, sc.default_seeds(Wp, Hp))
    seeds0 = rt.getSeeds()
    rt.setCounting(True)
    rt.rayTrace(out, W, H, 0, kernel=2)  # lists, probe, the counting kernel (its own symbol)
    cnt = rt.counters()
    rt.setCounting(False)
    rt.setSeeds(Wp, Hp, seeds0)
    rt.rayTrace(out, W, H, 0, kernel=2)  # ordered by the counting launch's measured costs
    rt.rayTrace(out, W, H, 0, kernel=2)
    rt.counterTotals(reset=True)
    torch.cuda.synchronize()
    for _ in range(args.frames):  # the steady state, enqueued back to back (bench.py's timed loop)
        rt.rayTrace(out, W, H, 0, kernel=2, sync=False)
    rt.synchronize()
    tot = rt.counterTotals(reset=True)
    alg = cnt["nodes_visited"] * 64 + cnt["tris_tested"] * 36 + W * H * 32
    print(json.dumps({"frames": args.frames, "renders_counted": tot["renders"],
                      "rays_per_frame": (tot["rays_closest"] + tot["rays_shadow"]) / max(tot["renders"], 1),
                      "algorithmic_bytes_per_launch": int(alg), "nodes_visited": int(cnt["nodes_visited"]),
                      "tris_tested": int(cnt["tris_tested"]),
                      "main_kernel": "k_tris<4, false, false, true>",
                      "main_dispatches": 2 + args.frames,
                      "steady_dispatches": f"the last {args.frames}"}))


if __name__ == "__main__":
    main()
