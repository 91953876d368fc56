"""A/B of librtmi builds on a whole frame, one process per build per round (in-process A/Bs of
several builds misread: DESIGN.md §7), builds alternating round by round: per build the median
kernel time of --frames frames of the same view (the first --skip dropped: schedule, lists), and
the frames' bits compared across builds.

    python profiles/frame_ab.py LABEL=path.so LABEL= LABEL=?K=V ... [--config bunny|dragon|spheres] [--rounds 3] [--frames 20]
    (LABEL= with an empty path: the in-tree build; ?K=V+K2=V2 after the path: environment of that child)
"""
import argparse
import hashlib
import json
import os
import statistics
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CONFIGS = {"bunny": (1024, 1024, 1), "dragon": (1920, 1080, 16), "spheres": (1024, 1024, 1)}


def child(args):
    sys.path.insert(0, str(ROOT))
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = CONFIGS[args.config]
    rt = pt.RayTracer(0, lib_path=args.lib or None)
    if args.config == "spheres":
        rt.setSpheres(sc.main_scene())
        c = sc.MAIN_CAMERA
        kernel = 0
    else:
        rt.setSpheres(sc.ply_scene())
        c = sc.PLY_CAMERA
        rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS[args.config]))
        kernel = 2
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    Wp, Hp = sc.padded_dims(W, H)
    seeds = sc.default_seeds(Wp, Hp)
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    ms = []
    for _ in range(args.frames):
        rt.setSeeds(Wp, Hp, seeds)  # every frame the same (progression 0 from the same seeds)
        rt.rayTrace(out, W, H, 0, kernel=kernel)
        ms.append(rt.lastKernelMs())
    h = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()
    ms = ms[args.skip:]
    print(json.dumps({"median_ms": statistics.median(ms), "min_ms": min(ms), "sha1": h}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--config", default="bunny", choices=sorted(CONFIGS))
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--skip", type=int, default=3)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--lib", default="")
    args = ap.parse_args()
    if args.child:
        return child(args)
    res = {}
    for rnd in range(args.rounds):
        for spec in (args.libs if rnd % 2 == 0 else list(reversed(args.libs))):
            label, _, path = spec.partition("=")
            path, _, envs = path.partition("?")
            env = dict(os.environ)
            for kv in filter(None, envs.split("+")):
                k, _, v = kv.partition("=")
                env[k] = v
            r = subprocess.run([sys.executable, "-u", __file__, "--child", "--lib", path, "--config", args.config,
                                "--frames", str(args.frames), "--skip", str(args.skip)],
                               capture_output=True, text=True, timeout=600, env=env)
            if r.returncode != 0:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(r.returncode)
            line = json.loads(r.stdout.strip().split("\n")[-1])
            res.setdefault(label, []).append(line)
            print(f"round {rnd + 1} {label}: median {line['median_ms']:.4f} ms min {line['min_ms']:.4f}", flush=True)
    out = {lab: {"median_ms": statistics.median(x["median_ms"] for x in v), "min_ms": min(x["min_ms"] for x in v)}
           for lab, v in res.items()}
    out["bit_identical"] = len({x["sha1"] for v in res.values() for x in v}) == 1
    print(json.dumps({"config": args.config, **out}))


if __name__ == "__main__":
    main()
