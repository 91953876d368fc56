"""A/B of librtmi builds on the sphere scene (BASELINE configs[1]: main.cpp scene, 1024x1024,
sampleRate 1, progressive frames), one process per build per round; per build the median kernel
time of --frames progressive frames, and the frames' bits compared across builds.

    python profiles/sphere_ab.py LABEL=path.so LABEL= ... [--rounds 3] [--frames 40] [--size 1024]
"""
import argparse
import hashlib
import json
import statistics
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def child(args):
    sys.path.insert(0, str(ROOT))
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W = H = args.size
    rt = pt.RayTracer(0, lib_path=args.lib or None)
    rt.setSpheres(sc.main_scene())
    c = sc.MAIN_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(1)
    rt.setMaxPathDepth(6)
    out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    ms = []
    for p in range(args.frames):
        rt.rayTrace(out, W, H, p, kernel=0)
        ms.append(rt.lastKernelMs())
    h = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()
    print(json.dumps({"median_ms": statistics.median(ms[3:]), "min_ms": min(ms[3:]), "sha1": h}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--lib", default="")
    args = ap.parse_args()
    if args.child:
        return child(args)
    res = {}
    for rnd in range(args.rounds):
        for spec in (args.libs if rnd % 2 == 0 else list(reversed(args.libs))):
            label, _, path = spec.partition("=")
            r = subprocess.run([sys.executable, "-u", __file__, "--child", "--lib", path, "--frames", str(args.frames),
                                "--size", str(args.size)], capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(r.returncode)
            line = json.loads(r.stdout.strip().split("\n")[-1])
            res.setdefault(label, []).append(line)
            print(f"round {rnd + 1} {label}: median {line['median_ms']:.4f} ms min {line['min_ms']:.4f}", flush=True)
    out = {lab: {"median_ms": statistics.median(x["median_ms"] for x in v), "min_ms": min(x["min_ms"] for x in v)}
           for lab, v in res.items()}
    out["bit_identical"] = len({x["sha1"] for v in res.values() for x in v}) == 1
    print(json.dumps(out))


if __name__ == "__main__":
    main()
