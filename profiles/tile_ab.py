"""A/B of librtmi builds on the N-way row-stripe tiles of the dragon frame, ONE PROCESS PER BUILD
per round (in-process A/Bs of several builds misread tiles: DESIGN.md §7), builds alternating
round by round so clock drift hits them alike.  Each child renders every rank's tile (best of
--reps) and reports the slowest; the parent prints per-build medians and checks that the builds'
tiles are bit-identical.

    python profiles/tile_ab.py LABEL=path.so LABEL= LABEL=?K=V ... [--n 8] [--rounds 3] [--reps 2] [--frame]
    (LABEL= with an empty path: the in-tree build; ?K=V+K2=V2 after the path: that child's environment)
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


def child(args):
    sys.path.insert(0, str(ROOT))
    for kv in args.env:
        k, _, v = kv.partition("=")
        os.environ[k] = v
    import torch
    import ptload

    pt = ptload.load()
    sc = pt.scenes
    W, H, sr = 1920, 1080, 16
    rt = pt.RayTracer(0, lib_path=args.lib or None)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS["dragon"]))
    Wp, Hp = sc.padded_dims(W, H)
    seeds = sc.default_seeds(Wp, Hp)
    ptdist = ptload.submodule("dist")
    times, h = [], hashlib.sha1()
    ranks = range(args.n) if args.n > 1 else [0]
    owner = rt.partitionStripes(W, H, 8, args.n) if args.balanced and args.n > 1 else None
    for r in ranks:
        tile = ((8, args.n, r) + ((owner,) if owner is not None else ())) if args.n > 1 else None
        rows = len(ptdist.tile_rows(H, 8, args.n, r, owner)) if args.n > 1 else H
        out = torch.zeros(rows * W * 4, dtype=torch.float32, device="cuda:0")
        best = 1e9
        for _ in range(args.reps):
            rt.setSeeds(Wp, Hp, seeds)
            rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
            best = min(best, rt.lastKernelMs())
        times.append(best)
        h.update(out.cpu().numpy().tobytes())
    frame = None
    if args.frame:
        out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
        frame = 1e9
        for _ in range(args.reps):
            rt.setSeeds(Wp, Hp, seeds)
            rt.rayTrace(out, W, H, 0, kernel=2)
            frame = min(frame, rt.lastKernelMs())
    print(json.dumps({"max_ms": max(times), "rank_ms": [round(t, 3) for t in times], "frame_ms": frame,
                      "sha1": h.hexdigest()}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--frame", action="store_true", help="also time the whole frame (best of --reps)")
    ap.add_argument("--balanced", action="store_true", help="the tiles under rt_partition_stripes' owner map")
    ap.add_argument("--env", action="append", default=[])
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--lib", default="")
    args = ap.parse_args()
    if args.child:
        return child(args)
    res = {}
    for rnd in range(args.rounds):
        order = args.libs if rnd % 2 == 0 else list(reversed(args.libs))
        for spec in order:
            label, _, path = spec.partition("=")
            path, _, envs = path.partition("?")  # LABEL=path?K=V+K2=V2: that child's environment too
            cmd = [sys.executable, "-u", __file__, "--child", "--lib", path, "--n", str(args.n), "--reps",
                   str(args.reps)] + (["--frame"] if args.frame else []) + (["--balanced"] if args.balanced else []) + sum(
                       (["--env", e] for e in args.env + [kv for kv in envs.split("+") if kv]), [])
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(r.returncode)
            line = json.loads(r.stdout.strip().split("\n")[-1])
            res.setdefault(label, []).append(line)
            print(f"round {rnd + 1} {label}: max {line['max_ms']:.3f} ms ranks {line['rank_ms']}"
                  + (f" frame {line['frame_ms']:.2f} ms" if line["frame_ms"] else ""), flush=True)
    shas = {lab: {x["sha1"] for x in v} for lab, v in res.items()}
    summary = {lab: {"median_max_ms": statistics.median(x["max_ms"] for x in v),
                     "min_max_ms": min(x["max_ms"] for x in v),
                     "median_frame_ms": statistics.median(x["frame_ms"] for x in v) if args.frame else None}
               for lab, v in res.items()}
    summary["bit_identical"] = len(set().union(*shas.values())) == 1
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
