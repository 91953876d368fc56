"""How much the reference's result depends on the OpenCL builtin library (container only;
TEST INFRASTRUCTURE, not product).

The reference's radiance goes through pow / sin / cos / exp / log (materials.h:190-196, :259;
rtcommon.h:287-289), whose accuracy OpenCL leaves to the implementation (sin/cos <= 4 ulp,
pow <= 16 ulp).  The parity bar here is bit equality under the pinned builtins
(include/rt_math.h), which the HIP kernels and oracle/_ref share.  This script renders the
same configurations with two builds of the UNCHANGED reference source:
  pinned  oracle/_ref/libptref.so       (clshim.c -> rt_math.h)
  libm    oracle/_ref_libm/libptref.so  (clshim.c -DCLSHIM_LIBM -> glibc sinf/cosf/expf/logf/powf)
and reports, per configuration, the share of RGB components that are bit-identical and that
lie within the north star's 1e-5 relative tolerance of each other, plus the largest relative
difference.  Since the GPU frames equal the pinned render bit for bit (tests/), the same
numbers describe the GPU against a reference built on glibc's libm.

    make -C oracle ref ref_libm && python oracle/libm_sensitivity.py [--out profiles/r03/libm_sensitivity.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(HERE))

import ptload  # noqa: E402
from oracle import LIBREF, LIBREF_LIBM, Reference  # noqa: E402


def compare(a: np.ndarray, b: np.ndarray, tol: float = 1e-5) -> dict:
    """RGB components of two RGBA32F buffers (alpha is always 0)."""
    a = a.reshape(-1, 4)[:, :3].astype(np.float64).reshape(-1)
    b = b.reshape(-1, 4)[:, :3].astype(np.float64).reshape(-1)
    same = a.view(np.uint64) == b.view(np.uint64)
    diff = np.abs(a - b)
    scale = np.maximum(np.abs(a), np.abs(b))
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = np.where(scale > 0, diff / scale, 0.0)
    within = diff <= tol * scale
    return {"components": int(a.size), "bit_identical": round(float(same.mean()), 6),
            "within_1e-5_rel": round(float(within.mean()), 6), "beyond_1e-5_rel": int((~within).sum()),
            "max_rel": float(rel.max()) if rel.size else 0.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r03" / "libm_sensitivity.json"))
    ap.add_argument("--dragon-pixels", type=int, default=16)
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    pt = ptload.load()
    sc = pt.scenes
    pinned = Reference(build_if_missing=False)
    libm = Reference(build_if_missing=False, path=LIBREF_LIBM)
    meta = json.loads((ROOT / "tests" / "golden" / "meta.json").read_text())
    res = {"pinned": str(LIBREF.relative_to(ROOT)), "libm": str(LIBREF_LIBM.relative_to(ROOT)),
           "tolerance": "north star: per-pixel radiance within 1e-5 relative", "configs": {}}

    # the golden configurations, every progressive frame (errors accumulate through the mix
    # and, for raytrace, through the seeds: a 1-ulp difference can change a later branch)
    for name, m in meta["cases"].items():
        if "kernel" not in m:
            continue
        with np.load(ROOT / "tests" / "golden" / f"{name}.npz", allow_pickle=False) as z:
            g = {k: z[k] for k in z.files}
        spheres = g["spheres"].view(pt._abi.SPHERE_DTYPE)
        W, H, Wp, Hp = m["W"], m["H"], m["Wpad"], m["Hpad"]
        verts = g.get("verts")
        idx = g.get("idx")
        outs = {}
        for who, ref in (("pinned", pinned), ("libm", libm)):
            out = np.zeros(W * H * 4, np.float32)
            sd = g["seeds_in"].copy()
            fr = []
            for p in range(m["frames"]):
                ref.launch(m["kernel"], out, g["camera"], spheres, W, H, Wp, Hp, m["sample_rate"], m["max_depth"], p,
                           sd, verts, idx, nthreads=args.threads)
                fr.append(out.copy())
            outs[who] = (fr, sd)
        assert all(np.array_equal(f.view(np.uint32), e.view(np.uint32)) for f, e in zip(outs["pinned"][0], g["frames"]))
        res["configs"][name] = {
            "frames": [compare(a, b) for a, b in zip(outs["pinned"][0], outs["libm"][0])],
            "seeds_identical": bool(np.array_equal(outs["pinned"][1], outs["libm"][1])),
        }

    # the headline configuration: dragon class, 1920x1080, sampleRate 16 (256 spp), a strided
    # subset of whole pixels (the reference's linear loop over 871,414 triangles)
    W, H, sr = 1920, 1080, 16
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS["dragon"])
    S = sc.ply_scene()
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    n = args.dragon_pixels
    pix = (np.arange(n, dtype=np.int64) * (W * H // n) + (W * H // n) // 2).astype(np.uint32)
    outs = {}
    t0 = time.time()
    for who, ref in (("pinned", pinned), ("libm", libm)):
        out = np.zeros(W * H * 4, np.float32)
        sd = sc.default_seeds(Wp, Hp)
        ref.launch_pixels(2, out, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, pix, verts, idx, nthreads=args.threads)
        outs[who] = out.reshape(-1, 4)[pix.astype(np.int64)].copy()
    res["configs"]["dragon_1920x1080_256spp_subset"] = {
        "pixels": int(n), "seconds": round(time.time() - t0, 1), **compare(outs["pinned"], outs["libm"])}

    # summary over every component compared
    tot = bit = win = 0
    for v in res["configs"].values():
        for f in v.get("frames", [v]):
            tot += f["components"]
            bit += f["bit_identical"] * f["components"]
            win += f["within_1e-5_rel"] * f["components"]
    res["all"] = {"components": tot, "bit_identical": round(bit / tot, 6), "within_1e-5_rel": round(win / tot, 6)}
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res["all"]))
    for k, v in res["configs"].items():
        last = v["frames"][-1] if "frames" in v else v
        print(k, json.dumps(last))


if __name__ == "__main__":
    main()
