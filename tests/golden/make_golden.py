"""Generate the golden fixtures from the reference kernel itself (container-only).

The reference has no tests, fixtures or golden vectors of its own, so the
pins are produced here from its own source: clrt/ocl/raytracer.cl compiled unchanged for
x86-64 (oracle/Makefile `ref` -> oracle/_ref/libptref.so, read in place from
/root/reference) under the pinned arithmetic model (include/rt_math.h), driven with
RayTracerCL's launch semantics (padded NDRange, glibc rand() seeds, progression 0..F-1).
The camera floats come from the reference's own host math compiled against its vendored
gmtl (oracle/ref_camera.cpp).

Outputs (committed): tests/golden/*.npz (inputs + expected outputs) and
tests/golden/meta.json.  Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import subprocess
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import ptload  # noqa: E402
from oracle import Reference  # noqa: E402

pt = ptload.load()
sc = pt.scenes
ab = pt._abi


def frames(ref, kernel, W, H, sr, depth, n_frames, spheres, cam, seeds, verts=None, idx=None, nd_y=8):
    Wp, Hp = sc.padded_dims(W, H, nd_y)
    out = np.zeros(W * H * 4, np.float32)
    sd = seeds.copy()
    per_frame = []
    for p in range(n_frames):
        ref.launch(kernel, out, cam, spheres, W, H, Wp, Hp, sr, depth, p, sd, verts, idx)
        per_frame.append(out.copy())
    return np.stack(per_frame), sd


def main():
    ref = Reference()
    meta = {"generator": "tests/golden/make_golden.py",
            "reference": "clrt/ocl/raytracer.cl compiled by ROCm clang (-x cl -cl-std=CL1.2 -O2 "
                         "-ffp-contract=off -cl-fp32-correctly-rounded-divide-sqrt, x86-64) + oracle/clshim.c",
            "cases": {}}
    rng = np.random.default_rng(20261015)

    # ---- whole-frame sphere kernels (raytrace / raytrace_ss), main.cpp scene ---------------
    S = sc.main_scene()
    for name, kernel, W, H, sr, nf in [("spheres_64x64_sr1", 0, 64, 64, 1, 4),
                                       ("spheres_48x40_sr2", 0, 48, 40, 2, 3),
                                       ("spheres_ss_64x64", 1, 64, 64, 1, 3)]:
        Wp, Hp = sc.padded_dims(W, H)
        cam = ref.camera_spherical(W, **sc.MAIN_CAMERA)
        seeds = sc.default_seeds(Wp, Hp)
        imgs, sd = frames(ref, kernel, W, H, sr, 6, nf, S, cam, seeds)
        np.savez_compressed(HERE / f"{name}.npz", spheres=S.view(np.uint8), camera=cam, seeds_in=seeds,
                            frames=imgs, seeds_out=sd)
        meta["cases"][name] = dict(kernel=kernel, W=W, H=H, Wpad=Wp, Hpad=Hp, nd_y=8, sample_rate=sr, max_depth=6,
                                   frames=nf, scene="main.cpp", camera=sc.MAIN_CAMERA, seeds="glibc rand() seed 1")

    # ---- whole-frame triangle kernel, plymain.cpp lights, 2000-tri synthetic mesh -----------
    S2 = sc.ply_scene()
    verts, idx = sc.make_mesh(2000)
    for name, W, H, sr, nf, nd_y in [("tris_64x48_sr1", 64, 48, 1, 3, 8), ("tris_40x30_sr2", 40, 30, 2, 2, 16)]:
        Wp, Hp = sc.padded_dims(W, H, nd_y)
        cam = ref.camera_spherical(W, **sc.PLY_CAMERA)
        seeds = sc.default_seeds(Wp, Hp)
        imgs, sd = frames(ref, 2, W, H, sr, 6, nf, S2, cam, seeds, verts, idx, nd_y)
        np.savez_compressed(HERE / f"{name}.npz", spheres=S2.view(np.uint8), camera=cam, seeds_in=seeds,
                            frames=imgs, seeds_out=sd, verts=verts, idx=idx)
        meta["cases"][name] = dict(kernel=2, W=W, H=H, Wpad=Wp, Hpad=Hp, nd_y=nd_y, sample_rate=sr, max_depth=6,
                                   frames=nf, scene="plymain.cpp", camera=sc.PLY_CAMERA,
                                   mesh="rt_make_mesh(2000) (verts/idx stored)")

    # ---- primary-hit triangle indices + t (scene_intersection_tri) -------------------------
    cam = ref.camera_spherical(64, **sc.PLY_CAMERA)
    rays = sc.camera_rays(cam, 64, 48)
    hit, t = ref.closest_hits(rays, verts, idx)
    # plus random rays from inside the box, including bounce-like origins on the mesh
    n = 4096
    rr = np.zeros(n, ab.RAY_DTYPE)
    rr["o"] = rng.uniform([-5, -4.9, -5], [5, 4.9, 5], (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    rr["d"] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rr["tmin"] = np.float32(1e-4)
    rr["tmax"] = np.float32(np.inf)
    h2, t2 = ref.closest_hits(rr, verts, idx)
    sh = rr.copy()
    sh["tmax"] = rng.uniform(0.0, 8.0, n).astype(np.float32)
    occ = ref.any_hits(sh, verts, idx)
    np.savez_compressed(HERE / "hits_2000.npz", verts=verts, idx=idx, primary_rays=rays.view(np.uint8),
                        primary_hit=hit, primary_t=t, random_rays=rr.view(np.uint8), random_hit=h2, random_t=t2,
                        shadow_rays=sh.view(np.uint8), shadow_occluded=occ)
    meta["cases"]["hits_2000"] = dict(what="scene_intersection_tri / visibility_test_tri on 64x48 primary rays "
                                           "and 4096 random rays", hit_fraction=float((hit >= 0).mean()))

    # ---- per-function known answers ---------------------------------------------------------
    L = ref.lib
    seeds = np.array([[2, 2], [12345, 67890], [0xFFFFFFFF, 0x80000001], [1804289383, 846930886]], np.uint32)
    frand = np.zeros((len(seeds), 64), np.float32)
    for k, s in enumerate(seeds):
        st = s.copy()
        L.ref_frand_seq(st.ctypes.data, frand[k].ctypes.data, 64)
    # ray/triangle (intersects_triangle + _p) on random triangles
    m = 2048
    tri = rng.uniform(-1, 1, (m, 9)).astype(np.float32)
    rays_t = np.zeros(m, ab.RAY_DTYPE)
    rays_t["o"] = rng.uniform(-2, 2, (m, 3)).astype(np.float32)
    dd = (tri[:, :3] + 0.3 * tri[:, 3:6] + 0.3 * tri[:, 6:9]) - rays_t["o"]
    dd += rng.normal(scale=0.2, size=dd.shape)
    rays_t["d"] = (dd / np.linalg.norm(dd, axis=1, keepdims=True)).astype(np.float32)
    rays_t["tmin"] = np.float32(1e-4)
    rays_t["tmax"] = np.where(rng.uniform(size=m) < 0.5, np.inf, rng.uniform(0.5, 4, m)).astype(np.float32)
    tri_hit = np.zeros(m, np.int32)
    tri_p = np.zeros(m, np.int32)
    tri_uvt = np.zeros((m, 3), np.float32)
    for k in range(m):
        r = rays_t[k:k + 1].copy()
        u = np.zeros(1, np.float32)
        v = np.zeros(1, np.float32)
        tr = tri[k].copy()
        tri_p[k] = L.ref_intersects_triangle_p(r.ctypes.data, tr.ctypes.data)
        tri_hit[k] = L.ref_intersects_triangle(r.ctypes.data, u.ctypes.data, v.ctypes.data, tr.ctypes.data)
        tri_uvt[k] = (u[0], v[0], r["tmax"][0])
    # ray/sphere and the box
    sph_c = rng.uniform(-3, 3, (m, 3)).astype(np.float32)
    sph_r = rng.uniform(0.2, 2, m).astype(np.float32)
    sph_d = np.zeros(m, np.float32)
    box_t = np.zeros(m, np.float32)
    box_n = np.zeros((m, 3), np.float32)
    rays_b = rays_t.copy()
    rays_b["o"] = rng.uniform([-5.9, -4.9, -5.9], [5.9, 4.9, 5.9], (m, 3)).astype(np.float32)
    rays_b["tmax"] = np.float32(np.inf)
    for k in range(m):
        c = sph_c[k].copy()
        sph_d[k] = L.ref_intersect_sphere(rays_t[k:k + 1].ctypes.data, c.ctypes.data, float(sph_r[k]))
        rb = rays_b[k:k + 1].copy()
        box_t[k] = L.ref_intersects_box(rb.ctypes.data, 6.0, 5.0, 6.0)
        hit = np.zeros(6, np.float32)
        hit[:3] = rb["o"][0] + rb["d"][0] * box_t[k]
        L.ref_box_normal(rb.ctypes.data, hit.ctypes.data, 6.0, 5.0, 6.0)
        box_n[k] = hit[3:]
    # sample_material over the main.cpp materials (+ a blurred-refraction material)
    mats = np.concatenate([S, sc.init_sphere(kt=1.0, ior=1.5, refExp=50.0)])
    k_mat = 512
    mat_in = np.zeros(k_mat, ab.RAY_DTYPE)
    mat_in["o"] = rng.uniform(-1, 1, (k_mat, 3)).astype(np.float32)
    dm = rng.normal(size=(k_mat, 3)).astype(np.float32)
    mat_in["d"] = dm / np.linalg.norm(dm, axis=1, keepdims=True)
    mat_in["tmin"] = np.float32(1e-4)
    mat_in["tmax"] = rng.uniform(0.5, 5, k_mat).astype(np.float32)
    mat_in["propagation"] = rng.uniform(0.1, 1, (k_mat, 3)).astype(np.float32)
    nrm = rng.normal(size=(k_mat, 3)).astype(np.float32)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    hits = np.concatenate([mat_in["o"] + 0.5, nrm], axis=1).astype(np.float32)
    mat_idx = rng.integers(0, len(mats), k_mat).astype(np.int32)
    mat_seed = rng.integers(2, 2**32 - 1, (k_mat, 2), dtype=np.uint64).astype(np.uint32)
    mat_out = mat_in.copy()
    mat_ret = np.zeros(k_mat, np.int32)
    mat_seed_out = mat_seed.copy()
    for k in range(k_mat):
        r = mat_in[k:k + 1].copy()
        h = hits[k].copy()
        mm = mats[mat_idx[k]:mat_idx[k] + 1].copy()
        s = mat_seed[k].copy()
        mat_ret[k] = L.ref_sample_material(r.ctypes.data, h.ctypes.data, mm.ctypes.data, s.ctypes.data)
        mat_out[k] = r[0]
        mat_seed_out[k] = s
    # sphereEmissiveRadiance
    em_rays = np.zeros(m, ab.RAY_DTYPE)
    em_rays["o"] = rng.uniform(-4, 4, (m, 3)).astype(np.float32)
    em_r12 = rng.uniform(0, 1, (m, 2)).astype(np.float32)
    em_out = em_rays.copy()
    light_c = np.array([2.2, 1.0, 2.0], np.float32)
    for k in range(m):
        r = em_rays[k:k + 1].copy()
        L.ref_sphere_emissive(r.ctypes.data, light_c.ctypes.data, 0.5, float(em_r12[k, 0]), float(em_r12[k, 1]))
        em_out[k] = r[0]
    # cameras
    cams_in = [(512, sc.MAIN_CAMERA), (1024, sc.MAIN_CAMERA), (1920, sc.PLY_CAMERA), (64, sc.PLY_CAMERA),
               (333, dict(target=(1.0, 2.0, -3.0), elevation=-20.0, azimuth=271.5, distance=7.25))]
    cams = np.stack([ref.camera_spherical(w, **c) for w, c in cams_in])
    np.savez_compressed(HERE / "kat.npz", frand_seeds=seeds, frand=frand, tri=tri, tri_rays=rays_t.view(np.uint8),
                        tri_hit=tri_hit, tri_p=tri_p, tri_uvt=tri_uvt, sph_c=sph_c, sph_r=sph_r, sph_d=sph_d,
                        box_rays=rays_b.view(np.uint8), box_t=box_t, box_n=box_n, mats=mats.view(np.uint8),
                        mat_in=mat_in.view(np.uint8), mat_hits=hits, mat_idx=mat_idx, mat_seed=mat_seed,
                        mat_out=mat_out.view(np.uint8), mat_ret=mat_ret, mat_seed_out=mat_seed_out,
                        em_rays=em_rays.view(np.uint8), em_r12=em_r12, em_out=em_out.view(np.uint8),
                        light_c=light_c, cam_widths=np.array([w for w, _ in cams_in], np.uint32), cams=cams)
    meta["cases"]["kat"] = dict(what="per-function known answers from the reference helpers "
                                     "(frand, intersects_triangle[_p], intersectSphere, intersectsBox/boxNormal, "
                                     "sample_material, sphereEmissiveRadiance) and the host camera (gmtl)",
                                cameras=[dict(width=w, **c) for w, c in cams_in])
    (HERE / "meta.json").write_text(json.dumps(meta, indent=1, default=list) + "\n")
    print("wrote", sorted(p.name for p in HERE.glob("*.npz")))


if __name__ == "__main__":
    main()
