"""Pin the oracle's independent BVH mode (oracle/pt_oracle.c `or_bvh_*`) — CPU only.

The BVH mode answers the reference's linear closest-hit and any-hit loops (rtcommon.h:39-52,
:59-68) in O(log N) per ray, so whole frames at the BASELINE sizes can be checked on the GPU
box in seconds (tests/test_gpu_fullframe.py).  It shares nothing with the product's traversal
(no quantised nodes, no determinant or unhittable-triangle culls, no candidate lists).  Here it
is pinned to:
  * the reference's own outputs: the golden triangle frames (every progressive pass and the
    seed planes) and the golden hit queries (tests/golden, recorded from the reference kernel
    compiled for x86-64);
  * the linear loop on adversarial rays: large random triangles with grazing rays aimed at their
    edges and vertices, rays tilted to |det| just above the 1e-4 threshold, exact ties
    (duplicated triangles), triangles around the determinant threshold, finite tmax;
  * the linear loop and the reference kernel itself on strided pixels of the dragon-class frame.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import bits

TRI_CASES = ["tris_64x48_sr1", "tris_40x30_sr2"]


@pytest.mark.parametrize("name", TRI_CASES)
def test_bvh_mode_golden_frames(name, golden, golden_meta, oracle, pt):
    g = golden(name)
    m = golden_meta["cases"][name]
    spheres = g["spheres"].view(pt._abi.SPHERE_DTYPE)
    bvh = oracle.build_bvh(g["verts"], g["idx"])
    out = np.zeros(m["W"] * m["H"] * 4, np.float32)
    seeds = g["seeds_in"].copy()
    for p in range(m["frames"]):
        oracle.render_tris(out, g["camera"], spheres, m["W"], m["H"], m["Wpad"], m["Hpad"], m["sample_rate"],
                           m["max_depth"], p, seeds, g["verts"], g["idx"], bvh=bvh)
        np.testing.assert_array_equal(bits(out), bits(g["frames"][p]), err_msg=f"frame {p}")
    np.testing.assert_array_equal(seeds, g["seeds_out"])


def test_bvh_mode_golden_hits(golden, oracle, pt):
    g = golden("hits_2000")
    R = pt._abi.RAY_DTYPE
    bvh = oracle.build_bvh(g["verts"], g["idx"])
    for key in ("primary", "random"):
        i, t = oracle.closest_hits_bvh(g[f"{key}_rays"].view(R), bvh)
        np.testing.assert_array_equal(i, g[f"{key}_hit"])
        np.testing.assert_array_equal(bits(t), bits(g[f"{key}_t"]))
    occ = oracle.any_hits_bvh(g["shadow_rays"].view(R), bvh)
    np.testing.assert_array_equal(occ, g["shadow_occluded"])


def _grazing_rays(rng, v, idx, n, R):
    """Rays through points on or just beside a triangle's edges and vertices (barycentric offsets
    of +-1e-7 .. 1e-3), tilted out of the triangle's plane so that |det| = |d . (e2 x e1)| lands
    just above or below the 1e-4 threshold, or at random angles."""
    nt = len(idx)
    k = rng.integers(0, nt, n)
    a, b, c = v[idx[k, 0]].astype(np.float64), v[idx[k, 1]].astype(np.float64), v[idx[k, 2]].astype(np.float64)
    e1, e2 = b - a, c - a
    nrm = np.cross(e2, e1)
    nl = np.linalg.norm(nrm, axis=1, keepdims=True)
    nh = nrm / np.maximum(nl, 1e-30)
    # barycentrics on an edge or at a vertex, pushed in or out by a tiny amount
    kind = rng.integers(0, 4, n)
    u = rng.uniform(0, 1, n)
    vv = rng.uniform(0, 1, n) * (1 - u)
    u = np.where(kind == 0, 0.0, u)
    vv = np.where(kind == 1, 0.0, vv)
    s = u + vv
    u = np.where(kind == 2, u / np.maximum(s, 1e-12), u)
    vv = np.where(kind == 2, vv / np.maximum(s, 1e-12), vv)
    u = np.where(kind == 3, rng.integers(0, 2, n).astype(np.float64), u)
    vv = np.where(kind == 3, 0.0, vv)
    eps = rng.choice([-1e-3, -1e-5, -1e-7, 0.0, 1e-7, 1e-5, 1e-3], n)
    p = a + (u + eps)[:, None] * e1 + (vv + rng.choice([-1, 1], n) * eps)[:, None] * e2
    # an in-plane direction plus a normal component giving |det| ~ 1e-4 x (1 +- small), or random
    t1 = e1 / np.maximum(np.linalg.norm(e1, axis=1, keepdims=True), 1e-30)
    t2 = np.cross(nh, t1)
    ang = rng.uniform(0, 2 * np.pi, n)
    inplane = np.cos(ang)[:, None] * t1 + np.sin(ang)[:, None] * t2
    target = 1e-4 * rng.choice([0.999, 1.0, 1.0001, 1.001, 1.01, 2.0], n)
    cz = np.clip(target / np.maximum(nl[:, 0], 1e-30), 0, 1)
    d = inplane * np.sqrt(1 - cz ** 2)[:, None] + (cz * rng.choice([-1, 1], n))[:, None] * nh
    rnd = rng.normal(size=(n, 3))
    rnd /= np.linalg.norm(rnd, axis=1, keepdims=True)
    d = np.where((rng.uniform(size=n) < 0.25)[:, None], rnd, d)
    t0 = rng.uniform(0.2, 8.0, n)
    o = p - d * t0[:, None]
    rr = np.zeros(n, R)
    rr["o"] = o.astype(np.float32)
    d32 = d.astype(np.float32)
    rr["d"] = d32 / np.linalg.norm(d32, axis=1, keepdims=True)
    rr["tmin"] = np.float32(1e-4)
    fin = rng.uniform(size=n) < 0.4
    rr["tmax"] = np.where(fin, (t0 * rng.uniform(0.9, 1.1, n)).astype(np.float32), np.float32(np.inf))
    return rr


def _check_vs_linear(oracle, rays, verts, idx):
    bvh = oracle.build_bvh(verts, idx)
    i_l, t_l = oracle.closest_hits(rays, verts, idx)
    i_b, t_b = oracle.closest_hits_bvh(rays, bvh)
    np.testing.assert_array_equal(i_b, i_l)
    np.testing.assert_array_equal(bits(t_b), bits(t_l))
    o_l = oracle.any_hits(rays, verts, idx)
    o_b = oracle.any_hits_bvh(rays, bvh)
    np.testing.assert_array_equal(o_b, o_l)
    return i_l, o_l


def test_bvh_mode_grazing_large_triangles(oracle, pt):
    """Large random triangles (edges up to ~14), exact duplicates and rotated duplicates (ties:
    the highest index must win), rays grazing their edges at |det| around the threshold."""
    rng = np.random.default_rng(5)
    nt = 2500
    v = rng.uniform(-4, 4, (nt * 3, 3)).astype(np.float32)
    idx = np.arange(nt * 3, dtype=np.int32).reshape(nt, 3)
    v[3:6] = v[0:3]  # duplicate: equal t, higher index wins
    v[9:12] = v[6:9][[1, 2, 0]]  # rotated duplicate: the same plane, other arithmetic
    v[15:18] = v[12:15]
    rays = _grazing_rays(rng, v, idx, 12000, pt._abi.RAY_DTYPE)
    hit, occ = _check_vs_linear(oracle, rays, v, idx)
    assert 0.1 < (hit >= 0).mean() < 0.999 and 0.1 < occ.mean() < 0.999


def test_bvh_mode_small_triangles_near_threshold(oracle, pt):
    """Tiny triangles whose |e2 x e1| straddles the 1e-4 determinant bound (most rays cannot be
    accepted at all, some only near normal incidence) and a dense dragon-like patch."""
    rng = np.random.default_rng(9)
    nt = 4000
    cr = np.exp(rng.uniform(np.log(2e-5), np.log(5e-4), nt))
    a = np.sqrt(cr) * np.exp(rng.uniform(-1.5, 1.5, nt))
    b = cr / a
    nrm = rng.normal(size=(nt, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    t1 = np.cross(nrm, rng.normal(size=(nt, 3)))
    t1 /= np.linalg.norm(t1, axis=1, keepdims=True)
    t2 = np.cross(nrm, t1)
    c0 = rng.uniform(-3, 3, (nt, 3))
    v = np.stack([c0, c0 + a[:, None] * t1, c0 + b[:, None] * t2], 1).reshape(-1, 3).astype(np.float32)
    idx = np.arange(nt * 3, dtype=np.int32).reshape(nt, 3)
    rays = _grazing_rays(rng, v, idx, 12000, pt._abi.RAY_DTYPE)
    # plus rays at normal incidence through the triangles' centroids
    n2 = 4000
    k = rng.integers(0, nt, n2)
    r2 = np.zeros(n2, pt._abi.RAY_DTYPE)
    cen = (v[idx[k, 0]] + v[idx[k, 1]] + v[idx[k, 2]]) / 3
    dd = np.where(rng.uniform(size=(n2, 1)) < 0.5, nrm[k], -nrm[k]).astype(np.float32)
    r2["o"] = (cen - dd * rng.uniform(0.5, 3, (n2, 1))).astype(np.float32)
    r2["d"] = dd / np.linalg.norm(dd, axis=1, keepdims=True)
    r2["tmin"] = np.float32(1e-4)
    r2["tmax"] = np.float32(np.inf)
    hit, _ = _check_vs_linear(oracle, np.concatenate([rays, r2]), v, idx)
    assert (hit >= 0).any()


def test_bvh_mode_dragon_class_rays(oracle, pt):
    """The dragon-class mesh (871,414 triangles): camera rays of the headline view, random box
    rays and shadow rays with finite tmax, BVH mode == the linear loop over every triangle."""
    sc = pt.scenes
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS["dragon"])
    cam = sc.camera_spherical(1920, **sc.PLY_CAMERA)
    rng = np.random.default_rng(3)
    prim = sc.camera_rays(cam, 1920, 1080)
    prim = prim[rng.choice(len(prim), 160, replace=False)]
    n = 160
    rr = np.zeros(n, pt._abi.RAY_DTYPE)
    rr["o"] = rng.uniform([-5.5, -4.9, -5.5], [5.5, 4.9, 5.5], (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    rr["d"] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rr["tmin"] = np.float32(1e-4)
    rr["tmax"] = np.where(rng.uniform(size=n) < 0.5, np.inf, rng.uniform(0, 8, n)).astype(np.float32)
    graze = _grazing_rays(rng, verts, idx.reshape(-1, 3), 160, pt._abi.RAY_DTYPE)
    hit, _ = _check_vs_linear(oracle, np.concatenate([prim, rr, graze]), verts, idx)
    assert (hit >= 0).mean() > 0.3


def test_bvh_mode_dragon_pixels_vs_linear_and_reference(oracle, pt):
    """Strided whole pixels of the dragon-class 1920x1080 frame at sampleRate 2: the BVH mode's
    radiance, seed words and ray counts == the linear oracle's; and == the reference kernel
    itself (oracle/_ref, when built) on the same pixels."""
    from oracle import LIBREF, Reference

    sc = pt.scenes
    W, H, sr = 1920, 1080, 2
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS["dragon"])
    S = sc.ply_scene()
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    seeds = sc.default_seeds(Wp, Hp)
    pix = (np.arange(12, dtype=np.int64) * (W * H // 12) + 104_729 % (W * H // 12)).astype(np.uint32)
    bvh = oracle.build_bvh(verts, idx)
    res = {}
    for who in ("bvh", "linear", "ref"):
        out = np.full(W * H * 4, -1.0, np.float32)
        sd = seeds.copy()
        if who == "ref":
            if not LIBREF.exists():
                continue
            Reference(build_if_missing=False).launch_pixels(2, out, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, pix, verts,
                                                            idx, nthreads=4)
            cnt = None
        else:
            cnt = oracle.render_tris(out, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, verts, idx, pixels=pix,
                                     bvh=bvh if who == "bvh" else None)
        res[who] = (out.reshape(-1, 4)[pix.astype(np.int64)].copy(), sd, cnt)
    np.testing.assert_array_equal(bits(res["bvh"][0]), bits(res["linear"][0]))
    np.testing.assert_array_equal(res["bvh"][1], res["linear"][1])
    assert res["bvh"][2] == res["linear"][2]
    if "ref" in res:
        np.testing.assert_array_equal(bits(res["bvh"][0]), bits(res["ref"][0]))
        np.testing.assert_array_equal(res["bvh"][1], res["ref"][1])
    assert (res["bvh"][0][:, :3] > 0).any()
