"""The padded mesh bounds behind k_tris's off-mesh box paths (rt_host.cpp `mesh_bounds`, DESIGN.md
§4.7) — CPU only.

A short frame answers a box-path query (a bounce off the box, or a shadow ray leaving it) without a
traversal when its segment misses the mesh's bounds padded by 1e-3 of their extent + 1e-4.  That is
exact only if every point the triangle test can accept lies deeper inside the padded box than the
slab test's rounding.  Pinned here against the oracle's independent BVH (itself pinned to the
reference, tests/test_oracle_bvh.py): for box-wall rays and for rays aimed at the mesh's extremal
vertices — the hits nearest the bounds — every ray the oracle finds a triangle for passes the
float32 slab test that the kernel applies, with its clamps to [tmin, tmax].
"""
from __future__ import annotations

import numpy as np

RT_SMALL_F = np.float32(1e-4)


def padded_bounds(verts, idx):
    """rt_host.cpp mesh_bounds: the used vertices' box, grown by 1e-3 of its extent + 1e-4 (float32)."""
    v = verts[np.unique(idx.reshape(-1))]
    lo, hi = v.min(axis=0).astype(np.float32), v.max(axis=0).astype(np.float32)
    pad = np.float32(1e-3) * np.float32((hi - lo).max()) + np.float32(1e-4)
    return lo - pad, hi + pad


def slab_misses(o, d, tmin, tmax, lo, hi):
    """k_tris segment_misses_box in float32 (IEEE reciprocals; the kernel's v_rcp_f32 is within 1 ulp)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = np.float32(1.0) / d
        t1 = (lo[None, :] - o) * inv
        t2 = (hi[None, :] - o) * inv
    # min / max that drop NaN, as v_min_f32 / v_max_f32 (0 x inf on a slab plane)
    mn = np.fmin(t1, t2)
    mx = np.fmax(t1, t2)
    tn = np.fmax(np.fmax(np.fmax(mn[:, 0], mn[:, 1]), mn[:, 2]), tmin)
    tf = np.fmin(np.fmin(np.fmin(mx[:, 0], mx[:, 1]), mx[:, 2]), tmax)
    return tn > tf


def _rays(o, d, tmax, pt):
    r = np.zeros(len(o), pt._abi.RAY_DTYPE)
    r["o"] = o
    r["d"] = d
    r["tmin"] = RT_SMALL_F
    r["tmax"] = tmax
    return r


def _unit(v):
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)


def test_off_mesh_segments_meet_no_triangle(oracle, pt):
    sc = pt.scenes
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS["bunny"])
    lo, hi = padded_bounds(verts, idx)
    bvh = oracle.build_bvh(verts, idx)
    rng = np.random.default_rng(5)
    bw, bh = 6.0, 5.0  # RT_BOX_WIDTH / RT_BOX_HEIGHT (include/rt_types.h)
    n = 40_000
    # box-wall origins (a bounce's hit point) toward random points around the mesh, and toward the
    # light (a shadow ray's segment, tmax = the light's distance)
    face = rng.integers(0, 6, n)
    o = rng.uniform(-1.0, 1.0, (n, 3)) * np.array([bw, bh, bw])
    ax = face // 2
    o[np.arange(n), ax] = np.where(face % 2 == 0, -1.0, 1.0) * np.array([bw, bh, bw])[ax]
    o = o.astype(np.float32)
    target = (lo + (hi - lo) * rng.uniform(-0.3, 1.3, (n, 3))).astype(np.float32)
    d = _unit(target - o)
    inf = np.float32(np.inf)
    # the mesh's extremal vertices (those on its bounds), each aimed at from many box-wall points
    v = verts[np.unique(idx.reshape(-1))]
    ext = np.concatenate([v[np.argsort(v[:, k])[:20]] for k in range(3)] +
                         [v[np.argsort(-v[:, k])[:20]] for k in range(3)])
    m = 6_000
    o2 = o[:m]
    t2 = ext[rng.integers(0, len(ext), m)] + rng.normal(0.0, 1e-3, (m, 3)).astype(np.float32)
    d2 = _unit(t2 - o2)
    light = np.array([0.0, 4.0, 2.0], np.float32)
    o3 = o[m:2 * m]
    d3 = _unit(light[None, :] - o3)
    tl = np.linalg.norm(light[None, :] - o3, axis=1).astype(np.float32)
    O = np.concatenate([o, o2, o3])
    D = np.concatenate([d, d2, d3])
    T = np.concatenate([np.full(n, inf, np.float32), np.full(m, inf, np.float32), tl])
    hit, _ = oracle.closest_hits_bvh(_rays(O, D, T, pt), bvh)
    miss = slab_misses(O, D, RT_SMALL_F, T, lo, hi)
    assert (hit >= 0).sum() > 5_000  # the rays do meet the mesh, many of them at its extremes
    assert miss.sum() > 5_000        # and many segments are answered off-mesh
    bad = np.nonzero((hit >= 0) & miss)[0]
    assert bad.size == 0, f"{bad.size} segments reported off the mesh meet a triangle (first {bad[:5]})"
