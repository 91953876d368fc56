"""GPU parity: the HIP kernels (through the C-ABI) against the reference fixtures and the oracle.

Bar: bit-exact radiance, seeds and hit indices (the arithmetic model is pinned, so the
north-star's 1e-5 relative tolerance is met with zero error).  Run on the
MI355X box with `pytest -m gpu`.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import bits

pytestmark = pytest.mark.gpu

SPHERE_CASES = ["spheres_64x64_sr1", "spheres_48x40_sr2", "spheres_ss_64x64"]
TRI_CASES = ["tris_64x48_sr1", "tris_40x30_sr2"]


def _setup(rt, pt, g, m, kernel_tris=False):
    rt.setSpheres(g["spheres"].view(pt._abi.SPHERE_DTYPE))
    rt.setCamera(g["camera"])
    rt.setSampleRate(m["sample_rate"])
    rt.setMaxPathDepth(m["max_depth"])
    rt.setNDRange(m["nd_y"])
    if kernel_tris:
        rt.setMesh(g["verts"], g["idx"])
    # a fresh size so the seed layout below is the one consumed
    rt.setSeeds(m["Wpad"], m["Hpad"], g["seeds_in"])


@pytest.mark.parametrize("name", SPHERE_CASES)
def test_golden_spheres(name, tracer, pt, golden, golden_meta):
    g, m = golden(name), golden_meta["cases"][name]
    rt = pt.RayTracer(0)
    _setup(rt, pt, g, m)
    out = np.zeros(m["W"] * m["H"] * 4, np.float32)
    for p in range(m["frames"]):
        rt.rayTrace(out, m["W"], m["H"], p, kernel=m["kernel"])
        np.testing.assert_array_equal(bits(out), bits(g["frames"][p]), err_msg=f"{name} frame {p}")
    np.testing.assert_array_equal(rt.getSeeds(), g["seeds_out"])
    rt.close()


TRAVERSALS = ["bvh", "bvh4f", "linear"]


@pytest.mark.parametrize("trav", TRAVERSALS)
@pytest.mark.parametrize("name", TRI_CASES)
def test_golden_tris(name, trav, tracer, pt, golden, golden_meta):
    g, m = golden(name), golden_meta["cases"][name]
    rt = pt.RayTracer(0)
    _setup(rt, pt, g, m, kernel_tris=True)
    rt.setTraversal(trav)
    out = np.zeros(m["W"] * m["H"] * 4, np.float32)
    for p in range(m["frames"]):
        rt.rayTrace(out, m["W"], m["H"], p, kernel=2)
        np.testing.assert_array_equal(bits(out), bits(g["frames"][p]), err_msg=f"{name} frame {p}")
    np.testing.assert_array_equal(rt.getSeeds(), g["seeds_out"])
    rt.close()


@pytest.mark.parametrize("trav", TRAVERSALS)
def test_golden_hit_indices(trav, tracer, pt, golden):
    g = golden("hits_2000")
    R = pt._abi.RAY_DTYPE
    tracer.setMesh(g["verts"], g["idx"])
    tracer.setTraversal(trav)
    for key in ("primary", "random"):
        idx, t = tracer.traceRays(g[f"{key}_rays"].view(R))
        np.testing.assert_array_equal(idx, g[f"{key}_hit"])
        np.testing.assert_array_equal(bits(t), bits(g[f"{key}_t"]))
    occ, _ = tracer.traceRays(g["shadow_rays"].view(R), any_hit=True)
    np.testing.assert_array_equal(occ, g["shadow_occluded"])
    tracer.setTraversal(False)


def test_spheres_vs_oracle_progressive(tracer, pt, oracle):
    sc = pt.scenes
    W, H, sr, frames = 200, 150, 2, 3
    Wp, Hp = sc.padded_dims(W, H)
    S = sc.main_scene()
    cam = sc.camera_spherical(W, **sc.MAIN_CAMERA)
    seeds = sc.default_seeds(Wp, Hp, skip=1234)
    rt = pt.RayTracer(0)
    rt.setSpheres(S)
    rt.setCamera(cam)
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setSeeds(Wp, Hp, seeds)
    got = np.zeros(W * H * 4, np.float32)
    exp = np.zeros_like(got)
    sd = seeds.copy()
    for p in range(frames):
        rt.rayTrace(got, W, H, p, kernel=0)
        c_or = oracle.render_spheres(exp, cam, S, W, H, Wp, Hp, sr, 6, p, sd)
        np.testing.assert_array_equal(bits(got), bits(exp), err_msg=f"frame {p}")
        c = rt.counters()
        assert (c["rays_closest"], c["rays_shadow"]) == c_or
    np.testing.assert_array_equal(rt.getSeeds(), sd)
    rt.close()


def test_sphere_config_full_size_progressive_vs_oracle(tracer, pt, oracle):
    """BASELINE configs[1] at its own size: the built-in sphere scene at 1024x1024, 8
    progressive frames (row-shifted seeds, mix 1/p) from the context's own glibc rand() seeds,
    every frame and the final seed planes equal to the oracle's, bit for bit; ray counts too."""
    sc = pt.scenes
    W = H = 1024
    Wp, Hp = sc.padded_dims(W, H)
    S = sc.main_scene()
    cam = sc.camera_spherical(W, **sc.MAIN_CAMERA)
    rt = pt.RayTracer(0)
    rt.setSpheres(S)
    c = sc.MAIN_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(1)
    rt.setMaxPathDepth(6)
    sd = sc.default_seeds(Wp, Hp)  # the stream a fresh context draws for its first size
    got = np.zeros(W * H * 4, np.float32)
    exp = np.zeros_like(got)
    for p in range(8):
        rt.rayTrace(got, W, H, p, kernel=0)
        c_or = oracle.render_spheres(exp, cam, S, W, H, Wp, Hp, 1, 6, p, sd)
        np.testing.assert_array_equal(bits(got), bits(exp), err_msg=f"frame {p}")
        cnt = rt.counters()
        assert (cnt["rays_closest"], cnt["rays_shadow"]) == c_or
    np.testing.assert_array_equal(rt.getSeeds(), sd)
    rt.close()


def test_bunny_config_full_size_vs_oracle(tracer, pt, oracle):
    """BASELINE configs[2] at its own size: the bunny-class mesh (69,451 triangles) at
    1024x1024, 1 spp, BVH traversal, from the context's own seeds; a strided subset of 2,048
    pixels (the oracle's linear loop) equals the GPU frame on those pixels and their seed slots,
    and the GPU frame's other pixels are filled."""
    sc = pt.scenes
    W = H = 1024
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS["bunny"])
    S = sc.ply_scene()
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    rt = pt.RayTracer(0)
    rt.setSpheres(S)
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(1)
    rt.setMaxPathDepth(6)
    rt.setMesh(verts, idx)
    got = np.zeros(W * H * 4, np.float32)
    rt.rayTrace(got, W, H, 0, kernel=2)
    s_got = rt.getSeeds()
    rt.close()
    sd = sc.default_seeds(Wp, Hp)
    pix = (np.arange(2048, dtype=np.int64) * (W * H // 2048) + 211).astype(np.uint32)
    exp = np.zeros(W * H * 4, np.float32)
    oracle.render_tris(exp, cam, S, W, H, Wp, Hp, 1, 6, 0, sd, verts, idx, pixels=pix)
    g = got.reshape(-1, 4)[pix.astype(np.int64)]
    e = exp.reshape(-1, 4)[pix.astype(np.int64)]
    np.testing.assert_array_equal(bits(g), bits(e))
    sl = pix.astype(np.int64) // W * Wp + pix % W
    plane = Wp * Hp
    np.testing.assert_array_equal(s_got[sl], sd[sl])
    np.testing.assert_array_equal(s_got[plane + sl], sd[plane + sl])
    assert (e[:, :3] > 0).any() and np.isfinite(got).all()


@pytest.mark.parametrize("n_tris", [69_451])
def test_tris_vs_oracle_mesh(n_tris, tracer, pt, oracle):
    """Bunny-class mesh, BVH traversal, against the oracle's linear loop."""
    sc = pt.scenes
    W, H, sr = 48, 36, 1
    Wp, Hp = sc.padded_dims(W, H)
    S = sc.ply_scene()
    verts, idx = sc.make_mesh(n_tris)
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    seeds = sc.default_seeds(Wp, Hp, skip=99)
    rt = pt.RayTracer(0)
    rt.setSpheres(S)
    rt.setCamera(cam)
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(verts, idx)
    rt.setSeeds(Wp, Hp, seeds)
    got = np.zeros(W * H * 4, np.float32)
    exp = np.zeros_like(got)
    sd = seeds.copy()
    rt.rayTrace(got, W, H, 0, kernel=2)
    c_or = oracle.render_tris(exp, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, verts, idx)
    np.testing.assert_array_equal(bits(got), bits(exp))
    c = rt.counters()
    assert (c["rays_closest"], c["rays_shadow"]) == c_or
    np.testing.assert_array_equal(rt.getSeeds(), sd)
    rt.close()


def test_bvh_equals_linear_dragon(tracer, pt):
    """Dragon-class mesh: closest-hit indices/t and any-hit flags, BVH vs the linear loop."""
    sc = pt.scenes
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS["dragon"])
    cam = sc.camera_spherical(320, **sc.PLY_CAMERA)
    rays = sc.camera_rays(cam, 320, 180)
    rng = np.random.default_rng(7)
    n = 16384
    rr = np.zeros(n, pt._abi.RAY_DTYPE)
    rr["o"] = rng.uniform([-5.5, -4.9, -5.5], [5.5, 4.9, 5.5], (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    rr["d"] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rr["tmin"] = np.float32(1e-4)
    rr["tmax"] = np.float32(np.inf)
    rs = rr.copy()
    rs["tmax"] = rng.uniform(0.0, 8.0, n).astype(np.float32)
    rt = tracer
    rt.setMesh(verts, idx)
    res = {}
    for trav in TRAVERSALS:
        rt.setTraversal(trav)
        res[trav] = (rt.traceRays(rays), rt.traceRays(rr), rt.traceRays(rs, any_hit=True))
    rt.setTraversal("bvh")
    for trav in ("bvh", "bvh4f"):
        for k in range(3):
            np.testing.assert_array_equal(res[trav][k][0], res["linear"][k][0])
            np.testing.assert_array_equal(bits(res[trav][k][1]), bits(res["linear"][k][1]))
    assert (res["bvh"][0][0] >= 0).mean() > 0.2  # visible


def test_bvh_equals_linear_fuzz_grazing(tracer, pt):
    """Large triangles and near-grazing rays stress the conservative culling margins."""
    rng = np.random.default_rng(11)
    nt = 3000
    v = rng.uniform(-4, 4, (nt * 3, 3)).astype(np.float32)
    idx = np.arange(nt * 3, dtype=np.int32).reshape(nt, 3)
    # a few exactly coplanar / duplicated triangles to exercise the tie rule
    v[3:6] = v[0:3]
    v[9:12] = v[6:9][[1, 2, 0]]
    n = 32768
    rr = np.zeros(n, pt._abi.RAY_DTYPE)
    tgt = v[rng.integers(0, nt * 3, n)] + rng.normal(scale=0.05, size=(n, 3)).astype(np.float32)
    o = rng.uniform(-6, 6, (n, 3)).astype(np.float32)
    d = tgt - o
    rr["o"] = o
    rr["d"] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rr["tmin"] = np.float32(1e-4)
    rr["tmax"] = np.where(rng.uniform(size=n) < 0.5, np.inf, rng.uniform(0, 10, n)).astype(np.float32)
    rt = tracer
    rt.setMesh(v, idx)
    out = {}
    for trav in TRAVERSALS:
        rt.setTraversal(trav)
        out[trav] = (rt.traceRays(rr), rt.traceRays(rr, any_hit=True))
    rt.setTraversal("bvh")
    for trav in ("bvh", "bvh4f"):
        np.testing.assert_array_equal(out[trav][0][0], out["linear"][0][0])
        np.testing.assert_array_equal(bits(out[trav][0][1]), bits(out["linear"][0][1]))
        np.testing.assert_array_equal(out[trav][1][0], out["linear"][1][0])


def test_unhittable_triangles_left_out_of_the_tree(tracer, pt, oracle):
    """The host build leaves out triangles no unit ray can accept (|det| < 1e-4 always,
    rt_bvh.cpp never_hit).  Triangles straddling that bound, hit at normal incidence and
    at random angles: BVH == linear for closest and any hit; non-unit directions fall back
    to the linear loop; a frame of a mesh whose triangles are mostly culled == oracle."""
    rng = np.random.default_rng(23)
    nt = 4000
    cr = np.exp(rng.uniform(np.log(2e-5), np.log(5e-4), nt))  # |e1 x e2| around the 1e-4 bound
    a = np.sqrt(cr) * np.exp(rng.uniform(-1.5, 1.5, nt))
    b = cr / a
    nrm = rng.normal(size=(nt, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    t1 = np.cross(nrm, rng.normal(size=(nt, 3)))
    t1 /= np.linalg.norm(t1, axis=1, keepdims=True)
    t2 = np.cross(nrm, t1)
    c = rng.uniform(-3, 3, (nt, 3))
    v = np.stack([c, c + a[:, None] * t1, c + b[:, None] * t2], axis=1).reshape(-1, 3).astype(np.float32)
    idx = np.arange(nt * 3, dtype=np.int32).reshape(nt, 3)
    n = 3 * nt
    rr = np.zeros(n, pt._abi.RAY_DTYPE)
    k = np.arange(n) % nt
    inplane = (rng.uniform(0.05, 0.3, (n, 1)) * a[k, None] * t1[k] + rng.uniform(0.05, 0.3, (n, 1)) * b[k, None] * t2[k])
    sgn = np.where(rng.uniform(size=(n, 1)) < 0.5, 1.0, -1.0)
    o = c[k] + inplane + sgn * 2.0 * nrm[k]
    d = -sgn * nrm[k]
    rnd = np.arange(n) >= 2 * nt  # the last third: random directions toward the triangle
    d[rnd] = (c[k[rnd]] + inplane[rnd]) - rng.uniform(-6, 6, (rnd.sum(), 3))
    o[rnd] = c[k[rnd]] + inplane[rnd] - d[rnd]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rr["o"] = o.astype(np.float32)
    rr["d"] = d.astype(np.float32)
    rr["tmin"] = np.float32(1e-4)
    rr["tmax"] = np.float32(np.inf)
    rs = rr.copy()
    rs["tmax"] = np.float32(10.0)
    rt = tracer
    rt.setMesh(v, idx)
    info = rt.meshInfo()
    assert 0 < info["n_tris_tree"] < nt
    out = {}
    for trav in ("linear", "bvh", "bvh4f"):
        rt.setTraversal(trav)
        out[trav] = (rt.traceRays(rr), rt.traceRays(rs, any_hit=True))
    for trav in ("bvh", "bvh4f"):
        np.testing.assert_array_equal(out[trav][0][0], out["linear"][0][0])
        np.testing.assert_array_equal(bits(out[trav][0][1]), bits(out["linear"][0][1]))
        np.testing.assert_array_equal(out[trav][1][0], out["linear"][1][0])
    hits = out["linear"][0][0] >= 0
    assert hits.sum() > 500  # triangles above the bound are hit
    # the hit triangles are all in the tree: |e1 x e2| >= ~1e-4
    assert cr[out["linear"][0][0][hits]].min() > 0.9e-4
    # longer directions can accept culled triangles: those queries take the linear loop
    rl = rr.copy()
    rl["d"] = (d * 50.0).astype(np.float32)
    rt.setTraversal("bvh")
    got = rt.traceRays(rl)
    rt.setTraversal("linear")
    exp = rt.traceRays(rl)
    rt.setTraversal("bvh")
    np.testing.assert_array_equal(got[0], exp[0])
    np.testing.assert_array_equal(bits(got[1]), bits(exp[1]))
    assert (cr[exp[0][exp[0] >= 0]] < 1e-4).any()
    # a frame of a shrunken bunny-class mesh (most triangles culled) == oracle
    sc = pt.scenes
    W, H, sr = 40, 30, 1
    Wp, Hp = sc.padded_dims(W, H)
    S = sc.ply_scene()
    mv, mi = sc.make_mesh(69_451)
    mv = mv.reshape(-1, 3)
    cen = mv.mean(axis=0)
    mv = (cen + (mv - cen) * np.float32(0.15)).astype(np.float32).reshape(-1)
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    seeds = sc.default_seeds(Wp, Hp, skip=5)
    r2 = pt.RayTracer(0)
    r2.setSpheres(S)
    r2.setCamera(cam)
    r2.setSampleRate(sr)
    r2.setMaxPathDepth(6)
    r2.setMesh(mv, mi)
    assert r2.meshInfo()["n_tris_tree"] < 69_451
    r2.setSeeds(Wp, Hp, seeds)
    got = np.zeros(W * H * 4, np.float32)
    exp = np.zeros_like(got)
    sd = seeds.copy()
    r2.rayTrace(got, W, H, 0, kernel=2)
    oracle.render_tris(exp, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, mv, mi)
    np.testing.assert_array_equal(bits(got), bits(exp))
    np.testing.assert_array_equal(r2.getSeeds(), sd)
    r2.close()


@pytest.mark.parametrize("kernel,prog", [(2, 0), (2, 3), (0, 0), (1, 2)])
def test_tiles_assemble_to_full_frame(kernel, prog, tracer, pt, oracle):
    """Row-stripe tiles (the multi-GPU partition) reassemble to the single-device frame,
    which equals the oracle's frame (and seeds) bit for bit."""
    sc = pt.scenes
    from importlib import import_module

    dist = import_module("pathtracer_cl_amd.dist")
    W, H, sr = 72, 53, 1
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(5000)
    seeds = sc.default_seeds(Wp, Hp)
    S = sc.ply_scene()
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    prev = np.random.default_rng(3).uniform(0, 1, (H, W, 4)).astype(np.float32)

    def make():
        rt = pt.RayTracer(0)
        rt.setSpheres(S)
        rt.setCamera(cam)
        rt.setSampleRate(sr)
        rt.setMaxPathDepth(6)
        rt.setMesh(verts, idx)
        rt.setSeeds(Wp, Hp, seeds)
        return rt

    rt = make()
    full = prev.copy().reshape(-1)
    rt.rayTrace(full, W, H, prog, kernel=kernel)
    full_seeds = rt.getSeeds()
    rt.close()
    # the single-device frame the tiles must reassemble to is itself the oracle's
    exp = prev.copy().reshape(-1)
    sd = seeds.copy()
    if kernel == 2:
        oracle.render_tris(exp, cam, S, W, H, Wp, Hp, sr, 6, prog, sd, verts, idx)
    else:
        oracle.render_spheres(exp, cam, S, W, H, Wp, Hp, sr, 6, prog, sd, single_sample=kernel == 1)
    np.testing.assert_array_equal(bits(full), bits(exp))
    np.testing.assert_array_equal(full_seeds, sd)
    for n_ranks, stripe in [(2, 8), (3, 5), (4, 16)]:
        tiles = []
        for r in range(n_ranks):
            rows = dist.tile_rows(H, stripe, n_ranks, r)
            rt = make()
            t = np.ascontiguousarray(prev[rows]).reshape(-1)
            rt.rayTrace(t, W, H, prog, kernel=kernel, tile=(stripe, n_ranks, r))
            s = rt.getSeeds().reshape(2, Hp, Wp)
            np.testing.assert_array_equal(s[:, rows], full_seeds.reshape(2, Hp, Wp)[:, rows])
            rt.close()
            tiles.append(t.reshape(len(rows), W, 4))
        frame = dist.assemble(tiles, H, W, stripe)
        np.testing.assert_array_equal(bits(frame.reshape(-1)), bits(full))


@pytest.mark.parametrize("n_ranks,stripe,H,owned", [(2, 8, 53, False), (3, 4, 45, False), (3, 4, 45, True)])
def test_progressive_sphere_tiles_with_seed_halo(n_ranks, stripe, H, owned, tracer, pt, oracle):
    """raytrace (row-shifted seeds) on row-stripe tiles over progressive frames, with the
    seed-row halo moved between contexts through device buffers (rt_pack/unpack_seed_rows,
    the path dist.exchange_seed_rows drives over RCCL): every frame reassembles bit-exactly
    to the single-device frame (itself equal to the oracle's frames and seeds), and every
    seed row equals the single-device seeds on its last writer.  Includes a restart
    (progression back to 0) and, with `owned`, owner-map partitions that change between frames
    (rt_tile.stripe_owner; the halo moves the rows of the stripes that changed owner too)."""
    import torch
    from importlib import import_module

    dist = import_module("pathtracer_cl_amd.dist")
    sc = pt.scenes
    W, sr = 72, 1
    Wp, Hp = sc.padded_dims(W, H)
    seeds = sc.default_seeds(Wp, Hp)
    cam = sc.camera_spherical(W, **sc.MAIN_CAMERA)

    def make():
        rt = pt.RayTracer(0)
        rt.setSpheres(sc.main_scene())
        rt.setCamera(cam)
        rt.setSampleRate(sr)
        rt.setMaxPathDepth(6)
        rt.setSeeds(Wp, Hp, seeds)
        return rt

    ref = make()
    ranks = [make() for _ in range(n_ranks)]
    halo = dist.SeedHalo(H, Hp, stripe, n_ranks)
    full = np.zeros(W * H * 4, np.float32)
    ns = (H + stripe - 1) // stripe
    maps = [None, dist.lpt_owner(np.arange(ns)[::-1] + 1, n_ranks), np.array([(3 * s_) % n_ranks for s_ in range(ns)])]
    owner = None
    rows = [dist.tile_rows(H, stripe, n_ranks, r) for r in range(n_ranks)]
    tiles = [torch.zeros(H * W * 4, dtype=torch.float32, device="cuda:0") for r in range(n_ranks)]
    moved = 0
    exp = np.zeros_like(full)
    sd = seeds.copy()
    try:
        for f, p in enumerate([0, 1, 2, 3, 4, 0, 1, 2]):
            if owned:  # the partition changes between frames; a tile keeps what it holds for progression
                new_owner = maps[f % 3]
                if f > 0 and p > 0:  # progression mixes into the tile's previous pixels: carry them over
                    prev = dist.assemble([t.cpu().numpy().reshape(-1, W, 4) for t in tiles], H, W, stripe, owner)
                    for r in range(n_ranks):
                        rr = dist.tile_rows(H, stripe, n_ranks, r, new_owner)
                        tiles[r][: len(rr) * W * 4] = torch.from_numpy(np.ascontiguousarray(prev[rr]).reshape(-1)).cuda()
                owner = new_owner
                halo.set_owner(owner)
            ref.rayTrace(full, W, H, p, kernel=0)
            # raytrace's row-shifted seeds (raytracer.cl:20-30) over the same progression
            oracle.render_spheres(exp, cam, sc.main_scene(), W, H, Wp, Hp, sr, 6, p, sd)
            np.testing.assert_array_equal(bits(full), bits(exp), err_msg=f"oracle, progression {p}")
            for (src, dst), rws in halo.plan(p).items():
                buf = torch.empty((2, len(rws), Wp), dtype=torch.int32, device="cuda:0")
                ranks[src].packSeedRows(rws, buf)
                ranks[dst].unpackSeedRows(rws, buf)
                moved += len(rws)
            for r in range(n_ranks):
                ranks[r].rayTrace(tiles[r], W, H, p, kernel=0, tile=(stripe, n_ranks, r, owner), halo=True)
            halo.commit(p)
            frame = dist.assemble([t.cpu().numpy().reshape(-1, W, 4) for t in tiles], H, W, stripe, owner)
            np.testing.assert_array_equal(bits(frame.reshape(-1)), bits(full), err_msg=f"progression {p}")
        ref_seeds = ref.getSeeds().reshape(2, Hp, Wp)
        np.testing.assert_array_equal(ref_seeds.reshape(-1), sd)
        got = [rk.getSeeds().reshape(2, Hp, Wp) for rk in ranks]
        for row in range(Hp):
            w = halo.writer[row]
            if w >= 0:
                np.testing.assert_array_equal(got[w][:, row], ref_seeds[:, row])
        assert moved > 0
        # without the halo flag a progressive sphere tile is refused
        with pytest.raises(pt.RtError):
            ranks[0].rayTrace(tiles[0], W, H, 1, kernel=0, tile=(stripe, n_ranks, 0))
    finally:
        ref.close()
        for rk in ranks:
            rk.close()


def test_owner_map_tiles_assemble_to_full_frame(tracer, pt, oracle):
    """Tiles under an owner-map partition (rt_tile.stripe_owner): the cost-balanced map of
    rt_partition_stripes (cached per view: a second call returns it without a probe) and a
    hand-made one with a rank that owns nothing.  Every rank's tile, on its own context and on one
    context that switches partitions (the stripe map and the schedule are re-keyed), reassembles
    bit-exactly — on the host and with rt_assemble_tiles — to the full frame, itself the oracle's,
    with every rank's seed rows equal to the full frame's."""
    import torch
    from importlib import import_module

    dist = import_module("pathtracer_cl_amd.dist")
    sc = pt.scenes
    W, H, stripe, sr = 72, 53, 8, 2
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(5000)
    seeds = sc.default_seeds(Wp, Hp)
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    S = sc.ply_scene()

    def make():
        rt = pt.RayTracer(0)
        rt.setSpheres(S)
        rt.setCamera(cam)
        rt.setSampleRate(sr)
        rt.setMaxPathDepth(6)
        rt.setMesh(verts, idx)
        rt.setSeeds(Wp, Hp, seeds)
        return rt

    rt = make()
    full = np.zeros(W * H * 4, np.float32)
    rt.rayTrace(full, W, H, 0, kernel=2)
    full_seeds = rt.getSeeds().reshape(2, Hp, Wp)
    exp = np.zeros_like(full)
    oracle.render_tris(exp, cam, S, W, H, Wp, Hp, sr, 6, 0, seeds.copy(), verts, idx)
    np.testing.assert_array_equal(bits(full), bits(exp))
    n = 3
    balanced = rt.partitionStripes(W, H, stripe, n)
    np.testing.assert_array_equal(rt.partitionStripes(W, H, stripe, n), balanced)
    assert balanced.shape == (7,) and balanced.max() < n
    rt.close()
    switching = make()
    for owner in (balanced, np.array([1, 1, 0, 1, 0, 0, 1], np.uint32), None):
        tiles = []
        for r in range(n):
            rows = dist.tile_rows(H, stripe, n, r, owner)
            for rk, fresh in ((make(), True), (switching, False)):
                rk.setSeeds(Wp, Hp, seeds)
                t = torch.zeros(max(len(rows), 1) * W * 4, dtype=torch.float32, device="cuda:0")
                rk.rayTrace(t, W, H, 0, kernel=2, tile=(stripe, n, r, owner))
                s_ = rk.getSeeds().reshape(2, Hp, Wp)
                np.testing.assert_array_equal(s_[:, rows], full_seeds[:, rows])
                got = t.cpu().numpy()[: len(rows) * W * 4]
                np.testing.assert_array_equal(bits(got), bits(full.reshape(H, W, 4)[rows].reshape(-1)),
                                              err_msg=f"owner {owner}, rank {r}, fresh {fresh}")
                if fresh:
                    rk.close()
                    tiles.append(t)
        frame = dist.assemble([t.cpu().numpy().reshape(-1, W, 4) for t in tiles], H, W, stripe, owner)
        np.testing.assert_array_equal(bits(frame.reshape(-1)), bits(full))
        dev_frame = torch.full((W * H * 4,), -1.0, dtype=torch.float32, device="cuda:0")
        dist.assemble_native(tiles, H, W, stripe, dev_frame, owner=owner)
        np.testing.assert_array_equal(bits(dev_frame.cpu().numpy()), bits(full))
    switching.close()


def test_native_comm_assembly_and_single_rank_render(tracer, pt):
    """The native host's sharding path (csrc/rt_comm.hip).  rt_assemble_tiles (the root's
    device-side scatter) rebuilds the full frame from 3 ranks' compact tiles; a 1-rank RCCL
    communicator's rt_comm_render equals rt_render over progressive frames of raytrace_tris
    and raytrace (halo bookkeeping on), and rt_comm_gather_frame moves the tile unchanged.
    (RCCL refuses two ranks on one GPU: the multi-rank exchange runs on the 8-GPU node.)"""
    import torch
    from importlib import import_module

    dist = import_module("pathtracer_cl_amd.dist")
    sc = pt.scenes
    W, H, stripe = 72, 53, 8
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(5000)
    seeds = sc.default_seeds(Wp, Hp)

    def make(kernel):
        rt = pt.RayTracer(0)
        rt.setSpheres(sc.ply_scene() if kernel == 2 else sc.main_scene())
        rt.setCamera(sc.camera_spherical(W, **(sc.PLY_CAMERA if kernel == 2 else sc.MAIN_CAMERA)))
        rt.setSampleRate(1)
        rt.setMaxPathDepth(6)
        if kernel == 2:
            rt.setMesh(verts, idx)
        rt.setSeeds(Wp, Hp, seeds)
        return rt

    dev = "cuda:0"
    rt = make(2)
    full = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
    rt.rayTrace(full, W, H, 0, kernel=2)
    rt.close()
    n = 3
    tiles = []
    for r in range(n):
        rows = dist.tile_rows(H, stripe, n, r)
        t = torch.zeros(len(rows) * W * 4, dtype=torch.float32, device=dev)
        rk = make(2)
        rk.rayTrace(t, W, H, 0, kernel=2, tile=(stripe, n, r))
        rk.close()
        tiles.append(t)
    frame = torch.full((W * H * 4,), -1.0, dtype=torch.float32, device=dev)
    dist.assemble_native(tiles, H, W, stripe, frame)
    torch.testing.assert_close(frame, full, rtol=0, atol=0)

    comm = dist.NativeComm(1, 0, 0, dist.NativeComm.unique_id())
    try:
        for kernel in (2, 0):
            ref, rk = make(kernel), make(kernel)
            exp = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
            got = torch.zeros_like(exp)
            for p in [0, 1, 2, 0, 1]:
                ref.rayTrace(exp, W, H, p, kernel=kernel)
                comm.render(rk, got, W, H, p, kernel, stripe=stripe)
                assert torch.equal(got.view(torch.int32), exp.view(torch.int32)), (kernel, p)
            np.testing.assert_array_equal(rk.getSeeds(), ref.getSeeds())
            ref.close()
            rk.close()
            comm.reset_halo()
        moved = torch.zeros_like(full)
        comm.gather(full, moved, W, H, stripe)
        assert torch.equal(moved, full)
    finally:
        comm.close()


def test_device_framebuffer_matches_host(tracer, pt):
    import torch

    sc = pt.scenes
    W, H = 96, 64
    Wp, Hp = sc.padded_dims(W, H)
    seeds = sc.default_seeds(Wp, Hp)
    rt = tracer
    rt.setSpheres(sc.ply_scene())
    rt.setCamera(sc.camera_spherical(W, **sc.PLY_CAMERA))
    rt.setSampleRate(2)
    rt.setMaxPathDepth(6)
    rt.setMesh(*sc.make_mesh(20000))
    host = np.zeros(W * H * 4, np.float32)
    dev = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    for out in (host, dev):
        rt.setSeeds(Wp, Hp, seeds)
        for p in range(2):
            rt.rayTrace(out, W, H, p, kernel=2)
    np.testing.assert_array_equal(bits(host), bits(dev.cpu().numpy()))
    # rt_read: the blocking readback of the last (device) frame
    back = np.full(W * H * 4, -1.0, np.float32)
    rt.read(back)
    np.testing.assert_array_equal(bits(host), bits(back))
    with pytest.raises(pt.RtError):
        rt.read(np.zeros(16, np.float32))


def test_dragon_full_size_properties(tracer, pt, oracle):
    """BASELINE config 4 at full size (1920x1080, 871k tris), sampleRate 1 for the oracle
    subset: a strided pixel subset is bit-exact against the oracle's linear loop; the frame
    is finite, alpha 0, deterministic, and every pixel's seed advanced."""
    sc = pt.scenes
    W, H, sr = 1920, 1080, 1
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS["dragon"])
    S = sc.ply_scene()
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    seeds = sc.default_seeds(Wp, Hp)
    rt = tracer
    rt.setSpheres(S)
    rt.setCamera(cam)
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(verts, idx)
    out = np.zeros(W * H * 4, np.float32)
    rt.setSeeds(Wp, Hp, seeds)
    rt.rayTrace(out, W, H, 0, kernel=2)
    s_gpu = rt.getSeeds()
    out2 = np.zeros_like(out)
    rt.setSeeds(Wp, Hp, seeds)
    rt.rayTrace(out2, W, H, 0, kernel=2)
    np.testing.assert_array_equal(bits(out), bits(out2))
    img = out.reshape(H, W, 4)
    assert np.isfinite(img).all() and (img[..., 3] == 0).all() and img[..., :3].max() > 0
    changed = (s_gpu.reshape(2, Hp, Wp)[:, :H, :W] != seeds.reshape(2, Hp, Wp)[:, :H, :W]).any(0)
    assert changed.all()
    pix = np.arange(0, W * H, 32_407, dtype=np.uint32)  # 64 pixels spread over the frame
    exp = np.zeros_like(out)
    sd = seeds.copy()
    oracle.render_tris(exp, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, verts, idx, pixels=pix)
    e = exp.reshape(-1, 4)[pix]
    gpx = out.reshape(-1, 4)[pix]
    np.testing.assert_array_equal(bits(gpx), bits(e))


def _pixel_seeds(seeds, pix, Wp, Hp, W):
    """The two seed-plane words of each pixel's slot (raytrace_tris: y * Wpad + x)."""
    s = seeds.reshape(2, Hp * Wp)
    slot = (pix // W) * Wp + pix % W
    return s[:, slot]


def test_dragon_headline_config_vs_oracle(tracer, pt, oracle):
    """The benchmark's own configuration (BASELINE config 4: 871k tris, 1920x1080,
    sampleRate 16 = 256 samples per pixel with strat_rand total = 16, maxDepth 6,
    raytracer.cl:184-243): a strided subset of 64 pixels (mesh, silhouette and box pixels) and
    their seed slots are bit-exact against the oracle's linear loop (16 oracle threads: about a
    minute on the GPU box)."""
    sc = pt.scenes
    W, H, sr = 1920, 1080, 16
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS["dragon"])
    S = sc.ply_scene()
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    seeds = sc.default_seeds(Wp, Hp)
    rt = tracer
    rt.setSpheres(S)
    rt.setCamera(cam)
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(verts, idx)
    rt.setSeeds(Wp, Hp, seeds)
    out = np.zeros(W * H * 4, np.float32)
    rt.rayTrace(out, W, H, 0, kernel=2)
    s_gpu = rt.getSeeds()
    pix = np.arange(4_321, W * H, 32_399, dtype=np.uint32)  # 64 pixels over the frame
    exp = np.zeros_like(out)
    sd = seeds.copy()
    oracle.render_tris(exp, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, verts, idx, pixels=pix)
    np.testing.assert_array_equal(bits(out.reshape(-1, 4)[pix]), bits(exp.reshape(-1, 4)[pix]))
    np.testing.assert_array_equal(_pixel_seeds(s_gpu, pix, Wp, Hp, W), _pixel_seeds(sd, pix, Wp, Hp, W))
    assert out.reshape(-1, 4)[pix, :3].max() > 0


@pytest.fixture(scope="module")
def lucy_mesh(pt):
    """BASELINE config 5's mesh (Lucy class, 28,055,742 triangles), made once per module."""
    return pt.scenes.make_mesh(pt.scenes.MESH_CONFIGS["lucy"])


@pytest.fixture(scope="module")
def lucy_culled(pt, tracer, lucy_mesh):
    """A context with the Lucy-class mesh on the default (host SAH) builder's tree."""
    verts, idx = lucy_mesh
    rt = pt.RayTracer(0)
    rt.setSpheres(pt.scenes.ply_scene())
    rt.setMaxPathDepth(6)
    rt.setBuilder("host")
    rt.setMesh(verts, idx)
    yield rt
    rt.close()


def test_lucy_class_28m_tris(tracer, pt, oracle, lucy_mesh, lucy_culled):
    """BASELINE config 5's mesh (Lucy class, 28,055,742 triangles) at reduced resolution.
    Under the reference's absolute |det| < 1e-4 rule (geometryFuncs.h:167) no unit ray can
    accept any of its triangles, so the host build's tree holds almost none of them
    (DESIGN §6); the GPU LBVH keeps all 28M.  Both trees render the same bits (16 spp);
    a pixel subset equals the oracle's linear loop over all 28M triangles; and on the full
    28M tree, rays long enough to pass the det rule hit real triangles with BVH == linear."""
    sc = pt.scenes
    verts, idx = lucy_mesh
    n = sc.MESH_CONFIGS["lucy"]
    S = sc.ply_scene()
    W, H = 192, 144
    Wp, Hp = sc.padded_dims(W, H)
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    seeds = sc.default_seeds(Wp, Hp, skip=11)

    culled = lucy_culled
    full = pt.RayTracer(0)
    full.setSpheres(S)
    full.setMaxPathDepth(6)
    full.setBuilder("gpu")
    full.setMesh(verts, idx)
    try:
        assert culled.meshInfo()["n_tris_tree"] < 16
        assert full.meshInfo()["n_tris_tree"] == n
        frames = []
        for rt in (culled, full):
            rt.setCamera(cam)
            rt.setSampleRate(4)
            rt.setSeeds(Wp, Hp, seeds)
            f = np.zeros(W * H * 4, np.float32)
            rt.rayTrace(f, W, H, 0, kernel=2)
            frames.append((f, rt.getSeeds()))
        np.testing.assert_array_equal(bits(frames[0][0]), bits(frames[1][0]))
        np.testing.assert_array_equal(frames[0][1], frames[1][1])
        # oracle subset at sampleRate 1 (the oracle walks all 28M triangles per ray)
        culled.setSampleRate(1)
        culled.setSeeds(Wp, Hp, seeds)
        got = np.zeros(W * H * 4, np.float32)
        culled.rayTrace(got, W, H, 0, kernel=2)
        pix = np.arange(97, W * H, W * H // 16, dtype=np.uint32)
        exp = np.zeros_like(got)
        sd = seeds.copy()
        oracle.render_tris(exp, cam, S, W, H, Wp, Hp, 1, 6, 0, sd, verts, idx, pixels=pix)
        np.testing.assert_array_equal(bits(got.reshape(-1, 4)[pix]), bits(exp.reshape(-1, 4)[pix]))
        np.testing.assert_array_equal(_pixel_seeds(culled.getSeeds(), pix, Wp, Hp, W),
                                      _pixel_seeds(sd, pix, Wp, Hp, W))
        # closest hits on the full 28M-triangle tree: directions 100x unit length
        rng = np.random.default_rng(5)
        m = 2048
        v = verts.reshape(-1, 3)
        tri = rng.integers(0, n, m)
        tgt = v[idx[tri]].mean(axis=1)
        o = tgt + rng.normal(size=(m, 3)) * 3.0
        d = tgt - o
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        rr = np.zeros(m, pt._abi.RAY_DTYPE)
        rr["o"] = o.astype(np.float32)
        rr["d"] = (d * 100.0).astype(np.float32)
        rr["tmin"] = np.float32(1e-6)
        rr["tmax"] = np.float32(np.inf)
        full.setTraversal("bvh")
        got_h = full.traceRays(rr)
        full.setTraversal("linear")
        exp_h = full.traceRays(rr)
        np.testing.assert_array_equal(got_h[0], exp_h[0])
        np.testing.assert_array_equal(bits(got_h[1]), bits(exp_h[1]))
        assert (exp_h[0] >= 0).sum() > m // 2
        # and the oracle agrees on a sample of them
        oh = oracle.closest_hits(rr[:64], verts, idx)
        np.testing.assert_array_equal(oh[0], exp_h[0][:64])
        np.testing.assert_array_equal(bits(oh[1]), bits(exp_h[1][:64]))
    finally:
        full.close()


def test_lucy_config5_at_size_eight_tiles(tracer, pt, oracle, lucy_mesh, lucy_culled):
    """BASELINE config 5 at its own size: the Lucy-class mesh (28,055,742 triangles), 4096x4096,
    sampleRate 4, as the 8 row-stripe tiles of an 8-GPU run (stripe 8; RayTracerCL.cpp:217-307 over
    raytracer.cl:184-243, sharded).  The whole frame is finite, alpha 0 and advances every seed;
    the 8 tiles, each rendered from the same seeds into a device tile and scattered by the root's
    device assembly (rt_assemble_tiles, the last step of rt_comm_gather_frame), equal the whole
    frame bit for bit, and so do the seed planes after them; a strided pixel subset rendered at
    sampleRate 1 equals the oracle's linear loop over all 28M triangles, frames and seeds."""
    import torch
    from importlib import import_module

    dist = import_module("pathtracer_cl_amd.dist")
    sc = pt.scenes
    verts, idx = lucy_mesh
    S = sc.ply_scene()
    W = H = 4096
    n_ranks, stripe = 8, 8
    Wp, Hp = sc.padded_dims(W, H)
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    seeds = sc.default_seeds(Wp, Hp, skip=13)
    rt = lucy_culled
    rt.setCamera(cam)
    rt.setSampleRate(4)
    rt.setSeeds(Wp, Hp, seeds)
    dev = torch.device("cuda", 0)
    whole = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
    rt.rayTrace(whole, W, H, 0, kernel=2)
    s_whole = rt.getSeeds()
    img = whole.cpu().numpy()
    f = img.reshape(H, W, 4)
    assert np.isfinite(f).all() and (f[..., 3] == 0).all() and f[..., :3].max() > 0
    changed = (s_whole.reshape(2, Hp, Wp)[:, :H, :W] != seeds.reshape(2, Hp, Wp)[:, :H, :W]).any(0)
    assert changed.all()
    del f
    # the 8 ranks' tiles on one GPU: tiles own disjoint rows and read / write only their own seed
    # slots (raytrace_tris: unshifted y * Wpad + x), so rendering them in turn from the same
    # starting planes is what 8 GPUs with replicated seeds do
    rt.setSeeds(Wp, Hp, seeds)
    rows_max = dist.max_tile_rows(H, stripe, n_ranks)
    tiles = []
    for r in range(n_ranks):
        t = torch.zeros(rows_max * W * 4, dtype=torch.float32, device=dev)
        rt.rayTrace(t, W, H, 0, kernel=2, tile=(stripe, n_ranks, r))
        tiles.append(t)
    s_tiles = rt.getSeeds()
    frame = torch.full((W * H * 4,), -1.0, dtype=torch.float32, device=dev)
    dist.assemble_native(tiles, H, W, stripe, frame, device=0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(bits(frame.cpu().numpy()), bits(img))
    np.testing.assert_array_equal(s_tiles, s_whole)
    del tiles, frame, whole, img
    # oracle subset at sampleRate 1 (the oracle walks all 28M triangles per ray)
    rt.setSampleRate(1)
    rt.setSeeds(Wp, Hp, seeds)
    got = np.zeros(W * H * 4, np.float32)
    rt.rayTrace(got, W, H, 0, kernel=2, tile=None)
    pix = np.arange(1_234, W * H, W * H // 24, dtype=np.uint32)
    exp = np.zeros_like(got)
    sd = seeds.copy()
    oracle.render_tris(exp, cam, S, W, H, Wp, Hp, 1, 6, 0, sd, verts, idx, pixels=pix)
    np.testing.assert_array_equal(bits(got.reshape(-1, 4)[pix]), bits(exp.reshape(-1, 4)[pix]))
    np.testing.assert_array_equal(_pixel_seeds(rt.getSeeds(), pix, Wp, Hp, W), _pixel_seeds(sd, pix, Wp, Hp, W))


@pytest.mark.parametrize("kernel", [0, 2])
def test_blurred_refraction_lobe_vs_oracle(kernel, tracer, pt, oracle):
    """sampleRefraction's blurred lobe (materials.h:183-199, taken when refExp < 1e5): the
    plymain glass sphere with refExp 40 and a Phong lobe on the mirror, over 3 progressive
    frames of raytrace and raytrace_tris, bit-exact against the oracle."""
    sc = pt.scenes
    S = sc.ply_scene().copy()
    S["refExp"][1] = 40.0  # the glass sphere (kt 0.8)
    S["specExp"][2] = 60.0
    assert S["kt"][1] > 0
    W, H, sr = 48, 40, 2
    Wp, Hp = sc.padded_dims(W, H)
    cam = sc.camera_spherical(W, **sc.MAIN_CAMERA)
    seeds = sc.default_seeds(Wp, Hp, skip=3)
    verts, idx = sc.make_mesh(3000)
    rt = pt.RayTracer(0)
    rt.setSpheres(S)
    rt.setCamera(cam)
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    if kernel == 2:
        rt.setMesh(verts, idx)
    rt.setSeeds(Wp, Hp, seeds)
    got = np.zeros(W * H * 4, np.float32)
    exp = np.zeros_like(got)
    sd = seeds.copy()
    for p in range(3):
        rt.rayTrace(got, W, H, p, kernel=kernel)
        if kernel == 2:
            oracle.render_tris(exp, cam, S, W, H, Wp, Hp, sr, 6, p, sd, verts, idx)
        else:
            oracle.render_spheres(exp, cam, S, W, H, Wp, Hp, sr, 6, p, sd)
        np.testing.assert_array_equal(bits(got), bits(exp), err_msg=f"progression {p}")
    np.testing.assert_array_equal(rt.getSeeds(), sd)
    rt.close()


def test_errors_are_loud(tracer, pt):
    rt = pt.RayTracer(0)
    out = np.zeros(16 * 16 * 4, np.float32)
    with pytest.raises(pt.RtError):
        rt.rayTrace(out, 16, 16, 0, kernel=0)  # no spheres
    rt.setSpheres(pt.scenes.main_scene())
    with pytest.raises(pt.RtError):
        rt.rayTrace(out, 16, 16, 0, kernel=2)  # no mesh
    with pytest.raises(pt.RtError):
        rt.rayTrace(out, 16, 16, 1, kernel=0, tile=(4, 2, 0))  # shifted seeds cross stripes
    with pytest.raises(pt.RtError):
        rt.setMesh(np.array([[0, 0, 0], [1, 0, 0], [np.nan, 1, 0]], np.float32), np.array([[0, 1, 2]], np.int32))
    with pytest.raises(pt.RtError):
        rt.setMesh(np.zeros((3, 3), np.float32), np.array([[0, 1, 3]], np.int32))
    for retired in (2, 3):  # the binary-tree and packet traversals were removed
        assert rt._lib.rt_set_traversal(rt._h, retired) == pt._abi.RT_ERR_ARG
    rt.close()


@pytest.mark.parametrize("args,name", [(["--scene", "main", "--width", "64", "--height", "64", "--frames", "4"],
                                        "spheres_64x64_sr1"),
                                       (["--mesh", "2000", "--width", "64", "--height", "48", "--frames", "3"],
                                        "tris_64x48_sr1")])
def test_cpp_host_replays_reference_app(args, name, tracer, golden, tmp_path):
    """The C++ host class (RayTracerHIP.hpp) driven like main.cpp / plymain.cpp + GlutCLWindow's
    progression loop reproduces the reference kernel's frames from the default glibc seeds."""
    import subprocess

    from conftest import ROOT

    raw = tmp_path / "out.f32"
    subprocess.run([str(ROOT / "pathtracer.cl_amd" / "rt_render"), *args, "--raw", str(raw)], check=True,
                   timeout=120)
    got = np.fromfile(raw, np.float32)
    exp = golden(name)["frames"][-1]
    np.testing.assert_array_equal(bits(got), bits(exp))


def test_cpp_host_shards(tracer, golden, tmp_path):
    """The C++ host's sharding paths (rt_render_cli.cpp): two separate processes each render
    one rank's row stripes (`--tile 8,2,r`), and the compact tiles reassemble to the reference
    kernel's frame; a native RCCL communicator (`--comm-ranks 1`: rt_comm_create,
    rt_comm_render, gather to rank 0) writes the same frame.  (RCCL refuses two ranks on one
    GPU; the multi-rank exchange runs on the 8-GPU node.)"""
    import subprocess
    from importlib import import_module

    from conftest import ROOT

    dist = import_module("pathtracer_cl_amd.dist")
    cli = str(ROOT / "pathtracer.cl_amd" / "rt_render")
    base = ["--mesh", "2000", "--width", "64", "--height", "48", "--frames", "3"]
    W, H = 64, 48
    exp = golden("tris_64x48_sr1")["frames"][-1]
    procs, tiles = [], []
    for r in range(2):
        raw = tmp_path / f"tile{r}.f32"
        procs.append(subprocess.Popen([cli, *base, "--tile", f"8,2,{r}", "--raw", str(raw)]))
        tiles.append(raw)
    for p in procs:
        assert p.wait(timeout=120) == 0
    parts = [np.fromfile(t, np.float32).reshape(-1, W, 4) for t in tiles]
    frame = dist.assemble(parts, H, W, 8)
    np.testing.assert_array_equal(bits(frame.reshape(-1)), bits(exp))
    raw = tmp_path / "comm.f32"
    subprocess.run([cli, *base, "--comm-ranks", "1", "--comm-rank", "0", "--comm-id", str(tmp_path / "id"),
                    "--raw", str(raw)], check=True, timeout=120)
    np.testing.assert_array_equal(bits(np.fromfile(raw, np.float32)), bits(exp))


def test_ply_mesh_cli_and_oracle(tracer, pt, oracle, tmp_path):
    """A PLY file (binary LE, Stanford-scan layout) through both hosts: the C++ CLI (--ply,
    plymain.cpp's scene with the mesh actually handed to the tracer) and the Python RayTracer
    agree bit for bit, and both equal the CPU oracle on the same normalised mesh."""
    import subprocess
    import struct

    from conftest import ROOT

    sc = pt.scenes
    verts, idx = sc.make_mesh(2000)
    e = "<"
    head = ("ply\nformat binary_little_endian 1.0\n"
            f"element vertex {len(verts)}\nproperty float x\nproperty float y\nproperty float z\n"
            "property float confidence\nproperty float intensity\n"
            f"element face {len(idx)}\nproperty list uchar int vertex_indices\nend_header\n").encode()
    body = b"".join(struct.pack(e + "fffff", *map(float, v), 1.0, 0.5) for v in verts)
    body += b"".join(struct.pack(e + "Biii", 3, *map(int, t)) for t in idx)
    ply = tmp_path / "mesh.ply"
    ply.write_bytes(head + body)
    W, H = 64, 48
    raw = tmp_path / "out.f32"
    subprocess.run([str(ROOT / "pathtracer.cl_amd" / "rt_render"), "--ply", str(ply), "--width", str(W),
                    "--height", str(H), "--frames", "1", "--raw", str(raw)], check=True, timeout=120)
    got_cli = np.fromfile(raw, np.float32)

    v, i = sc.load_ply(ply)
    Wp, Hp = sc.padded_dims(W, H)
    seeds = sc.default_seeds(Wp, Hp)
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    rt = tracer
    rt.setSpheres(sc.ply_scene())
    rt.setCamera(cam)
    rt.setSampleRate(1)
    rt.setMaxPathDepth(6)
    rt.setMesh(v, i)
    rt.setSeeds(Wp, Hp, seeds)
    got_py = np.zeros(W * H * 4, np.float32)
    rt.rayTrace(got_py, W, H, 0, kernel=2)
    exp = np.zeros(W * H * 4, np.float32)
    oracle.render_tris(exp, cam, sc.ply_scene(), W, H, Wp, Hp, 1, 6, 0, seeds, v, i)
    np.testing.assert_array_equal(bits(got_py), bits(exp))
    np.testing.assert_array_equal(bits(got_cli), bits(exp))


@pytest.mark.parametrize("n_tris,sr", [(2000, 1), (20_000, 2)])
def test_pixel_candidate_lists_vs_oracle(pt, oracle, monkeypatch, n_tris, sr):
    """Camera rays answered from the per-pixel candidate lists (k_pixel_lists: sorted, the
    early end on the next candidate's earliest accept t, blocks popped in list order) equal
    the oracle's linear loop bit for bit, lists forced on (RT_PIXEL_LISTS=1) at sample rates
    the automatic rule leaves them off for, and off; meshes whose pixels hold 1-32 candidates
    (the 2,000-triangle mesh: large triangles, many lists over 8)."""
    sc = pt.scenes
    W, H = 64, 48
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(n_tris)
    seeds = sc.default_seeds(Wp, Hp, skip=3)
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    exp = np.zeros(W * H * 4, np.float32)
    oracle.render_tris(exp, cam, sc.ply_scene(), W, H, Wp, Hp, sr, 6, 0, seeds.copy(), verts, idx)  # advances its seeds
    for mode, builder in (("1", "host"), ("1", "gpu"), ("0", "host")):
        monkeypatch.setenv("RT_PIXEL_LISTS", mode)
        rt = pt.RayTracer(0)  # read when the context is created
        rt.setSpheres(sc.ply_scene())
        rt.setCamera(cam)
        rt.setSampleRate(sr)
        rt.setMaxPathDepth(6)
        rt.setBuilder(builder)  # the GPU-built tree: never-culling normal boxes
        rt.setMesh(verts, idx)
        rt.setSeeds(Wp, Hp, seeds)
        got = np.zeros(W * H * 4, np.float32)
        rt.rayTrace(got, W, H, 0, kernel=2)
        rt.close()
        np.testing.assert_array_equal(bits(got), bits(exp), err_msg=f"RT_PIXEL_LISTS={mode} {builder}")


def test_pixel_candidate_lists_small_wide_frames(pt, oracle, monkeypatch):
    """The list frustum on frames whose pixels subtend a wide angle: a 24x20 frame
    at fov 100 (L = (W/2)/tan(fov/2) ~ 10, where normalising the corner rays misses interior
    directions by ~1/(8 L^2) ~ 1e-3) with the mesh filling the view, sampleRate 4, lists forced
    on — equal to the oracle.  Then a list area too small for every pixel (RT_LIST_MB: the
    pixels that do not fit take the tree) on the 64x48 frame: equal to the oracle, and the
    render reports the lists on with pixels on the tree."""
    sc = pt.scenes
    verts, idx = sc.make_mesh(2000)
    for (W, H, fov, dist, env) in ((24, 20, 100.0, 3.2, {}), (64, 48, 53.0, 5.0, {"RT_LIST_MB": "1"})):
        Wp, Hp = sc.padded_dims(W, H)
        seeds = sc.default_seeds(Wp, Hp, skip=11)
        c = dict(sc.PLY_CAMERA)
        c["distance"] = dist
        cam = sc.camera_spherical(W, fov=fov, **c)
        exp = np.zeros(W * H * 4, np.float32)
        oracle.render_tris(exp, cam, sc.ply_scene(), W, H, Wp, Hp, 4, 6, 0, seeds.copy(), verts, idx)
        monkeypatch.setenv("RT_PIXEL_LISTS", "1")
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        rt = pt.RayTracer(0)
        rt.setSpheres(sc.ply_scene())
        rt.setCamera(cam)
        rt.setSampleRate(4)
        rt.setMaxPathDepth(6)
        rt.setMesh(verts, idx)
        rt.setSeeds(Wp, Hp, seeds)
        got = np.zeros(W * H * 4, np.float32)
        rt.rayTrace(got, W, H, 0, kernel=2)
        info = rt.renderInfo()
        rt.close()
        for k in env:
            monkeypatch.delenv(k)
        np.testing.assert_array_equal(bits(got), bits(exp), err_msg=f"{W}x{H} fov {fov} {env}")
        assert info["lists"] == 1
        if env:
            assert 0 < info["list_pixels_tree"] and info["list_records"] <= info["list_capacity"], info


def test_pixel_candidate_lists_skewed_cameras(pt, oracle, monkeypatch):
    """The lists' pixel-square culling (k_pixel_lists: a candidate's widened triangle projected
    through the camera basis onto the pixel's (a, b) square) with camera bases the spherical camera
    never makes: right skewed toward up, up stretched, view off-axis (a general basis, inverted
    per pixel), and a basis with nonzero w lanes (camera_dir normalises over four lanes; the
    projection test is then skipped) — lists forced on, sampleRate 2, equal to the oracle."""
    sc = pt.scenes
    W, H = 48, 40
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(20_000)
    c = dict(sc.PLY_CAMERA)
    c["distance"] = 3.4
    base = sc.camera_spherical(W, fov=60.0, **c).reshape(4, 4).astype(np.float32)
    view, up, right = base[0].copy(), base[1].copy(), base[2].copy()
    skewed = base.copy()
    skewed[2] = right + np.float32(0.3) * up          # right leans toward up
    skewed[1] = up * np.float32(1.7)                   # up stretched
    skewed[0] = view + np.float32(0.2) * W * right     # the view axis off the frame's centre
    wlanes = base.copy()
    wlanes[0, 3], wlanes[1, 3], wlanes[2, 3] = np.float32(0.5), np.float32(0.01), np.float32(-0.02)
    monkeypatch.setenv("RT_PIXEL_LISTS", "1")
    for name, cam in (("skewed", skewed), ("w lanes", wlanes)):
        cam = np.ascontiguousarray(cam.reshape(16), np.float32)
        seeds = sc.default_seeds(Wp, Hp, skip=7)
        exp = np.zeros(W * H * 4, np.float32)
        oracle.render_tris(exp, cam, sc.ply_scene(), W, H, Wp, Hp, 2, 6, 0, seeds.copy(), verts, idx)
        rt = pt.RayTracer(0)
        rt.setSpheres(sc.ply_scene())
        rt.setCamera(cam)
        rt.setSampleRate(2)
        rt.setMaxPathDepth(6)
        rt.setMesh(verts, idx)
        rt.setSeeds(Wp, Hp, seeds)
        got = np.zeros(W * H * 4, np.float32)
        rt.rayTrace(got, W, H, 0, kernel=2)
        info = rt.renderInfo()
        rt.close()
        assert info["lists"] == 1, info
        np.testing.assert_array_equal(bits(got), bits(exp), err_msg=name)


def test_candidate_lists_reused_across_frames(pt, oracle, monkeypatch):
    """The candidate lists depend only on camera, mesh / tree, frame and tile: frames of one
    view reuse them (rt_render_info.lists_rebuilt 0) and a camera move rebuilds them.  Every
    frame of a progressive sequence, before and after a move, equals the oracle."""
    sc = pt.scenes
    W, H, sr = 64, 48, 2
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(20_000)
    monkeypatch.setenv("RT_PIXEL_LISTS", "1")
    rt = pt.RayTracer(0)
    rt.setSpheres(sc.ply_scene())
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(verts, idx)
    seeds = sc.default_seeds(Wp, Hp, skip=17)
    rt.setSeeds(Wp, Hp, seeds)
    sd = seeds.copy()
    got = np.zeros(W * H * 4, np.float32)
    exp = np.zeros_like(got)
    rebuilt = []
    for f, az in enumerate((105.0, 105.0, 105.0, 108.0, 108.0)):
        c = dict(sc.PLY_CAMERA)
        c["azimuth"] = az
        rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
        cam = sc.camera_spherical(W, **c)
        p = 0 if f in (0, 3) else f - (0 if f < 3 else 3)
        rt.rayTrace(got, W, H, p, kernel=2)
        rebuilt.append(rt.renderInfo()["lists_rebuilt"])
        oracle.render_tris(exp, cam, sc.ply_scene(), W, H, Wp, Hp, sr, 6, p, sd, verts, idx)
        np.testing.assert_array_equal(bits(got), bits(exp), err_msg=f"frame {f}")
    np.testing.assert_array_equal(rt.getSeeds(), sd)
    rt.close()
    assert rebuilt == [1, 0, 0, 1, 0], rebuilt


def test_traversal_switch_on_a_context_keeps_results(pt, oracle):
    """the cached schedule (LPT order, pixel classes, the long chains' slots)
    belongs to one traversal.  One context renders the same tile at sampleRate 4 (a
    sample-split render: few pixels per lane) with the compressed tree, then the full-precision
    tree, then the linear loop, then the compressed tree again; every render equals the oracle
    on the tile's rows."""
    sc = pt.scenes
    W, H, sr, tile = 96, 64, 4, (8, 4, 1)
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(2000)
    seeds = sc.default_seeds(Wp, Hp, skip=5)
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    rows = np.arange(H)[(np.arange(H) // tile[0]) % tile[1] == tile[2]]
    pix = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1).astype(np.uint32)
    exp = np.zeros(W * H * 4, np.float32)
    sd = seeds.copy()
    oracle.render_tris(exp, cam, sc.ply_scene(), W, H, Wp, Hp, sr, 6, 0, sd, verts, idx, pixels=pix)
    exp_tile = exp.reshape(H, W, 4)[rows].reshape(-1)
    rt = pt.RayTracer(0)
    rt.setSpheres(sc.ply_scene())
    rt.setCamera(cam)
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(verts, idx)
    split = []
    for trav in ("bvh", "bvh4f", "linear", "bvh"):
        rt.setTraversal(trav)
        rt.setSeeds(Wp, Hp, seeds)
        got = np.zeros(len(rows) * W * 4, np.float32)
        rt.rayTrace(got, W, H, 0, kernel=2, tile=tile)
        split.append(rt.renderInfo()["split_chunks"])
        np.testing.assert_array_equal(bits(got), bits(exp_tile), err_msg=trav)
        s_got = rt.getSeeds()
        sl = pix.astype(np.int64) // W * Wp + pix % W
        np.testing.assert_array_equal(s_got[sl], sd[sl], err_msg=trav)
    rt.close()
    assert split[0] > 0 and split[1] == 0 and split[2] == 0 and split[3] > 0, split


@pytest.mark.parametrize("width", [8, 16, 64, 3])
@pytest.mark.parametrize("sr", [2, 3, 5])
def test_sample_split_vs_oracle(tracer, pt, oracle, monkeypatch, sr, width):
    """Sample-split rendering forced on (RT_SPLIT=1): the seed pass stores each chunk's first
    seed from the pixel's closest-hit queries alone, k_tris renders the chunks as independent
    tasks and k_split_finish sums the samples in order.  Whole frames over two progressive
    frames and a row-stripe tile equal the oracle bit for bit, frames and seeds, with chunkings
    that do not divide the sample count evenly (sr 3: 9 chunks of 1 sample; sr 5: 13 chunks of
    2, the last of 1).  The long chains' seed pass runs with `width` lanes per chain: 8-64
    subtree-parallel lanes (k_chain_seeds, the default 8) or (3) 4 cooperative lanes (coop_round)."""
    monkeypatch.setenv("RT_SPLIT", "1")
    monkeypatch.setenv("RT_SEED_WIDTH", str(width))
    sc = pt.scenes
    W, H = 72, 40
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(20_000)
    seeds = sc.default_seeds(Wp, Hp, skip=3)
    S = sc.ply_scene()
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    spp = sr * sr
    csz = (spp + 15) // 16
    rt = pt.RayTracer(0)  # RT_SPLIT is read when the context is created
    rt.setSpheres(S)
    rt.setCamera(cam)
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(verts, idx)
    rt.setSeeds(Wp, Hp, seeds)
    got = np.zeros(W * H * 4, np.float32)
    exp = np.zeros_like(got)
    sd = seeds.copy()
    for p in range(2):
        rt.rayTrace(got, W, H, p, kernel=2)
        info = rt.renderInfo()
        assert info["split_chunks"] == (spp + csz - 1) // csz
        # the long chains ran on their own stream with `width` lanes per chain
        assert info["pixels_long"] > 0 and info["split_coop"] == width and info["split_guard"] == 0, info
        # the long chains' chunk tasks (single samples, either pass form) answer the box segments
        # from the seed pass's per-sample mesh-hit depths (no traversal for them)
        assert info["split_hit_depth"] == 1, info
        # the view's second frame: its tiles re-sorted by the first frame's measured chunk costs
        # (frames of >= 16 samples per pixel)
        assert info["schedule_measured"] == (1 if p == 1 and spp >= 16 else 0), info
        # the mesh pixels' chunk seeds jumped ahead from their frame seeds (no seed pass for them)
        assert info["split_spec"] == 1, info
        assert len(rt.longChains()) == info["pixels_long"]
        oracle.render_tris(exp, cam, S, W, H, Wp, Hp, sr, 6, p, sd, verts, idx)
        np.testing.assert_array_equal(bits(got), bits(exp), err_msg=f"frame {p}")
        np.testing.assert_array_equal(rt.getSeeds(), sd, err_msg=f"seeds after frame {p}")
    tile = (8, 2, 1)
    rows = np.arange(H)[(np.arange(H) // tile[0]) % tile[1] == tile[2]]
    pix = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1).astype(np.uint32)
    sd = seeds.copy()
    oracle.render_tris(exp, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, verts, idx, pixels=pix)
    rt.setSeeds(Wp, Hp, seeds)
    got = np.zeros(len(rows) * W * 4, np.float32)
    rt.rayTrace(got, W, H, 0, kernel=2, tile=tile)
    info = rt.renderInfo()
    assert info["split_chunks"] > 0 and info["pixels_long"] > 0 and info["split_coop"] == width, info
    np.testing.assert_array_equal(bits(got), bits(exp.reshape(H, W, 4)[rows].reshape(-1)), err_msg="tile")
    np.testing.assert_array_equal(rt.getSeeds(), sd, err_msg="tile seeds")
    rt.close()


@pytest.mark.parametrize("width", [8, 3])
@pytest.mark.parametrize("spec", ["2", "0"])
def test_speculated_pixels_repaired_vs_oracle(pt, oracle, monkeypatch, spec, width):
    """Speculated mesh pixels (their chunk seeds jumped ahead from the frame seed, DESIGN.md
    §4.5) whose camera rays miss the mesh after all are repaired: with RT_SPLIT_SPEC=2 every
    pixel whose probe rays all hit is speculated, silhouettes included, so some chunks meet a
    camera ray that misses; those pixels are listed and re-rendered (seed pass + chunks) and the
    frame and seeds equal the oracle bit for bit — the repair restarts each chain at its first
    chunk that saw a miss (the chunks before it stand) — and so does the view's next frame.  RT_SPLIT_SPEC=0 (no speculation, every mesh
    pixel through the seed pass) equals it too."""
    monkeypatch.setenv("RT_SPLIT", "1")
    monkeypatch.setenv("RT_SPLIT_SPEC", spec)
    monkeypatch.setenv("RT_SEED_WIDTH", str(width))  # the long chains' (and repairs') pass: 8 lanes / cooperative
    sc = pt.scenes
    W, H, sr = 128, 96, 8
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(20_000)
    seeds = sc.default_seeds(Wp, Hp, skip=5)
    S = sc.ply_scene()
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    rt = pt.RayTracer(0)
    rt.setSpheres(S)
    rt.setCamera(cam)
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(verts, idx)
    rt.setSeeds(Wp, Hp, seeds)
    got = np.zeros(W * H * 4, np.float32)
    rt.rayTrace(got, W, H, 0, kernel=2)
    info = rt.renderInfo()
    assert info["split_chunks"] > 0 and info["split_guard"] == 0, info
    if spec == "2":
        assert info["split_spec"] == 1 and info["split_repaired"] > 0, info
    else:
        assert info["split_spec"] == 0 and info["split_repaired"] == 0, info
    exp = np.zeros_like(got)
    sd = seeds.copy()
    oracle.render_tris(exp, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, verts, idx)
    np.testing.assert_array_equal(bits(got), bits(exp))
    np.testing.assert_array_equal(rt.getSeeds(), sd)
    # the next (progressive) frame of the same view, its schedule reused: repaired again where its
    # camera rays miss, the same bits as the oracle's frame 1
    rt.rayTrace(got, W, H, 1, kernel=2)
    info1 = rt.renderInfo()
    assert info1["split_guard"] == 0, info1
    if spec == "2":
        assert info1["split_repaired"] > 0, info1
    oracle.render_tris(exp, cam, S, W, H, Wp, Hp, sr, 6, 1, sd, verts, idx)
    np.testing.assert_array_equal(bits(got), bits(exp))
    np.testing.assert_array_equal(rt.getSeeds(), sd)
    rt.close()


def test_kernel_time_split(pt, monkeypatch):
    """rt_last_kernel_split_ms: a many-sample frame's device time splits into the candidate-list
    pre-pass and the main kernel, the two adding up to rt_last_kernel_ms; without lists
    (RT_PIXEL_LISTS=0) the pre-pass part is zero."""
    sc = pt.scenes
    W, H = 128, 96
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(20_000)
    for mode, has_pre in (("1", True), ("0", False)):
        monkeypatch.setenv("RT_PIXEL_LISTS", mode)
        rt = pt.RayTracer(0)
        rt.setSpheres(sc.ply_scene())
        c = sc.PLY_CAMERA
        rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
        rt.setSampleRate(4)
        rt.setMaxPathDepth(6)
        rt.setMesh(verts, idx)
        rt.setSeeds(Wp, Hp, sc.default_seeds(Wp, Hp))
        out = np.zeros(W * H * 4, np.float32)
        rt.rayTrace(out, W, H, 0, kernel=2)
        total = rt.lastKernelMs()
        pre, main = rt.lastKernelSplitMs()
        rt.close()
        assert main > 0.0 and abs(pre + main - total) <= 0.01 * total + 1e-3, (pre, main, total)
        assert (pre > 0.0) if has_pre else (pre < 0.05 * total), (mode, pre, total)


# ---- GPU BVH builder (csrc/rt_build_gpu.hip) ----------------------------------------------

@pytest.mark.parametrize("trav", ["bvh", "bvh4f"])
@pytest.mark.parametrize("name", TRI_CASES)
def test_gpu_builder_golden_tris(name, trav, pt, golden, golden_meta):
    """Frames from a GPU-built tree equal the reference kernel's (golden fixtures)."""
    g, m = golden(name), golden_meta["cases"][name]
    rt = pt.RayTracer(0)
    rt.setBuilder("gpu")
    _setup(rt, pt, g, m, kernel_tris=True)
    assert rt.meshInfo()["builder"] == pt._abi.RT_BUILD_GPU
    rt.setTraversal(trav)
    out = np.zeros(m["W"] * m["H"] * 4, np.float32)
    for p in range(m["frames"]):
        rt.rayTrace(out, m["W"], m["H"], p, kernel=2)
        np.testing.assert_array_equal(bits(out), bits(g["frames"][p]), err_msg=f"{name} frame {p}")
    np.testing.assert_array_equal(rt.getSeeds(), g["seeds_out"])
    rt.close()


def _query_sets(pt, verts, n=16384, seed=5):
    sc = pt.scenes
    cam = sc.camera_spherical(320, **sc.PLY_CAMERA)
    rays = sc.camera_rays(cam, 320, 180)
    rng = np.random.default_rng(seed)
    lo, hi = verts.min(0) - 1.0, verts.max(0) + 1.0
    rr = np.zeros(n, pt._abi.RAY_DTYPE)
    rr["o"] = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    rr["d"] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rr["tmin"] = np.float32(1e-4)
    rr["tmax"] = np.float32(np.inf)
    rs = rr.copy()
    rs["tmax"] = rng.uniform(0.0, 8.0, n).astype(np.float32)
    return rays, rr, rs


@pytest.mark.parametrize("case", ["dragon", "tiny1", "tiny2", "tiny7", "duplicates"])
def test_gpu_builder_equals_linear(case, pt):
    """Closest-hit index + t and any-hit flags from the GPU-built tree equal the linear loop
    (dragon class; 1/2/7-triangle meshes; many triangles with one centroid = equal Morton codes)."""
    sc = pt.scenes
    if case == "dragon":
        verts, idx = sc.make_mesh(sc.MESH_CONFIGS["dragon"])
    elif case.startswith("tiny"):
        verts, idx = sc.make_mesh(200)
        idx = idx[: int(case[4:])]
    else:
        rng = np.random.default_rng(2)
        nt = 5000
        # vertices a, -a and a point inside their box: every box centre (the Morton
        # centroid) is the origin, so all codes are equal
        a = rng.uniform(-2, 2, (nt, 3)).astype(np.float32)
        c = (a * rng.uniform(-0.9, 0.9, (nt, 3))).astype(np.float32)
        verts = np.stack([a, -a, c], axis=1).reshape(-1, 3)
        idx = np.arange(nt * 3, dtype=np.int32).reshape(nt, 3)
    rays, rr, rs = _query_sets(pt, verts)
    res = {}
    for builder, trav in [("host", "linear"), ("gpu", "bvh"), ("gpu", "bvh4f")]:
        rt = pt.RayTracer(0)
        rt.setBuilder(builder)
        rt.setMesh(verts, idx)
        rt.setTraversal(trav)
        res[(builder, trav)] = (rt.traceRays(rays), rt.traceRays(rr), rt.traceRays(rs, any_hit=True))
        if builder == "gpu":
            info = rt.meshInfo()
            assert info["builder"] == pt._abi.RT_BUILD_GPU and info["n_nodes4"] >= 1
        rt.close()
    ref = res[("host", "linear")]
    for key, got in res.items():
        for k in range(3):
            np.testing.assert_array_equal(got[k][0], ref[k][0], err_msg=f"{case} {key} set {k}")
            if k < 2:
                np.testing.assert_array_equal(bits(got[k][1]), bits(ref[k][1]), err_msg=f"{case} {key} t {k}")


def test_interactive_view_replay(tracer, pt, oracle, tmp_path):
    """f3: ProgressiveViewHIP (GlutCLWindow.cpp:136-301 without GL) driven through the C++ CLI by
    display / arrow-key / drag / reshape events.  Every displayed frame equals the oracle's render
    of the reference kernel for the state the window is in — camera from setCameraSpherical(
    (0,-4,0), elevation, azimuth, 5) at fov 53 once the orbit has moved it (main.cpp's camera
    before), progression 0 after a (re)allocation and +1 per refining display, the seed planes
    of the context's glibc rand() stream regenerated on every size change — bit for bit, frames
    and their progressive mix.  Every key / drag posts a redisplay exactly when refinement had
    finished (GlutCLWindow.cpp:294-301), and a display at maxProgression renders nothing."""
    import json
    import subprocess

    from conftest import ROOT

    max_prog = 4
    events = ("d,d,d,d,d,d,l,d,d,m:7:-4,d,u,u,d,d,d,d,d,d,m:3:2,d,s:48:40,d,d,n,d,r,d,m:-400:90,d,d,"
              "d,d,d,d,u,d")
    frames_path = tmp_path / "frames.f32"
    res = subprocess.run([str(ROOT / "pathtracer.cl_amd" / "rt_render"), "--scene", "main", "--width", "64",
                          "--height", "48", "--events", events, "--max-progression", str(max_prog),
                          "--frames-out", str(frames_path)], check=True, timeout=120, capture_output=True, text=True)
    lines = [json.loads(x) for x in res.stdout.strip().splitlines()]
    states, final = lines[:-1], lines[-1]
    shown = np.fromfile(frames_path, np.float32)

    sc = pt.scenes
    f32 = np.float32
    S = sc.main_scene()
    az, el = f32(105.0), f32(40.0)  # GlutCLWindow's constructor (:24-28)
    orbited = False
    W, H, prog, realloc = 64, 48, 0, True
    exp = sd = None
    consumed = 0  # values of the context's rand() stream used by earlier seed layouts
    off = 0
    n_rendered = n_post = 0
    evs = events.split(",")
    assert len(states) == len(evs)
    for ev, st in zip(evs, states):
        assert st["event"] == ev
        post = False
        rendered = False
        if ev == "d":
            if realloc:
                Wp, Hp = sc.padded_dims(W, H)
                sd = sc.default_seeds(Wp, Hp, skip=consumed)
                consumed += 2 * Wp * Hp
                exp = np.zeros(W * H * 4, np.float32)
                prog, realloc, rendered, post = 0, False, True, max_prog > 0
            elif prog < max_prog:
                prog, rendered, post = prog + 1, True, True
            if rendered:
                cam = (sc.camera_spherical(W, (0.0, -4.0, 0.0), float(el), float(az), 5.0) if orbited
                       else sc.camera_spherical(W, **sc.MAIN_CAMERA))
                oracle.render_spheres(exp, cam, S, W, H, Wp, Hp, 1, 6, prog, sd)
                got = shown[off:off + W * H * 4]
                off += W * H * 4
                np.testing.assert_array_equal(bits(got), bits(exp), err_msg=f"displayed frame {n_rendered} ({ev})")
                n_rendered += 1
        elif ev in ("l", "r", "u", "n") or ev[0] == "m":
            if ev == "l":
                az = np.fmod(f32(az + f32(3.0)), f32(360.0))
            elif ev == "r":
                az = np.fmod(f32(az - f32(3.0)), f32(360.0))
            elif ev == "u":
                el = min(f32(el + f32(3.0)), f32(90.0))
            elif ev == "n":
                el = max(f32(el - f32(3.0)), f32(10.0))
            else:
                dx, dy = map(int, ev[2:].split(":"))
                az = np.fmod(f32(az + f32(dx)), f32(360.0))
                el = max(min(f32(el + f32(dy)), f32(90.0)), f32(10.0))
            orbited = True
            post = prog >= max_prog  # restart(), GlutCLWindow.cpp:294-301
            prog = 0
        else:
            W, H = map(int, ev[2:].split(":"))
            realloc = True
        n_post += post and ev != "d"
        assert (st["rendered"], st["redisplay"], st["progression"]) == (rendered, post, prog), (ev, st)
        assert (st["width"], st["height"]) == (W, H)
        assert f32(st["azimuth"]) == az and f32(st["elevation"]) == el
    assert off == shown.size and n_rendered >= 20
    assert n_post >= 2  # drags / keys after refinement finished did post a redisplay
    assert (final["progression"], final["width"], final["height"]) == (prog, W, H)


def test_huge_coordinates_fall_back_to_full_precision_nodes(tracer, pt):
    """A mesh whose extent exceeds the compressed grid (255 * 2^7) cannot be encoded in
    48/64-B nodes: the default traversal falls back to the full-precision 4-wide nodes and
    still equals the linear loop."""
    sc = pt.scenes
    verts, idx = sc.make_mesh(3000)
    verts = (verts * np.float32(2.0e4)).astype(np.float32)  # extent ~1e5
    rng = np.random.default_rng(4)
    n = 4096
    rr = np.zeros(n, pt._abi.RAY_DTYPE)
    rr["o"] = rng.uniform(-1.5e5, 1.5e5, (n, 3)).astype(np.float32)
    tgt = verts[rng.integers(0, len(verts), n)]
    d = tgt - rr["o"]
    rr["d"] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rr["tmin"] = np.float32(1e-4)
    rr["tmax"] = np.float32(np.inf)
    res = {}
    for builder in ("host", "gpu"):
        for trav in ("bvh", "linear"):
            rt = pt.RayTracer(0)
            rt.setBuilder(builder)
            rt.setMesh(verts, idx)
            rt.setTraversal(trav)
            res[(builder, trav)] = rt.traceRays(rr)
            rt.close()
    ref = res[("host", "linear")]
    assert (ref[0] >= 0).sum() > n // 4
    for key, got in res.items():
        np.testing.assert_array_equal(got[0], ref[0], err_msg=str(key))
        np.testing.assert_array_equal(bits(got[1]), bits(ref[1]), err_msg=str(key))


def test_schedule_changes_no_bits(tracer, pt, monkeypatch):
    """The pixel queue's order (step-counting probe, LPT key) and the box-wave priority are
    scheduling only: a frame with box and mesh pixels, 16 spp, renders to the same bits and
    seeds with the queue row-major (RT_SCHEDULE=0), with the default schedule (a sample-split
    render: few pixels per lane), with whole-pixel tasks (RT_SPLIT=0), with the split forced
    on, with split buffers too small for the frame (RT_SPLIT_MB=1: whole pixels again), with
    camera rays traversing the tree instead of their candidate lists (RT_PIXEL_LISTS=0), and
    with a list area too small for every pixel (RT_LIST_MB=2)."""
    sc = pt.scenes
    W, H, sr = 160, 120, 4
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(20_000)
    seeds = sc.default_seeds(Wp, Hp, skip=7)
    frames = []
    for env in ({"RT_SCHEDULE": "0"}, {}, {"RT_SPLIT": "0"}, {"RT_SPLIT": "1"}, {"RT_SPLIT": "1", "RT_SPLIT_MB": "1"},
                {"RT_PIXEL_LISTS": "0"}, {"RT_LIST_MB": "2"}):
        for k in ("RT_SCHEDULE", "RT_SPLIT", "RT_SPLIT_MB", "RT_PIXEL_LISTS", "RT_LIST_MB"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        rt = pt.RayTracer(0)  # the knobs are read when the context is created
        rt.setSpheres(sc.ply_scene())
        c = sc.PLY_CAMERA
        rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
        rt.setSampleRate(sr)
        rt.setMaxPathDepth(6)
        rt.setMesh(verts, idx)
        rt.setSeeds(Wp, Hp, seeds)
        out = np.zeros(W * H * 4, np.float32)
        rt.rayTrace(out, W, H, 0, kernel=2)
        frames.append((bits(out).copy(), rt.getSeeds().copy()))
        rt.close()
    for f, s in frames[1:]:
        np.testing.assert_array_equal(f, frames[0][0])
        np.testing.assert_array_equal(s, frames[0][1])


def test_renders_on_alternating_streams(tracer, pt):
    """rt_render_async on a different stream from the previous render's: the new render
    is ordered after the previous one's counter hand-back (which reads and zeroes the counters and
    queue cursors it uses) and so after its seed and framebuffer writes.  Progressive frames enqueued
    without a host wait, alternately on the context's stream and on two torch streams, end in the same
    framebuffer, seeds and per-frame ray counts as the same frames rendered one by one, and the
    device-side counter totals (rt_counter_totals) add up every frame's counts."""
    import torch

    sc = pt.scenes
    W, H, sr = 128, 96, 2
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(20_000)
    seeds = sc.default_seeds(Wp, Hp, skip=13)

    def make():
        rt = pt.RayTracer(0)
        rt.setSpheres(sc.ply_scene())
        c = sc.PLY_CAMERA
        rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
        rt.setSampleRate(sr)
        rt.setMaxPathDepth(6)
        rt.setMesh(verts, idx)
        rt.setSeeds(Wp, Hp, seeds)
        return rt

    ref = make()
    exp = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    rays = 0
    for p in range(6):
        ref.rayTrace(exp, W, H, p, kernel=2)
        c = ref.counters()
        rays += c["rays_closest"] + c["rays_shadow"]
    exp_seeds = ref.getSeeds()
    ref.close()
    rt = make()
    got = torch.zeros_like(exp)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    rt.rayTrace(got, W, H, 0, kernel=2)  # the schedule and lists (host work) before the async frames
    rt.setSeeds(Wp, Hp, seeds)
    rt.counterTotals(reset=True)
    for p, st in enumerate([None, s1.cuda_stream, s2.cuda_stream, None, s2.cuda_stream, s1.cuda_stream]):
        rt.rayTrace(got, W, H, p, kernel=2, stream=st, sync=False)
    tot = rt.counterTotals(reset=True)
    torch.cuda.synchronize()
    assert tot["renders"] == 6 and tot["rays_closest"] + tot["rays_shadow"] == rays, tot
    assert torch.equal(got.view(torch.int32), exp.view(torch.int32))
    np.testing.assert_array_equal(rt.getSeeds(), exp_seeds)
    rt.close()


def test_pilot_order_changes_no_bits(tracer, pt, oracle, monkeypatch):
    """The first frame of a view of >= 64 samples per pixel is ordered by a pilot render (DESIGN
    §4.4: the same kernel at 2x2 samples per pixel from a copy of the seeds, into a scratch
    framebuffer, with its own counters and queue cursors).  Nothing of it may reach the frame: at
    sampleRate 8 (64 spp, whole pixels) the frame, both seed planes and the ray counts are the same
    with the pilot (default), with a 3x3 pilot and without one (RT_PILOT=0: the probe's order), and
    equal to the oracle's; the view's next frame is ordered by the first frame's measured costs."""
    sc = pt.scenes
    W, H, sr = 96, 72, 8
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(20_000)
    seeds = sc.default_seeds(Wp, Hp, skip=9)
    frames = []
    for pilot in (None, "3", "0"):
        monkeypatch.delenv("RT_PILOT", raising=False)
        monkeypatch.setenv("RT_SPLIT", "0")  # whole pixels (a 96x72 frame would render sample-split)
        if pilot is not None:
            monkeypatch.setenv("RT_PILOT", pilot)
        rt = pt.RayTracer(0)  # the knobs are read when the context is created
        rt.setSpheres(sc.ply_scene())
        c = sc.PLY_CAMERA
        rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
        rt.setSampleRate(sr)
        rt.setMaxPathDepth(6)
        rt.setMesh(verts, idx)
        rt.setSeeds(Wp, Hp, seeds)
        out = np.zeros(W * H * 4, np.float32)
        rt.rayTrace(out, W, H, 0, kernel=2)
        info = rt.renderInfo()
        assert info["split_chunks"] == 0 and info["schedule_pilot"] == (0 if pilot == "0" else 1), (pilot, info)
        cnt = rt.counters()
        frames.append((bits(out).copy(), rt.getSeeds().copy(), (cnt["rays_closest"], cnt["rays_shadow"])))
        rt.setSeeds(Wp, Hp, seeds)
        rt.rayTrace(out, W, H, 0, kernel=2)
        info = rt.renderInfo()
        assert info["schedule_pilot"] == 0 and info["schedule_measured"] == 1, (pilot, info)
        np.testing.assert_array_equal(bits(out), frames[-1][0])
        rt.close()
    for f, s_, c_ in frames[1:]:
        np.testing.assert_array_equal(f, frames[0][0])
        np.testing.assert_array_equal(s_, frames[0][1])
        assert c_ == frames[0][2]
    exp = np.zeros(W * H * 4, np.float32)
    sd = seeds.copy()
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    c_or = oracle.render_tris(exp, cam, sc.ply_scene(), W, H, Wp, Hp, sr, 6, 0, sd, verts, idx,
                              bvh=oracle.build_bvh(verts, idx))
    np.testing.assert_array_equal(frames[0][0], bits(exp))
    np.testing.assert_array_equal(frames[0][1], sd)
    assert frames[0][2] == tuple(c_or)


def test_tree_cull_knobs_change_no_bits(tracer, pt, monkeypatch):
    """The host build's two culls and its cost area are traversal savings only: a tree without the
    determinant cull's normal boxes (RT_DET_CULL=0), one that keeps the triangles no unit ray can hit
    (RT_CULL_UNHITTABLE=0), and shadow rays on the closest-hit tree (RT_BVH_LIGHT_W=0: one tree)
    or on a tree split by the lights' projected area alone (1) render a frame of the dragon-class mesh (871,414 triangles,
    66,533 of them under the |det| >= 1e-4 rule for every unit ray, geometryFuncs.h:167) to the same
    bits and seeds as the default tree, at sampleRate 4 with the candidate lists."""
    sc = pt.scenes
    W, H, sr = 160, 120, 4
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS["dragon"])
    seeds = sc.default_seeds(Wp, Hp, skip=5)
    frames = []
    for env in ({}, {"RT_DET_CULL": "0"}, {"RT_CULL_UNHITTABLE": "0"}, {"RT_DET_CULL": "0", "RT_CULL_UNHITTABLE": "0"},
                {"RT_BVH_LIGHT_W": "0"}, {"RT_BVH_LIGHT_W": "1"}):
        for k in ("RT_DET_CULL", "RT_CULL_UNHITTABLE", "RT_BVH_LIGHT_W"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        rt = pt.RayTracer(0)
        rt.setSpheres(sc.ply_scene())
        c = sc.PLY_CAMERA
        rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
        rt.setSampleRate(sr)
        rt.setMaxPathDepth(6)
        rt.setMesh(verts, idx)  # the knobs are read by the build
        info = rt.meshInfo()
        rt.setSeeds(Wp, Hp, seeds)
        out = np.zeros(W * H * 4, np.float32)
        rt.rayTrace(out, W, H, 0, kernel=2)
        frames.append((bits(out).copy(), rt.getSeeds().copy(), info["n_tris_tree"], info["n_nodes4_shadow"]))
        rt.close()
    assert frames[0][2] < len(idx) and frames[2][2] == len(idx) and frames[4][2] == frames[0][2], [f[2] for f in frames]
    assert frames[0][3] > 0 and frames[4][3] == 0 and frames[5][3] > 0, [f[3] for f in frames]  # the shadow tree built
    for f, s_, _, _ in frames[1:]:
        np.testing.assert_array_equal(f, frames[0][0])
        np.testing.assert_array_equal(s_, frames[0][1])


def test_stepping_knobs_change_no_bits(tracer, pt, monkeypatch):
    """k_tris's stepping-round exit rule and its grid are scheduling only: a short frame (1 spp,
    so the short-frame grid of 3 blocks per CU) renders to the same bits and seeds with a grid of
    7 blocks, with the round ending at every completed query, with it ending only when 64 have
    completed (no live-lane rule), and with the live-lane rule alone (RTMI_* knobs, read at every
    render)."""
    sc = pt.scenes
    W, H, sr = 256, 192, 1
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(20_000)
    seeds = sc.default_seeds(Wp, Hp, skip=3)
    rt = pt.RayTracer(0)
    rt.setSpheres(sc.ply_scene())
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(verts, idx)
    knobs = ("RTMI_GRID_BLOCKS", "RTMI_FETCH_K", "RTMI_FETCH_FRAC")
    frames = []
    for env in ({}, {"RTMI_GRID_BLOCKS": "7"}, {"RTMI_FETCH_K": "1"}, {"RTMI_FETCH_K": "64", "RTMI_FETCH_FRAC": "0"},
                {"RTMI_FETCH_K": "64", "RTMI_FETCH_FRAC": "16"}):
        for k in knobs:
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        rt.setSeeds(Wp, Hp, seeds)
        out = np.zeros(W * H * 4, np.float32)
        rt.rayTrace(out, W, H, 0, kernel=2)
        frames.append((bits(out).copy(), rt.getSeeds().copy()))
    rt.close()
    for f, s in frames[1:]:
        np.testing.assert_array_equal(f, frames[0][0])
        np.testing.assert_array_equal(s, frames[0][1])
