"""Whole frames at the BASELINE configurations' own sizes, bit for bit against the oracle.

The reference runs one work-item per pixel over the whole NDRange (raytracer.cl:184-243,
launched by RayTracerCL.cpp:289-292), so parity means every pixel and every seed slot.  The
oracle's linear loop costs O(871k) per ray — days for a dragon frame — so these tests use the
oracle's independent BVH mode (oracle/pt_oracle.c `or_bvh_*`: a plain binary tree with exact
binary64 boxes and conservative margins, none of the product's quantised nodes, culls or lists),
which tests/test_oracle_bvh.py pins to the golden fixtures, to the linear loop on adversarial
rays and to the reference kernel itself.  The oracle renders on the host's CPUs (16 threads on
the GPU box): the dragon frame at sampleRate 4 and one 8-way tile at sampleRate 16 take tens of
seconds each.

  * BASELINE configs[0]: the sphere scene at 512x512, 1 spp (main.cpp:123-127), from the
    context's own seeds (the padded 512x512 layout, RayTracerCL.cpp:229-232), three frames;
  * configs[2]: the bunny-class mesh at 1024x1024, 1 spp, three frames (the later ones with the
    camera-ray candidate lists of the unchanged view);
  * configs[3]: the dragon-class frame, 1920x1080, at sampleRate 4 (whole-pixel tasks);
  * one 8-way row-stripe tile of configs[3] at its own sampleRate 16 (256 spp): the sample-split
    path with its long chains, speculated mesh pixels and the repair pass;
  * the split path's buffers regrown on one context (a tile, then the whole frame) with more
    repaired pixels than the per-sample repair slots.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import bits

pytestmark = pytest.mark.gpu


def _seed_slots(pix, Wp, W):
    pix = np.asarray(pix, np.int64)
    return pix // W * Wp + pix % W


@pytest.fixture(scope="module")
def dragon(pt, oracle):
    sc = pt.scenes
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS["dragon"])
    bvh = oracle.build_bvh(verts, idx)
    W, H = 1920, 1080
    Wp, Hp = sc.padded_dims(W, H)
    return dict(verts=verts, idx=idx, bvh=bvh, W=W, H=H, Wp=Wp, Hp=Hp, S=sc.ply_scene(),
                cam=sc.camera_spherical(W, **sc.PLY_CAMERA), seeds=sc.default_seeds(Wp, Hp))


@pytest.fixture(scope="module")
def dragon_sr4(dragon, oracle):
    """The oracle's whole dragon frame at sampleRate 4 from the default seeds (and the seeds it
    leaves, and its ray counts)."""
    d = dragon
    exp = np.zeros(d["W"] * d["H"] * 4, np.float32)
    sd = d["seeds"].copy()
    cnt = oracle.render_tris(exp, d["cam"], d["S"], d["W"], d["H"], d["Wp"], d["Hp"], 4, 6, 0, sd, d["verts"],
                             d["idx"], bvh=d["bvh"])
    return exp, sd, cnt


def _tracer(pt, d, sr):
    rt = pt.RayTracer(0)
    rt.setSpheres(d["S"])
    c = pt.scenes.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    rt.setMesh(d["verts"], d["idx"])
    return rt


def _tile_rows(H, tile):
    stripe, n, r = tile[:3]
    owner = tile[3] if len(tile) > 3 else None
    s = np.arange(H) // stripe
    return np.arange(H)[(s % n if owner is None else np.asarray(owner)[s]) == r]


def _check_tile(got, got_seeds, exp, exp_seeds, d, rows):
    W, Wp, Hp = d["W"], d["Wp"], d["Hp"]
    np.testing.assert_array_equal(bits(got), bits(exp.reshape(d["H"], W, 4)[rows].reshape(-1)))
    pix = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1)
    sl = _seed_slots(pix, Wp, W)
    plane = Wp * Hp
    np.testing.assert_array_equal(got_seeds[sl], exp_seeds[sl])
    np.testing.assert_array_equal(got_seeds[plane + sl], exp_seeds[plane + sl])


def test_sphere_config1_512_vs_oracle(tracer, pt, oracle):
    """BASELINE configs[0] (main.cpp:123-127: sampleRate 1, maxDepth 6, the main.cpp camera) at
    its own 512x512, from the seeds a fresh context draws for that size: three progressive
    frames (row-shifted seeds, mix 1/p), every pixel, both seed planes and the ray counts equal
    to the oracle's."""
    sc = pt.scenes
    W = H = 512
    Wp, Hp = sc.padded_dims(W, H)
    assert (Wp, Hp) == (512, 512)
    S = sc.main_scene()
    cam = sc.camera_spherical(W, **sc.MAIN_CAMERA)
    rt = pt.RayTracer(0)
    rt.setSpheres(S)
    c = sc.MAIN_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(1)
    rt.setMaxPathDepth(6)
    sd = sc.default_seeds(Wp, Hp)
    got = np.zeros(W * H * 4, np.float32)
    exp = np.zeros_like(got)
    for p in range(3):
        rt.rayTrace(got, W, H, p, kernel=0)
        c_or = oracle.render_spheres(exp, cam, S, W, H, Wp, Hp, 1, 6, p, sd)
        np.testing.assert_array_equal(bits(got), bits(exp), err_msg=f"frame {p}")
        cnt = rt.counters()
        assert (cnt["rays_closest"], cnt["rays_shadow"]) == c_or
    np.testing.assert_array_equal(rt.getSeeds(), sd)
    assert np.isfinite(got).all() and (got.reshape(-1, 4)[:, 3] == 0).all()
    rt.close()


def test_bunny_config_whole_frame_vs_bvh_oracle(tracer, pt, oracle):
    """BASELINE configs[2]: the bunny-class mesh (69,451 triangles) at 1024x1024, 1 spp, from the
    context's own seeds: every pixel and seed slot of three progressive frames (the later ones reuse
    the view's schedule — a 1-spp frame keeps the probe's order — and the second builds its
    candidate lists) equal to the oracle's."""
    sc = pt.scenes
    W = H = 1024
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(sc.MESH_CONFIGS["bunny"])
    bvh = oracle.build_bvh(verts, idx)
    S = sc.ply_scene()
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    rt = pt.RayTracer(0)
    rt.setSpheres(S)
    c = sc.PLY_CAMERA
    rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
    rt.setSampleRate(1)
    rt.setMaxPathDepth(6)
    rt.setMesh(verts, idx)
    sd = sc.default_seeds(Wp, Hp)
    got = np.zeros(W * H * 4, np.float32)
    exp = np.zeros_like(got)
    for p in range(3):
        rt.rayTrace(got, W, H, p, kernel=2)
        info = rt.renderInfo()
        assert info["lists"] == (1 if p >= 1 else 0), info
        assert info["schedule_measured"] == 0, info  # 1 spp: the probe's order throughout
        c_or = oracle.render_tris(exp, cam, S, W, H, Wp, Hp, 1, 6, p, sd, verts, idx, bvh=bvh)
        np.testing.assert_array_equal(bits(got), bits(exp), err_msg=f"frame {p}")
        cnt = rt.counters()
        assert (cnt["rays_closest"], cnt["rays_shadow"]) == c_or
    np.testing.assert_array_equal(rt.getSeeds(), sd)
    assert (exp.reshape(-1, 4)[:, :3] > 0).mean() > 0.05
    rt.close()


def test_dragon_whole_frame_sr4_vs_bvh_oracle(tracer, pt, dragon, dragon_sr4):
    """BASELINE configs[3]'s frame (dragon class, 871,414 triangles, 1920x1080, maxDepth 6) at
    sampleRate 4: all 2,073,600 pixels, both seed planes and the ray counts equal to the oracle's —
    rendered under the probe's order, then again from the same seeds under the order re-sorted by
    the first render's measured per-pixel costs (16 spp, whole pixels: DESIGN §4.4)."""
    d = dragon
    exp, sd, c_or = dragon_sr4
    rt = _tracer(pt, d, 4)
    got = np.zeros(d["W"] * d["H"] * 4, np.float32)
    for k in range(2):
        if k:
            rt.setSeeds(d["Wp"], d["Hp"], d["seeds"])
        rt.rayTrace(got, d["W"], d["H"], 0, kernel=2)
        info = rt.renderInfo()
        assert info["lists"] == 1 and info["split_chunks"] == 0 and info["schedule_measured"] == k, info
        assert info["schedule_pilot"] == 0, info  # (16 spp: no pilot render, test_pilot_order_changes_no_bits)
        np.testing.assert_array_equal(bits(got), bits(exp), err_msg=f"render {k}")
        np.testing.assert_array_equal(rt.getSeeds(), sd, err_msg=f"render {k}")
        cnt = rt.counters()
        assert (cnt["rays_closest"], cnt["rays_shadow"]) == c_or
    rt.close()


def test_dragon_8way_tile_sr16_whole_tile_vs_bvh_oracle(tracer, pt, oracle, dragon):
    """One whole 8-way row-stripe tile (stripe 8, rank 3 of 8: BASELINE configs[4]'s sharding)
    of the headline frame at its own sampleRate 16 (256 spp): the sample-split path — speculated
    mesh pixels' chunks, the long chains' 8-lane subtree-parallel seed pass and single-sample
    chunks on the second stream (their box segments answered from the seed pass's mesh-hit
    depths), the repair pass of the speculated pixels whose camera rays missed, the in-order sums
    per part — against the oracle on every pixel and seed slot of the tile."""
    d = dragon
    tile = (8, 8, 3)
    rows = _tile_rows(d["H"], tile)
    rt = _tracer(pt, d, 16)
    got = np.zeros(len(rows) * d["W"] * 4, np.float32)
    rt.rayTrace(got, d["W"], d["H"], 0, kernel=2, tile=tile)
    info = rt.renderInfo()
    assert info["split_chunks"] == 16 and info["split_coop"] == 8 and info["split_spec"] == 1, info
    assert info["split_guard"] == 0 and info["pixels_long"] >= 1000, info
    assert info["split_repaired"] > 0, info  # the repair pass ran on this tile
    assert info["split_hit_depth"] == 1, info  # the long chains' box segments answered from the seed pass
    got_seeds = rt.getSeeds()
    rt.close()
    pix = (rows[:, None] * d["W"] + np.arange(d["W"])[None, :]).reshape(-1).astype(np.uint32)
    exp = np.zeros(d["W"] * d["H"] * 4, np.float32)
    sd = d["seeds"].copy()
    oracle.render_tris(exp, d["cam"], d["S"], d["W"], d["H"], d["Wp"], d["Hp"], 16, 6, 0, sd, d["verts"], d["idx"],
                       pixels=pix, bvh=d["bvh"])
    _check_tile(got, got_seeds, exp, sd, d, rows)


def test_dragon_balanced_8way_tile_sr16_whole_tile_vs_bvh_oracle(tracer, pt, oracle, dragon):
    """The headline frame's 8-way partition by probed stripe cost (rt_partition_stripes: a whole-frame
    probe, LPT over the 135 stripes — bench.py's default at N > 1): a valid owner map, the same from a
    fresh context, and the tile of the rank holding the frame's top stripe (where the box pixels'
    long chains crowd) at sampleRate 16 equal to the oracle on every pixel and seed slot — the
    tile-local rows map to the frame's rows and seed slots through the owner map
    (RtTriLaunch::stripe_map)."""
    d = dragon
    rt = _tracer(pt, d, 16)
    owner = rt.partitionStripes(d["W"], d["H"], 8, 8)
    assert owner.shape == (135,) and owner.max() < 8 and len(set(owner.tolist())) == 8
    rt2 = _tracer(pt, d, 16)
    np.testing.assert_array_equal(rt2.partitionStripes(d["W"], d["H"], 8, 8), owner)  # deterministic
    rt2.close()
    tile = (8, 8, int(owner[0]), owner)
    rows = _tile_rows(d["H"], tile)
    assert 0 in rows and not np.array_equal(rows, _tile_rows(d["H"], (8, 8, int(owner[0]))))
    got = np.zeros(len(rows) * d["W"] * 4, np.float32)
    rt.rayTrace(got, d["W"], d["H"], 0, kernel=2, tile=tile)
    info = rt.renderInfo()
    assert info["split_chunks"] == 16 and info["split_guard"] == 0 and info["pixels_long"] >= 1000, info
    got_seeds = rt.getSeeds()
    rt.close()
    pix = (rows[:, None] * d["W"] + np.arange(d["W"])[None, :]).reshape(-1).astype(np.uint32)
    exp = np.zeros(d["W"] * d["H"] * 4, np.float32)
    sd = d["seeds"].copy()
    oracle.render_tris(exp, d["cam"], d["S"], d["W"], d["H"], d["Wp"], d["Hp"], 16, 6, 0, sd, d["verts"], d["idx"],
                       pixels=pix, bvh=d["bvh"])
    _check_tile(got, got_seeds, exp, sd, d, rows)


def test_balanced_partition_evens_out_the_long_chains(pt, dragon):
    """What the cost-aware partition is for: under interleaved 8-row stripes the 8 ranks'
    long chains (box pixels, serial sample chains) run from ~7,400 down to ~4,900 — the box pixels
    crowd the frame's top rows — and the slowest rank follows them.  Under rt_partition_stripes' map
    every rank's count is within 10 % of the mean."""
    d = dragon
    rt = _tracer(pt, d, 16)
    owner = rt.partitionStripes(d["W"], d["H"], 8, 8)
    counts = {}
    for name, own in (("interleaved", None), ("balanced", owner)):
        c = []
        for r in range(8):
            rows = _tile_rows(d["H"], (8, 8, r, own))
            buf = np.zeros(len(rows) * d["W"] * 4, np.float32)
            rt.rayTrace(buf, d["W"], d["H"], 0, kernel=2, tile=(8, 8, r, own))
            c.append(rt.renderInfo()["pixels_long"])
        counts[name] = np.array(c, np.float64)
    rt.close()
    spread = {k: (v.max() - v.min()) / v.mean() for k, v in counts.items()}
    assert spread["balanced"] < 0.2 and counts["balanced"].max() < 1.1 * counts["balanced"].mean(), counts
    assert spread["balanced"] < spread["interleaved"], counts


def test_split_buffers_regrown_with_repairs_vs_oracle(pt, dragon, dragon_sr4, monkeypatch):
    """One context renders an 8-way tile and then the whole frame, both sample-split (RT_SPLIT=1)
    at sampleRate 4 with every probe-hit pixel speculated (RT_SPLIT_SPEC=2: silhouettes too, so
    many repairs) and only 4 per-sample repair slots (RT_REPAIR_SLOTS=4: the repairs beyond
    them take the per-pixel seeds, split_item_base > 0).  The whole frame has more long chains
    than the tile, so their seed buffer is regrown between the two renders, while the repair
    buffer from the first render is kept (the regrowth freed it and left it in use).
    Both renders equal the oracle on every pixel and seed slot."""
    monkeypatch.setenv("RT_SPLIT", "1")
    monkeypatch.setenv("RT_SPLIT_SPEC", "2")
    monkeypatch.setenv("RT_REPAIR_SLOTS", "4")
    d = dragon
    exp, sd_exp, _ = dragon_sr4
    rt = _tracer(pt, d, 4)  # the knobs are read when the context is created
    tile = (8, 8, 5)
    rows = _tile_rows(d["H"], tile)
    got = np.zeros(len(rows) * d["W"] * 4, np.float32)
    rt.rayTrace(got, d["W"], d["H"], 0, kernel=2, tile=tile)
    i1 = rt.renderInfo()
    assert i1["split_chunks"] > 0 and i1["split_spec"] == 1 and i1["split_guard"] == 0, i1
    assert i1["split_repaired"] > 4, i1
    _check_tile(got, rt.getSeeds(), exp, sd_exp, d, rows)
    rt.setSeeds(d["Wp"], d["Hp"], d["seeds"])
    got = np.zeros(d["W"] * d["H"] * 4, np.float32)
    rt.rayTrace(got, d["W"], d["H"], 0, kernel=2)
    i2 = rt.renderInfo()
    assert i2["split_chunks"] > 0 and i2["split_guard"] == 0, i2
    assert i2["pixels_long"] > i1["pixels_long"] and i2["split_repaired"] > i1["split_repaired"], (i1, i2)
    np.testing.assert_array_equal(bits(got), bits(exp))
    np.testing.assert_array_equal(rt.getSeeds(), sd_exp)
    rt.close()
