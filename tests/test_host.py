"""Host-side logic and the C-ABI library, CPU only (no compute calls need a GPU here)."""
from __future__ import annotations

import ctypes
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, gpu_available

HEADER = ROOT / "include" / "pathtracer_rt.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(pt):
    lib = pt.load_library()
    names = declared_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), f"librtmi.so does not export {n}"
        assert n in pt._abi.SIGNATURES, f"_abi.py does not bind {n}"
    nm = subprocess.run(["nm", "-D", "--defined-only", str(pt._abi.LIB_PATH)], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (rt_\w+)", nm))
    assert set(names) <= exported


def test_library_is_gfx950_code_object(pt):
    """The fat binary embeds a gfx950 (and only gfx950) device code object.  (Bare arch names
    such as "gfx942" do occur as host-side strings: rocPRIM's target-architecture table.)"""
    import re as _re

    data = pt._abi.LIB_PATH.read_bytes()
    targets = set(_re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", data))
    assert targets == {b"gfx950"}


def test_struct_layouts_match_reference(pt):
    ab = pt._abi
    assert ab.SPHERE_DTYPE.itemsize == 80 and ab.SPHERE_DTYPE.fields["center"][1] == 64
    assert ab.SPHERE_DTYPE.fields["emission_power"][1] == 44 and ab.SPHERE_DTYPE.fields["refExp"][1] == 60
    assert ab.RAY_DTYPE.itemsize == 60 and ab.RAY_DTYPE.fields["diffuse_bounce"][1] == 56


def test_glibc_rand_stream_matches_libc(pt):
    """rt_glibc_rand_fill restates glibc random(): compare with this libc's own rand()."""
    prog = r"""
import ctypes, sys
libc = ctypes.CDLL("libc.so.6")
print(" ".join(str(libc.rand()) for _ in range(5000)))
"""
    got = subprocess.run([__import__("sys").executable, "-c", prog], capture_output=True, text=True, check=True)
    libc_vals = np.array([int(v) for v in got.stdout.split()], np.uint32)
    np.testing.assert_array_equal(pt.scenes.glibc_rand(5000), libc_vals)
    np.testing.assert_array_equal(pt.scenes.glibc_rand(100, skip=4900), libc_vals[4900:])
    seeds = pt.scenes.default_seeds(64, 8)
    assert seeds.size == 2 * 64 * 8 and seeds.min() >= 2


@pytest.mark.parametrize("w,h,ndy,exp", [(512, 512, 8, (512, 512)), (1920, 1080, 8, (1920, 1080)),
                                        (1000, 1001, 8, (1024, 1008)), (33, 7, 32, (64, 32)), (64, 48, 16, (64, 48))])
def test_padded_dims(pt, w, h, ndy, exp):
    assert pt.scenes.padded_dims(w, h, ndy) == exp


@pytest.mark.parametrize("n", [1, 2, 7, 2000, 69_451])
def test_mesh_generator(pt, n):
    v, i = pt.scenes.make_mesh(n)
    assert i.shape == (n, 3) and np.isfinite(v).all()
    assert i.min() >= 0 and i.max() < len(v)
    if n >= 2000:
        a, b, c = v[i[:, 0]], v[i[:, 1]], v[i[:, 2]]
        nrm = np.cross(c - a, b - a)  # the reference's normal cross(e2, e1)
        outward = ((a - np.array(pt.scenes.MESH_CENTER, np.float32)) * nrm).sum(1)
        assert (outward > 0).mean() > 0.97
        assert v[:, 1].min() > -5.0  # rests inside the box floor
    v2, i2 = pt.scenes.make_mesh(n)
    assert v.tobytes() == v2.tobytes() and i.tobytes() == i2.tobytes()


def test_mesh_visibility_by_class(pt):
    """det >= 1e-4 (geometryFuncs.h:167) is absolute: record how many triangles can ever pass."""
    for name, expect_lo, expect_hi in [("bunny", 0.95, 1.0), ("dragon", 0.5, 1.0)]:
        v, i = pt.scenes.make_mesh(pt.scenes.MESH_CONFIGS[name])
        a, b, c = v[i[:, 0]], v[i[:, 1]], v[i[:, 2]]
        twice_area = np.linalg.norm(np.cross(b - a, c - a), axis=1)
        frac = (twice_area >= 1e-4).mean()
        assert expect_lo <= frac <= expect_hi, (name, frac)


@pytest.mark.parametrize("H,stripe,n", [(1080, 8, 1), (1080, 8, 2), (1080, 8, 8), (53, 5, 3), (7, 16, 4)])
def test_tile_rows_partition(pt, H, stripe, n):
    dist = __import__("ptload").submodule("dist")
    lib = pt.load_library()
    seen = []
    for r in range(n):
        rows = dist.tile_rows(H, stripe, n, r)
        t = pt._abi.RtTile(stripe, n, r)
        assert lib.rt_tile_rows(H, ctypes.byref(t)) == len(rows)
        assert np.all(np.diff(rows) > 0)
        seen.append(rows)
    allr = np.sort(np.concatenate(seen))
    np.testing.assert_array_equal(allr, np.arange(H))


def test_assemble_roundtrip():
    dist = __import__("ptload").submodule("dist")
    H, W, stripe, n = 37, 5, 4, 3
    full = np.random.default_rng(0).random((H, W, 4)).astype(np.float32)
    tiles = [full[dist.tile_rows(H, stripe, n, r)] for r in range(n)]
    np.testing.assert_array_equal(dist.assemble(tiles, H, W, stripe), full)


@pytest.mark.parametrize("H,stripe,n,seed", [(1080, 8, 8, 0), (1083, 8, 3, 1), (53, 5, 4, 2), (7, 16, 4, 3),
                                             (64, 8, 5, 4)])
def test_tile_rows_owner_map(pt, H, stripe, n, seed):
    """rt_tile with a stripe-owner map (rt_partition_stripes' output form): rt_tile_rows equals
    dist.tile_rows for every rank — including ranks that own no stripe and a short last stripe —
    the ranks' rows cover the frame once, and compact tiles assemble back to the frame."""
    dist = __import__("ptload").submodule("dist")
    lib = pt.load_library()
    ns = (H + stripe - 1) // stripe
    rng = np.random.default_rng(seed)
    owner = rng.integers(0, max(n - 1, 1), ns).astype(np.uint32)  # rank n - 1 owns nothing
    seen = []
    for r in range(n):
        rows = dist.tile_rows(H, stripe, n, r, owner)
        t, _keep = pt._abi.tile_struct((stripe, n, r, owner))
        assert lib.rt_tile_rows(H, ctypes.byref(t)) == len(rows)
        assert np.all(np.diff(rows) > 0)
        np.testing.assert_array_equal(dist.row_owner(H, stripe, n, owner)[rows], r)
        seen.append(rows)
    np.testing.assert_array_equal(np.sort(np.concatenate(seen)), np.arange(H))
    W = 3
    full = rng.random((H, W, 4)).astype(np.float32)
    tiles = [full[rows] for rows in seen]
    np.testing.assert_array_equal(dist.assemble(tiles, H, W, stripe, owner), full)


def test_lpt_owner_rule():
    """dist.lpt_owner — the rule rt_partition_stripes applies to its probed stripe costs: costliest
    stripe first (ties: lower index) to the least-loaded rank (ties: lower rank)."""
    dist = __import__("ptload").submodule("dist")
    np.testing.assert_array_equal(dist.lpt_owner([5, 9, 1, 9, 3], 2), [0, 0, 1, 1, 1])
    np.testing.assert_array_equal(dist.lpt_owner([1, 1, 1, 1], 4), [0, 1, 2, 3])
    rng = np.random.default_rng(7)
    c = rng.integers(1, 1000, 135)
    own = dist.lpt_owner(c, 8)
    loads = np.bincount(own, weights=c, minlength=8)
    assert loads.max() - loads.min() <= c.max()  # LPT: within one stripe of each other


def test_fails_loudly_without_gpu(pt):
    if gpu_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(pt.RtError):
        pt.RayTracer(0)


def test_camera_helper_defaults(pt):
    cam = pt.scenes.camera_spherical(512, **pt.scenes.MAIN_CAMERA).reshape(4, 4)
    # SURVEY.md §8a a27 probe values (main.cpp camera, 512 wide)
    np.testing.assert_allclose(cam[3, :3], [4.283601, -2.79039, 2.277631], rtol=1e-6)
    np.testing.assert_allclose(cam[0, :3], [-439.8886, -124.2164, -233.893], rtol=1e-6)
    assert np.all(cam[:, 3] == 0)
