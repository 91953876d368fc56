"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

- `Oracle`     — oracle/liboracle.so, the C restatement of the reference kernel
                 (oracle/pt_oracle.c).  Used by tests/, __graft_entry__.smoke() and the
                 cpu_baseline leg of bench.py — never by the product path.
- `Reference`  — oracle/_ref/libptref.so, the reference's own clrt/ocl/raytracer.cl compiled
                 for x86-64 (oracle/Makefile `ref`; needs /root/reference, container only).

Both take the same numpy records as librtmi (pathtracer.cl_amd/_abi.py dtypes).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIBORACLE = ORACLE_DIR / "liboracle.so"
LIBREF = ORACLE_DIR / "_ref" / "libptref.so"
LIBREF_LIBM = ORACLE_DIR / "_ref_libm" / "libptref.so"  # the same reference, glibc transcendentals
REFERENCE_ROOT = Path("/root/reference")

KERNEL_SPHERES, KERNEL_SPHERES_SS, KERNEL_TRIS = 0, 1, 2


class Counters(ctypes.Structure):
    _fields_ = [("closest", ctypes.c_uint64), ("shadow", ctypes.c_uint64)]


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def build(ref: bool = False) -> None:
    """Compile liboracle.so (and, if /root/reference exists and ref=True, oracle/_ref)."""
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)
    if ref and REFERENCE_ROOT.exists():
        subprocess.run(["make", "-s", "-C", str(ORACLE_DIR), "ref"], check=True)


class Oracle:
    def __init__(self, path: os.PathLike | None = None):
        p = Path(path) if path else LIBORACLE
        if not p.exists():
            build()
        self.lib = ctypes.CDLL(str(p))
        L = self.lib
        vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
        L.or_render_spheres.argtypes = [vp, vp, vp, u32, u32, u32, u32, u32, u32, u32, u32, vp, i32, i32, vp]
        L.or_render_spheres.restype = i32
        L.or_render_tris.argtypes = [vp, vp, vp, u32, u32, u32, u32, u32, u32, u32, u32, vp, vp, vp, u32, vp, u32,
                                     u32, i32, vp]
        L.or_render_tris.restype = i32
        L.or_closest_hits.argtypes = [vp, u32, vp, vp, u32, vp, vp]
        L.or_any_hits.argtypes = [vp, u32, vp, vp, u32, vp]
        L.or_render_tris_bvh.argtypes = L.or_render_tris.argtypes + [vp]
        L.or_render_tris_bvh.restype = i32
        L.or_bvh_build.argtypes = [vp, u32, vp, u32]
        L.or_bvh_build.restype = vp
        L.or_bvh_free.argtypes = [vp]
        L.or_bvh_free.restype = None
        L.or_bvh_nodes.argtypes = [vp]
        L.or_bvh_nodes.restype = u32
        L.or_bvh_depth.argtypes = [vp]
        L.or_bvh_depth.restype = u32
        L.or_closest_hits_bvh.argtypes = [vp, u32, vp, vp, vp, vp, vp]
        L.or_any_hits_bvh.argtypes = [vp, u32, vp, vp, vp, vp]
        for f in ("sin", "cos", "exp", "log"):
            fn = getattr(L, f"or_math_{f}")
            fn.argtypes = [ctypes.c_float]
            fn.restype = ctypes.c_float
        L.or_math_pow.argtypes = [ctypes.c_float, ctypes.c_float]
        L.or_math_pow.restype = ctypes.c_float
        L.or_math_vec.argtypes = [i32, vp, vp, vp, ctypes.c_size_t]
        L.or_math_vec.restype = None

    def render_spheres(self, out, cam, spheres, W, H, Wpad, Hpad, sample_rate, max_depth, progressive, seeds,
                       single_sample=False, nthreads=None):
        c = Counters()
        nthreads = nthreads or _threads()
        st = self.lib.or_render_spheres(_p(out), _p(cam), _p(spheres), len(spheres), W, H, Wpad, Hpad, sample_rate,
                                        max_depth, progressive, _p(seeds), int(single_sample), nthreads,
                                        ctypes.byref(c))
        assert st == 0
        return c.closest, c.shadow

    def render_tris(self, out, cam, spheres, W, H, Wpad, Hpad, sample_rate, max_depth, progressive, seeds, verts,
                    idx, pixels=None, max_samples=0, nthreads=None, bvh: "MeshBVH | None" = None):
        """raytrace_tris (raytracer.cl:184-243); bvh=None: the reference's linear loops, else the
        independent BVH mode over the same mesh (same results, O(log N) per ray)."""
        c = Counters()
        nthreads = nthreads or _threads()
        n_tris = idx.size // 3
        if pixels is not None:
            pixels = np.ascontiguousarray(pixels, np.uint32)  # a strided view would pass other pixels
        npx = 0 if pixels is None else len(pixels)
        args = (_p(out), _p(cam), _p(spheres), len(spheres), W, H, Wpad, Hpad, sample_rate, max_depth, progressive,
                _p(seeds), _p(verts), _p(idx), n_tris, _p(pixels), npx, max_samples, nthreads, ctypes.byref(c))
        if bvh is None:
            st = self.lib.or_render_tris(*args)
        else:
            assert bvh.n_tris == n_tris
            st = self.lib.or_render_tris_bvh(*args, ctypes.c_void_p(bvh.handle))
        assert st == 0
        return c.closest, c.shadow

    def build_bvh(self, verts, idx) -> "MeshBVH":
        """The oracle's own BVH over the mesh (oracle/pt_oracle.c or_bvh_build)."""
        return MeshBVH(self, verts, idx)

    def closest_hits_bvh(self, rays, bvh):
        n = len(rays)
        oi = np.empty(n, np.int32)
        ot = np.empty(n, np.float32)
        self.lib.or_closest_hits_bvh(_p(rays), n, _p(bvh.verts), _p(bvh.idx), ctypes.c_void_p(bvh.handle), _p(oi),
                                     _p(ot))
        return oi, ot

    def any_hits_bvh(self, rays, bvh):
        n = len(rays)
        oi = np.empty(n, np.int32)
        self.lib.or_any_hits_bvh(_p(rays), n, _p(bvh.verts), _p(bvh.idx), ctypes.c_void_p(bvh.handle), _p(oi))
        return oi

    MATH_FN = {"sin": 0, "cos": 1, "exp": 2, "log": 3, "pow": 4, "sincos_s": 5, "sincos_c": 6}

    def math(self, fn: str, x: np.ndarray, y: float = 0.0) -> np.ndarray:
        """The pinned builtin `fn` (include/rt_math.h) over every element of x (pow: x ** y)."""
        x = np.ascontiguousarray(x, np.float32)
        yy = np.array([y], np.float32)
        out = np.empty_like(x)
        self.lib.or_math_vec(self.MATH_FN[fn], _p(x), _p(yy), _p(out), x.size)
        return out

    def closest_hits(self, rays, verts, idx):
        n = len(rays)
        oi = np.empty(n, np.int32)
        ot = np.empty(n, np.float32)
        self.lib.or_closest_hits(_p(rays), n, _p(verts), _p(idx), idx.size // 3, _p(oi), _p(ot))
        return oi, ot

    def any_hits(self, rays, verts, idx):
        n = len(rays)
        oi = np.empty(n, np.int32)
        self.lib.or_any_hits(_p(rays), n, _p(verts), _p(idx), idx.size // 3, _p(oi))
        return oi


def _threads() -> int:
    """Worker threads for oracle renders: the CPUs this process may run on (the GPU box grants
    a share of a large machine, os.cpu_count() shows all of it), at most 16."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


class MeshBVH:
    """Handle of an or_bvh (the oracle's independent BVH mode); keeps the mesh arrays alive."""

    def __init__(self, orc: Oracle, verts, idx):
        self.lib = orc.lib
        self.verts = np.ascontiguousarray(verts, np.float32)
        self.idx = np.ascontiguousarray(idx, np.int32)
        self.n_tris = self.idx.size // 3
        self.handle = self.lib.or_bvh_build(_p(self.verts), self.verts.size // 3, _p(self.idx), self.n_tris)
        if not self.handle:
            raise ValueError("or_bvh_build failed (empty mesh or index out of range)")
        self.n_nodes = self.lib.or_bvh_nodes(ctypes.c_void_p(self.handle))
        self.depth = self.lib.or_bvh_depth(ctypes.c_void_p(self.handle))

    def close(self):
        if self.handle:
            self.lib.or_bvh_free(ctypes.c_void_p(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Reference:
    """The reference kernel itself (clrt/ocl/raytracer.cl compiled for x86-64) + KAT wrappers."""

    def __init__(self, build_if_missing: bool = True, path: os.PathLike | None = None):
        lib = Path(path) if path else LIBREF
        if not lib.exists() and build_if_missing:
            build(ref=True)
        if not lib.exists():
            raise FileNotFoundError(f"{lib} (needs /root/reference to build)")
        self.lib = ctypes.CDLL(str(lib))
        L = self.lib
        vp, u32, i32, f32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_float
        L.ref_launch_kernel.argtypes = [i32, vp, vp, vp, u32, u32, u32, u32, u32, u32, u32, u32, vp, vp, vp, u32, i32]
        L.ref_launch_kernel.restype = i32
        L.ref_launch_pixels.argtypes = [i32, vp, vp, vp, u32, u32, u32, u32, u32, u32, u32, u32, vp, vp, vp, u32,
                                        vp, u32, i32]
        L.ref_launch_pixels.restype = i32
        L.ref_camera_spherical.argtypes = [f32, f32, f32, f32, f32, f32, f32, u32, vp]
        L.ref_frand_seq.argtypes = [vp, vp, u32]
        L.ref_strat_seq.argtypes = [vp, vp, u32, i32]
        L.ref_intersect_sphere.argtypes = [vp, vp, f32]
        L.ref_intersect_sphere.restype = f32
        L.ref_intersects_box.argtypes = [vp, f32, f32, f32]
        L.ref_intersects_box.restype = f32
        L.ref_box_normal.argtypes = [vp, vp, f32, f32, f32]
        L.ref_intersects_triangle.argtypes = [vp, vp, vp, vp]
        L.ref_intersects_triangle.restype = i32
        L.ref_intersects_triangle_p.argtypes = [vp, vp]
        L.ref_intersects_triangle_p.restype = i32
        L.ref_sphere_emissive.argtypes = [vp, vp, f32, f32, f32]
        L.ref_sample_material.argtypes = [vp, vp, vp, vp]
        L.ref_sample_material.restype = i32
        L.ref_closest_hits.argtypes = [vp, u32, vp, vp, u32, vp, vp]
        L.ref_any_hits.argtypes = [vp, u32, vp, vp, u32, vp]

    def launch(self, kernel, out, cam, spheres, W, H, Wpad, Hpad, sample_rate, max_depth, progressive, seeds,
               verts=None, idx=None, nthreads=8):
        n_tris = 0 if idx is None else idx.size // 3
        st = self.lib.ref_launch_kernel(kernel, _p(out), _p(cam), _p(spheres), len(spheres), W, H, Wpad, Hpad,
                                        sample_rate, max_depth, progressive, _p(seeds), _p(verts), _p(idx), n_tris,
                                        nthreads)
        assert st == 0

    def launch_pixels(self, kernel, out, cam, spheres, W, H, Wpad, Hpad, sample_rate, max_depth, progressive, seeds,
                      pixels, verts=None, idx=None, nthreads=8):
        """The reference kernel on the work-items of `pixels` (y*W + x) only."""
        n_tris = 0 if idx is None else idx.size // 3
        px = np.ascontiguousarray(pixels, np.uint32)
        st = self.lib.ref_launch_pixels(kernel, _p(out), _p(cam), _p(spheres), len(spheres), W, H, Wpad, Hpad,
                                        sample_rate, max_depth, progressive, _p(seeds), _p(verts), _p(idx), n_tris,
                                        _p(px), px.size, nthreads)
        assert st == 0

    def camera_spherical(self, width, target, elevation, azimuth, distance, fov=53.0):
        cam = np.zeros(16, np.float32)
        self.lib.ref_camera_spherical(*[float(t) for t in target], float(elevation), float(azimuth), float(distance),
                                      float(fov), int(width), _p(cam))
        return cam

    def closest_hits(self, rays, verts, idx):
        n = len(rays)
        oi = np.empty(n, np.int32)
        ot = np.empty(n, np.float32)
        self.lib.ref_closest_hits(_p(rays), n, _p(verts), _p(idx), idx.size // 3, _p(oi), _p(ot))
        return oi, ot

    def any_hits(self, rays, verts, idx):
        n = len(rays)
        oi = np.empty(n, np.int32)
        self.lib.ref_any_hits(_p(rays), n, _p(verts), _p(idx), idx.size // 3, _p(oi))
        return oi
