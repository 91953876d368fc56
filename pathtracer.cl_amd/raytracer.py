"""`RayTracer` — the reference's host API over the MI355X C-ABI.

Mirrors clrt/RayTracer.h:51-70 (camera, settings, scene) and RayTracerCL::rayTrace
(clrt/RayTracerCL.h:111-112): same method names, same argument meaning, the same RGBA32F
framebuffer layout (W*H float4, row-major, alpha 0) and the same progression semantics
(0 overwrites, p > 0 mixes with weight 1/p — GlutCLWindow.cpp:144-158).  Errors raise
`RtError`, as the reference throws cl::Error.

The framebuffer may be a numpy array (host) or a torch CUDA tensor on the tracer's device
(rendered in place, no copy).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _abi


class RayTracer:
    KERNEL_SPHERES = _abi.RT_KERNEL_SPHERES
    KERNEL_SPHERES_SS = _abi.RT_KERNEL_SPHERES_SS
    KERNEL_TRIS = _abi.RT_KERNEL_TRIS

    def __init__(self, device: int = 0, lib_path=None):
        # lib_path: another build of librtmi.so (in-process A/B of kernel variants)
        self._lib = _abi.load(lib_path)
        h = ctypes.c_void_p()
        st = self._lib.rt_create(int(device), ctypes.byref(h))
        if st != _abi.RT_OK:
            raise _abi.RtError(st, f"rt_create(device={device}): {self._lib.rt_status_string(st).decode()}")
        self._h = h
        self.device = device
        self._spheres: list[np.ndarray] = []
        self._scene_dirty = True
        self._fov = 53.0
        self._sample_rate = 8
        self._max_depth = 4
        self._mesh = None

    # ---- lifetime --------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._lib.rt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, st: int, what: str):
        if st != _abi.RT_OK:
            detail = self._lib.rt_last_error(self._h).decode(errors="replace")
            raise _abi.RtError(st, f"{what}: {self._lib.rt_status_string(st).decode()} ({detail})")

    # ---- camera (RayTracer.h:56-60) ------------------------------------------------------
    def setCameraMatrix(self, m) -> None:
        """4x4 view matrix (rows = gmtl matrix rows); stored column-major across the ABI."""
        m = np.asarray(m, np.float32).reshape(4, 4)
        colmajor = np.ascontiguousarray(m.T).reshape(-1)
        self._check(self._lib.rt_set_view_matrix(self._h, _abi.ptr(colmajor)), "rt_set_view_matrix")

    def setCameraSpherical(self, target, elevationDeg: float, azimuthDeg: float, distance: float) -> None:
        t = [float(v) for v in target]
        self._check(self._lib.rt_set_camera_spherical(self._h, *t, float(elevationDeg), float(azimuthDeg),
                                                      float(distance)), "rt_set_camera_spherical")

    def setFoVAngle(self, fovDeg: float) -> None:
        self._fov = float(fovDeg)
        self._check(self._lib.rt_set_fov(self._h, self._fov), "rt_set_fov")

    def getFoVAngle(self) -> float:
        return self._fov

    def setCamera(self, cam16) -> None:
        """Explicit Camera struct (view, up, right, position float4s) — fixture replay."""
        cam = np.ascontiguousarray(cam16, np.float32).reshape(16)
        self._check(self._lib.rt_set_camera(self._h, _abi.ptr(cam)), "rt_set_camera")

    # ---- settings (RayTracer.h:62-66) ----------------------------------------------------
    def setSampleRate(self, sampleRate: int) -> None:
        self._sample_rate = int(sampleRate)
        self._check(self._lib.rt_set_params(self._h, self._sample_rate, self._max_depth), "rt_set_params")

    def getSampleRate(self) -> int:
        return self._sample_rate

    def setMaxPathDepth(self, depth: int) -> None:
        self._max_depth = int(depth)
        self._check(self._lib.rt_set_params(self._h, self._sample_rate, self._max_depth), "rt_set_params")

    def getMaxPathDepth(self) -> int:
        return self._max_depth

    def setTraversal(self, linear) -> None:
        """False/"bvh": 4-wide BVH, compressed nodes (default); "bvh4f": the same tree with full-precision
        nodes; True/"linear": the reference loop."""
        t = {False: _abi.RT_TRAVERSAL_BVH, True: _abi.RT_TRAVERSAL_LINEAR, "bvh": _abi.RT_TRAVERSAL_BVH,
             "linear": _abi.RT_TRAVERSAL_LINEAR, "bvh4f": _abi.RT_TRAVERSAL_BVH4F}[linear]
        self._check(self._lib.rt_set_traversal(self._h, t), "rt_set_traversal")

    def setBuilder(self, builder: str) -> None:
        """BVH builder for the next setMesh: "host" (binned SAH, default) or "gpu" (LBVH on the device)."""
        b = {"host": _abi.RT_BUILD_HOST, "gpu": _abi.RT_BUILD_GPU}[builder]
        self._check(self._lib.rt_set_builder(self._h, b), "rt_set_builder")

    def setNDRange(self, nd_y: int) -> None:
        """Work-group height of the reference launch (fixes the padded seed height)."""
        self._check(self._lib.rt_set_ndrange(self._h, int(nd_y)), "rt_set_ndrange")

    # ---- scene (RayTracer.h:68-70) --------------------------------------------------------
    def addSphere(self, sphere) -> None:
        s = np.asarray(sphere, _abi.SPHERE_DTYPE).reshape(-1)
        for rec in s:
            self._spheres.append(rec.copy())
        self._scene_dirty = True

    def removeSphere(self, sphere) -> None:
        """Removes the first sphere equal to `sphere` (a stub in the reference, RayTracer.cpp:55-58)."""
        s = np.asarray(sphere, _abi.SPHERE_DTYPE).reshape(-1)[0]
        for i, rec in enumerate(self._spheres):
            if rec.tobytes() == s.tobytes():
                del self._spheres[i]
                self._scene_dirty = True
                return

    def clearSpheres(self) -> None:
        self._spheres.clear()
        self._scene_dirty = True

    def setSpheres(self, spheres) -> None:
        self.clearSpheres()
        self.addSphere(spheres)

    def setMesh(self, verts, idx) -> None:
        """Triangle mesh for the raytrace_tris kernel; the BVH is built on the host, its cost area
        leaning toward the lights of the spheres added so far (uploaded first; culling only)."""
        self._sync_scene()
        v = np.ascontiguousarray(verts, np.float32).reshape(-1, 3)
        i = np.ascontiguousarray(idx, np.int32).reshape(-1, 3)
        self._check(self._lib.rt_set_mesh(self._h, _abi.ptr(v), v.shape[0], _abi.ptr(i), i.shape[0]), "rt_set_mesh")
        self._mesh = (v.shape[0], i.shape[0])

    def meshInfo(self) -> dict:
        st = _abi.RtMeshStats()
        self._check(self._lib.rt_mesh_info(self._h, ctypes.byref(st)), "rt_mesh_info")
        return {f: getattr(st, f) for f, _ in _abi.RtMeshStats._fields_}

    def _sync_scene(self):
        if self._scene_dirty:
            arr = np.array(self._spheres, dtype=_abi.SPHERE_DTYPE) if self._spheres else np.zeros(0, _abi.SPHERE_DTYPE)
            self._check(self._lib.rt_set_spheres(self._h, _abi.ptr(arr) if len(arr) else None, len(arr)),
                        "rt_set_spheres")
            self._scene_dirty = False

    # ---- seeds (RayTracerCL.cpp:147-171) --------------------------------------------------
    def setSeeds(self, wpad: int, hpad: int, seeds=None) -> None:
        self._check(self._lib.rt_set_seed_layout(self._h, int(wpad), int(hpad)), "rt_set_seed_layout")
        if seeds is not None:
            s = np.ascontiguousarray(seeds, np.uint32).reshape(-1)
            self._check(self._lib.rt_set_seeds(self._h, _abi.ptr(s), s.size), "rt_set_seeds")

    def packSeedRows(self, rows, buf) -> None:
        """Copy seed rows (both planes) into `buf` ([2, n, Wpad] uint32; numpy or torch CUDA)."""
        r = np.ascontiguousarray(rows, np.uint32)
        flags = _abi.RT_OUT_DEVICE if getattr(buf, "is_cuda", False) else 0
        self._check(self._lib.rt_pack_seed_rows(self._h, _abi.ptr(r), r.size, _abi.ptr(buf), flags),
                    "rt_pack_seed_rows")

    def unpackSeedRows(self, rows, buf) -> None:
        """Write seed rows (both planes) from `buf` ([2, n, Wpad] uint32; numpy or torch CUDA)."""
        r = np.ascontiguousarray(rows, np.uint32)
        flags = _abi.RT_OUT_DEVICE if getattr(buf, "is_cuda", False) else 0
        self._check(self._lib.rt_unpack_seed_rows(self._h, _abi.ptr(r), r.size, _abi.ptr(buf), flags),
                    "rt_unpack_seed_rows")

    def getSeeds(self) -> np.ndarray:
        w, h = ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self._lib.rt_seed_layout(self._h, ctypes.byref(w), ctypes.byref(h)), "rt_seed_layout")
        out = np.empty(2 * w.value * h.value, np.uint32)
        self._check(self._lib.rt_get_seeds(self._h, _abi.ptr(out), out.size), "rt_get_seeds")
        return out

    # ---- render (RayTracerCL::rayTrace) ---------------------------------------------------
    def rayTrace(self, out, width: int, height: int, progression: int, kernel: int = _abi.RT_KERNEL_SPHERES,
                 tile: tuple | None = None, stream=None, sync: bool = True, halo: bool = False) -> None:
        """Render into `out` (W*H*4 float32 — or tile rows*W*4 — numpy or torch CUDA tensor).
        tile = (stripe_rows, n_ranks, rank) for interleaved stripes, or (stripe_rows, n_ranks,
        rank, owner) with a per-stripe owner map (partitionStripes).
        halo=True: the caller keeps this tile's seed rows current (dist.SeedHalo), which
        permits progressive sphere frames on a tile."""
        self._sync_scene()
        flags = _abi.RT_SEEDS_HALO if halo else 0
        if not isinstance(out, np.ndarray):
            if getattr(out, "is_cuda", False):
                flags |= _abi.RT_OUT_DEVICE
            if out.dtype.__str__() not in ("torch.float32",):
                raise TypeError("framebuffer must be float32")
            if not out.is_contiguous():
                raise ValueError("framebuffer must be contiguous")
        else:
            if out.dtype != np.float32 or not out.flags["C_CONTIGUOUS"]:
                raise ValueError("framebuffer must be a contiguous float32 array")
        t, _keep = _abi.tile_struct(tile)  # (_keep: the owner map the struct points into)
        rows = self._lib.rt_tile_rows(height, ctypes.byref(t) if t else None)
        need = int(width) * int(rows) * 4
        n = out.size if isinstance(out, np.ndarray) else out.numel()
        if n < need:
            raise ValueError(f"framebuffer holds {n} floats, {need} needed")
        tp = ctypes.byref(t) if t else None
        if sync and stream is None:
            st = self._lib.rt_render(self._h, _abi.ptr(out), int(width), int(height), int(progression), int(kernel),
                                     tp, flags)
            self._check(st, "rt_render")
        else:
            sp = ctypes.c_void_p(stream) if isinstance(stream, int) else stream
            st = self._lib.rt_render_async(self._h, _abi.ptr(out), int(width), int(height), int(progression),
                                           int(kernel), tp, flags, sp)
            self._check(st, "rt_render_async")
            if sync:
                self.synchronize()

    def read(self, host: np.ndarray) -> None:
        """Blocking readback of the last frame into `host` (GlutCLWindow.cpp:214-225)."""
        if host.dtype != np.float32 or not host.flags["C_CONTIGUOUS"]:
            raise ValueError("host buffer must be a contiguous float32 array")
        self._check(self._lib.rt_read(self._h, _abi.ptr(host), host.size), "rt_read")

    def synchronize(self) -> None:
        self._check(self._lib.rt_synchronize(self._h), "rt_synchronize")

    def partitionStripes(self, width: int, height: int, stripe: int, n_ranks: int) -> np.ndarray:
        """rt_partition_stripes: the cost-balanced owner of each of the frame's row stripes for the
        current camera, mesh and lights (a whole-frame probe, LPT over the stripes; cached per view)."""
        self._sync_scene()
        ns = (int(height) + int(stripe) - 1) // int(stripe)
        owner = np.empty(max(ns, 1), np.uint32)
        made = ctypes.c_int(0)
        self._check(self._lib.rt_partition_stripes(self._h, int(width), int(height), int(stripe), int(n_ranks),
                                                   _abi.ptr(owner), ctypes.byref(made)), "rt_partition_stripes")
        return owner[:ns]

    # ---- instrumentation ------------------------------------------------------------------
    def setCounting(self, enable: bool) -> None:
        self._check(self._lib.rt_set_counting(self._h, int(bool(enable))), "rt_set_counting")

    def counters(self) -> dict:
        c = _abi.RtCounters()
        self._check(self._lib.rt_get_counters(self._h, ctypes.byref(c)), "rt_get_counters")
        return {f: getattr(c, f) for f, _ in _abi.RtCounters._fields_}

    def counterTotals(self, reset: bool = True) -> dict:
        """rt_counter_totals: the counters summed over every render since the last reset (waits for
        the renders; frames enqueued back to back each add their own counts), with `renders` = how
        many renders they cover.  Raises if a defect guard fired in any of them."""
        c = _abi.RtCounters()
        n = ctypes.c_uint64(0)
        self._check(self._lib.rt_counter_totals(self._h, ctypes.byref(c), ctypes.byref(n), int(bool(reset))),
                    "rt_counter_totals")
        d = {f: getattr(c, f) for f, _ in _abi.RtCounters._fields_}
        d["renders"] = n.value
        return d

    def lastKernelMs(self) -> float:
        ms = ctypes.c_float()
        self._check(self._lib.rt_last_kernel_ms(self._h, ctypes.byref(ms)), "rt_last_kernel_ms")
        return ms.value

    def lastKernelSplitMs(self) -> tuple[float, float]:
        """(candidate-list pre-pass, main kernel) device times of the last render, ms."""
        pre, main = ctypes.c_float(), ctypes.c_float()
        self._check(self._lib.rt_last_kernel_split_ms(self._h, ctypes.byref(pre), ctypes.byref(main)),
                    "rt_last_kernel_split_ms")
        return pre.value, main.value

    def renderInfo(self) -> dict:
        """rt_last_render_info: the last render's lists, sample split and schedule (no result depends
        on any of it)."""
        fn = getattr(self._lib, "rt_last_render_info", None)
        if fn is None:  # an older library loaded for an A/B run
            return {}
        i = _abi.RtRenderInfo()
        self._check(fn(self._h, ctypes.byref(i)), "rt_last_render_info")
        return {f: getattr(i, f) for f, _ in _abi.RtRenderInfo._fields_}

    def longChains(self) -> np.ndarray:
        """rt_last_long_chains: the last sample-split render's long chains (tile-local y * W + x),
        the pixels whose seed pass ran on the second stream (cooperative queries)."""
        n = ctypes.c_uint32(0)
        self._check(self._lib.rt_last_long_chains(self._h, None, 0, ctypes.byref(n)), "rt_last_long_chains")
        out = np.empty(n.value, np.uint32)
        if n.value:
            self._check(self._lib.rt_last_long_chains(self._h, _abi.ptr(out), n.value, ctypes.byref(n)),
                        "rt_last_long_chains")
        return out

    def traceRays(self, rays: np.ndarray, any_hit: bool = False) -> tuple[np.ndarray, np.ndarray]:
        r = np.ascontiguousarray(rays, _abi.RAY_DTYPE)
        idx = np.empty(r.size, np.int32)
        t = np.empty(r.size, np.float32)
        self._check(self._lib.rt_trace_rays(self._h, _abi.ptr(r), r.size, int(bool(any_hit)), _abi.ptr(idx),
                                            _abi.ptr(t)), "rt_trace_rays")
        return idx, t
