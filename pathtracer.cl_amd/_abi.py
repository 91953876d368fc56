"""ctypes binding of librtmi.so — the C-ABI boundary declared in include/pathtracer_rt.h.

This is the binding a Python host would add to drop the MI355X path tracer in
for RayTracerCL (clrt/RayTracerCL.h:111-112).  Structured numpy dtypes mirror
the byte layouts of include/rt_types.h (clrt/ocl/geometry.h:63-163).

There is deliberately no fallback: if librtmi.so is missing or fails to load,
`load()` raises.  Build it with `python __graft_entry__.py` or
`make -C pathtracer.cl_amd/csrc`.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "librtmi.so"

# --- status / enums (pathtracer_rt.h) -------------------------------------------------
RT_OK = 0
RT_ERR_ARG = -1
RT_ERR_HIP = -2
RT_ERR_NO_SCENE = -3
RT_ERR_NO_MESH = -4
RT_ERR_ALLOC = -5
RT_ERR_STATE = -6
RT_ERR_LIMIT = -7

RT_KERNEL_SPHERES = 0
RT_KERNEL_SPHERES_SS = 1
RT_KERNEL_TRIS = 2

RT_TRAVERSAL_BVH = 0
RT_TRAVERSAL_LINEAR = 1
RT_TRAVERSAL_BVH4F = 4

RT_BUILD_HOST = 0
RT_BUILD_GPU = 1

RT_OUT_DEVICE = 1
RT_SEEDS_HALO = 2

# --- record layouts (rt_types.h) --------------------------------------------------------
VEC3 = ("<f4", 3)
SPHERE_DTYPE = np.dtype(
    [
        ("diffuse", *VEC3),
        ("kd", "<f4"),
        ("extinction", *VEC3),
        ("kt", "<f4"),
        ("emission", *VEC3),
        ("emission_power", "<f4"),
        ("ks", "<f4"),
        ("specExp", "<f4"),
        ("ior", "<f4"),
        ("refExp", "<f4"),
        ("center", *VEC3),
        ("radius", "<f4"),
    ]
)
assert SPHERE_DTYPE.itemsize == 80

RAY_DTYPE = np.dtype(
    [
        ("o", *VEC3),
        ("d", *VEC3),
        ("tmin", "<f4"),
        ("tmax", "<f4"),
        ("propagation", *VEC3),
        ("extinction", *VEC3),
        ("diffuse_bounce", "<u4"),
    ]
)
assert RAY_DTYPE.itemsize == 60

# Camera = 4 x float4 (view, up, right, position); kept as a (16,) float32 array.
CAMERA_FLOATS = 16


class RtTile(ctypes.Structure):
    """rt_tile: stripe s of the frame belongs to rank stripe_owner[s] (a uint32 array of
    ceil(H / stripe_rows) entries), or with stripe_owner NULL to rank s % n_ranks."""
    _fields_ = [("stripe_rows", ctypes.c_uint32), ("n_ranks", ctypes.c_uint32), ("rank", ctypes.c_uint32),
                ("stripe_owner", ctypes.c_void_p)]


def tile_struct(tile):
    """RtTile from (stripe, n_ranks, rank) or (stripe, n_ranks, rank, owner), owner a uint32 array
    (or None); returns (struct, the owner array it points into, to be kept alive)."""
    if tile is None:
        return None, None
    stripe, n, r = (int(v) for v in tile[:3])
    owner = tile[3] if len(tile) > 3 else None
    if owner is None:
        return RtTile(stripe, n, r, None), None
    o = np.ascontiguousarray(owner, np.uint32)
    return RtTile(stripe, n, r, o.ctypes.data), o


class RtMeshStats(ctypes.Structure):
    _fields_ = [("n_tris", ctypes.c_uint32), ("n_nodes2", ctypes.c_uint32), ("depth2", ctypes.c_uint32),
                ("n_nodes4", ctypes.c_uint32), ("depth4", ctypes.c_uint32), ("stack4", ctypes.c_uint32),
                ("build_seconds", ctypes.c_double), ("builder", ctypes.c_uint32), ("n_tris_tree", ctypes.c_uint32),
                ("n_nodes4_shadow", ctypes.c_uint32)]


class RtCounters(ctypes.Structure):
    _fields_ = [
        ("rays_closest", ctypes.c_uint64),
        ("rays_shadow", ctypes.c_uint64),
        ("nodes_visited", ctypes.c_uint64),
        ("tris_tested", ctypes.c_uint64),
        ("leaves_visited", ctypes.c_uint64),
        ("lane_slots", ctypes.c_uint64),
        ("clocks_traversal", ctypes.c_uint64),
        ("clocks_total", ctypes.c_uint64),
        ("pixel_clocks_max", ctypes.c_uint64),
        ("pixel_rays_max", ctypes.c_uint64),
        ("pixel_steps_max", ctypes.c_uint64),
        ("rays_skipped", ctypes.c_uint64),
        ("clocks_shade", ctypes.c_uint64),
        ("pixels_long", ctypes.c_uint64),
    ]


class RtRenderInfo(ctypes.Structure):
    _fields_ = [
        ("kernel", ctypes.c_uint32),
        ("traversal", ctypes.c_uint32),
        ("grid_blocks", ctypes.c_uint32),
        ("lists", ctypes.c_uint32),
        ("list_capacity", ctypes.c_uint64),
        ("list_records", ctypes.c_uint64),
        ("list_pixels_tree", ctypes.c_uint32),
        ("pixels_long", ctypes.c_uint32),
        ("schedule_rebuilt", ctypes.c_uint32),
        ("lists_rebuilt", ctypes.c_uint32),
        ("schedule_host_ms", ctypes.c_double),
        ("split_chunks", ctypes.c_uint32),
        ("split_coop", ctypes.c_uint32),
        ("split_guard", ctypes.c_uint32),
        ("split_spec", ctypes.c_uint32),
        ("split_repaired", ctypes.c_uint32),
        ("split_hit_depth", ctypes.c_uint32),
        ("schedule_measured", ctypes.c_uint32),
        ("schedule_pilot", ctypes.c_uint32),
    ]


# Every symbol the header declares, with its ctypes signature.
_vp, _u32, _i32, _f32, _sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
SIGNATURES = {
    "rt_create": (_i32, [_i32, ctypes.POINTER(_vp)]),
    "rt_destroy": (_i32, [_vp]),
    "rt_last_error": (ctypes.c_char_p, [_vp]),
    "rt_status_string": (ctypes.c_char_p, [_i32]),
    "rt_set_spheres": (_i32, [_vp, _vp, _u32]),
    "rt_set_mesh": (_i32, [_vp, _vp, _u32, _vp, _u32]),
    "rt_mesh_info": (_i32, [_vp, ctypes.POINTER(RtMeshStats)]),
    "rt_set_view_matrix": (_i32, [_vp, _vp]),
    "rt_set_camera_spherical": (_i32, [_vp, _f32, _f32, _f32, _f32, _f32, _f32]),
    "rt_set_fov": (_i32, [_vp, _f32]),
    "rt_set_camera": (_i32, [_vp, _vp]),
    "rt_camera_spherical": (_i32, [_f32, _f32, _f32, _f32, _f32, _f32, _f32, _u32, _vp]),
    "rt_set_params": (_i32, [_vp, _u32, _u32]),
    "rt_set_traversal": (_i32, [_vp, _i32]),
    "rt_set_builder": (_i32, [_vp, _i32]),
    "rt_set_ndrange": (_i32, [_vp, _u32]),
    "rt_set_seed_layout": (_i32, [_vp, _u32, _u32]),
    "rt_set_seeds": (_i32, [_vp, _vp, _sz]),
    "rt_get_seeds": (_i32, [_vp, _vp, _sz]),
    "rt_seed_layout": (_i32, [_vp, ctypes.POINTER(_u32), ctypes.POINTER(_u32)]),
    "rt_glibc_rand_fill": (_i32, [_u32, _vp, _sz, _u32]),
    "rt_pack_seed_rows": (_i32, [_vp, _vp, _u32, _vp, _i32]),
    "rt_unpack_seed_rows": (_i32, [_vp, _vp, _u32, _vp, _i32]),
    "rt_render": (_i32, [_vp, _vp, _u32, _u32, _u32, _i32, ctypes.POINTER(RtTile), _i32]),
    "rt_render_async": (_i32, [_vp, _vp, _u32, _u32, _u32, _i32, ctypes.POINTER(RtTile), _i32, _vp]),
    "rt_synchronize": (_i32, [_vp]),
    "rt_tile_rows": (_u32, [_u32, ctypes.POINTER(RtTile)]),
    "rt_partition_stripes": (_i32, [_vp, _u32, _u32, _u32, _u32, _vp, ctypes.POINTER(_i32)]),
    "rt_read": (_i32, [_vp, _vp, _sz]),
    "rt_get_counters": (_i32, [_vp, ctypes.POINTER(RtCounters)]),
    "rt_set_counting": (_i32, [_vp, _i32]),
    "rt_counter_totals": (_i32, [_vp, ctypes.POINTER(RtCounters), ctypes.POINTER(ctypes.c_uint64), _i32]),
    "rt_last_kernel_ms": (_i32, [_vp, ctypes.POINTER(_f32)]),
    "rt_last_kernel_split_ms": (_i32, [_vp, ctypes.POINTER(_f32), ctypes.POINTER(_f32)]),
    "rt_last_render_info": (_i32, [_vp, ctypes.POINTER(RtRenderInfo)]),
    "rt_last_long_chains": (_i32, [_vp, _vp, _u32, ctypes.POINTER(_u32)]),
    "rt_trace_rays": (_i32, [_vp, _vp, _u32, _i32, _vp, _vp]),
    "rt_mesh_vertex_count": (_u32, [_u32]),
    "rt_make_mesh": (_i32, [_u32, _f32, _f32, _f32, _f32, _vp, _vp]),
    "rt_ply_open": (_i32, [ctypes.c_char_p, ctypes.POINTER(_vp), ctypes.POINTER(_u32), ctypes.POINTER(_u32)]),
    "rt_ply_read": (_i32, [_vp, _vp, _vp]),
    "rt_ply_dropped_faces": (_u32, [_vp]),
    "rt_ply_close": (_i32, [_vp]),
    "rt_ply_last_error": (ctypes.c_char_p, []),
    "rt_normalize_mesh": (_i32, [_vp, _u32, _f32, _f32]),
    # multi-GPU from the native host (csrc/rt_comm.hip, RCCL)
    "rt_comm_get_unique_id": (_i32, [_vp]),
    "rt_comm_create": (_i32, [_vp, _i32, _i32, _i32, ctypes.POINTER(_vp)]),
    "rt_comm_destroy": (_i32, [_vp]),
    "rt_comm_last_error": (ctypes.c_char_p, [_vp]),
    "rt_comm_count": (_i32, [_vp, ctypes.POINTER(_i32)]),
    "rt_comm_gather_frame": (_i32, [_vp, _vp, _vp, _u32, _u32, _u32, _vp, _i32]),
    "rt_assemble_tiles": (_i32, [_vp, _u32, _u32, _u32, _u32, _vp, _vp, _i32]),
    "rt_seed_halo_plan": (_i32, [_vp, _u32, _u32, _u32, _u32, _vp, _u32, _vp, _vp, _vp, ctypes.POINTER(_u32)]),
    "rt_seed_halo_peer_blocks": (_i32, [_vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp, _vp, _vp]),
    "rt_comm_render": (_i32, [_vp, _vp, _vp, _u32, _u32, _u32, _i32, _u32, _i32]),
    "rt_comm_reset_halo": (_i32, [_vp]),
    "rt_comm_set_partition": (_i32, [_vp, _i32]),
    "rt_comm_last_partition": (_i32, [_vp, _vp, _u32, ctypes.POINTER(_u32)]),
}
RT_PARTITION_INTERLEAVED = 0
RT_PARTITION_BALANCED = 1
RT_COMM_ID_BYTES = 128

_LIB = None


def load(path: str | os.PathLike | None = None) -> ctypes.CDLL:
    """Load librtmi.so (in-tree).  Raises if it is absent: there is no CPU fallback."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    # RTMI_LIB: an alternative in-tree build of the same library (A/B experiments)
    p = Path(path) if path else Path(os.environ.get("RTMI_LIB", LIB_PATH))
    if not p.exists():
        raise RuntimeError(
            f"{p} not found: the HIP library is required (build with `python __graft_entry__.py` "
            "or `make -C pathtracer.cl_amd/csrc`); there is no CPU fallback"
        )
    lib = ctypes.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if p == LIB_PATH:
                raise RuntimeError(f"{p} lacks {name}: rebuild it (`make -C pathtracer.cl_amd/csrc`)")
            continue  # an older build loaded for an A/B run: only its own entry points
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _LIB = lib
    return lib


def ptr(a) -> ctypes.c_void_p | None:
    """Raw pointer of a numpy array (host) or a torch tensor (device or host)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return ctypes.c_void_p(a.ctypes.data)
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    if isinstance(a, int):
        return ctypes.c_void_p(a)
    raise TypeError(f"cannot take the address of {type(a)!r}")


class RtError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"librtmi status {status}: {msg}")
        self.status = status
