"""MI355X-native path tracer — drop-in for the per-pixel kernel of krisher/PathTracer.cl.

The product is the C-ABI library `librtmi.so` (include/pathtracer_rt.h) built from
`csrc/` for gfx950; this package is its Python host mirror:

- `RayTracer`   the reference's RayTracer / RayTracerCL API (raytracer.py)
- `scenes`      the reference scenes, seeds, camera helper and synthetic meshes
- `dist`        one-process-per-GPU row-stripe rendering with an RCCL gather

Loading fails loudly when librtmi.so is missing — there is no CPU fallback.
The package directory is `pathtracer.cl_amd/`; import it through `ptload.load()`
(a dotted directory name is not a plain Python identifier).
"""
from . import _abi, scenes
from ._abi import RtError, load as load_library
from .raytracer import RayTracer

__all__ = ["RayTracer", "RtError", "scenes", "load_library"]
