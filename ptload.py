"""Import helper for the `pathtracer.cl_amd/` package (its directory name contains a dot).

    import ptload
    pt = ptload.load()          # the package, registered as `pathtracer_cl_amd`
    rt = pt.RayTracer(0)
"""
from __future__ import annotations

import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG_DIR = ROOT / "pathtracer.cl_amd"
NAME = "pathtracer_cl_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(NAME, PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        del sys.modules[NAME]
        raise
    return mod


def submodule(name: str):
    load()
    return importlib.import_module(f"{NAME}.{name}")
