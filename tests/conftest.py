"""Shared test fixtures.

Markers: `gpu` — needs an MI355X (run with `-m gpu` on the GPU box).  Everything else runs
on the CPU-only container: the oracle against the golden fixtures, the host logic, the
C-ABI symbol table and the multi-process (gloo) sharding path.
"""
from __future__ import annotations

import json
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an MI355X GPU (HIP)")


@pytest.fixture(scope="session")
def pt():
    # torch's HIP runtime first: a process whose first HIP call came from librtmi (the system
    # ROCm) sees no device through torch afterwards, whichever GPU test happens to run first
    gpu_available()
    lib = ROOT / "pathtracer.cl_amd" / "librtmi.so"
    if not lib.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "pathtracer.cl_amd" / "csrc")], check=True)
    import ptload

    return ptload.load()


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle, build

    build()
    return Oracle()


@pytest.fixture(scope="session")
def golden_meta():
    return json.loads((GOLDEN / "meta.json").read_text())


def load_golden(name: str) -> dict:
    with np.load(GOLDEN / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden():
    return load_golden


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available() and torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def tracer(pt):
    if not gpu_available():
        pytest.fail("GPU test run without a visible GPU")
    rt = pt.RayTracer(0)
    yield rt
    rt.close()


def bits(a: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(a).view(np.uint32)
