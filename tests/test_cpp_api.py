"""The C++ drop-in keeps the reference's RayTracer API (RayTracer.h:56-70).

tests/cpp/ref_main_replay.cpp is the reference's clrt/main.cpp / plymain.cpp call
sequence written against the reference's own types (`Sphere` from clrt/ocl/geometry.h,
`gmtl::Point3f`, `gmtl::Matrix44f`), compiled against include/RayTracerHIP.hpp with the
reference headers read in place.  CPU: it compiles and fails loudly without a GPU.
GPU: its frames equal the reference kernel's golden frames and the oracle, bit for bit,
through both camera overloads.
"""
from __future__ import annotations

import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import ROOT, bits

REF = Path("/root/reference")
BIN = ROOT / "tests" / "cpp" / "ref_main_replay"


@pytest.mark.skipif(not (REF / "clrt" / "ocl" / "geometry.h").exists(), reason="reference headers absent")
def test_reference_caller_compiles_and_fails_loudly_without_gpu(pt, tmp_path):
    subprocess.run(["make", "-s", "-B", "-C", str(ROOT / "tests" / "cpp")], check=True, timeout=300)
    assert BIN.exists()
    from conftest import gpu_available

    if gpu_available():
        pytest.skip("a GPU is visible: the GPU test covers the run")
    r = subprocess.run([str(BIN), "main", "16", "16", "1", str(tmp_path / "o.f32")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 3 and "rt_create" in r.stderr  # no CPU fallback


def _replay(tmp_path, *args):
    if not BIN.exists():
        pytest.fail("tests/cpp/ref_main_replay was not built (build() builds it where the reference is)")
    raw = tmp_path / "out.f32"
    subprocess.run([str(BIN), args[0], *map(str, args[1:4]), str(raw), *args[4:]], check=True, timeout=120)
    return np.fromfile(raw, np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("camera", ["spherical", "matrix"])
def test_reference_main_replay_equals_golden(camera, tracer, golden, tmp_path):
    """main.cpp's calls through RayTracerHIP == the reference kernel's frame (golden,
    main.cpp scene and camera, default glibc seeds, 4 progressive frames)."""
    got = _replay(tmp_path, "main", 64, 64, 4, camera)
    exp = golden("spheres_64x64_sr1")["frames"][-1]
    np.testing.assert_array_equal(bits(got), bits(exp))


@pytest.mark.gpu
def test_reference_plymain_replay_equals_oracle(tracer, pt, oracle, tmp_path):
    """plymain.cpp's scene and camera (its mesh is never handed over by the reference)
    through RayTracerHIP == the oracle's sphere frames over 3 progressive passes."""
    sc = pt.scenes
    W, H, frames = 48, 40, 3
    got = _replay(tmp_path, "ply", W, H, frames)
    Wp, Hp = sc.padded_dims(W, H)
    sd = sc.default_seeds(Wp, Hp)
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    exp = np.zeros(W * H * 4, np.float32)
    for p in range(frames):
        oracle.render_spheres(exp, cam, sc.ply_scene(), W, H, Wp, Hp, 1, 6, p, sd)
    np.testing.assert_array_equal(bits(got), bits(exp))


def test_gl_pbo_adapter_builds_and_fails_loudly_without_gpu(pt):
    """f3, the display side of GlutCLWindow::rayTrace (GlutCLWindow.cpp:190-227):
    include/GlPboTargetHIP.hpp (PBO shared through hipGraphicsGLRegisterBuffer, or the
    glMapBuffer + rt_read readback) compiles and links against libGL, the HIP runtime and
    librtmi.  No GL context exists here or on the GPU box, so its two paths are not run;
    without a GPU the program fails at rt_create (no CPU fallback)."""
    subprocess.run(["make", "-s", "-B", "-C", str(ROOT / "tests" / "cpp"), "gl_pbo_target"], check=True, timeout=300)
    exe = ROOT / "tests" / "cpp" / "gl_pbo_target"
    assert exe.exists()
    from conftest import gpu_available

    if gpu_available():
        pytest.skip("a GPU is visible: nothing to check without a GL context")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 3 and "rt_create" in r.stderr
