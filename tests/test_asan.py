"""The host C++ under AddressSanitizer + UndefinedBehaviorSanitizer — CPU only.

`make -C tests/cpp asan` compiles every source of librtmi with -fsanitize=address,undefined on
the host side (device code as usual) and the oracle likewise, into tests/cpp/asan_host, which
drives: the PLY reader over the malformed corpus (tests/ply_corpus.py), the host helpers (camera,
glibc rand, tiles, synthetic mesh, the host BVH builder and its input checks, the seed-halo
planner for N = 2..8, rt_create without a device, the C ABI's exception guard), and oracle frames
(spheres; triangles through the linear loop and the BVH mode, equal).  Any sanitizer report
(heap/stack overflow, use after free, leak, signed overflow, invalid shift, float-cast overflow,
misaligned access …) fails the run.
"""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
EXE = ROOT / "tests" / "cpp" / "asan_host"

ENV = dict(os.environ,
           ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0:allocator_may_return_null=1:"
                        "detect_stack_use_after_return=1:strict_string_checks=1",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
           LSAN_OPTIONS="suppressions=" + str(ROOT / "tests" / "cpp" / "lsan.supp"))


@pytest.fixture(scope="module")
def asan_exe():
    r = subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "cpp"), "asan"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail("ASan build failed:\n" + r.stdout[-4000:] + r.stderr[-4000:])
    return EXE


def _run(exe, *args, timeout=600):
    r = subprocess.run([str(exe), *args], capture_output=True, text=True, env=ENV, timeout=timeout)
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, r.stderr[-6000:]
    assert "ERROR: LeakSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    return r.stdout


def test_asan_ply_corpus(asan_exe, tmp_path, pt):
    from ply_corpus import cases

    names = {getattr(pt._abi, n): n for n in dir(pt._abi) if n.startswith("RT_ERR_") or n == "RT_OK"}
    cs = cases()
    paths = []
    for name, data, _ in cs:
        p = tmp_path / f"{name}.ply"
        p.write_bytes(data)
        paths.append(str(p))
    # plus real meshes in the three encodings (the round-trip writer of test_ply.py)
    from test_ply import _write

    verts, idx = pt.scenes.make_mesh(2000)
    for fmt in ("ascii", "binary_little_endian", "binary_big_endian"):
        p = tmp_path / f"mesh_{fmt}.ply"
        _write(p, fmt, verts, [list(map(int, t)) for t in idx])
        paths.append(str(p))
    out = _run(asan_exe, "ply", *paths).strip().split("\n")
    assert len(out) == len(paths)
    for (name, _, want), line in zip(cs, out):
        st = int(line.split("\t")[0])
        got = "ok" if st == 0 else names.get(st, str(st))
        assert got == want, (name, line)
    for line in out[len(cs):]:
        st, nv, nt = (int(x) for x in line.split("\t")[:3])
        assert st == 0 and nv == len(verts) and nt == len(idx), line


def test_asan_host(asan_exe):
    assert "host ok" in _run(asan_exe, "host")


def test_asan_oracle(asan_exe):
    assert "oracle ok" in _run(asan_exe, "oracle")
