"""PLY reader (csrc/rt_ply.cpp; PLYLoader.cpp:4-90 semantics over ply.c) — host code, CPU tests.

Files are written here in the three PLY encodings with the layout of the Stanford scans the
reference's plymain.cpp loads (dragon_vrip.ply: vertex x, y, z, confidence, intensity; face
`list uchar int vertex_indices`), plus extra elements/properties, quads and degenerate faces.
The reference's own loader keeps only 2-vertex faces (PLYLoader.cpp:74) and its result is never
handed to the tracer (plymain.cpp), so there is no reference output to pin against: parity here
is against the arrays the files were written from ("parity unpinned" w.r.t. the reference).
"""
from __future__ import annotations

import struct

import numpy as np
import pytest


def _mesh(pt, n=600):
    verts, idx = pt.scenes.make_mesh(n)
    return verts, idx


def _write(path, fmt, verts, faces, extra_edge=True):
    """faces: list of index lists (any length)."""
    nv = len(verts)
    conf = np.linspace(0.0, 1.0, nv, dtype=np.float32)
    inten = np.arange(nv, dtype=np.float64) * 0.5
    hdr = ["ply", f"format {fmt} 1.0", "comment written by tests/test_ply.py", "obj_info synthetic",
           f"element vertex {nv}", "property float x", "property float y", "property float z",
           "property float confidence", "property double intensity"]
    if extra_edge:
        hdr += ["element edge 2", "property int vertex1", "property list ushort int extra_list"]
    hdr += [f"element face {len(faces)}", "property list uchar int vertex_indices", "property uchar flags",
            "end_header"]
    head = ("\n".join(hdr) + "\n").encode()
    edges = [(0, [1, 2, 3]), (2, [])]
    if fmt == "ascii":
        lines = []
        for i in range(nv):
            lines.append(" ".join(repr(float(v)) for v in verts[i]) + f" {float(conf[i])!r} {float(inten[i])!r}")
        if extra_edge:
            for v1, lst in edges:
                lines.append(f"{v1} {len(lst)} " + " ".join(map(str, lst)))
        for f in faces:
            lines.append(f"{len(f)} " + " ".join(map(str, f)) + " 7")
        body = ("\n".join(lines) + "\n").encode()
    else:
        e = "<" if fmt == "binary_little_endian" else ">"
        parts = []
        for i in range(nv):
            parts.append(struct.pack(e + "ffffd", *[float(v) for v in verts[i]], float(conf[i]), float(inten[i])))
        if extra_edge:
            for v1, lst in edges:
                parts.append(struct.pack(e + "iH" + "i" * len(lst), v1, len(lst), *lst))
        for f in faces:
            parts.append(struct.pack(e + "B" + "i" * len(f) + "B", len(f), *f, 7))
        body = b"".join(parts)
    path.write_bytes(head + body)


@pytest.mark.parametrize("fmt", ["ascii", "binary_little_endian", "binary_big_endian"])
def test_ply_roundtrip_exact(fmt, tmp_path, pt):
    verts, idx = _mesh(pt)
    faces = [list(map(int, t)) for t in idx]
    p = tmp_path / f"m_{fmt}.ply"
    _write(p, fmt, verts, faces)
    v, i = pt.scenes.load_ply(p, normalize=False)
    np.testing.assert_array_equal(v.view(np.uint32), verts.view(np.uint32))
    np.testing.assert_array_equal(i, idx)


@pytest.mark.parametrize("fmt", ["ascii", "binary_little_endian"])
def test_ply_polygons_fan_and_degenerate_faces(fmt, tmp_path, pt):
    verts = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [0.5, 2, 0]], np.float32)
    faces = [[0, 1, 2, 3], [1, 2], [0, 1, 2, 3, 4], [4, 3, 2]]
    p = tmp_path / "poly.ply"
    _write(p, fmt, verts, faces, extra_edge=False)
    v, i = pt.scenes.load_ply(p, normalize=False)
    want = [[0, 1, 2], [0, 2, 3], [0, 1, 2], [0, 2, 3], [0, 3, 4], [4, 3, 2]]
    np.testing.assert_array_equal(i, np.array(want, np.int32))


def test_ply_errors(tmp_path, pt):
    lib = pt.load_library()
    verts = np.zeros((3, 3), np.float32)
    p = tmp_path / "bad.ply"
    _write(p, "binary_little_endian", verts, [[0, 1, 5]], extra_edge=False)  # index out of range
    with pytest.raises(pt.RtError, match="out of range"):
        pt.scenes.load_ply(p)
    p.write_bytes(b"not a ply\n")
    with pytest.raises(pt.RtError, match="magic"):
        pt.scenes.load_ply(p)
    _write(p, "binary_little_endian", verts, [[0, 1, 2]], extra_edge=False)
    p.write_bytes(p.read_bytes()[:-3])  # truncated body
    with pytest.raises(pt.RtError, match="truncated"):
        pt.scenes.load_ply(p)
    with pytest.raises(pt.RtError, match="cannot open"):
        pt.scenes.load_ply(tmp_path / "missing.ply")
    assert lib.rt_normalize_mesh(None, 0, 3.0, -5.0) != 0


def test_ply_normalisation(tmp_path, pt):
    verts, idx = _mesh(pt, 300)
    verts = verts * np.float32(7.0) + np.float32(3.0)
    p = tmp_path / "n.ply"
    _write(p, "binary_little_endian", verts, [list(map(int, t)) for t in idx])
    v, _ = pt.scenes.load_ply(p)
    lo, hi = v.min(0), v.max(0)
    assert abs(float((hi - lo).max()) - pt.scenes.PLY_MAX_EXTENT) < 1e-5
    assert abs(float(lo[1]) - pt.scenes.PLY_FLOOR_Y) < 1e-6
    assert abs(float(lo[0] + hi[0])) < 1e-5 and abs(float(lo[2] + hi[2])) < 1e-5


def _status_names(pt):
    return {getattr(pt._abi, n): n for n in dir(pt._abi) if n.startswith("RT_ERR_") or n == "RT_OK"}


def test_ply_malformed_corpus_returns_status(tmp_path, pt):
    """Every malformed file of tests/ply_corpus.py comes back as RT_ERR_ARG with a message from
    rt_ply_open — huge header counts (the r04 verdict's `element face 4000000000000000000`, which
    used to escape the C ABI as std::length_error and abort the caller), truncated bodies,
    negative / huge list lengths, out-of-range and non-integer indices, non-finite coordinates,
    header defects — and the well-formed ones load."""
    import ctypes

    from ply_corpus import cases

    lib = pt.load_library()
    names = _status_names(pt)
    for name, data, want in cases():
        p = tmp_path / f"{name}.ply"
        p.write_bytes(data)
        h = ctypes.c_void_p()
        nv, nt = ctypes.c_uint32(), ctypes.c_uint32()
        st = lib.rt_ply_open(str(p).encode(), ctypes.byref(h), ctypes.byref(nv), ctypes.byref(nt))
        if st == pt._abi.RT_OK:
            lib.rt_ply_close(h)
        got = "ok" if st == pt._abi.RT_OK else names.get(st, str(st))
        assert got == want, (name, got, lib.rt_ply_last_error())
        if st != pt._abi.RT_OK:
            assert lib.rt_ply_last_error(), name
    p = tmp_path / "face_count_4e18.ply"
    with pytest.raises(pt.RtError, match="declares 4000000000000000000"):
        pt.scenes.load_ply(p)


def test_abi_entries_are_exception_guarded():
    """No C++ exception crosses the C ABI: every `int rt_*` entry defined in the
    extern "C" blocks of the host sources is a function-try-block ending in RT_CATCH (the
    exception in flight mapped to a status and a message, csrc/rt_internal.h)."""
    import re
    from pathlib import Path

    csrc = Path(__file__).resolve().parent.parent / "pathtracer.cl_amd" / "csrc"
    n = 0
    for f in ("rt_host.cpp", "rt_ply.cpp", "rt_comm.hip"):
        lines = (csrc / f).read_text().split("\n")
        in_c = False
        for i, ln in enumerate(lines):
            if ln.startswith('extern "C" {'):
                in_c = True
            if in_c and re.match(r"^int rt_\w+\(", ln):
                j = i
                while lines[j] not in ("{", "try {"):
                    j += 1
                assert lines[j] == "try {", (f, ln)
                k = j + 1
                while not lines[k].startswith("}"):
                    k += 1
                assert lines[k].startswith("} RT_CATCH("), (f, ln)
                n += 1
    assert n >= 45, n
