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
