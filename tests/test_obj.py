"""Wavefront OBJ scenes behind model_path.

The library's loader (scene.cpp LoadObj, through srtReadScene) is checked against an
independent Python restatement of the same OBJ subset (below), on hand-written files that
cover fan triangulation, relative indices, i/t/n index forms, materials, the srt comment
directives, the automatic camera, and the error messages. CPU only (no GPU needed).
"""
from __future__ import annotations

import math

import numpy as np
import pytest

import simpleraytracer_amd as srt
from scenefile import read_scene as read_binary


def py_parse_obj(text, mtl=None):
    """Independent restatement: (vertices N x 9, albedo N x 3, camera or None, background)."""
    pos, tris, alb = [], [], []
    mats = mtl or {}
    cur = (0.8, 0.8, 0.8)
    cam, bg = None, (0.0, 0.0, 0.0)
    for line in text.splitlines():
        parts = line.split()
        if not parts:
            continue
        if parts[0].startswith("#"):
            body = line[line.index("#") + 1:].split()
            if len(body) >= 2 and body[0] == "srt":
                if body[1] == "camera":
                    cam = [float(x) for x in body[2:12]]
                elif body[1] == "background":
                    bg = tuple(float(x) for x in body[2:5])
            continue
        if parts[0] == "v":
            pos.append([float(x) for x in parts[1:4]])
        elif parts[0] == "f":
            idx = []
            for tok in parts[1:]:
                i = int(tok.split("/")[0])
                idx.append(i - 1 if i > 0 else len(pos) + i)
            for k in range(1, len(idx) - 1):
                tris.append(pos[idx[0]] + pos[idx[k]] + pos[idx[k + 1]])
                alb.append(cur)
        elif parts[0] == "usemtl":
            cur = mats.get(parts[1], (0.8, 0.8, 0.8))
    return np.array(tris, np.float32), np.array(alb, np.float32), cam, bg


QUAD_OBJ = """# a quad, a pentagon fan and relative indices
mtllib scene.mtl
v -1 -1 3
v 1 -1 3
v 1 1 3
v -1 1 3
usemtl red
f 1 2 3 4
v 0 0 2.5
v 0.5 0 2.5
v 0.6 0.4 2.5
v 0.2 0.7 2.5
v -0.2 0.4 2.5
usemtl unknown_material
f -5/1 -4/2/3 -3//1 -2 -1
usemtl green
f 5/1/1 6/2/2 7/3/3
# srt background 0.1 0.2 0.3
"""

MTL = """newmtl red
Kd 0.9 0.1 0.1
newmtl green
Kd 0.1 0.8 0.2
"""


def test_obj_matches_python_restatement(tmp_path):
    (tmp_path / "scene.mtl").write_text(MTL)
    obj = tmp_path / "scene.obj"
    obj.write_text(QUAD_OBJ)
    got = srt.read_scene(str(obj))
    v, a, cam, bg = py_parse_obj(QUAD_OBJ, {"red": (0.9, 0.1, 0.1), "green": (0.1, 0.8, 0.2)})
    assert got["vertices"].shape == (2 + 3 + 1, 9)
    assert np.array_equal(got["vertices"], v)
    assert np.array_equal(got["albedo"], a)
    assert np.array_equal(got["background"], np.array(bg, np.float32))
    assert got["flags"] == 0
    # automatic camera: looks along +z at the bounding-box centre, bounding sphere in a 60 deg view
    lo, hi = v.reshape(-1, 3).min(0).astype(np.float64), v.reshape(-1, 3).max(0).astype(np.float64)
    c = (lo + hi) / 2
    r = 0.5 * np.linalg.norm(hi - lo)
    d = r / math.sin(math.radians(30))
    want = np.array([c[0], c[1], c[2] - d, c[0], c[1], c[2], 0, 1, 0, 60], np.float32)
    assert np.array_equal(got["camera"], want)


def test_obj_camera_directive_and_crlf(tmp_path):
    text = "# srt camera 0 0 -5 0 0 0 0 1 0 45\r\nv 0 0 0\r\nv 1 0 0\r\nv 0 1 0\r\nf 1 2 3\r\n"
    obj = tmp_path / "c.OBJ"
    obj.write_bytes(text.encode())
    got = srt.read_scene(str(obj))
    assert np.array_equal(got["camera"], np.array([0, 0, -5, 0, 0, 0, 0, 1, 0, 45], np.float32))
    assert np.array_equal(got["albedo"], np.full((1, 3), 0.8, np.float32))


@pytest.mark.parametrize("body,msg", [
    ("v 0 0 0\nv 1 0 0\nf 1 2 3\n", "line 3: face index 3 out of range (2 vertices so far)"),
    ("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2\n", "line 4: face needs at least 3 vertices"),
    ("v 0 0\n", "line 1: vertex needs 3 coordinates"),
    ("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 x 3\n", "line 4: bad face index 'x'"),
    ("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n", "line 4: face index 0 out of range"),
    ("v 0 0 0\n", "no faces"),
    ("# srt camera 1 2 3\nv 0 0 0\n", "line 1: srt camera needs 10 numbers"),
    ("# srt zoom 2\n", "line 1: unknown srt directive 'zoom'"),
    ("# srt camera 0 0 -5 0 0 0 0 1 0 190\nv 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n", "bad camera vfov"),
])
def test_obj_errors(tmp_path, body, msg):
    obj = tmp_path / "bad.obj"
    obj.write_text(body)
    with pytest.raises(srt.SrtError) as e:
        srt.read_scene(str(obj))
    assert str(e.value).startswith(f"Error reading scene file: {obj}: ")
    assert msg in str(e.value)


def test_obj_through_ml_create_model(tmp_path):
    """model_path may name an OBJ file; mlCreateModel loads it (no GPU needed to create)."""
    obj = tmp_path / "tri.obj"
    obj.write_text("v -0.5 -0.5 2\nv 0.5 -0.5 2\nv 0 0.5 2\nf 1 2 3\n")
    ctx = srt.Context()
    model = ctx.create_model(str(obj))
    (idt, _, _, ic), (odt, _, _, oc) = model.info()
    assert (idt, ic, odt, oc) == (0, 2, 0, 4)
    model.close()
    ctx.close()


def test_convert_scene_roundtrip_and_flags(tmp_path):
    (tmp_path / "scene.mtl").write_text(MTL)
    obj = tmp_path / "scene.obj"
    obj.write_text(QUAD_OBJ)
    dst = srt.convert_scene(str(obj), str(tmp_path / "scene.srt"), input_dtype=-1, output_dtype=1)
    cam, bg, v, a = read_binary(dst)
    got = srt.read_scene(str(obj))
    assert np.array_equal(v, got["vertices"]) and np.array_equal(a, got["albedo"])
    assert np.array_equal(cam, got["camera"]) and np.array_equal(bg, got["background"])
    assert srt.read_scene(dst)["flags"] == 1
    back = srt.convert_scene(dst, str(tmp_path / "b.srt"), input_dtype=1, output_dtype=0)
    assert srt.read_scene(back)["flags"] == 2
    with pytest.raises(srt.SrtError, match="Bad output data type 7"):
        srt.convert_scene(dst, str(tmp_path / "c.srt"), output_dtype=7)


def test_binary_loader_rejects_trailing_bytes_and_unknown_flags(tmp_path):
    from scenefile import write_custom_scene

    p = write_custom_scene(tmp_path / "t.srt", [[-0.5, -0.5, 2, 0.5, -0.5, 2, 0, 0.5, 2]])
    with open(p, "ab") as f:
        f.write(b"\0")
    with pytest.raises(srt.SrtError, match="trailing bytes"):
        srt.read_scene(p)
    p2 = write_custom_scene(tmp_path / "u.srt", [[-0.5, -0.5, 2, 0.5, -0.5, 2, 0, 0.5, 2]])
    raw = bytearray(open(p2, "rb").read())
    raw[12] = 8  # flags field (offset 12): unknown bit
    open(p2, "wb").write(bytes(raw))
    with pytest.raises(srt.SrtError, match="unknown flags 8"):
        srt.read_scene(p2)
