"""Known-answer tests of the CPU oracle on hand-built scenes.

No reference render code exists to pin against, so these analytic
cases pin the oracle: exact ray generation, t of a head-on hit, misses, behind-eye rejection,
depth order, tie-break to the lowest id, disabled (edge-on / degenerate) triangles, watertight
shared edges, two-sided hits and head-on shading.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle.srt_oracle import OracleScene, closest_hit, pixel_position
from scenefile import write_custom_scene

TRI_Z2 = [-0.5, -0.5, 2, 0.5, -0.5, 2, 0, 0.5, 2]


def scene(tmp_path, tris, name="s.srt", **kw):
    return OracleScene(write_custom_scene(tmp_path / name, tris, **kw))


def test_pixel_position_is_exact():
    assert pixel_position(0, 0, 0.5, 0.5, 256, 256) == (np.float32(0.5 / 256), np.float32(0.5 / 256))
    fx, fy = pixel_position(1919, 1079, 0.5, 0.5, 1920, 1080)
    assert fx == np.float32(np.float32(1919.5) / np.float32(1920))
    assert fy == np.float32(np.float32(1079.5) / np.float32(1080))


def test_frame_centre_ray_is_forward(tmp_path):
    s = scene(tmp_path, [TRI_Z2])
    f = s.frame(256, 256)
    d = f[3:6] + np.float32(0.5) * f[6:9] + np.float32(0.5) * f[9:12]
    assert np.allclose(d, [0, 0, 1], atol=1e-7)
    assert np.allclose(np.linalg.norm(f[9:12]) / 2, np.tan(np.radians(30)), rtol=1e-6)


def test_head_on_hit_t_and_shading(tmp_path):
    s = scene(tmp_path, [TRI_Z2], albedo=[[0.9, 0.6, 0.3]])
    e = s.edges(256, 256)
    i, t, det = closest_hit(e, 0.5, 0.5)
    assert i == 0 and det > 0
    assert t == pytest.approx(2.0, rel=1e-6)  # |d| = 1 at the centre, plane z = 2
    img = s.render(256, 256)
    assert img[128, 128, 3] == 0.0
    assert np.allclose(img[128, 128, :3], [0.9, 0.6, 0.3], rtol=1e-5)


def test_miss_outside_and_background(tmp_path):
    s = scene(tmp_path, [TRI_Z2], background=(0.1, 0.2, 0.3))
    assert closest_hit(s.edges(64, 64), 0.02, 0.02)[0] == -1
    img = s.render(64, 64)
    assert img[0, 0].tolist() == pytest.approx([0.1, 0.2, 0.3, -1.0])


def test_behind_the_eye_never_hits(tmp_path):
    s = scene(tmp_path, [[-5, -5, -2, 5, -5, -2, 0, 5, -2]])
    assert np.all(s.render(48, 48)[..., 3] == -1)


def test_nearer_wins_regardless_of_id(tmp_path):
    far = [-1, -1, 3, 1, -1, 3, 0, 1, 3]
    near = [-0.2, -0.2, 2, 0.2, -0.2, 2, 0, 0.2, 2]
    s = scene(tmp_path, [far, near])
    i, t, _ = closest_hit(s.edges(64, 64), 0.5, 0.5)
    assert i == 1 and t == pytest.approx(2.0, rel=1e-6)
    s2 = scene(tmp_path, [near, far], name="s2.srt")
    assert closest_hit(s2.edges(64, 64), 0.5, 0.5)[0] == 0


def test_tie_keeps_lowest_id(tmp_path):
    s = scene(tmp_path, [TRI_Z2, TRI_Z2, TRI_Z2])
    ids = s.render(64, 64)[..., 3]
    assert set(np.unique(ids)) == {-1.0, 0.0}


def test_disabled_triangles(tmp_path):
    edge_on = [0, -1, 1, 0, 1, 1, 0, 0, 3]          # plane x = 0 contains the eye
    degenerate = [0.1, 0.1, 2, 0.1, 0.1, 2, 0.3, 0.2, 2]  # repeated vertex: zero area
    s = scene(tmp_path, [edge_on, degenerate])
    e = s.edges(32, 32)
    assert np.all(np.isnan(e[0, :10]))  # vol == 0 exactly: disabled
    # repeated vertex: vol is rounding noise, but nC == 0 and nA == -nB exactly, so any ray
    # passing the sign test has det == 0 and is rejected
    assert np.array_equal(e[1, 6:9], np.zeros(3, np.float32))
    assert np.array_equal(e[1, 0:3], -e[1, 3:6])
    assert np.all(s.render(32, 32)[..., 3] == -1)


def test_two_sided(tmp_path):
    front = TRI_Z2
    back = [TRI_Z2[3], TRI_Z2[4], TRI_Z2[5], TRI_Z2[0], TRI_Z2[1], TRI_Z2[2], *TRI_Z2[6:]]
    for tri in (front, back):
        s = scene(tmp_path, [tri], name=f"t{tri[0]}.srt")
        i, t, _ = closest_hit(s.edges(64, 64), 0.5, 0.5)
        assert i == 0 and t == pytest.approx(2.0, rel=1e-6)


def test_shared_edge_is_watertight(tmp_path):
    """A quad split along its diagonal: no sample inside the quad misses both triangles, even
    samples placed exactly on the diagonal (its edge normals are exact negatives)."""
    q = [(-0.5, -0.5, 2), (0.5, -0.5, 2), (0.5, 0.5, 2), (-0.5, 0.5, 2)]
    t0 = [*q[0], *q[1], *q[2]]
    t1 = [*q[0], *q[2], *q[3]]
    s = scene(tmp_path, [t0, t1])
    e = s.edges(100, 100)
    g = np.linspace(0.36, 0.64, 141, dtype=np.float32)
    misses = [(fx, fy) for fx in g for fy in g if closest_hit(e, float(fx), float(fy))[0] < 0]
    assert misses == []
    # along the projected diagonal both triangles' shared-edge functions are exact negatives
    assert np.array_equal(e[0, 6:9], -e[1, 3:6]) or np.array_equal(e[0, 0:3], -e[1, 6:9]) or \
        any(np.array_equal(e[0, 3 * a:3 * a + 3], -e[1, 3 * b:3 * b + 3]) for a in range(3) for b in range(3))


def test_sample_offsets_move_the_ray(tmp_path):
    s = scene(tmp_path, [TRI_Z2])
    w = h = 64
    base = s.render(w, h)
    offs = np.full((h, w, 2), 0.5, np.float32)
    offs[..., 0] = 0.0
    shifted = s.render(w, h, offs)
    assert not np.array_equal(base[..., 3], shifted[..., 3])


def test_row_subset_matches_full_frame(tmp_path):
    s = scene(tmp_path, [TRI_Z2, [-1, -1, 3, 1, -1, 3, 0, 1, 3]])
    full = s.render(80, 60)
    part = s.render(80, 60, row_begin=7, row_count=40, row_step=3)
    rows = np.arange(7, 47, 3)
    assert np.array_equal(full[rows].view(np.uint32), part[rows].view(np.uint32))
    other = np.setdiff1d(np.arange(60), rows)
    assert np.all(np.isnan(part[other]))
