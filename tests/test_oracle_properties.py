"""The oracle against an independent float64 Moller-Trumbore restatement (hypothesis).

The float64 reference below shares nothing with the oracle except the camera frame floats:
it intersects the ray eye + t*d, d = base + fx*du + fy*dv (float64), with each triangle by the
textbook Moller-Trumbore algorithm (two-sided, t > 0) and picks the smallest t. Disagreements
are allowed only where float32 cannot decide: the ray within 1e-4 (relative barycentric) of an
edge of either candidate, or two candidates within 1e-5 relative depth.
"""
from __future__ import annotations

import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from oracle.srt_oracle import OracleScene, closest_hit
from scenefile import write_custom_scene

EDGE_EPS = 1e-4
DEPTH_EPS = 1e-5


def mt64(eye, d, tris):
    """Per triangle: (t, u, v) in float64 or None."""
    out = []
    for v in tris.astype(np.float64):
        v0, v1, v2 = v[0:3], v[3:6], v[6:9]
        e1, e2 = v1 - v0, v2 - v0
        p = np.cross(d, e2)
        det = e1 @ p
        if abs(det) < 1e-300:
            out.append(None)
            continue
        s = eye - v0
        u = (s @ p) / det
        q = np.cross(s, e1)
        w = (d @ q) / det
        t = (e2 @ q) / det
        if u >= 0 and w >= 0 and u + w <= 1 and t > 0:
            out.append((t, u, w))
        else:
            out.append((None, u, w))
    return out


def mt64_all(eye, d, tris):
    """Vectorised over triangles: arrays t (inf where no hit), u, v."""
    v = tris.astype(np.float64)
    v0, e1, e2 = v[:, 0:3], v[:, 3:6] - v[:, 0:3], v[:, 6:9] - v[:, 0:3]
    p = np.cross(d, e2)
    det = np.einsum("ij,ij->i", e1, p)
    with np.errstate(divide="ignore", invalid="ignore"):
        s = eye - v0
        u = np.einsum("ij,ij->i", s, p) / det
        q = np.cross(s, e1)
        w = (q @ d) / det
        t = np.einsum("ij,ij->i", e2, q) / det
    ok = (u >= 0) & (w >= 0) & (u + w <= 1) & (t > 0) & (np.abs(det) > 1e-300)
    return np.where(ok, t, np.inf), u, w


def margin(hit):
    if hit is None:
        return 0.0
    _, u, w = hit
    return min(abs(u), abs(w), abs(1 - u - w))


tri_strategy = st.lists(
    st.tuples(
        st.floats(-0.6, 0.6), st.floats(-0.6, 0.6), st.floats(1.0, 4.0),   # centroid
        st.lists(st.floats(-0.4, 0.4), min_size=9, max_size=9),             # vertex offsets
    ),
    min_size=1, max_size=8)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(tris=tri_strategy, rays=st.lists(st.tuples(st.floats(0.05, 0.95), st.floats(0.05, 0.95)), min_size=1,
                                         max_size=16))
def test_oracle_matches_float64_moller_trumbore(tmp_path, tris, rays):
    verts = np.array([[c[0] + o[0], c[1] + o[1], c[2] + o[2], c[0] + o[3], c[1] + o[4], c[2] + o[5],
                       c[0] + o[6], c[1] + o[7], c[2] + o[8]] for (*c, o) in [(a, b, z, off) for a, b, z, off in tris]],
                     np.float32)
    path = write_custom_scene(tmp_path / "h.srt", verts)
    s = OracleScene(path)
    w, h = 96, 64
    frame = s.frame(w, h).astype(np.float64)
    eye, base, du, dv = frame[0:3], frame[3:6], frame[6:9], frame[9:12]
    edges = s.edges(w, h)
    for fx, fy in rays:
        fx, fy = float(np.float32(fx)), float(np.float32(fy))
        got, t32, _ = closest_hit(edges, fx, fy)
        d = base + fx * du + fy * dv
        hits = mt64(eye, d, verts)
        valid = [(hh[0], i) for i, hh in enumerate(hits) if hh is not None and hh[0] is not None]
        want = min(valid)[1] if valid else -1
        if got == want:
            # depth accuracy away from edges; on an edge (or vertex) of a sliver, float32
            # edge functions cancel and t = vol / det is ill-conditioned
            if got >= 0 and margin(hits[got]) >= EDGE_EPS:
                assert abs(t32 - hits[got][0]) <= 1e-4 * hits[got][0]
            continue
        # disagreement: must be a float32-undecidable configuration
        near_edge = any(hits[i] is not None and margin(hits[i]) < EDGE_EPS for i in (got, want) if i >= 0)
        ts = sorted(v[0] for v in valid)
        near_tie = len(ts) > 1 and (ts[1] - ts[0]) <= DEPTH_EPS * ts[0]
        assert near_edge or near_tie, f"oracle {got} vs float64 {want} at {(fx, fy)}"


def test_oracle_matches_float64_on_dense_soup(tmp_path):
    """Seeded 300-triangle soup, every pixel of a 64x48 frame: id agreement except on
    float32-undecidable pixels, and enough hits that the comparison is not vacuous."""
    rng = np.random.default_rng(5)
    c = np.stack([rng.uniform(-0.8, 0.8, 300), rng.uniform(-0.5, 0.5, 300), rng.uniform(2, 4, 300)], 1)
    verts = (np.repeat(c, 3, 0) + rng.uniform(-0.25, 0.25, (900, 3))).reshape(300, 9).astype(np.float32)
    s = OracleScene(write_custom_scene(tmp_path / "d.srt", verts))
    w, h = 64, 48
    frame = s.frame(w, h).astype(np.float64)
    img = s.render(w, h)
    hits = undecidable = 0
    for y in range(h):
        for x in range(w):
            fx = float(np.float32(np.float32(x + 0.5) / np.float32(w)))
            fy = float(np.float32(np.float32(y + 0.5) / np.float32(h)))
            d = frame[3:6] + fx * frame[6:9] + fy * frame[9:12]
            t, u, v = mt64_all(frame[0:3], d, verts)
            want = int(np.argmin(t)) if np.isfinite(t).any() else -1
            got = int(img[y, x, 3])
            hits += got >= 0
            if got != want:
                marg = np.minimum(np.minimum(np.abs(u), np.abs(v)), np.abs(1 - u - v))
                near_edge = any(marg[i] < EDGE_EPS for i in (got, want) if i >= 0)
                ts = np.sort(t[np.isfinite(t)])
                near_tie = len(ts) > 1 and (ts[1] - ts[0]) <= DEPTH_EPS * ts[0]
                assert near_edge or near_tie, (x, y, got, want)
                undecidable += 1
    assert hits > 0.1 * w * h, hits
    assert undecidable <= 3
