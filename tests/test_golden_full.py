"""Full-size golden fixtures of the headline configs (tests/golden/fullframes.*, made by
tests/golden/make_fullframes.py with the CPU oracle, brute force).

CPU: the oracle's deferred shading of the stored ids reproduces the SHA-256 of the oracle's own
RGBA rows (so the stored ids + shading are the whole oracle frame); the oracle still renders a
sample of the stored rows identically; and the C3 fixture agrees with an independent float64
Moller-Trumbore restatement on sampled pixels wherever float32 can decide.
GPU: every stored pixel -- the whole C3 and C2 frames, C3 with per-pixel jitter every 8th row, 64
rows of C5 (1M triangles, 4K) -- rendered by the HIP path: ids bit-exact, RGB <= 1e-5 of the
oracle's shading of those ids.
"""
from __future__ import annotations

import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

import simpleraytracer_amd as srt

GOLDEN = Path(__file__).resolve().parent / "golden"
META = json.loads((GOLDEN / "fullframes.json").read_text())
RGB_TOL = 1e-5


@pytest.fixture(scope="module")
def ids():
    return dict(np.load(GOLDEN / "fullframes.npz"))


@pytest.fixture(scope="module")
def paths(tmp_path_factory):
    d = tmp_path_factory.mktemp("full")
    out = {}
    for name, m in META.items():
        key = (m["scene"], m["triangles"])
        if key not in out:
            p = str(d / f"{m['scene']}_{m['triangles']}.srt")
            out[key] = srt.write_scene(p, "soup", m["triangles"]) if m["scene"] == "soup" else \
                srt.write_scene(p, m["scene"])
    return {name: out[(m["scene"], m["triangles"])] for name, m in META.items()}


def rows_of(m):
    b, step, count = m["rows"]
    return np.arange(b, b + step * count, step)


def offsets_for(m):
    w, h = m["width"], m["height"]
    if m["offsets_seed"] is None:
        return np.full((h, w, 2), 0.5, np.float32)
    return np.random.default_rng(m["offsets_seed"]).random((h, w, 2), dtype=np.float32)


def oracle_rgba(path, m, stored_ids):
    """The oracle's deferred shading of the stored ids (stage 3 of the oracle), stored rows only."""
    from oracle.srt_oracle import OracleScene

    w, h = m["width"], m["height"]
    frame_ids = np.full((h, w), -1, np.int32)
    rows = rows_of(m)
    frame_ids[rows] = stored_ids
    return OracleScene(path).shade(w, h, frame_ids, offsets_for(m))[rows]


@pytest.mark.parametrize("name", sorted(META))
def test_stored_ids_and_shading_are_the_oracle_frame(paths, ids, name):
    m = META[name]
    got = oracle_rgba(paths[name], m, ids[name])
    assert hashlib.sha256(np.ascontiguousarray(got).tobytes()).hexdigest() == m["rgba_sha256"]
    assert abs(float((ids[name] >= 0).mean()) - m["hit_fraction"]) < 1e-4


@pytest.mark.parametrize("name", sorted(META))
def test_oracle_still_computes_the_stored_ids(paths, ids, name):
    """The oracle's closest-hit scan (srto_closest_hit over its edge records, the loop its renders
    run) at 256 sampled stored pixels, ray positions from its own pixel_position."""
    from oracle.srt_oracle import OracleScene, closest_hit, pixel_position

    m = META[name]
    w, h = m["width"], m["height"]
    rows = rows_of(m)
    edges = OracleScene(paths[name]).edges(w, h)
    off = offsets_for(m)
    rng = np.random.default_rng(11)
    for i, x in zip(rng.integers(0, len(rows), 256), rng.integers(0, w, 256)):
        y = int(rows[i])
        fx, fy = pixel_position(int(x), y, float(off[y, x, 0]), float(off[y, x, 1]), w, h)
        assert closest_hit(edges, fx, fy)[0] == ids[name][i, x], (name, x, y)


def test_c3_fixture_agrees_with_float64_moller_trumbore(paths, ids):
    """300 sampled pixels of the full C3 fixture against an independent float64 closest hit over
    all 100k triangles (tests/test_oracle_properties.py mt64_all): equal ids except where float32
    cannot decide (within 1e-4 barycentric of an edge, or two depths within 1e-5)."""
    from test_oracle_properties import DEPTH_EPS, EDGE_EPS, mt64_all

    name = "c3_soup100k_1080p"
    m = META[name]
    w, h = m["width"], m["height"]
    sc = srt.read_scene(paths[name])
    frame = np.array(srt.scene_frame(paths[name], w, h), np.float64)
    eye, base, du, dv = frame
    rng = np.random.default_rng(3)
    # half the samples where the fixture has a hit (the hits are the interesting part)
    hit_px = np.argwhere(ids[name] >= 0)
    pick = np.concatenate([hit_px[rng.choice(len(hit_px), 200, replace=False)],
                           np.stack([rng.integers(0, h, 100), rng.integers(0, w, 100)], 1)])
    undecidable = 0
    for y, x in pick:
        fx = float(np.float32(np.float32(x + 0.5) / np.float32(w)))
        fy = float(np.float32(np.float32(y + 0.5) / np.float32(h)))
        t, u, v = mt64_all(eye, base + fx * du + fy * dv, sc["vertices"])
        want = int(np.argmin(t)) if np.isfinite(t).any() else -1
        got = int(ids[name][y, x])
        if got != want:
            marg = np.minimum(np.minimum(np.abs(u), np.abs(v)), np.abs(1 - u - v))
            near_edge = any(marg[i] < EDGE_EPS for i in (got, want) if i >= 0)
            ts = np.sort(t[np.isfinite(t)])
            near_tie = len(ts) > 1 and (ts[1] - ts[0]) <= DEPTH_EPS * ts[0]
            assert near_edge or near_tie, (x, y, got, want)
            undecidable += 1
    assert undecidable <= 3


def gpu_frame(path, m, variant="cull"):
    import torch

    w, h = m["width"], m["height"]
    ds = srt.DeviceScene(path, 0)
    s = torch.cuda.current_stream()
    ds.prepare(w, h, s)
    off = torch.from_numpy(offsets_for(m)).cuda()
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    ds.trace(off, out, 0, h, variant=variant, stream=s)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    ds.close()
    return got


def assert_full_parity(got_rows, path, m, stored_ids, name):
    bad = np.argwhere(got_rows[..., 3].view(np.uint32) != stored_ids.astype(np.float32).view(np.uint32))
    assert bad.size == 0, f"{name}: {len(bad)} tri_id mismatches of {stored_ids.size}, first {bad[:5].tolist()}"
    want = oracle_rgba(path, m, stored_ids)
    d = np.abs(got_rows[..., :3] - want[..., :3])
    assert float(d.max()) <= RGB_TOL, f"{name}: max rgb delta {d.max()}"


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(META))
def test_gpu_reproduces_full_fixture(gpu, paths, ids, name):
    m = META[name]
    got = gpu_frame(paths[name], m)
    assert_full_parity(got[rows_of(m)], paths[name], m, ids[name], name)


@pytest.mark.gpu
def test_gpu_engine_bands_reproduce_full_c3_fixture(gpu, paths, ids):
    """The headline frame through the frame engine's multi-device path (8 interleaved bands,
    all-to-all id exchange, compositor shading; fake devices on one GPU), every pixel."""
    from simpleraytracer_amd.engine import FrameEngine

    name = "c3_soup100k_1080p"
    m = META[name]
    with FrameEngine(paths[name], m["width"], m["height"], devices=[0] * 8, batch=8, queues=1) as e:
        e.set_inputs(offsets_for(m))
        e.run(1)
        for k in (0, 5):  # composited on devices 0 and 5
            assert_full_parity(e.read_frame(k), paths[name], m, ids[name], name)


@pytest.mark.gpu
@pytest.mark.parametrize("p", [2, 8])
def test_gpu_engine_rotated_bands_reproduce_full_c3_fixture(gpu, paths, ids, p):
    """The headline frame as P rotated contiguous bands (all-to-all, the band record pass skipping the
    record blocks that cannot reach a band; fake devices on one GPU), every pixel of every frame."""
    from simpleraytracer_amd.engine import FrameEngine

    name = "c3_soup100k_1080p"
    m = META[name]
    with FrameEngine(paths[name], m["width"], m["height"], devices=[0] * p, batch=p, queues=1, rows="rotated") as e:
        e.set_inputs(offsets_for(m))
        e.run(1)
        for k in range(p):  # composited on every device: every device traced every band once
            assert_full_parity(e.read_frame(k), paths[name], m, ids[name], name)
