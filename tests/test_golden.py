"""Committed golden fixtures (tests/golden/, made by tests/golden/make_golden.py).

CPU: the scene generators reproduce the committed SHA-256, and the oracle reproduces the
committed frames bit-for-bit. GPU: the HIP path reproduces the same fixtures (ids bit-exact,
RGB within 1e-5) without running the oracle.
"""
from __future__ import annotations

import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

import simpleraytracer_amd as srt

GOLDEN = Path(__file__).resolve().parent / "golden"
SCENES = json.loads((GOLDEN / "scenes.json").read_text())
FRAMES = json.loads((GOLDEN / "frames.json").read_text())


@pytest.fixture(scope="module")
def golden_paths(tmp_path_factory):
    d = tmp_path_factory.mktemp("golden")
    out = {}
    for name, spec in SCENES.items():
        kw = {k: v for k, v in spec.items() if k in ("triangles", "seed", "size")}
        out[name] = srt.write_scene(str(d / f"{name}.srt"), spec["kind"], **kw)
    return out


@pytest.fixture(scope="module")
def fixtures():
    return dict(np.load(GOLDEN / "frames.npz"))


def offsets_for(seed, w, h):
    if seed is None:
        return np.full((h, w, 2), 0.5, np.float32)
    return np.random.default_rng(seed).random((h, w, 2), dtype=np.float32)


@pytest.mark.parametrize("name", sorted(SCENES))
def test_scene_generators_are_deterministic(golden_paths, name):
    assert hashlib.sha256(Path(golden_paths[name]).read_bytes()).hexdigest() == SCENES[name]["sha256"]


@pytest.mark.parametrize("name", sorted(FRAMES))
def test_oracle_reproduces_golden(golden_paths, fixtures, name):
    from oracle.srt_oracle import OracleScene

    scene, w, h, r0, rc, step, seed = FRAMES[name]
    img = OracleScene(golden_paths[scene]).render(w, h, offsets_for(seed, w, h), row_begin=r0, row_count=rc,
                                                  row_step=step)
    rows = fixtures[f"{name}__rows"]
    assert np.array_equal(rows, np.arange(r0, r0 + rc, step))
    assert np.array_equal(img[rows].view(np.uint32), fixtures[f"{name}__rgba"].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(FRAMES))
def test_gpu_reproduces_golden(gpu, golden_paths, fixtures, name):
    import torch

    scene, w, h, r0, rc, step, seed = FRAMES[name]
    ds = srt.DeviceScene(golden_paths[scene], 0)
    s = torch.cuda.current_stream()
    ds.prepare(w, h, s)
    off = torch.from_numpy(offsets_for(seed, w, h)).cuda()
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    ds.trace(off, out, 0, h, stream=s)
    torch.cuda.synchronize()
    got = out.cpu().numpy()[fixtures[f"{name}__rows"]]
    want = fixtures[f"{name}__rgba"]
    assert np.array_equal(got[..., 3].view(np.uint32), want[..., 3].view(np.uint32))
    assert float(np.abs(got[..., :3] - want[..., :3]).max()) <= 1e-5
    ds.close()
