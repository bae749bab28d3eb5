#!/usr/bin/env python3
"""Regenerate tests/golden/ fixtures (run from the repo root: python tests/golden/make_golden.py).

What they are: SHA-256 of the generated scene files (the generators are part of the product
and must stay deterministic), and small CPU-oracle frames/rows of every config. The reference
holds no render fixture of its own, so these freeze the oracle
(DESIGN.md section 8); they are data, not reference source.
"""
from __future__ import annotations

import hashlib
import json
import sys
import tempfile
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))

import simpleraytracer_amd as srt  # noqa: E402
from oracle.srt_oracle import OracleScene  # noqa: E402

OUT = REPO / "tests" / "golden"

SCENES = {
    "triangle": dict(kind="triangle"),
    "cornell": dict(kind="cornell"),
    "soup100k": dict(kind="soup", triangles=100_000),
    "soup1m": dict(kind="soup", triangles=1_000_000),
    "soup2k_seed7": dict(kind="soup", triangles=2_000, seed=7),
}

# (scene, width, height, row_begin, row_count, row_step, offsets seed or None)
FRAMES = {
    "c1_triangle_256": ("triangle", 256, 256, 0, 256, 1, None),
    "c2_cornell_192x108": ("cornell", 192, 108, 0, 108, 1, None),
    "c2_cornell_1080p_rows": ("cornell", 1920, 1080, 5, 1075, 97, None),
    "c3_soup100k_1080p_rows": ("soup100k", 1920, 1080, 0, 1080, 359, None),
    "soup2k_160x90_random_offsets": ("soup2k_seed7", 160, 90, 0, 90, 1, 42),
}


def sha256(path):
    return hashlib.sha256(Path(path).read_bytes()).hexdigest()


def offsets_for(seed, w, h):
    if seed is None:
        return np.full((h, w, 2), 0.5, np.float32)
    return np.random.default_rng(seed).random((h, w, 2), dtype=np.float32)


def build(tmp):
    paths = {}
    for name, kw in SCENES.items():
        p = Path(tmp) / f"{name}.srt"
        kind = kw.pop("kind")
        srt.write_scene(str(p), kind, **kw)
        kw["kind"] = kind
        paths[name] = str(p)
    return paths


def render_fixture(paths, spec):
    scene, w, h, r0, rc, step, seed = spec
    img = OracleScene(paths[scene]).render(w, h, offsets_for(seed, w, h), row_begin=r0, row_count=rc,
                                           row_step=step)
    rows = np.arange(r0, r0 + rc, step)
    return rows, img[rows]


def main():
    with tempfile.TemporaryDirectory() as tmp:
        paths = build(tmp)
        scenes = {name: {"sha256": sha256(p), **SCENES[name]} for name, p in paths.items()}
        (OUT / "scenes.json").write_text(json.dumps(scenes, indent=1, sort_keys=True) + "\n")
        arrays = {}
        for name, spec in FRAMES.items():
            rows, img = render_fixture(paths, spec)
            arrays[f"{name}__rows"] = rows
            arrays[f"{name}__rgba"] = img
        np.savez_compressed(OUT / "frames.npz", **arrays)
        (OUT / "frames.json").write_text(json.dumps({k: list(v[:6]) + [v[6]] for k, v in FRAMES.items()},
                                                    indent=1) + "\n")
    print("wrote", OUT / "scenes.json", OUT / "frames.npz")


if __name__ == "__main__":
    main()
