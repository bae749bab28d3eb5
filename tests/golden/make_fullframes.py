#!/usr/bin/env python3
"""Regenerate tests/golden/fullframes.* (run from the repo root: python tests/golden/make_fullframes.py).

Full-size fixtures of the headline configs, made by the CPU oracle (test infrastructure, brute
force over every triangle; a few minutes on 8 cores):
  * c3_soup100k_1080p  -- every pixel of the C3 frame (1920 x 1080, 100k triangles), uniform offsets
  * c2_cornell_1080p   -- every pixel of the C2 frame
  * c3_random_rows     -- C3 with seeded U[0,1) per-pixel offsets, every 8th row
  * c5_soup1m_4k_rows  -- C5 (3840 x 2160, 1M triangles), 64 evenly spaced rows
Stored: the hit ids (int32, the bit-exact channel) of the rendered rows, and the SHA-256 of the
oracle's RGBA bytes of those rows; the RGB channels are re-derived at test time by the oracle's
deferred shading of the stored ids (tests/test_golden_full.py checks that this reproduces the
SHA-256), so the fixture stays small. The reference holds no render fixture of its own
(SURVEY.md sections 0, 8c); these freeze the oracle at full size. Data, not reference source.
"""
from __future__ import annotations

import hashlib
import json
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))

import simpleraytracer_amd as srt  # noqa: E402
from oracle.srt_oracle import OracleScene  # noqa: E402

OUT = REPO / "tests" / "golden"

# name: (scene kind, triangles, width, height, rows spec (begin, step, count), offsets seed or None)
FULL = {
    "c3_soup100k_1080p": ("soup", 100_000, 1920, 1080, (0, 1, 1080), None),
    "c2_cornell_1080p": ("cornell", 0, 1920, 1080, (0, 1, 1080), None),
    "c3_random_rows": ("soup", 100_000, 1920, 1080, (3, 8, 135), 42),
    "c5_soup1m_4k_rows": ("soup", 1_000_000, 3840, 2160, (17, 33, 64), None),
}


def rows_of(spec):
    b, step, count = spec
    return np.arange(b, b + step * count, step)


def offsets_for(seed, w, h):
    if seed is None:
        return np.full((h, w, 2), 0.5, np.float32)
    return np.random.default_rng(seed).random((h, w, 2), dtype=np.float32)


def scene_file(tmp, kind, tri):
    p = Path(tmp) / f"{kind}_{tri}.srt"
    if not p.exists():
        if kind == "soup":
            srt.write_scene(str(p), "soup", tri)
        else:
            srt.write_scene(str(p), kind)
    return str(p)


def main():
    meta, arrays = {}, {}
    with tempfile.TemporaryDirectory() as tmp:
        for name, (kind, tri, w, h, rspec, seed) in FULL.items():
            t0 = time.time()
            o = OracleScene(scene_file(tmp, kind, tri))
            rows = rows_of(rspec)
            img = o.render(w, h, offsets_for(seed, w, h), row_begin=int(rows[0]), row_count=int(rows[-1] - rows[0] + 1),
                           row_step=int(rspec[1]))[rows]
            ids = img[..., 3].astype(np.int32)
            assert np.array_equal(ids.astype(np.float32).view(np.uint32), img[..., 3].view(np.uint32))
            arrays[name] = ids
            meta[name] = {"scene": kind, "triangles": tri, "width": w, "height": h, "rows": list(rspec),
                          "offsets_seed": seed, "rgba_sha256": hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest(),
                          "hit_fraction": round(float((ids >= 0).mean()), 4)}
            print(f"{name}: {time.time() - t0:.1f} s, hit fraction {meta[name]['hit_fraction']}", flush=True)
    np.savez_compressed(OUT / "fullframes.npz", **arrays)
    (OUT / "fullframes.json").write_text(json.dumps(meta, indent=1) + "\n")
    print("wrote", OUT / "fullframes.npz", (OUT / "fullframes.npz").stat().st_size, "bytes")


if __name__ == "__main__":
    main()
