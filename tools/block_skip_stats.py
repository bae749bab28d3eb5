#!/usr/bin/env python3
"""How many 256-record blocks of the spatial (Morton) order a band's record pass needs (the block skip,
render.hip BandMayReach), per band layout, for the C3 soup at 1080p: contiguous (rotated) bands vs
interleaved 16-row tile rows. Block extents approximated by the projected vertex rows (the kernels use
the exact screen boxes, slightly larger); the numbers quoted in DESIGN.md section 7.

    python tools/block_skip_stats.py
"""
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import simpleraytracer_amd as srt
from test_gpu_parity import morton_order_numpy
d = tempfile.mkdtemp()
path = srt.write_scene(os.path.join(d, "s.srt"), "soup", 100_000)
order = morton_order_numpy(path)
sc = srt.read_scene(path)
v = sc["vertices"].astype(np.float64)[order]
H = 1080
# projected vertex y in rows (camera at origin looking +z, vfov 60: y_img = (0.5 - y/(z*2*tan30)) * H)
t = np.tan(np.radians(30))
ys = np.stack([(0.5 - v[:, 3*k+1] / (v[:, 3*k+2] * 2 * t)) * H for k in range(3)], 1)
lo, hi = ys.min(1), ys.max(1)
n = len(v); nb = (n + 255) // 256
blo = np.array([lo[i*256:(i+1)*256].min() for i in range(nb)]); bhi = np.array([hi[i*256:(i+1)*256].max() for i in range(nb)])
print("blocks", nb, "mean y extent rows", (bhi - blo).mean())
for P in (2, 4, 8):
    b = -(-H // P)
    need = []
    for j in range(P):
        r0, r1 = j * b, min(H, (j + 1) * b) - 1
        need.append(((bhi >= r0 - 1) & (blo <= r1 + 1)).sum())
    print("P", P, "needed blocks per band", need, "mean frac", np.mean(need) / 400)
    # interleaved 16-row tile rows
    need = []
    for j in range(P):
        rows = np.zeros(H, bool)
        for tr in range(j, -(-H // 16), P):
            rows[tr*16:(tr+1)*16] = True
        cum = np.concatenate([[0], np.cumsum(rows)])
        a = np.clip(np.floor(blo) - 1, 0, H - 1).astype(int); bb = np.clip(np.floor(bhi) + 1, 0, H - 1).astype(int)
        need.append(((cum[bb + 1] - cum[a]) > 0).sum())
    print("P", P, "interleaved needed", need, "mean frac", np.mean(need) / 400)
