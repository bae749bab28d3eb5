#!/usr/bin/env python3
"""How much of the trace kernel's pixel-test work could a front-to-back depth cull remove? (VERDICT r05
"next" 1, step (a): on the CPU, before any kernel work.)

Model of the trace kernel's work (render.hip TraceCullKernel): a block is one
64 x 16 tile part; its candidates are the records whose screen box meets the tile; a candidate costs
one exact test per pixel of its range = its screen box clipped to the tile (columns x rows). The
screen box is taken here as the projected triangle's pixel bounding box (the kernel's box is that up to
rounding slack), uniform 0.5 offsets (the headline).

A depth cull visits the tile's candidates nearest-first by a lower bound of their depth (here the
smallest vertex depth; the BVH variant's DepthLowerBound is this bound over the screen box) and drops a
candidate when the bound exceeds -- strictly -- the largest best t over the cells of the tile its range
touches (so it can neither win nor tie). With candidates in bound order, every pixel whose final winner
has a smaller bound already holds its final t when the candidate is reached, so the final frame's per-
pixel t (from the oracle's ids) gives the ideal cull exactly. Cells: whole 64-pixel row segments (the
verdict's proposal), 16 / 8 / 4-pixel row segments, 8 x 4 and 4 x 4 pixel boxes, and the exact per-range
maximum (the best any cull of this kind can do). Batches: the kernel walks 128 candidates per batch
between barriers, so a cull known only after a batch removes only candidates of later batches; `batched`
applies the per-cell cull with the t values of the batches before (bound order).

    python tools/depth_cull_study.py [--out profiles/r06/depth_cull/study.json]

Prints the histogram (candidates per tile) and, per cell size, the share of pixel tests removed over
the centre tiles (the heaviest tenth by candidates: the critical path) and over the frame.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def frame_vectors(cam, W, H):
    eye, look, up, vfov = np.array(cam[:3], np.float64), np.array(cam[3:6], np.float64), np.array(cam[6:9]), cam[9]
    f = look - eye
    f /= np.linalg.norm(f)
    r = np.cross(f, up)
    r /= np.linalg.norm(r)
    u = np.cross(r, f)
    hh = np.tan(np.radians(vfov) / 2)
    hw = hh * W / H
    base = f - hw * r + hh * u
    return eye, f, r, u, hh, hw, base


def render_ids(path, W, H):
    import simpleraytracer_amd as srt

    os.environ["ML_VISIBLE_DEVICES"] = "cpu"
    return srt.render(path, W, H)[..., 3].astype(np.int64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--triangles", type=int, default=100_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import simpleraytracer_amd as srt
    from oracle.srt_oracle import OracleScene

    W, H = a.width, a.height
    with tempfile.TemporaryDirectory() as d:
        path = srt.write_scene(os.path.join(d, "soup.srt"), "soup", a.triangles)
        sc = OracleScene(path)
        t0 = time.time()
        ids = render_ids(path, W, H)
        edges = sc.edges(W, H).astype(np.float64)
        verts = sc.vertices.astype(np.float64).reshape(-1, 3, 3)
        cam = sc.camera
    eye, f, r, u, hh, hw, base = frame_vectors(cam, W, H)
    # per-pixel best t (the hit's depth along f; the ray's f component is 1): t = vol / det
    ys, xs = np.mgrid[0:H, 0:W]
    fx = (xs + 0.5) / W
    fy = (ys + 0.5) / H
    hit = ids >= 0
    e = edges[np.where(hit, ids, 0)]
    det = (e[..., 0] + fx * e[..., 1] + fy * e[..., 2]) + (e[..., 3] + fx * e[..., 4] + fy * e[..., 5]) + \
          (e[..., 6] + fx * e[..., 7] + fy * e[..., 8])
    tbest = np.where(hit, e[..., 9] / np.where(hit, det, 1.0), np.inf)
    # triangles: projected pixel boxes (pixel centres x + 0.5 = fx W), depth lower bound
    P = verts - eye
    z = P @ f
    q = P / z[..., None] - base
    px = (q @ r) / (2 * hw) * W - 0.5
    py = (q @ u) / (-2 * hh) * H - 0.5
    x0 = np.ceil(px.min(1)).astype(np.int64)
    x1 = np.floor(px.max(1)).astype(np.int64)
    y0 = np.ceil(py.min(1)).astype(np.int64)
    y1 = np.floor(py.max(1)).astype(np.int64)
    lb = z.min(1)
    ok = (z.min(1) > 0) & (x0 <= x1) & (y0 <= y1) & (x1 >= 0) & (y1 >= 0) & (x0 < W) & (y0 < H)
    x0, x1, y0, y1 = np.clip(x0, 0, W - 1), np.clip(x1, 0, W - 1), np.clip(y0, 0, H - 1), np.clip(y1, 0, H - 1)
    TW, TH = 64, 16
    tx0, tx1, ty0, ty1 = x0 // TW, x1 // TW, y0 // TH, y1 // TH
    ntx, nty = (W + TW - 1) // TW, (H + TH - 1) // TH
    # (tile, triangle) pairs
    pairs = []
    for i in np.nonzero(ok)[0]:
        for ty in range(ty0[i], ty1[i] + 1):
            for tx in range(tx0[i], tx1[i] + 1):
                pairs.append((ty * ntx + tx, i))
    pairs = np.array(pairs, np.int64)
    order = np.lexsort((lb[pairs[:, 1]], pairs[:, 0]))  # per tile, nearest bound first
    pairs = pairs[order]
    tiles = pairs[:, 0]
    starts = np.searchsorted(tiles, np.arange(ntx * nty + 1))
    cells = {"row64": (64, 1), "row16": (16, 1), "row8": (8, 1), "row4": (4, 1), "box8x4": (8, 4),
             "box4x4": (4, 4), "pixel": (1, 1)}
    tot = {k: 0.0 for k in ["tests", "range_exact"] + [c for c in cells] + [c + "_batched" for c in cells]}
    centre = {k: 0.0 for k in tot}
    cand_hist = np.zeros(ntx * nty, np.int64)
    counts = np.diff(starts)
    centre_min = int(np.percentile(counts[counts > 0], 90))  # the heaviest tenth of the listed tiles
    for t in range(ntx * nty):
        s, e_ = starts[t], starts[t + 1]
        if s == e_:
            continue
        ty, tx = divmod(t, ntx)
        X0, Y0 = tx * TW, ty * TH
        tri = pairs[s:e_, 1]
        cand_hist[t] = len(tri)
        tb = tbest[Y0:Y0 + TH, X0:X0 + TW]
        th, tw = tb.shape
        cx0 = np.clip(x0[tri] - X0, 0, tw - 1)
        cx1 = np.clip(x1[tri] - X0, 0, tw - 1)
        cy0 = np.clip(y0[tri] - Y0, 0, th - 1)
        cy1 = np.clip(y1[tri] - Y0, 0, th - 1)
        inside = (x1[tri] >= X0) & (x0[tri] < X0 + tw) & (y1[tri] >= Y0) & (y0[tri] < Y0 + th)
        n = np.where(inside, (cx1 - cx0 + 1) * (cy1 - cy0 + 1), 0)
        lbt = lb[tri]
        big = len(tri) >= centre_min
        # candidate rank of each pixel's winner in this tile's bound order (1 << 30: a miss / not listed)
        rank_of = np.full(int(tri.max()) + 1, 1 << 30, np.int64)
        rank_of[tri] = np.arange(len(tri))
        idt = ids[Y0:Y0 + th, X0:X0 + tw]
        rank_pix = np.where((idt >= 0) & (idt <= tri.max()), rank_of[np.clip(idt, 0, tri.max())], 1 << 30)
        tests = float(n.sum())
        tot["tests"] += tests
        if big:
            centre["tests"] += tests
        # exact: max of tbest over each candidate's range
        rm = np.array([tb[cy0[k]:cy1[k] + 1, cx0[k]:cx1[k] + 1].max() if inside[k] else -np.inf
                       for k in range(len(tri))])
        kept = float(n[~(lbt > rm)].sum())
        tot["range_exact"] += tests - kept
        if big:
            centre["range_exact"] += tests - kept
        for name, (cw, ch) in cells.items():
            gh, gw = (th + ch - 1) // ch, (tw + cw - 1) // cw
            pad = np.full((gh * ch, gw * cw), np.inf)
            pad[:th, :tw] = tb
            cmax = pad.reshape(gh, ch, gw, cw).max(axis=(1, 3))
            cmv = np.array([cmax[cy0[k] // ch:cy1[k] // ch + 1, cx0[k] // cw:cx1[k] // cw + 1].max() if inside[k]
                            else -np.inf for k in range(len(tri))])
            removed = float(n[lbt > cmv].sum())
            tot[name] += removed
            if big:
                centre[name] += removed
            # batched: the cells' t after the batches before (128 candidates per batch, bound order): a
            # pixel's running t = its final t if its winner is in an earlier batch, else +inf (a lower bound
            # of the removal: the running t of an unfinished pixel may be finite)
            removed_b = 0.0
            for k in range(len(tri)):
                if not inside[k]:
                    continue
                b0 = (k // 128) * 128
                sub = tb[cy0[k] // ch * ch:(cy1[k] // ch + 1) * ch, cx0[k] // cw * cw:(cx1[k] // cw + 1) * cw]
                rp = rank_pix[cy0[k] // ch * ch:(cy1[k] // ch + 1) * ch, cx0[k] // cw * cw:(cx1[k] // cw + 1) * cw]
                run = np.where(rp < b0, sub, np.inf)
                if lbt[k] > run.max():
                    removed_b += n[k]
            tot[name + "_batched"] += removed_b
            if big:
                centre[name + "_batched"] += removed_b
    frac = lambda d: {k: round(v / d["tests"], 4) for k, v in d.items() if k != "tests"}
    hist_edges = [0, 1, 50, 100, 200, 300, 400, 500, 600, 700, 800, 1000, 10**9]
    hist = np.histogram(cand_hist, bins=hist_edges)[0].tolist()
    out = {"workload": f"soup-{a.triangles} {W}x{H}", "tile": "64x16", "tiles": int(ntx * nty),
           "pairs": int(len(pairs)), "pixel_tests": tot["tests"], "centre_min_candidates": centre_min,
           "centre_tiles": int((cand_hist >= centre_min).sum()), "max_candidates": int(cand_hist.max()),
           "centre_pixel_tests": centre["tests"],
           "removed_frac_frame": frac(tot), "removed_frac_centre": frac(centre),
           "candidates_histogram": {"edges": hist_edges[:-1], "tiles": hist},
           "seconds": round(time.time() - t0, 1)}
    print(json.dumps(out, indent=1))
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
