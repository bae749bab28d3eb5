#!/usr/bin/env python3
"""Per-block phase breakdown of the cull kernel (diagnostic build; run on the GPU box).

    make diag && SRT_LIB=simpleraytracer_amd/lib_diag/libModelRunner.so python tools/diag_cull.py

Renders the headline frame with the `make diag` library (s_memtime stamps around the cull
kernel's phases, render.hip SRT_DIAG) and prints the distribution of stream / gather /
filter+walk cycles and survivor counts over the blocks, heaviest blocks first.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    assert os.environ.get("SRT_LIB"), "set SRT_LIB to the diag library"
    import torch

    import simpleraytracer_amd as srt
    from simpleraytracer_amd import _native

    w, h = int(os.environ.get("W", 1920)), int(os.environ.get("H", 1080))
    tri = int(os.environ.get("TRI", 100_000))
    lib = _native.lib()
    lib.srtDiagRead.restype = ctypes.c_int
    lib.srtDiagRead.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    with tempfile.TemporaryDirectory() as d:
        path = srt.write_scene(os.path.join(d, "s.srt"), "soup", tri)
        scene = srt.DeviceScene(path, 0)
        stream = torch.cuda.current_stream()
        off = torch.full((h, w, 2), 0.5, dtype=torch.float32, device="cuda")
        out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
        scene.prepare(w, h, stream)
        for _ in range(3):
            scene.trace(off, out, 0, h, variant="cull", stream=stream)
        torch.cuda.synchronize()
        buf = np.zeros((65536, 8), np.uint64)
        assert lib.srtDiagRead(buf.ctypes.data, buf.nbytes) == 0, _native.last_error()
        scene.close()
    shape = "8x4 tiles, bins " + os.environ.get("SRT_CULL_BIN", "1")
    parts = int(os.environ.get("PARTS", 2))  # trace blocks per cull tile (render.hip kParts)
    gx, gy = (w + 63) // 64, (h + 31) // 32
    nb = gx * gy * parts
    allb = buf[:nb].astype(np.float64)
    ran = allb[:, 6] > 0
    d = allb[ran]
    # packet-walk blocks: [1] gather, [2] walk, [3] survivors, [4] packets, [5] batches, [6] total
    names = ["stream", "gather", "walk", "surv", "packets", "batches", "total"]
    summary = {"shape": f"{gx}x{gy} tiles x {parts} parts, bins " + os.environ.get("SRT_CULL_BIN", "1"),
               "blocks": nb, "blocks_run": int(ran.sum())}
    for i, n in enumerate(names):
        col = d[:, i]
        summary[n] = {"mean": float(col.mean()), "p50": float(np.median(col)), "p90": float(np.percentile(col, 90)),
                      "max": float(col.max()), "sum": float(col.sum())}
    mode = buf[:nb, 7].astype(np.int64)
    cnt = (mode >> 16) & 0xFFFFFF
    summary["tile_list"] = {"mean": float(cnt.mean()), "p50": float(np.median(cnt)), "p90": float(np.percentile(cnt, 90)),
                            "max": int(cnt.max()), "sum": int(cnt.sum()) // parts, "large": int((mode >> 40).max())}
    # Balance: total block-cycles spread over 256 CUs x 4 SIMDs vs the heaviest block.
    summary["balance"] = {"sum_cycles_per_simd": float(d[:, 6].sum() / 1024), "max_block_cycles": float(d[:, 6].max())}
    idx = np.nonzero(ran)[0]
    heavy = idx[np.argsort(-allb[idx, 6])[:8]]
    summary["heaviest"] = [{"block": int(b), **{n: int(allb[b, i]) for i, n in enumerate(names)}} for b in heavy]
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
