#!/usr/bin/env python3
"""Timeline of one frame's setup and trace kernels (diagnostic build; run on the GPU box).

    make diag && SRT_LIB=simpleraytracer_amd/lib_diag/libModelRunner.so python tools/diag_setup.py

Renders a few frames (headline config; env W, H, TRI) with the `make diag` library and reads the
last frame's stamps (s_memrealtime, 100 MHz, thread 0 of each block): PrepareBinKernel's phase
boundaries per block (render.hip SRT_SETUP_MARK: 0 start, 1 record computed, 2 tile bounds, 3 records
stored + histogram zeroed, 4 bins in LDS, 5 list reservations, 6 list stores; tile-info blocks: 0
start, 1 end), WorkOrderKernel's (0 start, 1 tile items in LDS, 2 totals, 3 bucket bases, 4 end) and
the trace kernel's block start / end. Times in us from the bin launch's first block start.
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
COLS = 16
ORDER_ROW, BIN_ROW = 60000, 61000  # render.hip kDiagOrderRow, kDiagBinRow


def q(v):
    v = np.asarray(v, np.float64)
    if v.size == 0:
        return None
    return [round(float(x), 2) for x in (v.min(), np.median(v), np.percentile(v, 90), v.max())]


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
        for _ in range(5):
            scene.prepare(w, h, stream)
            scene.trace(off, out, 0, h, variant="cull", stream=stream)
        torch.cuda.synchronize()
        buf = np.zeros((65536, COLS), np.uint64)
        assert lib.srtDiagRead(buf.ctypes.data, buf.nbytes) == 0, _native.last_error()
        scene.close()
    binr = buf[BIN_ROW:BIN_ROW + 4096]
    ordr = buf[ORDER_ROW:ORDER_ROW + 1000]
    bin_rows = binr[binr[:, 15] > 0]
    ord_rows = ordr[ordr[:, 15] > 0]
    t0 = float(bin_rows[:, 0].min())
    us = lambda v: (v.astype(np.float64) - t0) / 100.0  # noqa: E731
    info = bin_rows[bin_rows[:, 15] == 2]
    rec = bin_rows[bin_rows[:, 15] >= 6]
    out = {"frame": f"{w}x{h}, {tri} triangles", "bin_blocks": int(len(bin_rows)),
           "tile_info_blocks": {"n": int(len(info)), "start": q(us(info[:, 0])), "end": q(us(info[:, 1]))},
           "record_blocks": {"n": int(len(rec))}}
    names = ["start", "record", "bounds", "stored", "bins_lds", "reserved", "listed"]
    for k, n in enumerate(names):
        out["record_blocks"][n] = q(us(rec[:, k]))
    out["order_blocks"] = {"n": int(len(ord_rows))}
    for k, n in enumerate(["start", "items", "totals", "bases", "end"]):
        out["order_blocks"][n] = q(us(ord_rows[:, k]))
    tr = buf[:65536 - 6000]
    tr = tr[(tr[:, 9] > 0) & (tr[:, 8] >= bin_rows[:, 0].min())]
    out["trace_blocks"] = {"n": int(len(tr)), "start": q(us(tr[:, 8])), "end": q(us(tr[:, 9]))}
    print("quantiles: [min, median, p90, max] us from the first bin block's start")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
