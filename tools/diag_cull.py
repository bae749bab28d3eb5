#!/usr/bin/env python3
"""Per-block timeline of the cull trace kernel (diagnostic build; run on the GPU box).

    make diag && SRT_LIB=simpleraytracer_amd/lib_diag/libModelRunner.so python tools/diag_cull.py

Renders one frame (headline config by default; env W, H, TRI, OFFSETS=random; BATCH=8: one launch
of 8 frames, the headline's launch shape) with the `make diag` library, whose trace kernel stamps every block's start and end (s_memrealtime,
100 MHz), its work item (tile part, chunk of a split part, last arriver) and the packet-walk
phase cycles (render.hip SRT_DIAG). Prints the kernel span, block durations, how many blocks
run over time, the critical chains of split parts and the blocks that finish last.
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
COLS = 16  # render.hip kDiagCols


def stats(col):
    col = np.asarray(col, np.float64)
    if col.size == 0:
        return {}
    return {"mean": round(float(col.mean()), 2), "p50": round(float(np.median(col)), 2),
            "p90": round(float(np.percentile(col, 90)), 2), "max": round(float(col.max()), 2),
            "sum": round(float(col.sum()), 1)}


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
        if os.environ.get("OFFSETS") == "random":
            g = torch.Generator().manual_seed(0x5EED)
            off = torch.rand((h, w, 2), generator=g, dtype=torch.float32).cuda()
        else:
            off = torch.full((h, w, 2), 0.5, dtype=torch.float32, device="cuda")
        nb = int(os.environ.get("BATCH", "1"))
        out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
        outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in range(nb)]
        for _ in range(3):
            scene.prepare(w, h, stream)
            if nb == 1:
                scene.trace(off, out, 0, h, variant="cull", stream=stream)
            else:
                scene.trace_batch([off] * nb, outs, 0, h, variant="cull", stream=stream)
        torch.cuda.synchronize()
        buf = np.zeros((65536, COLS), np.uint64)
        assert lib.srtDiagRead(buf.ctypes.data, buf.nbytes) == 0, _native.last_error()
        scene.close()
    ran = np.nonzero(buf[:, 9] > 0)[0]
    if os.environ.get("DIAG_RAW"):  # every stamped block's row, for offline analysis
        np.save(os.environ["DIAG_RAW"], buf[ran])
    b = buf[ran].astype(np.float64)
    t0 = b[:, 8].min()
    start = (b[:, 8] - t0) / 100.0  # us
    end = (b[:, 9] - t0) / 100.0
    dur = end - start
    info = buf[ran, 11]
    chunk, nch, last = info & 0xFFFF, (info >> 16) & 0xFFFF, (info >> 32) & 1
    item = buf[ran, 10]
    summary = {"frame": f"{w}x{h}, {tri} triangles, offsets {os.environ.get('OFFSETS', 'uniform')}",
               "blocks": int(ran.size), "span_us": round(float(end.max()), 2),
               "duration_us": stats(dur), "split_blocks": int((nch > 1).sum()),
               "split_parts": int(len(set(item[nch > 1].tolist())))}
    pk = buf[ran, 7] & 8 != 0  # packet-walk blocks
    summary["packet_walk"] = {"blocks": int(pk.sum()), "gather_cycles": stats(b[pk, 1]), "walk_cycles": stats(b[pk, 2]),
                              "survivors": stats(b[pk, 3]), "packets": stats(b[pk, 4]),
                              "candidates": stats(buf[ran][pk, 7] >> 40)}
    # blocks running over time (1 us bins)
    nbins = int(np.ceil(end.max())) + 1
    active = np.zeros(nbins)
    for s0, e0 in zip(start, end):
        active[int(s0):int(np.ceil(e0))] += 1
    summary["active_blocks_per_us"] = [int(x) for x in active]
    # split parts: start of the first chunk to the end of the last arriver
    chains = {}
    for i in np.nonzero(nch > 1)[0]:
        c = chains.setdefault(int(item[i]), [1e9, 0.0, 0])
        c[0] = min(c[0], start[i])
        c[1] = max(c[1], end[i])
        c[2] = int(nch[i])
    top = sorted(chains.items(), key=lambda kv: -kv[1][1])[:8]
    summary["split_chains_latest"] = [{"item": k, "first_start": round(v[0], 2), "end": round(v[1], 2), "chunks": v[2]}
                                      for k, v in top]
    # where a block's time goes (gather / walk in shader cycles at the measured clock ratio, the rest
    # = descriptor / epilogue: split merge, shading loads, stores)
    cyc = b[:, 1] + b[:, 2]
    ok = (dur > 0.5) & (cyc > 0)
    ghz = float(np.median(cyc[ok] / (dur[ok] * 1e3))) if ok.any() else 0.0
    summary["phases_us"] = {"clock_ghz_lower_bound": round(ghz, 3)}
    for name, sel in (("split", nch > 1), ("whole", (nch <= 1) & (buf[ran, 7] & 8 != 0))):
        if sel.any():
            g = b[sel, 1] / 2400.0
            wk = b[sel, 2] / 2400.0
            summary["phases_us"][name] = {"blocks": int(sel.sum()), "dur": stats(dur[sel]), "gather": stats(g),
                                          "walk": stats(wk), "rest": stats(dur[sel] - g - wk)}
    # block classes by work-item flags (render.hip kItemRegular 1, kItemFull 2, kItemEmpty 4)
    fl = buf[ran, 12] & 0xFFFFFFFF
    classes = {"empty": (fl & 4) != 0, "full": ((fl & 2) != 0) & ((fl & 4) == 0),
               "list_whole": ((fl & 6) == 0) & (nch <= 1), "list_split": ((fl & 6) == 0) & (nch > 1)}
    summary["classes"] = {k: {"blocks": int(v.sum()), "dur_us": stats(dur[v]),
                              "gather_us": stats(b[v, 1] / 2400.0), "walk_us": stats(b[v, 2] / 2400.0)}
                          for k, v in classes.items() if v.any()}
    slots = int(os.environ.get("SLOTS", "1536"))
    summary["occupancy"] = {"block_us": round(float(dur.sum()), 1), "slots": slots,
                            "busy_frac": round(float(dur.sum() / (end.max() * slots)), 3),
                            "note": "sum of block lifetimes / (span x resident block slots)"}
    order = np.argsort(-end)[:12]
    summary["last_to_finish"] = [{"grid_block": int(ran[i]), "item": int(item[i]), "chunk": int(chunk[i]),
                                  "chunks": int(nch[i]), "last": int(last[i]), "start": round(float(start[i]), 2),
                                  "end": round(float(end[i]), 2), "candidates": int(buf[ran[i], 7] >> 40),
                                  "packets": int(buf[ran[i], 4])} for i in order]
    order = np.argsort(-dur)[:8]
    summary["longest"] = [{"grid_block": int(ran[i]), "item": int(item[i]), "chunks": int(nch[i]),
                           "start": round(float(start[i]), 2), "dur": round(float(dur[i]), 2),
                           "candidates": int(buf[ran[i], 7] >> 40), "survivors": int(buf[ran[i], 3]),
                           "packets": int(buf[ran[i], 4])} for i in order]
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
