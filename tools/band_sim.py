#!/usr/bin/env python3
"""Per-rank work of the multi-GPU band pipeline, measured on one GPU (no interconnect).

    python tools/band_sim.py [--ranks 2,4,8] [--queues 3] [--steps 2000] [--batch 8]

For P ranks, rank r's per-frame work in bench.py --mode bands is: the edge-record setup and
bins for the whole frame's records, the trace of band r (hit ids), and -- on every P-th frame,
as the rotating compositor -- the deferred shading of the whole frame. This runs exactly that
stream of kernels for one band at a time with --queues frames in flight and reports the frame
rate each rank could sustain if the gather were free, as Mrays/s of whole frames (W x H per
frame): the compute ceiling of bands x P. The gather's own cost is
modelled there from its bytes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--queues", type=int, default=3)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--triangles", type=int, default=100_000)
    ap.add_argument("--batch", type=int, default=16, help="frames per gather / shading launch (bench.py --batch)")
    ap.add_argument("--rows", default="interleaved", choices=["interleaved", "contiguous"], help="bench.py --rows")
    a = ap.parse_args()
    import torch

    import simpleraytracer_amd as srt
    from simpleraytracer_amd.bands import (band_range, band_rows, interleaved_band_rows, interleaved_frame_rows,
                                           interleaved_range)

    W, H, G = a.width, a.height, max(1, a.batch)
    L = min(G, srt.MAX_BATCH)  # frames per batched trace call
    dev = torch.device("cuda", 0)
    tmp = tempfile.TemporaryDirectory()
    path = srt.write_scene(os.path.join(tmp.name, "soup.srt"), "soup", a.triangles)
    off = torch.full((H, W, 2), 0.5, dtype=torch.float32, device=dev)
    # the frame's real ids, for realistic compositor shading work
    ref_scene = srt.DeviceScene(path, 0)
    ref_scene.prepare(W, H)
    frame_ids = torch.empty((H, W), dtype=torch.int32, device=dev)
    ref_scene.trace_ids(off, frame_ids, 0, H)
    torch.cuda.synchronize()
    ref_scene.close()
    qs = [{"scene": srt.DeviceScene(path, 0), "stream": torch.cuda.Stream(dev),
           "ids": torch.full((G, H, W), -1, dtype=torch.int32, device=dev),
           "rgba": torch.empty((G, H, W, 4), dtype=torch.float32, device=dev)} for _ in range(a.queues)]
    for q in qs:
        q["scene"].prepare(W, H)
    out = {"workload": f"soup-{a.triangles} {W}x{H}", "queues": a.queues, "batch": G, "rows": a.rows, "ranks": {}}
    for P in [int(x) for x in a.ranks.split(",")]:
        per = []
        inter = P if (P > 1 and a.rows == "interleaved") else 0
        B = interleaved_band_rows(H, P) if inter else band_rows(H, P)
        gathered = torch.full((P, G, B, W), -1, dtype=torch.int32, device=dev)  # band-major, as gathered
        band_rows_of = []
        for p in range(P):
            fr = torch.from_numpy(interleaved_frame_rows(H, P, p)).to(dev) if inter else None
            b0, c = interleaved_range(H, P, p) if inter else band_range(H, P, p)
            gathered[p, :, :c] = frame_ids.index_select(0, fr) if inter else frame_ids[b0:b0 + c]
            band_rows_of.append((b0, c, off.index_select(0, fr).contiguous() if inter else off[b0:b0 + c]))
        for r in range(P):
            r0, rows, band_off = band_rows_of[r]
            for q in qs:
                q["runs"] = []
                for s0 in range(0, G, L):
                    n = min(L, G - s0)
                    if P == 1:
                        q["runs"].append(q["scene"].bind_trace_batch([off] * n, [q["rgba"][j] for j in range(s0, s0 + n)],
                                                                     0, H, stream=q["stream"]))
                    elif rows:
                        q["runs"].append(q["scene"].bind_trace_batch([band_off] * n,
                                                                     [q["ids"][j, :rows] for j in range(s0, s0 + n)],
                                                                     r0, rows, stream=q["stream"], ids=True,
                                                                     row_interleave=max(1, inter)))

            def step(k):  # batch k: G frames
                q = qs[k % a.queues]
                for run in q["runs"]:
                    run()
                if P > 1 and k % P == r:  # this rank composites batch k
                    q["scene"].shade_bands(off, gathered, q["rgba"], B, stream=q["stream"], interleaved=inter)

            batches = max(1, a.steps // G)
            for k in range(max(2, a.warmup // G) * a.queues):
                step(k)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(batches):
                step(k)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            frames = batches * G
            per.append({"rank": r, "rows": rows, "us_per_frame": round(dt / frames * 1e6, 2),
                        "frame_mrays_per_s": round(W * H * frames / dt / 1e6, 1)})
        worst = min(p["frame_mrays_per_s"] for p in per)
        out["ranks"][P] = {"per_rank": per, "ceiling_mrays_per_s": worst, "band_rows": band_rows(H, P)}
        print(json.dumps({"P": P, "ceiling_mrays_per_s": worst, "per_rank": per}), flush=True)
    print(json.dumps(out))
    for q in qs:
        q["scene"].close()
    tmp.cleanup()


if __name__ == "__main__":
    main()
