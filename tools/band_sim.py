#!/usr/bin/env python3
"""Per-rank work of the multi-GPU band pipeline, measured on one GPU (no interconnect).

    python tools/band_sim.py [--ranks 2,4,8] [--queues 3] [--steps 2000]

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
    a = ap.parse_args()
    import torch

    import simpleraytracer_amd as srt
    from simpleraytracer_amd.bands import band_range, band_rows

    W, H = a.width, a.height
    dev = torch.device("cuda", 0)
    tmp = tempfile.TemporaryDirectory()
    path = srt.write_scene(os.path.join(tmp.name, "soup.srt"), "soup", a.triangles)
    off = torch.full((H, W, 2), 0.5, dtype=torch.float32, device=dev)
    qs = [{"scene": srt.DeviceScene(path, 0), "stream": torch.cuda.Stream(dev),
           "ids": torch.full((H, W), -1, dtype=torch.int32, device=dev),
           "rgba": torch.empty((H, W, 4), dtype=torch.float32, device=dev)} for _ in range(a.queues)]
    out = {"workload": f"soup-{a.triangles} {W}x{H}", "queues": a.queues, "ranks": {}}
    for P in [int(x) for x in a.ranks.split(",")]:
        per = []
        for r in range(P):
            r0, rows = band_range(H, P, r)

            def step(k):
                q = qs[k % a.queues]
                q["scene"].prepare(W, H, q["stream"])
                if P == 1:
                    q["scene"].trace(off, q["rgba"], 0, H, stream=q["stream"])
                    return
                if rows:
                    q["scene"].trace_ids(off[r0:r0 + rows], q["ids"][:rows], r0, rows, stream=q["stream"])
                if k % P == r:  # this rank composites frame k
                    q["scene"].shade(off, q["ids"], q["rgba"], 0, H, stream=q["stream"])

            for k in range(a.warmup * a.queues):
                step(k)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(a.steps):
                step(k)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            per.append({"rank": r, "rows": rows, "us_per_frame": round(dt / a.steps * 1e6, 2),
                        "frame_mrays_per_s": round(W * H * a.steps / dt / 1e6, 1)})
        worst = min(p["frame_mrays_per_s"] for p in per)
        out["ranks"][P] = {"per_rank": per, "ceiling_mrays_per_s": worst, "band_rows": band_rows(H, P)}
        print(json.dumps({"P": P, "ceiling_mrays_per_s": worst, "per_rank": per}), flush=True)
    print(json.dumps(out))
    for q in qs:
        q["scene"].close()
    tmp.cleanup()


if __name__ == "__main__":
    main()
