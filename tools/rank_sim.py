#!/usr/bin/env python3
"""Per-rank GPU time of the multi-GPU band pipeline, measured on one GPU with the frame engine
(srtEngineCreateRank with simulate=1: the rank's exact kernel stream -- its band's batched traces and
its share of the compositing -- without the exchange). For every P and rank: us of GPU time per
frame; the slowest rank bounds the job: gpu ceiling = W x H / slowest (Mrays/s).

The exchange, modelled (it cannot be measured on a one-GPU box): per frame the P - 1 ranks that do
not composite it send their band of hit ids (the engine's payload: id_bytes per pixel, 2 for 16-bit
codes) to its compositor; the all-to-all deals the compositors round-robin, so every one of the
P (P - 1) directed xGMI links of a fully connected node carries bytes_frame / (P (P - 1)) per frame
on average (share likewise; rotating: a batch's P - 1 senders use their links into its compositor,
the min(Q, P) batches in flight distinct ones), and the link-bound time per frame is that over the
per-direction link rate. ASSUMED
rate, not measured: --link-gbs (default 64 GB/s per direction; MI355X_MICROARCH.md has no xGMI figure,
SURVEY.md section 5 quotes 153.6 GB/s per link, bidirectional, so about 77 GB/s each way at peak;
RCCL point-to-point reaching ~85 % of it gives ~64). A sweep of rates is printed beside it. The job
ceiling = W x H / max(slowest rank's GPU time, link time) -- the exchange overlaps the other queue's
compute (its RCCL kernels' CU time is inside neither figure).

    python tools/rank_sim.py [--ranks 1,2,4,8] [--steps 16] [--batch 256] [--queues 2] [--link-gbs 64]
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
    # batches (warmup and timed) multiples of 8: under the rotating compositor roles (rotating)
    # every rank then composites the same number of batches at P = 2, 4, 8; 256-frame batches, as
    # bench.py's steps (its --frames-per-step)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--queues", type=int, default=2)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--triangles", type=int, default=100_000)
    ap.add_argument("--rows", default="interleaved")
    ap.add_argument("--exchange", default="share", choices=["alltoall", "rotating", "share"])
    ap.add_argument("--share", type=int, default=0,
                    help="share exchange: the compositor's tile rows per cycle, a power of two (0: srtShareAuto)")
    ap.add_argument("--launch", type=int, default=0, help="frames per trace launch (0: library default)")
    ap.add_argument("--all-ranks", action="store_true", help="every rank (default: ranks 0, P/2 and P-1)")
    ap.add_argument("--link-gbs", type=float, default=64.0, help="ASSUMED xGMI rate per direction (module doc)")
    ap.add_argument("--sweep-gbs", default="32,64,100,150", help="link rates of the printed sensitivity sweep")
    a = ap.parse_args()
    import numpy as np
    import torch

    from simpleraytracer_amd.device import write_scene
    from simpleraytracer_amd.engine import FrameEngine

    tmp = tempfile.TemporaryDirectory()
    path = write_scene(os.path.join(tmp.name, "soup.srt"), "soup", a.triangles)
    inputs = np.full((1, a.height, a.width, 2), 0.5, np.float32)
    out = {"batch": a.batch, "launch": a.launch, "queues": a.queues, "triangles": a.triangles, "width": a.width, "height": a.height,
           "rows": a.rows, "exchange": a.exchange, "share": a.share, "ranks": {}}
    for P in [int(x) for x in a.ranks.split(",")]:
        per = {}
        xbytes = 0.0
        ranks = range(P) if a.all_ranks else sorted({0, P // 2, P - 1})
        for r in ranks:
            if P == 1:
                eng = FrameEngine(path, a.width, a.height, devices=[0], queues=a.queues, batch=a.batch,
                                  launch=a.launch)
            else:
                eng = FrameEngine.rank(path, a.width, a.height, 0, r, P, None, queues=a.queues, batch=a.batch,
                                       rows=a.rows, simulate=True, launch=a.launch, exchange=a.exchange,
                                       share=a.share)
            eng.set_inputs(inputs)
            xbytes = eng.info()["exchange_bytes_per_frame"] if P > 1 else 0.0
            eng.run(a.warmup)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run(a.steps)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            per[r] = round(dt / (a.steps * a.batch) * 1e6, 3)
            eng.close()
        slow = max(per.values())
        # all-to-all and share (frame f composited on f % P): every directed link carries 1/(P (P - 1))
        # of a frame's payload; rotating: a batch's P - 1 senders each use their link into its
        # compositor, and the queues' batches in flight (on min(queues, P) distinct compositors) use
        # distinct links
        links = P * (P - 1) if a.exchange in ("alltoall", "share") else (P - 1) * min(a.queues, P)
        link_bytes = xbytes / links if P > 1 else 0.0
        link_us = link_bytes / (a.link_gbs * 1e3)
        bound = max(slow, link_us)
        out["ranks"][P] = {"us_per_frame": per, "slowest_us": slow,
                           "ceiling_mrays": round(a.width * a.height / slow, 1),
                           "exchange_bytes_per_frame": int(xbytes), "bytes_per_link_per_frame": int(link_bytes),
                           "link_us_per_frame": round(link_us, 3), "link_gbs_assumed": a.link_gbs,
                           "job_ceiling_mrays": round(a.width * a.height / bound, 1),
                           "bound": "link" if link_us > slow else "gpu",
                           "job_ceiling_sweep": {g: round(a.width * a.height / max(slow, link_bytes / (float(g) * 1e3)), 1)
                                                 for g in a.sweep_gbs.split(",")}}
        print(json.dumps({"P": P, **out["ranks"][P]}), flush=True)
    base = out["ranks"].get(1, {}).get("ceiling_mrays")
    if base:
        for P, r in out["ranks"].items():
            r["gpu_x_p1"] = round(r["ceiling_mrays"] / base, 3)
            r["job_x_p1"] = round(r["job_ceiling_mrays"] / base, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
