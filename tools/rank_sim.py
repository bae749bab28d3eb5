#!/usr/bin/env python3
"""Per-rank GPU time of the multi-GPU band pipeline, measured on one GPU with the frame engine
(srtEngineCreateRank with simulate=1: the rank's exact kernel stream -- its band's batched traces and
its share of the compositing -- without the exchange). For every P and rank: us of GPU time per
frame; the slowest rank bounds the job: ceiling = W x H / slowest (Mrays/s, exchange not included).

    python tools/rank_sim.py [--ranks 1,2,4,8] [--steps 30] [--batch 64] [--queues 2]
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
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--queues", type=int, default=2)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--triangles", type=int, default=100_000)
    ap.add_argument("--rows", default="interleaved")
    ap.add_argument("--launch", type=int, default=0, help="frames per trace launch (0: library default)")
    ap.add_argument("--all-ranks", action="store_true", help="every rank (default: ranks 0, P/2 and P-1)")
    a = ap.parse_args()
    import numpy as np
    import torch

    from simpleraytracer_amd.device import write_scene
    from simpleraytracer_amd.engine import FrameEngine

    tmp = tempfile.TemporaryDirectory()
    path = write_scene(os.path.join(tmp.name, "soup.srt"), "soup", a.triangles)
    inputs = np.full((1, a.height, a.width, 2), 0.5, np.float32)
    out = {"batch": a.batch, "launch": a.launch, "queues": a.queues, "triangles": a.triangles, "width": a.width, "height": a.height,
           "rows": a.rows, "ranks": {}}
    for P in [int(x) for x in a.ranks.split(",")]:
        per = {}
        ranks = range(P) if a.all_ranks else sorted({0, P // 2, P - 1})
        for r in ranks:
            if P == 1:
                eng = FrameEngine(path, a.width, a.height, devices=[0], queues=a.queues, batch=a.batch,
                                  launch=a.launch)
            else:
                eng = FrameEngine.rank(path, a.width, a.height, 0, r, P, None, queues=a.queues, batch=a.batch,
                                       rows=a.rows, simulate=True, launch=a.launch)
            eng.set_inputs(inputs)
            eng.run(a.warmup)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run(a.steps)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            per[r] = round(dt / (a.steps * a.batch) * 1e6, 3)
            eng.close()
        slow = max(per.values())
        out["ranks"][P] = {"us_per_frame": per, "slowest_us": slow,
                           "ceiling_mrays": round(a.width * a.height / slow, 1)}
        print(json.dumps({"P": P, **out["ranks"][P]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
