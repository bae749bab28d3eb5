#!/usr/bin/env python3
"""GPU time per frame of the cull pipeline's per-frame setup vs its trace (run on the GPU box).

    python tools/setup_probe.py [--rows 1,34,135,270,540,1080] [--queues 3] [--steps 2400]

For each band height, --queues frame queues each trace batches of 8 frames of rows [0, rows)
(srtTraceBatchAsync, hit ids: record setup, tile info, bins, work list and trace per frame), and
the loop reports us per frame with the chip shared by the queues. A 1-row band's trace is almost
empty, so its time is the per-frame setup every band of a multi-GPU frame repeats; the growth
with rows is the trace. (Host submission is 4 launches per 8 frames, far below these times.)
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
    ap.add_argument("--rows", default="1,34,135,270,540,1080")
    ap.add_argument("--queues", type=int, default=3)
    ap.add_argument("--steps", type=int, default=2400)
    ap.add_argument("--triangles", type=int, default=100_000)
    a = ap.parse_args()
    import torch

    import simpleraytracer_amd as srt

    W, H, G = 1920, 1080, srt.MAX_BATCH
    dev = torch.device("cuda", 0)
    tmp = tempfile.TemporaryDirectory()
    path = srt.write_scene(os.path.join(tmp.name, "soup.srt"), "soup", a.triangles)
    off = torch.full((H, W, 2), 0.5, dtype=torch.float32, device=dev)
    qs = [{"scene": srt.DeviceScene(path, 0), "stream": torch.cuda.Stream(dev),
           "ids": torch.full((G, H, W), -1, dtype=torch.int32, device=dev)} for _ in range(a.queues)]
    for q in qs:
        q["scene"].prepare(W, H)
    out = {"queues": a.queues, "batch": G, "us_per_frame": {}}
    for rows in [int(x) for x in a.rows.split(",")]:
        runs = [q["scene"].bind_trace_batch([off[:rows]] * G, [q["ids"][j, :rows] for j in range(G)], 0, rows,
                                            stream=q["stream"], ids=True) for q in qs]
        batches = max(a.queues, a.steps // G)
        for k in range(2 * a.queues):
            runs[k % a.queues]()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(batches):
            runs[k % a.queues]()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out["us_per_frame"][rows] = round(dt / (batches * G) * 1e6, 2)
        print(json.dumps({"rows": rows, "us_per_frame": out["us_per_frame"][rows]}), flush=True)
    print(json.dumps(out))
    for q in qs:
        q["scene"].close()


if __name__ == "__main__":
    main()
