#!/usr/bin/env python3
"""Is the frame-queue loop bound by host submission? (run on the GPU box)

Times K frames of bench.py's loop (prepare + trace per frame over Q queues) three ways:
submission only (the host loop, no wait), the loop plus the wait (what bench.py times), and
the per-call cost of the two ctypes entry points. If submission alone takes about as long as
the whole loop, the GPU is waiting for the host.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch

    import simpleraytracer_amd as srt

    W, H, K, Q = 1920, 1080, int(os.environ.get("K", 3000)), int(os.environ.get("Q", 3))
    tmp = tempfile.TemporaryDirectory()
    path = srt.write_scene(os.path.join(tmp.name, "s.srt"), "soup", 100_000)
    off = torch.full((H, W, 2), 0.5, dtype=torch.float32, device="cuda")
    qs = [(srt.DeviceScene(path, 0), torch.cuda.Stream(), torch.empty((H, W, 4), dtype=torch.float32, device="cuda"))
          for _ in range(Q)]
    out = {"frames": K, "queues": Q}
    for rep in range(3):
        for k in range(60):
            sc, st, o = qs[k % Q]
            sc.prepare(W, H, st)
            sc.trace(off, o, 0, H, stream=st)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            sc, st, o = qs[k % Q]
            sc.prepare(W, H, st)
            sc.trace(off, o, 0, H, stream=st)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[f"rep{rep}"] = {"submit_us_per_frame": round((t1 - t0) / K * 1e6, 2),
                            "total_us_per_frame": round((t2 - t0) / K * 1e6, 2)}
    # cost of the calls alone: prepare() (no GPU work) and a trace of a 1-row band
    sc, st, o = qs[0]
    t0 = time.perf_counter()
    for _ in range(2000):
        sc.prepare(W, H, st)
    out["prepare_call_us"] = round((time.perf_counter() - t0) / 2000 * 1e6, 2)
    torch.cuda.synchronize()
    print(json.dumps(out))
    for sc, _, _ in qs:
        sc.close()


if __name__ == "__main__":
    main()
