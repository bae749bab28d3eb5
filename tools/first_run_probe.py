#!/usr/bin/env python3
"""Probe: per-run wall time of consecutive timed runs of one simulated rank (tools/rank_sim.py's
engine), to find one-time costs that land inside a timed region.

    python tools/first_run_probe.py [--ranks 2] [--rank 0] [--exchange share] [--runs 4]

With SRT_PROBE_HOST=1 the engine also prints every trace / shade phase whose host time exceeds
300 us (engine.cpp RunWorker).
"""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--exchange", default="share")
    ap.add_argument("--runs", type=int, default=4)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--first", type=int, default=0, help="batches of the first run (0: --batches)")
    ap.add_argument("--torch-first", action="store_true", help="initialise torch's HIP context before the engine")
    a = ap.parse_args()
    import numpy as np
    import torch

    from simpleraytracer_amd.device import write_scene
    from simpleraytracer_amd.engine import FrameEngine

    if a.torch_first:
        torch.cuda.synchronize()
    tmp = tempfile.TemporaryDirectory()
    path = write_scene(os.path.join(tmp.name, "soup.srt"), "soup", 100_000)
    eng = FrameEngine.rank(path, 1920, 1080, 0, a.rank, a.ranks, None, queues=2, batch=64, simulate=True,
                           exchange=a.exchange)
    eng.set_inputs(np.full((1, 1080, 1920, 2), 0.5, np.float32))
    for i in range(a.runs):
        t0 = time.perf_counter()
        n = a.first if i == 0 and a.first else a.batches
        eng.run(n)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"run {i}: {(t1 - t0) * 1e3:.2f} ms run, {(t2 - t1) * 1e3:.2f} ms sync, "
              f"{(t1 - t0) / (n * 64) * 1e6:.2f} us/frame", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
