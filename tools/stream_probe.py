#!/usr/bin/env python3
"""Throughput of S concurrent frame queues on one GPU: S DeviceScene copies (own edge records,
bins and framebuffer), each on its own HIP stream, frames issued round-robin. S = 1 is the
bench.py frame loop.

    python tools/stream_probe.py [--queues 1,2,3] [--steps 60]
"""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queues", default="1,2,3")
    ap.add_argument("--steps", type=int, default=60)
    a = ap.parse_args()
    import torch

    import simpleraytracer_amd as srt

    W, H = 1920, 1080
    with tempfile.TemporaryDirectory() as d:
        path = srt.write_scene(os.path.join(d, "s.srt"), "soup", 100_000)
        for q in [int(x) for x in a.queues.split(",")]:
            scenes = [srt.DeviceScene(path, 0) for _ in range(q)]
            streams = [torch.cuda.Stream() for _ in range(q)]
            offs = [torch.full((H, W, 2), 0.5, dtype=torch.float32, device="cuda") for _ in range(q)]
            outs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(q)]

            def frame(i):
                k = i % q
                scenes[k].prepare(W, H, streams[k])
                scenes[k].trace(offs[k], outs[k], 0, H, stream=streams[k])

            for i in range(3 * q):
                frame(i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                frame(i)
            t_issue = time.perf_counter() - t0
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(f"queues {q}: {a.steps * W * H / dt / 1e6:.0f} Mrays/s, {dt / a.steps * 1e6:.1f} us per frame, "
                  f"host issue {t_issue / a.steps * 1e6:.1f} us per frame",
                  flush=True)
            for s in scenes:
                s.close()


if __name__ == "__main__":
    main()
