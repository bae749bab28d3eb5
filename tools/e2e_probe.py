#!/usr/bin/env python3
"""mlInfer end-to-end time per frame for several pipelined chunk counts (SRT_E2E_CHUNKS).

    python tools/e2e_probe.py [--width 1920 --height 1080 --triangles 100000]
"""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--triangles", type=int, default=100_000)
    ap.add_argument("--chunks", default="1,2,3,4,5,8")
    ap.add_argument("--torch", action="store_true", help="initialise torch's HIP context first (as bench.py does)")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--node", type=int, default=-1, help="pin this process to the CPUs of NUMA node N first")
    a = ap.parse_args()
    import glob

    nodes = {}
    for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        try:
            nodes[int(d.rsplit("node", 1)[1])] = open(d + "/cpulist").read().strip()
        except OSError:
            pass
    gpus = {}
    for d in sorted(glob.glob("/sys/class/drm/card*/device/numa_node")):
        try:
            gpus[d.split("/")[4]] = open(d).read().strip()
        except OSError:
            pass
    print(f"numa nodes {nodes}; gpu numa_node {gpus}; affinity {len(os.sched_getaffinity(0))} cpus "
          f"(first {sorted(os.sched_getaffinity(0))[:4]})", flush=True)
    if a.node >= 0 and a.node in nodes:
        cpus = set()
        for part in nodes[a.node].split(","):
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
        allowed = cpus & os.sched_getaffinity(0)
        if allowed:
            os.sched_setaffinity(0, allowed)
        print(f"pinned to node {a.node}: {len(allowed)} cpus", flush=True)
    import numpy as np

    if a.torch:
        import torch

        torch.cuda.init()
        torch.zeros(1, device="cuda")

    import simpleraytracer_amd as srt

    with tempfile.TemporaryDirectory() as d:
        path = srt.write_scene(os.path.join(d, "s.srt"), "soup", a.triangles)
        for c in a.chunks.split(","):
            os.environ["SRT_E2E_CHUNKS"] = c
            ctx = srt.Context()
            model = ctx.create_model(path)
            model.set_input_info(a.width, a.height)
            (idt, iw, ih, ic), (odt, ow, oh, oc) = model.info()
            inp = ctx.create_image(idt, iw, ih, ic)
            out = ctx.create_image(odt, ow, oh, oc)
            inp.array()[...] = np.float32(0.5)
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                model.infer(inp, out)
                ts.append((time.perf_counter() - t0) * 1e3)
            print(f"chunks {c}: ms per frame {[round(t, 3) for t in ts]}", flush=True)
            inp.close()
            out.close()
            model.close()
            ctx.close()


if __name__ == "__main__":
    main()
