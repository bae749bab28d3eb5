#!/usr/bin/env python3
"""Host cost of bench.py's band step (run under torch.distributed.run, 1 rank, on the GPU box).

    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 tools/host_probe_bands.py

Times, per frame, the host submission of a P = 8 band (135 rows of 1920) on Q = 3 frame queues:
  checked      prepare + trace_ids through DeviceScene (shape / dtype / device checks per call)
  raw          the same two C-ABI calls with cached pointers (4 kernel launches per frame)
  gather       raw + a dist.gather of the band's ids per frame on an RCCL process group (one
               rank: only the host side of the collective is measured)
  batch8       per 8 frames one srtTraceBatchAsync call (4 launches), one dist.gather of the
               (8, B, W) id batch and one srtShadeBandsAsync launch
  batch16      bench.py's step at N > 1: per 16 frames two batched trace calls, one gather of the
               (16, B, W) batch and one shading launch
Each is reported as submission-only and submission + drain (us per frame): with one rank the GPU
work of a P = 8 band is small, so these are the host's costs. Env: ROWS (band height, default
135), K (frames), Q (queues).
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
    import torch.distributed as dist

    import simpleraytracer_amd as srt
    from simpleraytracer_amd import _native
    from simpleraytracer_amd.bands import gather_band_batch, gather_band_ids

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    Q = int(os.environ.get("Q", 3))
    groups = [dist.new_group([0]) for _ in range(Q)]
    W, H, K, G = 1920, 1080, int(os.environ.get("K", 2400)), srt.MAX_BATCH
    r0, rows = 0, int(os.environ.get("ROWS", 135))
    tmp = tempfile.TemporaryDirectory()
    path = srt.write_scene(os.path.join(tmp.name, "s.srt"), "soup", 100_000)
    off = torch.full((H, W, 2), 0.5, dtype=torch.float32, device=dev)
    qs = []
    for q in range(Q):
        qd = {"scene": srt.DeviceScene(path, 0), "stream": torch.cuda.Stream(dev),
              "ids": torch.full((2 * G, rows, W), -1, dtype=torch.int32, device=dev),
              "frame": torch.empty((2 * G, rows, W), dtype=torch.int32, device=dev),
              "rgba": torch.empty((2 * G, rows, W, 4), dtype=torch.float32, device=dev), "group": groups[q],
              "fill": 0, "shade_scene": srt.DeviceScene(path, 0)}
        qd["scene"].prepare(W, H)
        qd["shade_scene"].prepare(W, rows)  # world 1: the gathered batch is one band, shaded as a frame
        qd["batch"] = [qd["scene"].bind_trace_batch([off[:rows]] * G, [qd["ids"][j] for j in range(s0, s0 + G)], r0,
                                                    rows, stream=qd["stream"], ids=True) for s0 in (0, G)]
        qs.append(qd)
    L = _native.lib()

    def frame(q, mode):
        sc, st = q["scene"], q["stream"]
        if mode == "checked":
            sc.prepare(W, H, st)
            sc.trace_ids(off[r0:r0 + rows], q["ids"][0], r0, rows, stream=st)
            return
        if mode in ("batch8", "batch16"):
            n = G if mode == "batch8" else 2 * G
            q["fill"] += 1
            if q["fill"] < n:
                return
            q["fill"] = 0
            for b in range(n // G):
                q["batch"][b]()
            with torch.cuda.stream(st):
                ids, work = gather_band_batch(q["ids"][:n], rows, dst=0, group=q["group"], out=q["frame"],
                                              async_op=True)
                work.wait()
            q["shade_scene"].shade_bands(off[:rows], ids, q["rgba"][:n], rows, stream=st)
            return
        L.srtPrepareAsync(sc.handle, W, H, st.cuda_stream)
        L.srtTraceIdsAsync(sc.handle, off.data_ptr(), q["ids"][0].data_ptr(), r0, rows, 2, st.cuda_stream)
        if mode == "gather":
            with torch.cuda.stream(st):
                _, work = gather_band_ids(q["ids"][0], rows, dst=0, group=q["group"], out=q["frame"][0],
                                          async_op=True)
                work.wait()

    out = {"frames": K, "queues": Q, "band_rows": rows, "batch": G}
    for mode in ("checked", "raw", "gather", "batch8", "batch16"):
        for k in range(Q * G * 4):
            frame(qs[k % Q], mode)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            frame(qs[k % Q], mode)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[mode] = {"submit_us": round((t1 - t0) / K * 1e6, 2), "total_us": round((t2 - t0) / K * 1e6, 2)}
    print(json.dumps(out))
    for q in qs:
        q["scene"].close()
        q["shade_scene"].close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
