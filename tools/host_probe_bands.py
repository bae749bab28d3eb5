#!/usr/bin/env python3
"""Host cost of bench.py's band step (run under torch.distributed.run, 1 rank, on the GPU box).

    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 tools/host_probe_bands.py

Times, per frame, the host submission of a P=8 band (135 rows of 1920) on Q=3 frame queues:
  checked       prepare + trace_ids through DeviceScene (shape / dtype / device checks per call)
  raw           the same two C-ABI calls with cached pointers
  gather        raw + a dist.gather of the band's ids per frame on an RCCL process group (one
                rank: only the host side of the collective is measured)
  gather_shade  gather + the deferred shading of every 8th frame
  batch<G>      raw + one gather of G frames' bands per G frames + one shade_bands launch
  batch<G>_thr  batch<G>, each queue submitted by its own Python thread (ctypes and c10d calls
                release the GIL, so HIP launches on different streams can overlap)
Each is reported as submission-only and submission + drain (us per frame). Env: ROWS (band
height, default 135 = P 8), MODES (comma list), K (frames), Q (queues).
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import threading
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
    W, H, K, G = 1920, 1080, int(os.environ.get("K", 2400)), 8
    r0, rows = 0, int(os.environ.get("ROWS", 135))
    tmp = tempfile.TemporaryDirectory()
    path = srt.write_scene(os.path.join(tmp.name, "s.srt"), "soup", 100_000)
    off = torch.full((H, W, 2), 0.5, dtype=torch.float32, device=dev)
    qs = []
    for q in range(Q):
        qs.append({"scene": srt.DeviceScene(path, 0), "stream": torch.cuda.Stream(dev),
                   "ids": torch.full((G, rows, W), -1, dtype=torch.int32, device=dev),
                   "frame": torch.empty((G, rows, W), dtype=torch.int32, device=dev),
                   "rgba": torch.empty((G, rows, W, 4), dtype=torch.float32, device=dev), "group": groups[q],
                   "fill": 0, "shade_scene": srt.DeviceScene(path, 0)})
    for q in qs:  # world 1: the gathered batch is one band, shaded as a frame of `rows` rows
        q["shade_scene"].prepare(W, rows)
    L = _native.lib()

    def frame(q, k, mode):
        sc, st = q["scene"], q["stream"]
        if mode == "checked":
            sc.prepare(W, H, st)
            sc.trace_ids(off[r0:r0 + rows], q["ids"][0], r0, rows, stream=st)
            return
        j = q["fill"]
        L.srtPrepareAsync(sc.handle, W, H, st.cuda_stream)
        L.srtTraceIdsAsync(sc.handle, off.data_ptr(), q["ids"][j].data_ptr(), r0, rows, 2, st.cuda_stream)
        if mode in ("gather", "gather_shade"):
            with torch.cuda.stream(st):
                _, work = gather_band_ids(q["ids"][0], rows, dst=0, group=q["group"], out=q["frame"][0],
                                          async_op=True)
                work.wait()
            if mode == "gather_shade" and k % 8 == 0:
                L.srtShadeAsync(q["shade_scene"].handle, off.data_ptr(), q["frame"].data_ptr(), q["rgba"].data_ptr(), 0, rows,
                                st.cuda_stream)
        elif mode.startswith("batch"):
            q["fill"] = j + 1
            if q["fill"] == G:
                q["fill"] = 0
                with torch.cuda.stream(st):
                    ids, work = gather_band_batch(q["ids"], rows, dst=0, group=q["group"], out=q["frame"],
                                                  async_op=True)
                    work.wait()
                L.srtShadeBandsAsync(q["shade_scene"].handle, off.data_ptr(), ids.data_ptr(), q["rgba"].data_ptr(), G, rows,
                                     st.cuda_stream)

    def loop(mode, ks):
        for k in ks:
            frame(qs[k % Q], k, mode)

    def loop_thread(mode, qi, count, go):
        go.wait()
        for i in range(count):
            frame(qs[qi], i * Q + qi, mode)

    out = {"frames": K, "queues": Q, "band_rows": rows, "batch": G}
    modes = os.environ.get("MODES", "checked,raw,gather,gather_shade,batch8,batch8_thr").split(",")
    for mode in modes:
        loop(mode.replace("_thr", ""), range(Q * G * 4))
        torch.cuda.synchronize()
        if mode.endswith("_thr"):
            go = threading.Barrier(Q + 1)
            th = [threading.Thread(target=loop_thread, args=(mode, qi, K // Q, go)) for qi in range(Q)]
            for t in th:
                t.start()
            go.wait()
            t0 = time.perf_counter()
            for t in th:
                t.join()
        else:
            t0 = time.perf_counter()
            loop(mode, range(K))
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
