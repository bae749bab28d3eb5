#!/usr/bin/env python3
"""Headline benchmark: Mrays/s rendering the 100k-triangle synthetic soup at 1920x1080, 1 spp.

    python bench.py [--gpus N --steps K --warmup W]        (N > 1: launched by torch.distributed.run)

One step = one complete frame of the hot path on device-resident inputs (SURVEY.md section 8
rows a9-a13): tile info, record setup and bins, the trace work list, the closest-hit trace
(TraceCullKernel; its frame is bit-identical to brute force, DESIGN.md section 5,
tests/test_gpu_parity.py), shading and the framebuffer store. Nothing is cached across frames.

Each GPU keeps --queues frame queues (default: 3 at N > 1 and for runs of at most 24 frames, else 2), each its own DeviceScene, HIP stream and buffers, and a
queue takes --batch frames at a time: up to 8 of them go through one srtTraceBatchAsync call (the
same per-frame work, one launch per stage for the batch). N = 1: batches of 8 frames, each frame
shaded into its own RGBA framebuffer; the single_queue pass runs one frame per launch on one
queue (the per-frame latency).

Multi-GPU, one rank per GPU over RCCL:
  --mode bands (default; BASELINE config C4): every frame is split into P bands -- the frame's
      16-row tile rows dealt round-robin (--rows interleaved, default) or contiguous blocks --,
      rank r traces its band (hit ids, 4 B per pixel; deferred shading, bit-identical), a batch
      of 16 frames' bands is gathered over RCCL in ONE collective (a torch-RCCL gather costs
      ~40 us of host time per call, more than a band's trace: tools/host_probe_bands.py) to
      the batch's compositor, rank (batch index) % P (--root rotate, default) or rank 0 (--root
      fixed), which shades the 16 frames in one launch (srtShadeBandsAsync). value = frames x W x
      H / the max-over-ranks time: "scaling": "strong". After the timed loop every compositing
      rank compares its last batch's frames with a one-GPU render bit for bit ("verified").
  --mode frames: every rank renders whole frames of a temporal-jitter sequence (no collective);
      "scaling": "weak". Reported beside the bands line at N > 1 ("frames").
At N = 1 the two modes coincide (one band = the frame, shaded in the trace).

Prints ONE JSON line on rank 0 (fields in DESIGN.md section 6).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
FP32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md chip table (spec, vector fp32, packed)
SIMDS, CLOCK_GHZ = 1024, 2.4  # 256 CUs x 4 SIMD-32; wave64 VALU issue = 2 cycles per instruction
EDGE_BYTES_PER_TRI = 36      # 9 fp32 edge coefficients per ray-triangle test
CULL_RECORD_BYTES = 64       # one cull record per triangle (render.hip CullRecord)
PIXEL_IO_BYTES = 8 + 16      # sample offsets in + RGBA out per ray
FLOPS_PER_TEST = 12          # 3 edge functions x 2 FMA
GOLDEN = 0.6180339887498949  # temporal jitter sequence step
KERNEL_NAMES = {"lds": "TraceLdsKernel", "scalar": "TraceScalarKernel", "cull": "TraceCullKernel",
                "bvh": "TraceBvhKernel"}
PROFILES = REPO / "profiles"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # 3000 frames = ~0.1 s timed at C3: 1000 frames (36 ms) read ~2.5 % low, the clocks still
    # settling (profiles/r01/ab/README.md)
    p.add_argument("--steps", type=int, default=3000)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--scene", default="soup", choices=["soup", "cornell", "triangle"])
    p.add_argument("--triangles", type=int, default=100_000)
    p.add_argument("--variant", default=os.environ.get("SRT_BENCH_VARIANT", "cull"), choices=list(KERNEL_NAMES))
    p.add_argument("--mode", default="bands", choices=["bands", "frames"], help="multi-GPU split (module doc)")
    p.add_argument("--root", default="rotate", choices=["rotate", "fixed"], help="bands: compositing rank")
    p.add_argument("--rows", default="interleaved", choices=["interleaved", "contiguous"],
                   help="bands: each rank's rows, the frame's 16-row tile rows dealt round-robin or one block")
    p.add_argument("--queues", type=int, default=int(os.environ.get("SRT_BENCH_QUEUES", "0")),
                   help="frames in flight per GPU (own scene buffers, HIP stream, process group each); 0 = 3 at "
                        "N > 1 or when the run is at most one 8-frame batch per queue, else 2")
    p.add_argument("--batch", type=int, default=int(os.environ.get("SRT_BENCH_BATCH", "0")),
                   help="frames per batch: traced in srtTraceBatchAsync calls of <= 8 frames and, bands at "
                        "N > 1, gathered in one collective and shaded in one launch; 0 = 16 at N > 1, 8 at N = 1")
    p.add_argument("--offsets", default="uniform", choices=["uniform", "random"],
                   help="sample offsets: uniform 0.5 (headline) or seeded U[0,1) per-pixel jitter")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample length")
    p.add_argument("--brute-steps", type=int, default=5, help="timed frames of the brute-force LDS kernel (0 = skip)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive ml* API measurement")
    p.add_argument("--no-extras", action="store_true", help="only the main line (no secondary legs)")
    return p.parse_args()


def workload_name(a, scene=None, triangles=None):
    scene = scene or a.scene
    triangles = triangles or a.triangles
    if scene == "soup":
        tri = f"{triangles // 1000}k" if triangles % 1000 == 0 else str(triangles)
        return f"soup-{tri} {a.width}x{a.height} 1spp"
    return f"{scene} {a.width}x{a.height} 1spp"


def jitter(rank: int) -> float:
    """Uniform sub-pixel offset of rank r's frames in frames mode (r = 0: 0.5, the headline frame)."""
    import numpy as np

    return float(np.float32((0.5 + rank * GOLDEN) % 1.0))


def make_offsets(torch, a, dev, value=0.5, kind="uniform", seed=0x5EED):
    if kind == "random":  # seeded per-pixel jitter, U[0, 1)
        g = torch.Generator(device="cpu").manual_seed(seed)
        return torch.rand((a.height, a.width, 2), generator=g, dtype=torch.float32).to(dev)
    return torch.full((a.height, a.width, 2), value, dtype=torch.float32, device=dev)


class Ctx:
    """This rank's process-wide state: torch, the process groups, the device, the scene files."""

    def __init__(self, a):
        import torch
        import torch.distributed as dist

        import simpleraytracer_amd as srt

        self.torch, self.dist, self.srt, self.a = torch, dist, srt, a
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if os.environ.get("SRT_BENCH_ONE_DEVICE"):  # rehearsal of N > 1 ranks on a one-GPU box (with gloo)
            local = 0
        if self.world != a.gpus:
            raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={self.world}")
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        self.backend = None
        self.groups = []
        if self.world > 1:
            self.backend = os.environ.get("SRT_BENCH_BACKEND", "nccl")  # gloo: CPU-side rehearsal on one GPU
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=self.dev)
            else:
                dist.init_process_group(self.backend)
            # one process group (RCCL communicator, NCCL stream) per frame queue: the gathers of
            # different frames in flight run concurrently
            self.groups = [dist.new_group(list(range(self.world))) for _ in range(max(1, a.queues))]
        self.tmp = tempfile.TemporaryDirectory()
        self.paths = {}

    def scene_path(self, kind, triangles=None):
        key = (kind, triangles)
        if key not in self.paths:
            path = os.path.join(self.tmp.name, f"{kind}_{triangles}_rank{self.rank}.srt")
            if kind == "soup":
                self.srt.write_scene(path, "soup", triangles)
            else:
                self.srt.write_scene(path, kind)
            self.paths[key] = path
        return self.paths[key]

    def max_over_ranks(self, x):
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64,
                              device=self.dev if self.backend != "gloo" else "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()


class Pipeline:
    """Frames over `queues` frame queues on this rank (module doc). mode "bands": rank r traces
    band r of every frame (P > 1: hit ids, gathered to the compositor, which shades); mode
    "frames": whole frames, each rank its own jitter; P == 1: the two coincide."""

    def __init__(self, ctx, path, mode="bands", queues=3, variant="cull", offsets="uniform", rotate=True, batch=1,
                 rows="interleaved"):
        from simpleraytracer_amd.bands import (band_range, band_rows, interleaved_band_rows, interleaved_frame_rows,
                                               interleaved_range)

        torch, a = ctx.torch, ctx.a
        self.ctx, self.mode, self.variant, self.rotate = ctx, mode, variant, rotate
        self.W, self.H = a.width, a.height
        P = ctx.world if mode == "bands" else 1
        self.P = P
        self.G = max(1, batch)  # frames per batch: per gather + shading launch at P > 1
        self.L = min(self.G, ctx.srt.MAX_BATCH)  # frames per batched trace call
        self.interleave = P if (P > 1 and rows == "interleaved") else 1
        if self.interleave > 1:
            self.row_begin, self.row_count = interleaved_range(self.H, P, ctx.rank)
            self.B = interleaved_band_rows(self.H, P)
        else:
            self.row_begin, self.row_count = band_range(self.H, P, ctx.rank) if P > 1 else (0, self.H)
            self.B = band_rows(self.H, P)
        self.offsets = make_offsets(torch, a, ctx.dev, jitter(ctx.rank) if mode == "frames" else 0.5, offsets,
                                    seed=0x5EED + (ctx.rank if mode == "frames" else 0))
        if self.interleave > 1:  # the band's rows of the frame's offsets, in band order (one copy)
            rows_t = torch.from_numpy(interleaved_frame_rows(self.H, P, ctx.rank)).to(ctx.dev)
            self.band_off = self.offsets.index_select(0, rows_t).contiguous()
        else:
            self.band_off = self.offsets[self.row_begin:self.row_begin + self.row_count]
        self.timing = False
        self.queues = []
        for q in range(max(1, queues)):
            qd = {"scene": ctx.srt.DeviceScene(path, ctx.dev.index), "stream": torch.cuda.Stream(ctx.dev),
                  "root": None, "index": q, "fill": 0, "traced": 0, "batches": 0, "shaded": 0, "runs": {}}
            qd["scene"].prepare(self.W, self.H)
            qd["rgba"] = torch.zeros((self.G, self.H, self.W, 4), dtype=torch.float32, device=ctx.dev)
            if P > 1:
                qd["band_ids"] = torch.full((self.G, self.B, self.W), -1, dtype=torch.int32, device=ctx.dev)
                qd["frame_ids"] = torch.empty(P * self.G * self.B * self.W, dtype=torch.int32, device=ctx.dev)
                qd["group"] = ctx.groups[q % len(ctx.groups)]
            self.queues.append(qd)
        self.triangles = self.queues[0]["scene"].triangles
        # Grow every queue's frame slots to the largest batched call now (allocation, zero fill):
        # a batch larger than the warm-up's partial ones must not allocate inside a timed loop.
        if self.row_count:
            for q in self.queues:
                self._batch_run(q, self.L)()
            torch.cuda.synchronize(ctx.dev)

    def _batch_run(self, q, f, slot=0):
        """The queue's batched trace of f slots from `slot` (one srtTraceBatchAsync call), bound once."""
        key = (f, slot)
        if key not in q["runs"]:
            sc, st = q["scene"], q["stream"]
            if self.P > 1:
                q["runs"][key] = sc.bind_trace_batch([self.band_off] * f, [q["band_ids"][j, :self.row_count]
                                                                           for j in range(slot, slot + f)],
                                                     self.row_begin, self.row_count, self.variant, st, ids=True,
                                                     row_interleave=self.interleave)
            else:
                q["runs"][key] = sc.bind_trace_batch([self.offsets] * f, [q["rgba"][j] for j in range(slot, slot + f)],
                                                     0, self.H, self.variant, st)
        return q["runs"][key]

    def step(self, k, nq):
        """Frame k on queue k % nq: into the queue's next batch slot; a full batch is traced
        (one call for all its frames), then at P > 1 gathered and shaded. With stage timing
        on, each frame is traced on its own (the single-frame calls bind the HIP events)."""
        q = self.queues[k % nq]
        sc, st = q["scene"], q["stream"]
        j = q["fill"]
        if self.timing and self.row_count:  # one frame per call: the stage events time one frame
            self._batch_run(q, 1, j)()
            q["traced"] = j + 1
        q["fill"] = j + 1
        if q["fill"] == self.G:
            self.flush(q, nq)

    def flush(self, q, nq):
        """Trace the queue's filled slots (if not yet), then at P > 1 gather them (one collective
        for all of them) to the batch's compositor, which shades every frame in one launch."""
        from simpleraytracer_amd.bands import compositor, gather_band_batch

        ctx, torch = self.ctx, self.ctx.torch
        f = q["fill"]
        if f == 0:
            return
        sc, st = q["scene"], q["stream"]
        if q["traced"] < f and self.row_count:
            for slot in range(0, f, self.L):
                self._batch_run(q, min(self.L, f - slot), slot)()
        q["fill"] = q["traced"] = 0
        if self.P == 1:
            q["root"], q["shaded"] = 0, f
            return
        root = compositor(q["batches"] * nq + q["index"], self.P, self.rotate)
        batch = q["band_ids"][:f]
        if ctx.backend == "gloo":  # CPU rehearsal: gloo gathers host tensors, synchronously
            st.synchronize()
            host_out = torch.empty(self.P * f * self.B * self.W, dtype=torch.int32) if ctx.rank == root else None
            ids, _ = gather_band_batch(batch.cpu(), self.H, dst=root, group=q["group"], out=host_out,
                                       interleaved=self.interleave > 1)
            if ids is not None:
                dev_ids = q["frame_ids"][:ids.numel()].view(ids.shape)
                dev_ids.copy_(ids.to(ctx.dev))
                torch.cuda.synchronize(ctx.dev)
                ids = dev_ids
        else:
            with torch.cuda.stream(st):
                ids, work = gather_band_batch(batch, self.H, dst=root, group=q["group"], out=q["frame_ids"],
                                              async_op=True, interleaved=self.interleave > 1)
                work.wait()  # the queue's stream waits for the gather (ids consumed / slots reusable)
        if ctx.rank == root:
            sc.shade_bands(self.offsets, ids, q["rgba"][:f], self.B, stream=st,
                           interleaved=self.interleave if self.interleave > 1 else 0)
            q["shaded"] = f
        q["root"] = root
        q["batches"] += 1

    def drain(self, nq=None):
        for q in self.queues[:nq or len(self.queues)]:  # partial batches
            self.flush(q, nq or len(self.queues))
        for q in self.queues:
            q["stream"].synchronize()

    def run(self, steps, warmup, queues=None, timing=False, batch=None):
        """`steps` timed frames after `warmup` per queue; stage timing binds events on queue 0's
        scene (use queues=1 then); `batch` (<= the pipeline's) overrides the frames per batch."""
        G, L = self.G, self.L
        if batch:
            self.G = min(batch, G)
            self.L = min(self.G, L)
        try:
            return self._run(steps, warmup, queues, timing)
        finally:
            self.G, self.L = G, L

    def _run(self, steps, warmup, queues, timing):
        torch, ctx = self.ctx.torch, self.ctx
        nq = min(queues or len(self.queues), len(self.queues))
        for k in range(warmup * nq):
            self.step(k, nq)
        self.drain(nq)
        sc0 = self.queues[0]["scene"]
        sc0.take_stage_times()
        sc0.set_stage_timing(timing)
        self.timing = timing
        ctx.barrier()
        torch.cuda.synchronize(ctx.dev)
        t0 = time.perf_counter()
        for k in range(steps):
            self.step(warmup * nq + k, nq)
        self.drain(nq)
        torch.cuda.synchronize(ctx.dev)
        ctx.barrier()
        elapsed = ctx.max_over_ranks(time.perf_counter() - t0)
        sc0.set_stage_timing(False)
        self.timing = False
        launches, prep_ms, bin_ms, trace_ms = sc0.take_stage_times()
        units = self.W * self.H * steps * (ctx.world if self.mode == "frames" else 1)
        return {"elapsed": elapsed, "mrays": units / elapsed / 1e6, "prepare_ms": prep_ms, "bin_ms": bin_ms,
                "trace_ms": trace_ms, "launches": launches, "ms_per_step": elapsed / steps * 1e3, "queues": nq}

    def verify(self):
        """Every rank that composited a batch compares its frames with a one-GPU render of the
        same frame (fused trace, this device), bit for bit; True on every rank iff all agree."""
        ctx, torch = self.ctx, self.ctx.torch
        ok = True
        for q in self.queues:
            if q["root"] == ctx.rank:
                ref_scene = ctx.srt.DeviceScene(q["scene"].path, ctx.dev.index)
                ref = torch.empty((self.H, self.W, 4), dtype=torch.float32, device=ctx.dev)
                st = torch.cuda.current_stream(ctx.dev)
                ref_scene.prepare(self.W, self.H, st)
                ref_scene.trace(self.offsets, ref, 0, self.H, variant=self.variant, stream=st)
                torch.cuda.synchronize(ctx.dev)
                for fr in q["rgba"][:q["shaded"]]:  # every frame of the queue's last composited batch
                    ok = ok and bool(torch.equal(ref.view(torch.int32), fr.view(torch.int32)))
                ref_scene.close()
                break
        return ctx.max_over_ranks(0.0 if ok else 1.0) == 0.0

    def close(self):
        for q in self.queues:
            q["scene"].close()


def stage_times_all_ranks(ctx, r):
    """[prepare, bin, trace] ms of every rank (instrumented single-queue pass)."""
    torch = ctx.torch
    mine = torch.tensor([r["prepare_ms"], r["bin_ms"], r["trace_ms"]], dtype=torch.float64,
                        device=ctx.dev if ctx.backend != "gloo" else "cpu")
    if ctx.world == 1:
        return [mine.tolist()]
    out = [torch.zeros_like(mine) for _ in range(ctx.world)]
    ctx.dist.all_gather(out, mine)
    return [t.tolist() for t in out]


def cpu_baseline(scene_path, a):
    """The oracle ('port') on this host's cores over a bounded, evenly spaced row sample."""
    from oracle import srt_oracle

    # OMP_NUM_THREADS is the GPU box's CPU share for one GPU (16 of its 256 host CPUs; gpurun
    # and the driver set it); os.cpu_count() reports the whole machine.
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    sc = srt_oracle.OracleScene(scene_path)
    h = a.height
    step = max(1, h // threads)  # calibration: one row per thread
    t0 = time.perf_counter()
    sc.render(a.width, h, row_begin=0, row_count=h, row_step=step, threads=threads)
    cal = time.perf_counter() - t0
    rows_cal = (h + step - 1) // step
    per_row = cal / rows_cal
    want_rows = max(rows_cal, min(h, int(a.cpu_seconds / max(per_row, 1e-9))))
    step = max(1, h // want_rows)
    t0 = time.perf_counter()
    sc.render(a.width, h, row_begin=0, row_count=h, row_step=step, threads=threads)
    dt = time.perf_counter() - t0
    rows = (h + step - 1) // step
    # single-thread scalar variant (BASELINE.md CPU plan (1)): a short row sample
    step1 = max(1, h // max(1, int(min(a.cpu_seconds / 3.0, 3.0) / max(per_row * threads, 1e-9))))
    t1 = time.perf_counter()
    sc.render(a.width, h, row_begin=0, row_count=h, row_step=step1, threads=1)
    dt1 = time.perf_counter() - t1
    rows1 = (h + step1 - 1) // step1
    model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "single_thread": {"value": round(rows1 * a.width / dt1 / 1e6, 6), "unit": "Mrays/s", "cores": 1,
                          "sample": f"{rows1} rows (every {step1}th), {dt1:.1f} s"},
        "cpu_model": model,
        "host_cpus": os.cpu_count(),
        "value": round(rows * a.width / dt / 1e6, 6),
        "unit": "Mrays/s",
        "cores": srt_oracle.threads(threads),
        "kind": "port",
        "sample": f"{rows} of {h} rows (every {step}th, all {a.width} columns) of {workload_name(a)}; "
                  f"{dt:.1f} s; OpenMP scalar C oracle (oracle/srt_oracle.c), brute force",
        "cores_note": "OMP_NUM_THREADS = this GPU's share of the box's host CPUs (host_cpus counts the "
                      "whole machine)",
    }


def committed_profile(name, key):
    """An entry of a committed profiles/ summary (rocprofv3 PMC passes), or None."""
    f = PROFILES / name
    if not f.exists():
        return None
    try:
        return json.loads(f.read_text()).get(key)
    except Exception:
        return None


def roofline_fields(wl, variant, launch_rays, n_tri, kernel_ms, band_ids):
    """The trace kernel's roofline (algorithmic bytes: each ray's offsets in + its output, each
    triangle's cull record once), the measured VALU issue from the committed PMC summary, and
    the section 8(d) brute-force-equivalent figures, clearly separated."""
    kernel_s = kernel_ms * 1e-3
    out_bytes = 4 if band_ids else 16
    alg = launch_rays * (8 + out_bytes) + n_tri * CULL_RECORD_BYTES
    achieved = alg / kernel_s / 1e9
    pmc = committed_profile("pmc_traffic.json", f"{wl}|{variant}") or {}
    roof = {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": pmc.get("hbm_bytes_per_launch"),
        "kernel": KERNEL_NAMES[variant],
        "kernel_ms": round(kernel_ms, 5),
        "bytes_per_launch": alg,
        "note": f"algorithmic bytes = launch rays x (8 B offsets in + {out_bytes} B out) + triangles x 64 B "
                "(each cull record once), over the trace kernel's HIP-event time; traffic = measured HBM "
                "bytes per launch (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE, profiles/pmc_traffic.json)",
    }
    sq = committed_profile("pmc_sq.json", f"{wl}|{variant}")
    valu = None
    if sq and sq.get("sq_insts_valu_per_launch"):
        issue_s = sq["sq_insts_valu_per_launch"] * 2 / (SIMDS * CLOCK_GHZ * 1e9)
        valu = {"valu_insts_per_launch": sq["sq_insts_valu_per_launch"], "issue_us": round(issue_s * 1e6, 2),
                "frac": round(issue_s / kernel_s, 4),
                "note": "SQ_INSTS_VALU (rocprofv3, profiles/pmc_sq.json) x 2 cycles per wave64 instruction "
                        "/ (1024 SIMDs x 2.4 GHz), over the kernel time"}
    tests = launch_rays * n_tri
    bf_bytes = launch_rays * (EDGE_BYTES_PER_TRI * n_tri + PIXEL_IO_BYTES)
    bfe = {"bytes_per_launch": bf_bytes, "tests_per_launch": tests,
           "hbm_equivalent_gbs": round(bf_bytes / kernel_s / 1e9, 1),
           "hbm_equivalent_frac": round(bf_bytes / kernel_s / 1e9 / HBM_PEAK_GBS, 2),
           "valu_equivalent_tflops": round(tests * FLOPS_PER_TEST / kernel_s / 1e12, 1),
           "note": "SURVEY 8(d) brute-force figures (36 B and 12 flops per ray-triangle test) over the cull "
                   "kernel's time: the work a brute-force kernel would do for the same bit-identical frame; "
                   "not a utilisation (the cull kernel proves most pairs miss without testing them)"}
    return roof, valu, bfe


def leg_summary(r):
    return {"mrays_per_s": round(r["mrays"], 3), "ms_per_step": round(r["ms_per_step"], 5), "queues": r["queues"]}


def main():
    a = parse()
    leg_queues = a.queues if a.queues > 0 else 3  # the secondary legs (random offsets, Cornell, variants)
    if a.queues <= 0:
        # Measured at C3 (profiles/r02/queues): long runs 2 / 3 / 1 queues 112.3 / 106.6 / 95.8
        # Grays/s (with 8-frame launches two queues already fill the chip, a third adds L2
        # contention); the driver's 20-step runs 91.8 / 96.9 / 83.6 (3 queues take one batch each,
        # 2 queues leave a 2-frame tail batch each). The secondary legs keep 3: random offsets
        # 78.1 vs 87.7, Cornell 143 vs 154, the BVH 15.1 vs 20.8 Grays/s with 2 vs 3.
        a.queues = 3 if a.gpus > 1 or -(-a.steps // 3) <= 8 else 2
    if a.batch <= 0:
        # 16 frames per gather at N > 1, 8 per launch at N = 1, at most one batch per queue's
        # share of the run: a short run (the driver's 20 steps over 3 queues) then traces, gathers
        # and shades its frames in ~one batch per queue instead of per-frame collectives (~45 us
        # of host time each) or a tail of partial batches
        a.batch = max(1, min(16 if a.gpus > 1 else 8, -(-a.steps // max(1, a.queues))))
    ctx = Ctx(a)
    world, rank = ctx.world, ctx.rank
    path = ctx.scene_path(a.scene, a.triangles if a.scene == "soup" else None)
    wl = workload_name(a)
    rotate = a.root == "rotate"
    main_run = Pipeline(ctx, path, a.mode, a.queues, a.variant, a.offsets, rotate, a.batch, a.rows)
    n_tri = main_run.triangles
    _, order_build_ms = main_run.queues[0]["scene"].spatial_order()
    W, H = a.width, a.height
    extras = not a.no_extras
    # Secondary passes first (they also bring the clocks up before the timed value loop): one
    # frame in flight (per-frame latency), then the same with HIP events bound to the kernels'
    # dispatch packets for the stage times (each event-bound dispatch leaves a 5-10 us bubble,
    # so that pass is slower; its kernel durations are not inflated by frame overlap).
    # (one frame per launch at N = 1: this pass is the per-frame latency)
    r1 = main_run.run(a.steps, a.warmup, queues=1, batch=1 if world == 1 else None) if len(main_run.queues) > 1 else None
    rt = main_run.run(min(a.steps, 1000), 2, queues=1, timing=True)
    ranks_stages = stage_times_all_ranks(ctx, rt)
    # value: uninstrumented frames over the frame queues
    r = main_run.run(a.steps, a.warmup)
    verified = main_run.verify() if (world > 1 and a.mode == "bands") else None
    main_run.close()
    legs = {}
    if world > 1 and extras:  # the other split and the other compositor choice, same steps
        try:
            om = "frames" if a.mode == "bands" else "bands"
            o = Pipeline(ctx, path, om, a.queues, a.variant, a.offsets, rotate, a.batch, a.rows)
            legs[om] = {**leg_summary(o.run(a.steps, a.warmup)), "scaling": "weak" if om == "frames" else "strong"}
            o.close()
            if a.mode == "bands":
                o = Pipeline(ctx, path, "bands", a.queues, a.variant, a.offsets, not rotate, a.batch, a.rows)
                legs["fixed_root" if rotate else "rotating_root"] = leg_summary(o.run(a.steps, a.warmup))
                o.close()
                other = "contiguous" if a.rows == "interleaved" else "interleaved"
                o = Pipeline(ctx, path, "bands", a.queues, a.variant, a.offsets, rotate, a.batch, other)
                legs[f"{other}_rows"] = leg_summary(o.run(a.steps, a.warmup))
                o.close()
        except Exception as e:  # noqa: BLE001 -- the primary line must still be printed
            legs["secondary_error"] = f"{type(e).__name__}: {e}"
    if world == 1 and extras:
        if a.offsets == "uniform":  # per-pixel jitter: the irregular-offset path
            o = Pipeline(ctx, path, "bands", leg_queues, a.variant, "random", batch=a.batch)
            rr = o.run(min(a.steps, 1000), a.warmup)
            rt2 = o.run(min(a.steps, 300), 2, queues=1, timing=True)
            o.close()
            legs["offsets_random"] = {**leg_summary(rr), "trace_kernel_ms": round(rt2["trace_ms"], 5),
                                      "note": "seeded U[0,1) per-pixel sample offsets (every tile irregular)"}
        if a.scene == "soup":  # C2: the Cornell box at the same resolution
            o = Pipeline(ctx, ctx.scene_path("cornell"), "bands", leg_queues, a.variant, a.offsets, batch=a.batch)
            legs["c2_cornell"] = {**leg_summary(o.run(min(a.steps, 1000), a.warmup)),
                                  "workload": workload_name(a, "cornell")}
            o.close()
        if a.brute_steps > 0 and a.variant != "lds":
            o = Pipeline(ctx, path, "bands", 1, "lds", a.offsets)
            legs["brute_force"] = o.run(a.brute_steps, 1, queues=1, timing=True)
            o.close()
        if a.brute_steps > 0:  # the other exact accelerator, same frame
            for v in ("cull", "bvh"):
                if v != a.variant:
                    o = Pipeline(ctx, path, "bands", leg_queues, v, a.offsets)
                    vr = o.run(min(a.steps, 1000), a.warmup)
                    vt = o.run(min(a.steps, 300), 2, queues=1, timing=True)
                    o.close()
                    legs[f"variant_{v}"] = {**leg_summary(vr), "kernel": KERNEL_NAMES[v],
                                            "stages_ms": {"prepare": round(vt["prepare_ms"], 5),
                                                          "bin": round(vt["bin_ms"], 5),
                                                          "trace_kernel": round(vt["trace_ms"], 5)},
                                            "note": "bit-identical frame (tests/test_gpu_parity.py)"}

    if rank == 0:
        band_ids = world > 1 and a.mode == "bands"
        launch_rays = main_run.row_count * W
        roof, valu, bfe = roofline_fields(wl, a.variant, launch_rays, n_tri, rt["trace_ms"], band_ids)
        if band_ids:
            par = (f"bands x{world} ({a.rows} rows) + RCCL gather of hit ids to the "
                   f"{'rotating' if rotate else 'rank-0'} compositor")
        else:
            par = f"{a.mode} x{world}"
        line = {
            "metric": "Mrays/s at 1920x1080 on 100k-tri synthetic mesh",
            "value": round(r["mrays"], 4),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(r["ms_per_step"], 5),
            "higher_is_better": True,
            "scaling": "strong" if a.mode == "bands" else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (PCG32 triangle soup, seed 0x5EED; {a.offsets} sample offsets resident in HBM)",
            "config": {
                "workload": wl,
                "triangles": int(n_tri),
                "width": W,
                "height": H,
                "spp": 1,
                "parallelism": par,
                "trace_variant": a.variant,
                "frame_queues": r["queues"],
                "frames_per_launch": main_run.L,
                "frames_per_batch": main_run.G,
                "offsets": a.offsets,
            },
            "roofline": roof,
            "stages_ms": {"prepare": round(rt["prepare_ms"], 5), "bin": round(rt["bin_ms"], 5),
                          "trace_kernel": round(rt["trace_ms"], 5), "frame": round(r["ms_per_step"], 5),
                          "frame_instrumented": round(rt["ms_per_step"], 5), "timed_launches": rt["launches"],
                          "note": "one frame per launch in flight, HIP events bound to the kernels' dispatches: "
                                  "prepare = TileInfoKernel (tile ray boxes), bin = PrepareBinKernel (record setup + "
                                  "bins) + WorkOrderKernel, trace_kernel = TraceCullKernel (rank 0's band at N > 1); "
                                  "frame = uninstrumented time per frame with config.frame_queues in flight"},
        }
        line["scene_build"] = {"spatial_order_ms": round(order_build_ms, 4),
                               "note": "once per scene at load, on the device (Morton codes + rocPRIM radix sort, "
                                       "csrc/spatial.hip); not per frame"}
        if valu is not None:
            line["valu_issue"] = valu
        line["brute_force_equivalent"] = bfe
        if r1 is not None:
            line["single_queue"] = {"mrays_per_s": round(r1["mrays"], 4), "ms_per_step": round(r1["ms_per_step"], 5),
                                    "note": "the same frames with one frame in flight (N = 1: one frame per launch, "
                                            "the per-frame latency)"}
        if world > 1:
            line["ranks_stages_ms"] = [{"rank": i, "prepare": round(s[0], 5), "bin": round(s[1], 5),
                                        "trace_kernel": round(s[2], 5)} for i, s in enumerate(ranks_stages)]
            line["verified"] = verified
            if band_ids:
                line["gather"] = {"payload": "int32 hit id per pixel (deferred shading on the compositor)",
                                  "frames_per_collective": main_run.G,
                                  "bytes_per_frame": (world - 1) * main_run.B * W * 4,
                                  "rgba_f32_equivalent": (world - 1) * main_run.B * W * 16}
        for k, v in legs.items():
            if k == "brute_force":
                bs = v["trace_ms"] * 1e-3
                tf = launch_rays * n_tri * FLOPS_PER_TEST / bs / 1e12
                line["brute_force"] = {
                    "variant": "lds", "kernel": "TraceLdsKernel", "mrays_per_s": round(v["mrays"], 3),
                    "kernel_ms": round(v["trace_ms"], 4), "steps": a.brute_steps,
                    "valu_equivalent_tflops": round(tf, 2), "valu_equivalent_frac": round(tf / FP32_PEAK_TFLOPS, 4),
                    "note": "north_star design taken literally: every ray tests every triangle, records tiled "
                            "through LDS; valu_equivalent counts 12 flops per test (DESIGN.md 5: ~5.25 VALU "
                            "instructions per test are issued)"}
            else:
                line[k] = v
        if world == 1 and not a.no_e2e and extras:
            line["e2e_ml_api"] = e2e_ml_api(path, W, H)
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(path, a)
        print(json.dumps(line), flush=True)
    if world > 1:
        ctx.dist.destroy_process_group()
    ctx.tmp.cleanup()


def e2e_ml_api(scene_path, W, H, reps=10, warmup=3):
    """PCIe-inclusive rate through the ml* API (host images in, host framebuffer out): median
    of `reps` frames after `warmup` (first frames pay one-time allocations)."""
    import numpy as np

    import simpleraytracer_amd as srt

    ctx = srt.Context()
    model = ctx.create_model(scene_path)
    model.set_input_info(W, H)
    (idt, iw, ih, ic), (odt, ow, oh, oc) = model.info()
    inp = ctx.create_image(idt, iw, ih, ic)
    out = ctx.create_image(odt, ow, oh, oc)
    inp.array()[...] = np.float32(0.5)
    for _ in range(warmup):
        model.infer(inp, out)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        model.infer(inp, out)
        times.append(time.perf_counter() - t0)
    dt = sorted(times)[len(times) // 2]
    inp.close()
    out.close()
    model.close()
    ctx.close()
    return {"mrays_per_s": round(W * H / dt / 1e6, 4), "ms_per_frame": round(dt * 1e3, 3),
            "path": "mlInfer: H2D offsets + prepare + trace + D2H framebuffer (pinned host images), "
                    "single device: 4 row chunks pipelined over three streams (SRT_E2E_CHUNKS)"}


if __name__ == "__main__":
    main()
