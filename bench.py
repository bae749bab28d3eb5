#!/usr/bin/env python3
"""Headline benchmark: Mrays/s rendering the 100k-triangle synthetic soup at 1920x1080, 1 spp.

    python bench.py [--gpus N --steps K --warmup W]

Runs with or without a launcher:
  * no WORLD_SIZE (or WORLD_SIZE=1): one process drives all N GPUs (devices 0..N-1) through the
    library's frame engine, one C++ worker thread per GPU, RCCL communicators from ncclCommInitAll;
  * python -m torch.distributed.run --nproc-per-node N bench.py --gpus N: one rank per GPU; the
    ranks share an RCCL unique id over torch.distributed (gloo: control plane only -- barriers, the
    id, max-over-ranks) and the engine's native communicator carries the data.
SRT_BENCH_ONE_DEVICE=1 puts every "device" on GPU 0 (single process: the bands are then exchanged
by device copies -- the multi-GPU rehearsal on a one-GPU box).

One step = one batch of --frames-per-step frames (default 256: a 256-frame sequence of the same
view; a timed region of a few tens of ms loses a fixed ~1 ms start cost -- 20 steps of 64 frames
read 114.6-116.5 Grays/s against 120.4 for 50 steps, 20 steps of 256 frames 122.4 -- so a step
carries 256), each frame a complete pass of the hot path on device-resident inputs (SURVEY.md
section 8 rows a9-a13): tile info, record setup and bins, the trace work list, the closest-hit
trace (TraceCullKernel; bit-identical to brute force), shading and the
framebuffer store. Nothing is cached across frames. Each GPU keeps --queues batches in flight.

Multi-GPU (BASELINE config C4), --mode bands (default): every frame is split
over the N GPUs in its 16-row tile rows, frame f composited on GPU f % N -- --exchange share
(default): the compositor traces k of every k + N - 1 tile rows itself (k = 32 at 1080p), fused with
the shading, every other GPU one, as packed hit ids; alltoall: N even interleaved bands --; the
bands go to the compositors over RCCL (the batch's N gathers fused into one ncclSend/ncclRecv
group), and each compositor shades its frames' received rows in one launch (deferred shading,
bit-identical). value = frames x W x H / the max-over-ranks time
of the timed steps: "scaling": "strong". --mode frames: every GPU renders whole frames of its own
(no exchange): "scaling": "weak" (a leg of the N > 1 line). After the timed steps every compositor
compares its last batches' frames with a single-GPU render by another kernel, bit for bit
("verified").

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
VERTEX_BYTES = 36            # 9 fp32 per triangle, read by the record pass
PIXEL_IO_BYTES = 8 + 16      # sample offsets in + RGBA out per ray
FLOPS_PER_TEST = 12          # 3 edge functions x 2 FMA
KERNEL_NAMES = {"lds": "TraceLdsKernel", "scalar": "TraceScalarKernel", "cull": "TraceCullKernel",
                "bvh": "TraceBvhKernel"}
PROFILES = REPO / "profiles"
METRIC = "Mrays/s at 1920x1080 on 100k-tri synthetic mesh"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # 50 steps x 256 frames = 12 800 frames, ~0.2 s timed at C3 on one GPU. (256 frames per step: a
    # timed region of 20 steps of 64 frames, ~23 ms, lost ~5 % to a fixed start cost -- 114.6 / 116.5
    # against 120.4 Grays/s at 50 steps; 20 steps of 128 / 256 frames: 120.3 / 122.4, profiles/r04/bench)
    p.add_argument("--steps", type=int, default=50, help="timed steps (batches of --frames-per-step frames)")
    p.add_argument("--warmup", type=int, default=2, help="untimed steps first")
    p.add_argument("--frames-per-step", type=int, default=256,
                   help="frames per step = per batch (a multiple of the GPU count for the all-to-all exchange)")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--scene", default="soup", choices=["soup", "cornell", "triangle"])
    p.add_argument("--triangles", type=int, default=100_000)
    p.add_argument("--variant", default=os.environ.get("SRT_BENCH_VARIANT", "cull"), choices=list(KERNEL_NAMES))
    p.add_argument("--mode", default="bands", choices=["bands", "frames"], help="multi-GPU split (module doc)")
    p.add_argument("--exchange", default="auto", choices=["auto", "alltoall", "rotating", "root", "share"],
                   help="bands: where frames are composited (module doc; auto: share)")
    p.add_argument("--share", type=int, default=0,
                   help="share exchange: the compositor's tile rows per cycle of share + N - 1, a power of two "
                        "(0: the library's srtShareAuto, 32 at 1080p)")
    p.add_argument("--rows", default="auto", choices=["auto", "interleaved", "contiguous", "rotated"],
                   help="bands: each GPU's rows -- the frame's 16-row tile rows dealt round-robin (interleaved), one "
                        "block (contiguous), or one block per GPU rotated by the frame's compositor (rotated; "
                        "all-to-all only); auto: rotated for all-to-all, interleaved otherwise")
    p.add_argument("--queues", type=int, default=int(os.environ.get("SRT_BENCH_QUEUES", "2")),
                   help="batches in flight per GPU (own scene buffers and HIP stream each)")
    p.add_argument("--offsets", default="uniform", choices=["uniform", "random"],
                   help="sample offsets: uniform 0.5 (headline) or seeded U[0,1) per-pixel jitter")
    p.add_argument("--launch", type=int, default=0,
                   help="frames per trace launch (0: the library's default, env SRT_LAUNCH_FRAMES)")
    p.add_argument("--inputs", type=int, default=1, help="distinct resident input images frames cycle through")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample length")
    p.add_argument("--brute-steps", type=int, default=5, help="timed frames of the brute-force LDS kernel (0 = skip)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive ml* API measurement")
    p.add_argument("--no-extras", action="store_true", help="only the main line (no secondary legs)")
    a = p.parse_args()
    if a.exchange == "auto":
        # Even framebuffer tiling (north_star: tiles over the GPUs + a gather): every frame split into
        # N contiguous bands of H / N rows, GPU d tracing band (d + c) % N of a frame composited on GPU
        # c = f % N (even load over any N frames), the bands' hit ids exchanged all-to-all. share
        # (the compositor tracing k of every k + N - 1 tile rows itself) and frames (whole frames
        # per GPU, no exchange) are legs beside it.
        a.exchange = "alltoall"
    if a.rows == "auto":
        a.rows = "rotated" if a.exchange == "alltoall" else "interleaved"
    return a


def workload_name(a, scene=None, triangles=None, width=None, height=None):
    scene = scene or a.scene
    triangles = triangles or a.triangles
    w, h = width or a.width, height or a.height
    if scene == "soup":
        tri = f"{triangles // 1000}k" if triangles % 1000 == 0 else str(triangles)
        return f"soup-{tri} {w}x{h} 1spp"
    return f"{scene} {w}x{h} 1spp"


def make_offsets(a, kind="uniform", count=1, seed=0x5EED):
    """(count, H, W, 2) float32 host offsets: uniform 0.5, or seeded U[0, 1) per-pixel jitter."""
    import numpy as np

    if kind == "random":
        rng = np.random.default_rng(seed)
        return rng.random((count, a.height, a.width, 2), dtype=np.float32)
    return np.full((count, a.height, a.width, 2), 0.5, dtype=np.float32)


class Job:
    """How this process takes part: one process for all GPUs, or one rank of a torchrun job."""

    def __init__(self, a):
        import torch

        self.torch = torch
        env_world = int(os.environ.get("WORLD_SIZE", "1") or 1)
        self.one_device = bool(os.environ.get("SRT_BENCH_ONE_DEVICE"))
        self.dist = None
        if env_world > 1:
            if env_world != a.gpus:
                raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={env_world}")
            import torch.distributed as dist

            self.dist = dist
            self.rank = int(os.environ.get("RANK", "0"))
            local = 0 if self.one_device else int(os.environ.get("LOCAL_RANK", "0"))
            import datetime

            # control plane only (the engine's RCCL communicator moves the data); a dead peer ends a
            # barrier after SRT_DIST_TIMEOUT_S instead of gloo's 30 minutes
            dist.init_process_group("gloo", timeout=datetime.timedelta(
                seconds=float(os.environ.get("SRT_DIST_TIMEOUT_S", "300"))))
            self.world = env_world
            self.devices = [local]
        else:
            self.rank = 0
            self.world = a.gpus
            self.devices = [0] * a.gpus if self.one_device else list(range(a.gpus))
        self.launch = "torchrun" if self.dist is not None else "single-process"
        self.tmp = tempfile.TemporaryDirectory()
        self.paths = {}

    @property
    def ranked(self):
        return self.dist is not None

    def scene_path(self, kind, triangles=None):
        import simpleraytracer_amd as srt

        key = (kind, triangles)
        if key not in self.paths:
            path = os.path.join(self.tmp.name, f"{kind}_{triangles}_rank{self.rank}.srt")
            if kind == "soup":
                srt.write_scene(path, "soup", triangles)
            else:
                srt.write_scene(path, kind)
            self.paths[key] = path
        return self.paths[key]

    def engine(self, path, a, mode=None, exchange=None, rows=None, queues=None, batch=None, variant=None,
               width=None, height=None, rccl_self=False):
        from simpleraytracer_amd.engine import FrameEngine, unique_id

        kw = dict(variant=variant or a.variant, queues=queues or a.queues, batch=batch or a.frames_per_step,
                  rows=rows or a.rows, exchange=exchange or a.exchange, split=mode or a.mode, launch=a.launch,
                  share=a.share)
        w, h = width or a.width, height or a.height
        if rccl_self:  # one device, the bands path with its ids sent to itself over a one-rank communicator
            return FrameEngine(path, w, h, devices=self.devices, rccl_self=True, **kw)
        if not self.ranked:
            return FrameEngine(path, w, h, devices=self.devices, **kw)
        return FrameEngine.rank(path, w, h, self.devices[0], self.rank, self.world, self.share_uid(unique_id), **kw)

    def share_uid(self, make):
        """Rank 0's make() (the RCCL unique id), on every rank."""
        uid = [make() if self.rank == 0 else None]
        self.dist.broadcast_object_list(uid, src=0)
        return uid[0]

    def sync(self):
        for d in sorted(set(self.devices)):
            self.torch.cuda.synchronize(d)

    def barrier(self):
        if self.ranked:
            self.dist.barrier()

    def max_over_ranks(self, x):
        if not self.ranked:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, values):
        """Every rank's list of floats (rank order)."""
        if not self.ranked:
            return [values]
        out = [None] * self.world
        self.dist.all_gather_object(out, values)
        return out

    def close(self):
        if self.ranked:
            self.dist.destroy_process_group()
        self.tmp.cleanup()


def timed(job, eng, steps, warmup):
    """`warmup` untimed batches, then exactly `steps` batches bracketed by a barrier + device
    synchronisation on both sides; elapsed = max over ranks. Returns (elapsed s, Mrays/s)."""
    eng.run(warmup)
    job.sync()
    job.barrier()
    t0 = time.perf_counter()
    eng.run(steps)  # returns once every local device has finished
    job.sync()
    elapsed = job.max_over_ranks(time.perf_counter() - t0)
    job.barrier()
    frames = steps * eng.batch * (job.world if eng.options["split"] == "frames" else 1)
    return elapsed, frames * eng.width * eng.height / elapsed / 1e6


def run_leg(job, a, path, inputs, steps, warmup, **kw):
    eng = job.engine(path, a, **kw)
    try:
        eng.set_inputs(inputs)
        el, mr = timed(job, eng, steps, warmup)
        return {"mrays_per_s": round(mr, 3), "ms_per_step": round(el / steps * 1e3, 5),
                "ms_per_frame": round(el / (steps * eng.batch) * 1e3, 6), "queues": eng.options["queues"],
                "frames_per_step": eng.batch}
    finally:
        eng.close()


def c5_leg(job, a, steps=10, warmup=2, batch=64, queues=1, launch=64):
    """BASELINE config C5 on this GPU: the 1M-triangle soup (seed 0x5EED + 1) at 3840 x 2160 in 64-frame
    steps, with a roofline block of its own for the trace kernel in the leg's launch shape (one launch in
    flight, HIP events on its dispatch) and the whole-frame figure. Frame loop: one queue, one 64-frame
    launch per step -- at 4K a record / bin launch and a trace launch each fill the chip, so a second queue
    only contends (three alternating rounds, profiles/r06/c5_ab/: 59 111 - 59 335 against 57 925 - 58 271
    Mrays/s with the headline's 2 queues x 8 frames), and fewer launch boundaries drain the chip fewer
    times (profiles/r06/c5_launch/: 16 / 32 / 64 frames per launch 59 576 - 59 653 / 60 003 - 60 127 /
    60 150 - 60 413); one queue also has the trace recompute its records (render.h RecordMode). (C5 proper
    is 8 GPUs: SCALE runs it; this is its one-GPU leg.)"""
    import copy

    a5 = copy.copy(a)
    a5.width, a5.height, a5.triangles, a5.frames_per_step = 3840, 2160, 1_000_000, batch
    a5.queues, a5.launch = queues, launch
    path = job.scene_path("soup", 1_000_000)
    wl = workload_name(a5)
    eng = job.engine(path, a5, batch=batch, width=a5.width, height=a5.height, queues=queues)
    try:
        eng.set_inputs(make_offsets(a5, a.offsets, 1))
        el, mr = timed(job, eng, steps, warmup)
        bad, checked = eng.verify()  # before the stage timing, which reuses queue 0's frames
        launch_frames = frames_per_launch(a5, 1)
        st = eng.stage_times(0, 24, launch_frames)
    finally:
        eng.close()
    import simpleraytracer_amd as srt

    n_tri = srt.scene_triangles(path)
    ms_frame = el / (steps * batch) * 1e3
    roof, _, _ = roofline_fields(wl, a.variant, a5.width * a5.height, launch_frames, n_tri, st[3], False, 1.0,
                                 profile_key(wl, a.variant, 1, a.rows, launch_frames), a.offsets != "uniform",
                                 f"C5 launch shape ({launch_frames} frames per launch), one launch in flight, {st[0]} "
                                 "launches, HIP events bound to the kernel's dispatch")
    return {"workload": wl, "mrays_per_s": round(mr, 3), "ms_per_frame": round(ms_frame, 6), "frames_per_step": batch,
            "queues": queues, "records": records_mode(queues, launch_frames, a.variant), "steps": steps, "roofline": roof, "whole_frame": whole_frame_fields(a5.width, a5.height, n_tri, ms_frame, 1),
            "stages_ms": {"bin": round(st[2], 5), "trace_kernel": round(st[3], 5), "frames_per_launch": launch_frames},
            "verified": bad == 0 and checked > 0}


def cpu_binned(scene_path, a, threads, seconds, oracle_rows=None):
    """The product's own CPU render path -- the backend the GPU path drops in for: mlInfer with
    ML_VISIBLE_DEVICES=cpu (csrc/cpu_render.cpp: records binned to 16 x 16 pixel tiles, the kernels'
    canonical math, threads over tiles) -- timed over whole frames on `threads` host threads (env
    SRT_CPU_THREADS), at least one and as many as fit `seconds`. oracle_rows = (rows, frame) of the
    brute-force oracle on the same offsets: the binned frame's ids are compared there bit for bit."""
    import numpy as np

    import simpleraytracer_amd as srt

    keep = {k: os.environ.get(k) for k in ("ML_VISIBLE_DEVICES", "SRT_CPU_THREADS")}
    os.environ["ML_VISIBLE_DEVICES"] = "cpu"
    os.environ["SRT_CPU_THREADS"] = str(threads)
    try:
        ctx = srt.Context()
        model = ctx.create_model(scene_path)
        model.set_input_info(a.width, a.height)
        (idt, iw, ih, ic), (odt, ow, oh, oc) = model.info()
        inp = ctx.create_image(idt, iw, ih, ic)
        out = ctx.create_image(odt, ow, oh, oc)
        inp.array()[...] = np.float32(0.5)
        times = []
        t_end = time.perf_counter() + seconds
        while not times or time.perf_counter() < t_end:
            t0 = time.perf_counter()
            model.infer(inp, out)
            times.append(time.perf_counter() - t0)
        frame = out.array().copy()
        for o in (inp, out, model, ctx):
            o.close()
    finally:
        for k, v in keep.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    dt = sorted(times)[len(times) // 2]
    res = {"value": round(a.width * a.height / dt / 1e6, 4), "unit": "Mrays/s", "cores": threads,
           "kind": "port", "frames": len(times), "ms_per_frame": round(dt * 1e3, 2),
           "sample": f"{len(times)} whole frames of {workload_name(a)} (median), uniform 0.5 offsets",
           "path": "mlInfer with ML_VISIBLE_DEVICES=cpu (csrc/cpu_render.cpp): screen-box binning to 16x16 pixel "
                   "tiles, exact canonical test, host threads over tiles -- the algorithm-matched CPU path the GPU "
                   "path drops in for (same culling idea, same bit-identical output)"}
    if oracle_rows is not None:
        rows, ref = oracle_rows
        res["parity_rows"] = len(rows)
        res["parity_vs_oracle"] = bool(np.array_equal(frame[rows, :, 3].view(np.uint32),
                                                      ref[rows, :, 3].view(np.uint32)))
    return res


def cpu_baseline(scene_path, a):
    """The oracle ('port') on this host's cores over a bounded, evenly spaced row sample, and beside it
    the product's binned CPU path (cpu_binned) on the same threads."""
    from oracle import srt_oracle

    # OMP_NUM_THREADS is the GPU box's CPU share for one GPU (16 of its 256 host CPUs; gpurun and
    # the driver set it); os.cpu_count() reports the whole machine.
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
    ref = sc.render(a.width, h, row_begin=0, row_count=h, row_step=step, threads=threads)
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
    try:
        binned = cpu_binned(scene_path, a, threads, max(1.0, a.cpu_seconds / 2),
                            (list(range(0, h, step)), ref))
    except Exception as e:  # noqa: BLE001 -- the baseline beside it must still be reported
        binned = {"error": f"{type(e).__name__}: {e}"}
    return {
        "single_thread": {"value": round(rows1 * a.width / dt1 / 1e6, 6), "unit": "Mrays/s", "cores": 1,
                          "sample": f"{rows1} rows (every {step1}th), {dt1:.1f} s"},
        "binned": binned,
        "cpu_model": model,
        "host_cpus": os.cpu_count(),
        "value": round(rows * a.width / dt / 1e6, 6),
        "unit": "Mrays/s",
        "cores": srt_oracle.threads(threads),
        "kind": "port",
        "sample": f"{rows} of {h} rows (every {step}th, all {a.width} columns) of {workload_name(a)}; "
                  f"{dt:.1f} s; OpenMP scalar C oracle (oracle/srt_oracle.c), brute force",
        "cores_note": "threads = OMP_NUM_THREADS, the CPU share the GPU box gives one GPU (16 of the machine's "
                      "host_cpus); BASELINE.md's 'all host cores' is not available to one GPU's job, so the "
                      "all-core rate would be about host_cpus / cores times this (scalar, linear in threads)",
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


def profile_key(wl, variant, world, rows_mode, launch_frames=1):
    """PMC summaries are keyed by the exact launch shape: the full frame at N = 1, the band at N > 1,
    and the frames per launch when more than one."""
    key = f"{wl}|{variant}" if world == 1 else f"{wl}|{variant}|bands{world}|{rows_mode}"
    return key if launch_frames == 1 else f"{key}|launch{launch_frames}"


def frames_per_launch(a, world):
    """engine.h EngineOptions::launch: --launch, else env SRT_LAUNCH_FRAMES, else 8 for whole frames
    and 64 for bands over more than one GPU; at most the batch and 256."""
    default = 64 if world > 1 and a.mode == "bands" else 8
    return min(a.launch or int(os.environ.get("SRT_LAUNCH_FRAMES") or default), a.frames_per_step, 256)


def records_mode(queues, launch_frames, variant="cull"):
    """Which records the binned trace reads (render.h RecordMode; renderer.cpp RecomputeRecords): env
    SRT_TRACE_RECORDS, else recomputed by the trace in a one-queue engine or one-frame launches, else stored."""
    if variant != "cull":
        return None
    env = os.environ.get("SRT_TRACE_RECORDS") or "auto"
    if env in ("stored", "recompute"):
        return env
    return "recompute" if queues == 1 or launch_frames == 1 else "stored"


def roofline_fields(wl, variant, launch_rays, launch_frames, n_tri, kernel_ms, band_ids, height_frac, key,
                    offsets_read, measured_in):
    """The trace kernel's roofline: its algorithmic bytes per launch over its HIP-event time.

    Algorithmic bytes per frame = the framebuffer it must write (16 B RGBA per ray, or the 4-B hit id
    on the band path) + each cull record read once (64 B; the band's pro-rata share at N > 1) + the
    sample offsets only where the trace reads them (8 B per ray of an irregular tile: jittered
    inputs; uniform inputs give regular tiles whose rays are computed, their offsets read once by
    the tile-info blocks of the bin launch, counted there). Measured traffic and VALU issue from
    committed rocprofv3 summaries of the same launch shape, else null."""
    kernel_s = kernel_ms * 1e-3
    out_bytes = 4 if band_ids else 16
    off_bytes = 8 if offsets_read else 0
    rec_bytes = int(round(n_tri * CULL_RECORD_BYTES * height_frac))
    frame_bytes = launch_rays * (off_bytes + out_bytes) + rec_bytes
    alg = launch_frames * frame_bytes
    achieved = alg / kernel_s / 1e9
    pmc = committed_profile("pmc_traffic.json", key) or {}
    roof = {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": pmc.get("hbm_bytes_per_launch"),
        "kernel": KERNEL_NAMES[variant],
        "kernel_ms": round(kernel_ms, 5),
        "frames_per_launch": launch_frames,
        "bytes_per_launch": alg,
        "bytes_per_frame": frame_bytes,
        "measured_in": measured_in,
        "profile_key": key,
        "note": f"algorithmic bytes per frame = rays x ({off_bytes} B offsets read by the trace + {out_bytes} B out) + "
                f"cull records x 64 B (stored: the 64-B record; recomputed, one-queue engines: 48 B of spatial "
                f"inputs + the 16-B screen box){'' if height_frac == 1 else ' x the band share of the rows'}; offsets count "
                "only where the trace loads them (irregular tiles); traffic = measured HBM bytes per launch of this "
                "launch shape (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE, profiles/pmc_traffic.json), null when no "
                "committed pass matches it",
    }
    sq = committed_profile("pmc_sq.json", key)
    valu = None
    if sq and sq.get("sq_insts_valu_per_launch"):
        issue_s = sq["sq_insts_valu_per_launch"] * 2 / (SIMDS * CLOCK_GHZ * 1e9)
        valu = {"valu_insts_per_launch": sq["sq_insts_valu_per_launch"], "issue_us": round(issue_s * 1e6, 2),
                "frac": round(issue_s / kernel_s, 4),
                "note": "SQ_INSTS_VALU (rocprofv3, profiles/pmc_sq.json) x 2 cycles per wave64 instruction "
                        "/ (1024 SIMDs x 2.4 GHz), over the kernel time"}
    tests = launch_frames * launch_rays * n_tri
    bf_bytes = launch_frames * launch_rays * (EDGE_BYTES_PER_TRI * n_tri + PIXEL_IO_BYTES)
    bfe = {"bytes_per_launch": bf_bytes, "tests_per_launch": tests,
           "hbm_equivalent_gbs": round(bf_bytes / kernel_s / 1e9, 1),
           "hbm_equivalent_frac": round(bf_bytes / kernel_s / 1e9 / HBM_PEAK_GBS, 2),
           "valu_equivalent_tflops": round(tests * FLOPS_PER_TEST / kernel_s / 1e12, 1),
           "note": "SURVEY 8(d) brute-force figures (36 B and 12 flops per ray-triangle test) over the cull "
                   "kernel's time: the work a brute-force kernel would do for the same bit-identical frame; "
                   "not a utilisation (the cull kernel proves most pairs miss without testing them)"}
    return roof, valu, bfe


def whole_frame_fields(W, H, n_tri, ms_per_frame, world):
    """The overlapped run as a whole: a frame's compulsory bytes (offsets in, RGBA framebuffer out,
    vertices read by the record pass) per frame time, against the HBM peak of the GPUs used."""
    bytes_frame = W * H * PIXEL_IO_BYTES + n_tri * VERTEX_BYTES
    gbs = bytes_frame / (ms_per_frame * 1e-3) / 1e9
    return {"bytes_per_frame": bytes_frame, "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS * world,
            "unit": "GB/s", "frac": round(gbs / (HBM_PEAK_GBS * world), 4),
            "note": "per frame: W x H x (8 B offsets + 16 B RGBA) + triangles x 36 B vertices, over ms_per_frame of "
                    "the timed (overlapped) run; peak = 8 TB/s x GPUs"}


def compositor_fraction(H, world, exchange, rows, share, own_rows=0):
    """Fraction of a frame's rows its compositor traces itself (straight into the frame as RGBA); the
    rest arrives as hit ids from the other GPUs. own_rows: the engine's two-device split (srtEngineSplit)."""
    from simpleraytracer_amd import _native
    from simpleraytracer_amd.bands import band_range, interleaved_range, rotate_own_rows, share_frame_rows

    if exchange == "share":
        k = share or _native.lib().srtShareAuto(H, world)
        return round(len(share_frame_rows(H, world, k, 0, 0)) / H, 5)
    if rows == "interleaved":
        return round(interleaved_range(H, world, 0)[1] / H, 5)
    if rows == "rotated" and world == 2:  # the compositor's band 0 (engine.cpp EngineSplit)
        return round((own_rows or rotate_own_rows(H)) / H, 5)
    return round(band_range(H, world, 0)[1] / H, 5)


def host_link_peaks(nbytes=64 << 20, reps=8):
    """Pinned host <-> device copy rates on this box (hipMemcpyAsync through torch's pinned copies, the
    path mlInfer's chunk pipeline takes): H2D alone, D2H alone, and both at once on two streams
    (duplex). GB/s; the e2e_ml_api roofline's denominator (measured, not the PCIe Gen5 x16 spec)."""
    import torch

    h_in = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d_b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()

    def run(h2d, d2h):
        for _ in range(2):  # warm-up
            if h2d:
                with torch.cuda.stream(s_in):
                    d_a.copy_(h_in, non_blocking=True)
            if d2h:
                with torch.cuda.stream(s_out):
                    h_out.copy_(d_b, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            if h2d:
                with torch.cuda.stream(s_in):
                    d_a.copy_(h_in, non_blocking=True)
            if d2h:
                with torch.cuda.stream(s_out):
                    h_out.copy_(d_b, non_blocking=True)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    t_in, t_out, t_both = run(True, False), run(False, True), run(True, True)
    gbs = lambda b, t: round(b / t / 1e9, 2)
    return {"h2d_gbs": gbs(nbytes * reps, t_in), "d2h_gbs": gbs(nbytes * reps, t_out),
            "duplex_gbs_each": gbs(nbytes * reps, t_both), "duplex_gbs_total": gbs(2 * nbytes * reps, t_both),
            "bytes_per_copy": nbytes, "copies": reps,
            "note": "torch pinned copies (hipMemcpyAsync) on two non-default streams, wall time of `copies` copies "
                    "after 2 untimed; duplex = H2D and D2H concurrently"}


def e2e_roofline(e2e, peaks, W, H, in_bytes_px=8, out_bytes_px=16):
    """mlInfer's host-link roofline: its bytes in and out over the measured one-way copy peaks.
    floor_duplex_ms = max(in / H2D, out / D2H): both directions at their full one-way rate at once (a
    full-duplex link, the render hidden) -- the bound the verdict asks for; floor_serial_ms = in / H2D
    + out / D2H (one direction at a time: what two concurrent copies achieved on the copy engines,
    host_link.duplex_gbs_total); frac = floor_duplex / measured."""
    bin_, bout = W * H * in_bytes_px, W * H * out_bytes_px
    duplex = max(bin_ / (peaks["h2d_gbs"] * 1e9), bout / (peaks["d2h_gbs"] * 1e9)) * 1e3
    serial = (bin_ / (peaks["h2d_gbs"] * 1e9) + bout / (peaks["d2h_gbs"] * 1e9)) * 1e3
    # what the box delivered with both directions busy at once (host_link.duplex_gbs_total): the link's
    # measured aggregate, the floor a pipelined frame can reach on this box
    agg = (bin_ + bout) / (peaks["duplex_gbs_total"] * 1e9) * 1e3
    return {"bytes_in": bin_, "bytes_out": bout, "floor_duplex_ms": round(duplex, 4), "floor_serial_ms": round(serial, 4),
            "floor_aggregate_ms": round(agg, 4),
            "frac": round(duplex / e2e["ms_per_frame"], 4), "frac_serial": round(serial / e2e["ms_per_frame"], 4),
            "frac_aggregate": round(agg / e2e["ms_per_frame"], 4),
            "achieved_gbs": round((bin_ + bout) / (e2e["ms_per_frame"] * 1e-3) / 1e9, 2),
            "note": "floor_duplex = both directions at their one-way rates at once (a full-duplex link); "
                    "floor_aggregate = in + out at the rate both directions reached together on this box "
                    "(host_link.duplex_gbs_total): the copy engines and the CU stores to host memory both "
                    "measured ~57 GB/s in total, however the bytes split between the directions"}


def e2e_ml_api(scene_path, W, H, reps=10, warmup=3, devices=None):
    """PCIe-inclusive rate through the ml* API (host images in, host framebuffer out): median of
    `reps` frames after `warmup`. devices: ML_VISIBLE_DEVICES for a multi-GPU mlInfer."""
    import numpy as np

    import simpleraytracer_amd as srt

    old = os.environ.get("ML_VISIBLE_DEVICES")
    if devices is not None:
        os.environ["ML_VISIBLE_DEVICES"] = ",".join(str(d) for d in devices)
    try:
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
        frame = out.array().copy()
        inp.close()
        out.close()
        model.close()
        ctx.close()
    finally:
        if devices is not None:
            if old is None:
                os.environ.pop("ML_VISIBLE_DEVICES", None)
            else:
                os.environ["ML_VISIBLE_DEVICES"] = old
    dt = sorted(times)[len(times) // 2]
    return {"mrays_per_s": round(W * H / dt / 1e6, 4), "ms_per_frame": round(dt * 1e3, 3)}, frame


def ml_multi_fields(path, W, H, devices, one_device):
    """mlInfer over `devices` (ML_VISIBLE_DEVICES) with the RCCL gather (device copies when a device
    repeats) and with per-device D2H into disjoint rows (direct): SURVEY 8(e)'s "report both"."""
    out = {}
    old_gather = os.environ.get("SRT_GATHER")
    for mode in ("copy" if one_device else "rccl", "direct"):
        try:
            os.environ["SRT_GATHER"] = mode
            e2e, _ = e2e_ml_api(path, W, H, devices=devices)
            out[mode] = {
                **e2e, "devices": devices,
                "path": ("mlInfer over ML_VISIBLE_DEVICES: H2D band offsets + interleaved band traces (hit ids) "
                         "+ gather to device 0 + shading + one D2H") if mode != "direct" else
                        ("mlInfer over ML_VISIBLE_DEVICES: H2D band offsets + band traces + shading on every "
                         "device + per-device D2H into disjoint rows of the host image (no gather)")}
        except Exception as e:  # noqa: BLE001
            out[mode] = {"error": f"{type(e).__name__}: {e}"}
        finally:
            if old_gather is None:
                os.environ.pop("SRT_GATHER", None)
            else:
                os.environ["SRT_GATHER"] = old_gather
    return out


def ml_multi_child(path, W, H, devices, timeout_s=240):
    """ml_multi_fields in a child process (rank 0 of a one-rank-per-GPU job), bounded by timeout_s."""
    import subprocess

    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    arg = json.dumps({"path": str(path), "W": W, "H": H, "devices": devices})
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--ml-multi-child", arg], env=env,
                           capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"error": f"mlInfer over {len(devices)} GPUs did not finish in {timeout_s} s (child killed)"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"child exit {r.returncode}: {(r.stderr or r.stdout)[-400:]}"}
    return json.loads(lines[-1])


def main():
    a = parse()
    if a.frames_per_step < 1 or a.queues < 1:
        raise SystemExit("--frames-per-step and --queues must be positive")
    job = Job(a)
    world, rank = job.world, job.rank
    path = job.scene_path(a.scene, a.triangles if a.scene == "soup" else None)
    wl = workload_name(a)
    W, H = a.width, a.height
    extras = not a.no_extras
    inputs = make_offsets(a, a.offsets, max(1, a.inputs))

    # value: the timed steps on the main engine
    eng = job.engine(path, a)
    info = eng.info()
    split = eng.split()
    n_tri = None
    eng.set_inputs(inputs)
    elapsed, mrays = timed(job, eng, a.steps, a.warmup)
    frames = a.steps * a.frames_per_step
    bad, checked = eng.verify()
    verified = job.gather([bad, checked])
    # The dominant kernel as the timed run launches it (launch_frames frames per launch), one launch
    # in flight: the roofline's kernel time (HIP events bound to the kernels' dispatches).
    launch_frames = frames_per_launch(a, world)
    n_launch = max(20, min(250, frames // launch_frames))
    st_launch = eng.stage_times(0, n_launch, launch_frames)
    # stage times of every rank's band (single-frame launches, events on the dispatches)
    n_stage = min(1000, max(20, frames))
    st = eng.stage_times(0, n_stage)
    if job.ranked:
        ranks_stages = job.gather(list(st))
    else:  # every device of this process, in band order
        ranks_stages = [list(st)] + [list(eng.stage_times(i, n_stage)) for i in range(1, info["local_devices"])]
    # the timed run's exchange, per device (HIP events on each device's exchange stream)
    xstats = [eng.exchange_stats(i) for i in range(info["local_devices"])] if world > 1 else []
    if job.ranked:
        xstats = [x for r in job.gather(xstats) for x in r]
    eng.close()
    import simpleraytracer_amd as srt

    n_tri = srt.scene_triangles(path)

    legs = {}
    if world == 1 and extras:
        # one frame per launch, one in flight: the per-frame latency
        legs["single_queue"] = run_leg(job, a, path, inputs, min(a.steps * a.frames_per_step, 2000), 20,
                                       queues=1, batch=1)
        legs["single_queue"]["note"] = "one frame per launch and in flight (the per-frame latency)"
        if a.inputs == 1:  # inputs that cannot stay in the 256 MB Infinity Cache
            ring = make_offsets(a, a.offsets, 16)
            legs["rotating_inputs"] = {**run_leg(job, a, path, ring, a.steps, a.warmup), "inputs": 16,
                                       "input_bytes": int(ring.nbytes),
                                       "note": "frames cycle through 16 distinct resident input images (265 MB > the "
                                               "256 MB MALL), same values as the headline's"}
        # The exchange code path over RCCL on one GPU: every frame's ids sent to itself with ncclSend /
        # ncclRecv inside the group, the groups timed as at N > 1 (a device-local copy through RCCL, not
        # an xGMI link: the rehearsal of the N > 1 exchange fields on hardware)
        try:
            e = job.engine(path, a, rccl_self=True, rows="interleaved", exchange="alltoall", batch=64)
            e.set_inputs(inputs)
            _, mr = timed(job, e, min(a.steps, 10), 1)
            xs, xi = e.exchange_stats(0), e.info()
            bad, checked = e.verify()
            e.close()
            legs["rccl_self_exchange"] = {
                "mrays_per_s": round(mr, 3), "transport": "RCCL" if xi["rccl"] else "none",
                "groups": xs["groups"], "ms_per_batch": round(xs["ms_mean"], 5),
                "bytes_per_batch": int(xs["bytes_sent"]),
                "gbs": round(xs["bytes_sent"] / (xs["ms_mean"] * 1e-3) / 1e9, 2) if xs["ms_mean"] else None,
                "verified": bad == 0 and checked > 0,
                "note": "one GPU, bands path with a one-rank RCCL communicator: each 64-frame batch's packed ids "
                        "sent to itself (ncclSend / ncclRecv to self inside one group, timed by HIP events on the "
                        "exchange stream) and shaded from the received copy; a device-local copy, not a link rate"}
        except Exception as exc:  # noqa: BLE001 -- the primary line must still be printed
            legs["rccl_self_exchange"] = {"error": f"{type(exc).__name__}: {exc}"}
        if a.offsets == "uniform":
            legs["offsets_random"] = {**run_leg(job, a, path, make_offsets(a, "random"), min(a.steps, 60), a.warmup),
                                      "note": "seeded U[0,1) per-pixel sample offsets (every tile irregular)"}
        if a.scene == "soup":
            legs["c2_cornell"] = {**run_leg(job, a, job.scene_path("cornell"), inputs, min(a.steps, 60), a.warmup),
                                  "workload": workload_name(a, "cornell")}
        if a.scene == "soup" and a.triangles == 100_000 and (W, H) == (1920, 1080):
            try:
                legs["c5_one_gpu"] = c5_leg(job, a)
            except Exception as exc:  # noqa: BLE001 -- the primary line must still be printed
                legs["c5_one_gpu"] = {"error": f"{type(exc).__name__}: {exc}"}
        if a.brute_steps > 0 and a.variant != "lds":
            e = job.engine(path, a, variant="lds", queues=1, batch=1)
            e.set_inputs(inputs)
            el, mr = timed(job, e, a.brute_steps, 1)
            n, _, _, kt = e.stage_times(0, a.brute_steps)
            e.close()
            tf = W * H * n_tri * FLOPS_PER_TEST / (kt * 1e-3) / 1e12
            legs["brute_force"] = {
                "variant": "lds", "kernel": "TraceLdsKernel", "mrays_per_s": round(mr, 3), "kernel_ms": round(kt, 4),
                "steps": a.brute_steps, "valu_equivalent_tflops": round(tf, 2),
                "valu_equivalent_frac": round(tf / FP32_PEAK_TFLOPS, 4),
                "note": "north_star design taken literally: every ray tests every triangle, records tiled through "
                        "LDS; valu_equivalent counts 12 flops per test (DESIGN.md 5: ~5.25 VALU instructions per "
                        "test are issued)"}
        if a.brute_steps > 0:
            for v in ("cull", "bvh"):
                if v != a.variant:
                    e = job.engine(path, a, variant=v, queues=3)
                    e.set_inputs(inputs)
                    _, mr = timed(job, e, min(a.steps, 30), 2)
                    n, pm, bm, tm = e.stage_times(0, 100)
                    e.close()
                    legs[f"variant_{v}"] = {"mrays_per_s": round(mr, 3), "kernel": KERNEL_NAMES[v],
                                            "stages_ms": {"prepare": round(pm, 5), "bin": round(bm, 5),
                                                          "trace_kernel": round(tm, 5)},
                                            "note": "bit-identical frame (tests/test_gpu_parity.py)"}
    if world > 1 and extras:
        main = (a.mode, a.exchange, a.rows)
        for name, kw in (("frames", {"mode": "frames"}),
                         ("share_exchange", {"mode": "bands", "exchange": "share", "rows": "interleaved"}),
                         ("interleaved_alltoall", {"mode": "bands", "exchange": "alltoall", "rows": "interleaved"}),
                         ("rotated_alltoall", {"mode": "bands", "exchange": "alltoall", "rows": "rotated"})):
            if (kw.get("mode"), kw.get("exchange", a.exchange), kw.get("rows", a.rows)) == main or \
                    (name == "frames" and a.mode == "frames"):
                continue
            try:
                legs[name] = run_leg(job, a, path, inputs, a.steps, a.warmup, **kw)
                legs[name]["scaling"] = "weak" if name == "frames" else "strong"
                if name != "frames":
                    legs[name]["compositor_fraction"] = compositor_fraction(H, world, kw["exchange"], kw["rows"],
                                                                            a.share)
            except Exception as e:  # noqa: BLE001 -- the primary line must still be printed
                legs[name] = {"error": f"{type(e).__name__}: {e}"}
        if main == ("bands", "alltoall", "rotated") and world == 2:
            # the two-device split at even halves (the value's split keeps the compositor's band 0 at the
            # share the measured link allows -- engine.cpp RotateSplitForLink -- or 4/5 without RCCL)
            prev = os.environ.get("SRT_ROTATE_OWN")
            os.environ["SRT_ROTATE_OWN"] = "50"
            try:
                legs["rotated_even_halves"] = run_leg(job, a, path, inputs, a.steps, a.warmup)
                legs["rotated_even_halves"].update(scaling="strong", compositor_fraction=0.5)
            except Exception as e:  # noqa: BLE001
                legs["rotated_even_halves"] = {"error": f"{type(e).__name__}: {e}"}
            finally:
                if prev is None:
                    os.environ.pop("SRT_ROTATE_OWN", None)
                else:
                    os.environ["SRT_ROTATE_OWN"] = prev
        if a.mode == "bands":
            # one frame in flight across the N GPUs: the per-frame latency of the split
            try:
                legs["one_frame_in_flight"] = {
                    **run_leg(job, a, path, inputs, min(a.steps * a.frames_per_step, 400), 20, queues=1, batch=1),
                    "note": "one frame per batch, one batch in flight: every GPU traces its band of it, the bands "
                            "are exchanged and composited on GPU 0 (per-frame latency across the N GPUs; "
                            "single_queue at N = 1 is the one-GPU figure)"}
            except Exception as e:  # noqa: BLE001
                legs["one_frame_in_flight"] = {"error": f"{type(e).__name__}: {e}"}

    if rank == 0:
        band = world > 1 and a.mode == "bands"
        rows0 = info["band_rows"] if band else H
        launch_rays = rows0 * W
        key = profile_key(wl, a.variant, world if band else 1, a.rows, launch_frames)
        offsets_read = a.offsets != "uniform"
        roof, valu, bfe = roofline_fields(
            wl, a.variant, launch_rays, launch_frames, n_tri, st_launch[3], band, rows0 / H, key, offsets_read,
            f"the timed run's launch shape ({launch_frames} frames per launch), one launch in flight, "
            f"{st_launch[0]} launches, HIP events bound to the kernel's dispatch")
        roof1, _, _ = roofline_fields(
            wl, a.variant, launch_rays, 1, n_tri, st[3], band, rows0 / H, profile_key(wl, a.variant, world if band
                                                                                      else 1, a.rows, 1),
            offsets_read, f"latency pass: one frame per launch, one in flight, {st[0]} launches")
        ms_frame = elapsed / frames * 1e3
        if band:
            par = (f"bands x{world} ({a.rows} rows) + {'RCCL' if info['rccl'] else 'device-copy'} "
                   f"{a.exchange} exchange of hit ids to the compositors")
        else:
            par = f"{a.mode} x{world}"
        line = {
            "metric": METRIC,
            "value": round(mrays, 4),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 5),
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
                "launch": job.launch,
                "devices": job.devices if not job.ranked else f"rank {rank} of {world}",
                "trace_variant": a.variant,
                "frames_per_step": a.frames_per_step,
                "frame_queues": a.queues,
                # engine.h EngineOptions::launch defaults when neither --launch nor SRT_LAUNCH_FRAMES is set
                "frames_per_launch": launch_frames,
                "records": records_mode(a.queues, launch_frames, a.variant),
                "inputs": max(1, a.inputs),
                "offsets": a.offsets,
            },
            "ms_per_frame": round(ms_frame, 6),
            "roofline": roof,
            "roofline_single_frame": roof1,
            "whole_frame": whole_frame_fields(W, H, n_tri, ms_frame, world if a.mode == "bands" else 1),
            "stages_ms": {"prepare": round(st[1], 5), "bin": round(st[2], 5), "trace_kernel": round(st[3], 5),
                          "timed_launches": st[0],
                          "note": "single-frame launches of rank 0's band, HIP events bound to the kernels' dispatches: "
                                  "prepare = TileInfoKernel (0 for a full frame: its tile info runs inside the bin "
                                  "launch), bin = PrepareBinKernel (record setup + bins [+ tile info]) + "
                                  "WorkOrderKernel, trace_kernel = TraceCullKernel"},
        }
        if valu is not None:
            line["valu_issue"] = valu
        line["brute_force_equivalent"] = bfe
        line["verified"] = all(v[0] == 0 and v[1] > 0 for v in verified)
        line["verify"] = {"frames_checked": sum(v[1] for v in verified), "mismatches": sum(v[0] for v in verified),
                          "note": "up to 4 frames composited in each queue's last batch, on every GPU, vs a single-GPU "
                                  "full-frame render of their inputs by another trace kernel (lds for cull), bit for "
                                  "bit"}
        if world > 1:
            line["ranks_stages_ms"] = [{"rank": i, "prepare": round(s[1], 5), "bin": round(s[2], 5),
                                        "trace_kernel": round(s[3], 5)} for i, s in enumerate(ranks_stages)]
            if band:
                from simpleraytracer_amd import _native

                share_k = a.share or _native.lib().srtShareAuto(H, world)
                xb = info["exchange_bytes_per_frame"]
                px = max(1, (world - 1) * info["buffer_rows"] * W)
                ms_x = [x["ms_mean"] for x in xstats if x["groups"]]
                sent = [x["bytes_sent"] for x in xstats if x["groups"]]
                ms_mean = sum(ms_x) / len(ms_x) if ms_x else None
                per_link = (sum(sent) / len(sent)) / (world - 1) if sent else None
                line["exchange"] = {"pattern": a.exchange, "rows": a.rows,
                                    "transport": "RCCL" if info["rccl"] else "device copies",
                                    "share": share_k if a.exchange == "share" else None,
                                    "compositor_fraction": compositor_fraction(H, world, a.exchange, a.rows, a.share,
                                                                               split["own_rows"]),
                                    "split": {**split, "note": "own_rows: the compositor's own band over two GPUs "
                                              "(rotated rows); link_gbs: RCCL send/receive groups of 32 MB timed at "
                                              "engine creation, per direction of the slowest GPU; source 'link' = "
                                              "the split derived from it (srtRotateSplitForLink, DESIGN.md 7)"},
                                    "ms_per_batch": round(ms_mean, 5) if ms_mean else None,
                                    "ms_per_batch_by_device": [round(x, 5) for x in ms_x],
                                    "bytes_per_link_per_batch": int(per_link) if per_link else None,
                                    "gbs_per_directed_link": round(per_link / (ms_mean * 1e-3) / 1e9, 2)
                                    if ms_mean and per_link else None,
                                    "timing_note": "HIP events on each GPU's exchange stream around every batch's "
                                                   "ncclSend / ncclRecv group (device copies on fake devices), from the "
                                                   "stream reaching the group to its end -- waits for late peers "
                                                   "included, so the rate is a lower bound of the link's; per directed "
                                                   "link = a GPU's bytes sent per batch / (N - 1)",
                                    "payload": "packed hit ids (16 + k bits per pixel: a u16 plane and k bit planes, "
                                               "render.h PackedIds) or int32 ids; deferred shading on the compositor, "
                                               "whose own band is traced to RGBA in place",
                                    "bytes_per_pixel": round(xb / px, 4),
                                    "bytes_per_frame": int(xb),
                                    "int32_ids_equivalent": int(px * 4),
                                    "rgba_f32_equivalent": int(px * 16)}
        for k, v in legs.items():
            line[k] = v
        if world == 1 and not a.no_e2e and extras:
            e2e, _ = e2e_ml_api(path, W, H)
            peaks = host_link_peaks()
            line["e2e_ml_api"] = {**e2e, "path": "mlInfer: H2D offsets (copy engine, row chunks pipelined: "
                                                 "SRT_E2E_CHUNKS) + trace storing each chunk's framebuffer rows "
                                                 "straight into the page-locked host image (SRT_E2E_DIRECT)",
                                  "host_link": peaks, "roofline": e2e_roofline(e2e, peaks, W, H)}
        if world > 1 and not a.no_e2e and extras:
            # the drop-in path over the N GPUs: the bands gathered to GPU 0 (RCCL; device copies on fake
            # devices) and one D2H, or every GPU copying its rows straight into the host image (direct).
            # One rank per GPU (the other ranks wait at the barrier below, their engines closed): rank 0
            # runs it over every GPU in a child process under a time limit, so a stuck GPU call there
            # cannot hold the job.
            if job.ranked:
                line["ml_multi"] = ml_multi_child(path, W, H, list(range(world)))
            else:
                line["ml_multi"] = ml_multi_fields(path, W, H, job.devices, job.one_device)
        if not a.no_cpu_baseline:  # on every line, from rank 0 (the other ranks wait at the barrier below)
            line["cpu_baseline"] = cpu_baseline(path, a)
        print(json.dumps(line), flush=True)
    job.barrier()
    job.close()


def error_line(e):
    """A failed run's record: the same keys as the result line with value null and the error.
    Every rank that fails prints one (the engine turns a dead peer into an error, engine.h)."""
    return {"metric": METRIC, "value": None, "unit": "Mrays/s", "higher_is_better": True,
            "n_gpus": int(os.environ.get("WORLD_SIZE", "0") or 0) or None, "rank": int(os.environ.get("RANK", "0") or 0),
            "error": f"{type(e).__name__}: {e}"}


if __name__ == "__main__":
    if len(sys.argv) == 3 and sys.argv[1] == "--ml-multi-child":  # bench.ml_multi_child
        _c = json.loads(sys.argv[2])
        print(json.dumps(ml_multi_fields(_c["path"], _c["W"], _c["H"], _c["devices"],
                                         len(set(_c["devices"])) < len(_c["devices"]))), flush=True)
        sys.exit(0)
    try:
        main()
    except SystemExit:
        raise
    except BaseException as exc:  # noqa: BLE001 -- a JSON error record and a non-zero exit, never a hang
        import traceback

        traceback.print_exc()
        print(json.dumps(error_line(exc)), flush=True)
        sys.stderr.flush()
        # No destructors or atexit hooks: a device left in a failed state must not turn the exit
        # into a hang (this process is never re-executed; it ends here).
        os._exit(1)
