#!/usr/bin/env python3
"""Headline benchmark: Mrays/s rendering the 100k-triangle synthetic soup at 1920x1080, 1 spp.

    python bench.py [--gpus N --steps K --warmup W]        (N > 1: launched by torch.distributed.run)

One step = one frame of the hot path on device-resident inputs (SURVEY.md section 8 rows
a9-a12): edge-record setup (prepare kernel) + the closest-hit trace with its cull bins
(TileInfo / BinTriangles / TileOrder kernels, then TraceCullKernel, which also shades and
stores the framebuffer). The trace result is bit-identical to brute force (every ray against
every triangle; DESIGN.md section 5, tests/test_gpu_parity.py).

Multi-GPU, one rank per GPU:
  --mode frames (default): every rank renders whole 1920x1080 frames of a temporal-jitter
      sequence (rank r's frames use the uniform sub-pixel offset J_r; J_0 = 0.5 = the headline
      frame); no collective in the timed region; "scaling": "weak". Each rank keeps --queues
      frames in flight (default 3): frame k goes to queue k % Q, a DeviceScene with its own edge
      records, bins and framebuffer on its own HIP stream, so one frame's stages fill the CUs
      another frame's heavy-tile tail leaves idle. The one-frame-in-flight rate is reported
      beside it ("single_queue").
  --mode bands: the frame's rows are split into P bands (north_star row bands), each rank
      traces its band, and the bands are gathered to rank 0 over RCCL every step (double
      buffered, so step k's gather overlaps step k+1's render); "scaling": "strong".
  For N > 1 the line also carries the other mode's measurement under "bands" / "frames".

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
EDGE_BYTES_PER_TRI = 36      # 9 fp32 edge coefficients per ray-triangle test
PIXEL_IO_BYTES = 8 + 16      # sample offsets in + RGBA out per ray
FLOPS_PER_TEST = 12          # 3 edge functions x 2 FMA
GOLDEN = 0.6180339887498949  # temporal jitter sequence step
KERNEL_NAMES = {"lds": "TraceLdsKernel", "scalar": "TraceScalarKernel", "cull": "TraceCullKernel",
                "bvh": "TraceBvhKernel"}


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
    p.add_argument("--mode", default="frames", choices=["frames", "bands"], help="multi-GPU split (see module doc)")
    p.add_argument("--queues", type=int, default=int(os.environ.get("SRT_BENCH_QUEUES", "3")),
                   help="frames mode: frame queues in flight per GPU (own scene buffers + HIP stream each)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample length")
    p.add_argument("--brute-steps", type=int, default=5, help="timed frames of the brute-force LDS kernel (0 = skip)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive ml* API measurement")
    return p.parse_args()


def workload_name(a):
    if a.scene == "soup":
        tri = f"{a.triangles // 1000}k" if a.triangles % 1000 == 0 else str(a.triangles)
        return f"soup-{tri} {a.width}x{a.height} 1spp"
    return f"{a.scene} {a.width}x{a.height} 1spp"


def jitter(rank: int) -> float:
    """Uniform sub-pixel offset of rank r's frames (r = 0: 0.5, the headline frame)."""
    import numpy as np

    return float(np.float32((0.5 + rank * GOLDEN) % 1.0))


def cpu_baseline(scene_path, a):
    """The oracle ('port') on this host's cores over a bounded, evenly spaced row sample."""
    from oracle import srt_oracle

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
    }


def pmc_traffic(workload, variant):
    """HBM bytes per trace launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    f = REPO / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None
    try:
        e = json.loads(f.read_text()).get(f"{workload}|{variant}")
        return None if e is None else float(e["hbm_bytes_per_launch"])
    except Exception:
        return None


class Frames:
    """Timed loop of one multi-GPU mode on this rank (module doc)."""

    def __init__(self, torch, dist, srt, scene, a, mode, world, rank, dev, variant, queues=1):
        from simpleraytracer_amd.bands import band_range, band_rows

        self.torch, self.dist, self.scene, self.a = torch, dist, scene, a
        self.mode, self.world, self.rank, self.variant = mode, world, rank, variant
        W, H = a.width, a.height
        if mode == "bands":
            self.row_begin, self.row_count = band_range(H, world, rank)
            B = band_rows(H, world)
            off = 0.5
        else:
            self.row_begin, self.row_count = 0, H
            B = H
            off = jitter(rank)
        self.offsets = torch.full((B, W, 2), off, dtype=torch.float32, device=dev)
        nbuf = 2 if (mode == "bands" and world > 1) else 1
        self.bands = [torch.zeros((B, W, 4), dtype=torch.float32, device=dev) for _ in range(nbuf)]
        self.frames = None
        if mode == "bands" and world > 1 and rank == 0:
            self.frames = [torch.empty((world * B, W, 4), dtype=torch.float32, device=dev) for _ in range(nbuf)]
        self.pending = [None] * nbuf
        self.stream = torch.cuda.current_stream(dev)
        self.dev = dev
        # Frame queues (frames mode): queue q = its own DeviceScene (edge records, bins, BVH)
        # + framebuffer + HIP stream; frame k goes to queue k % Q, so up to Q frames are in
        # flight and one frame's prepare/bin/trace fills the CUs another frame's heavy-tile
        # tail leaves idle. Queue 0 is `scene` (on the current stream in the Q = 1 loop).
        self.queues = [(scene, self.stream, self.offsets, self.bands[0])]
        if mode == "frames" and queues > 1:
            self.queues[0] = (scene, torch.cuda.Stream(dev), self.offsets, self.bands[0])  # all on side streams
            for _ in range(max(1, queues) - 1):
                self.queues.append((srt.DeviceScene(scene.path, dev.index), torch.cuda.Stream(dev),
                                    self.offsets.clone(), torch.zeros_like(self.bands[0])))

    def step(self, k, queues=1):
        from simpleraytracer_amd.bands import gather_bands

        a, W, H = self.a, self.a.width, self.a.height
        if queues > 1:  # frames mode, no collective
            scene, stream, offsets, band = self.queues[k % queues]
            scene.prepare(W, H, stream)
            scene.trace(offsets, band, 0, H, variant=self.variant, stream=stream)
            return
        slot = k % len(self.bands)
        if self.pending[slot] is not None:
            self.pending[slot].wait()  # the gather still reading this band buffer
            self.pending[slot] = None
        self.scene.prepare(W, H, self.stream)
        band = self.bands[slot]
        self.scene.trace(self.offsets[:self.row_count], band[:self.row_count], self.row_begin, self.row_count,
                         variant=self.variant, stream=self.stream)
        if self.mode == "bands" and self.world > 1:
            out = self.frames[slot] if self.frames is not None else None
            if self.dist.get_backend() == "gloo":  # CPU rehearsal only: gloo gathers host tensors
                gather_bands(band.cpu(), H, dst=0)
            else:
                self.pending[slot] = self.dist.gather(band, gather_list=None if out is None else
                                                      [out[r * band.shape[0]:(r + 1) * band.shape[0]]
                                                       for r in range(self.world)], dst=0, async_op=True)

    def run(self, steps, warmup, timing=True, queues=1):
        """K timed frames over `queues` frame queues (stage timing: queue 0's events, so
        timing runs use queues=1)."""
        torch, dist = self.torch, self.dist
        queues = min(queues, len(self.queues))
        for k in range(warmup * queues):
            self.step(k, queues)
        self.drain()
        self.scene.take_stage_times()
        self.scene.set_stage_timing(timing)
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        for k in range(steps):
            self.step(warmup * queues + k, queues)
        self.drain()
        torch.cuda.synchronize(self.dev)
        if self.world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        self.scene.set_stage_timing(False)
        if self.world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=self.dev if dist.get_backend() != "gloo" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        launches, prep_ms, bin_ms, trace_ms = self.scene.take_stage_times()
        units = self.a.width * self.a.height * steps * (self.world if self.mode == "frames" else 1)
        return {"elapsed": elapsed, "mrays": units / elapsed / 1e6, "prepare_ms": prep_ms, "bin_ms": bin_ms,
                "trace_ms": trace_ms, "launches": launches, "ms_per_step": elapsed / steps * 1e3, "queues": queues}

    def close(self):
        for q in self.queues[1:]:
            q[0].close()
        self.queues = self.queues[:1]

    def drain(self):
        for i, h in enumerate(self.pending):
            if h is not None:
                h.wait()
                self.pending[i] = None


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    import simpleraytracer_amd as srt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("SRT_BENCH_ONE_DEVICE"):  # rehearsal of N > 1 ranks on a one-GPU box (with gloo)
        local = 0
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("SRT_BENCH_BACKEND", "nccl")  # gloo: CPU-side rehearsal on one GPU
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    tmp = tempfile.TemporaryDirectory()
    scene_path = os.path.join(tmp.name, f"scene_rank{rank}.srt")
    if a.scene == "soup":
        srt.write_scene(scene_path, "soup", a.triangles)
    else:
        srt.write_scene(scene_path, a.scene)
    scene = srt.DeviceScene(scene_path, local)
    n_tri = scene.triangles
    W, H = a.width, a.height
    wl = workload_name(a)

    main_run = Frames(torch, dist, srt, scene, a, a.mode, world, rank, dev, a.variant, a.queues)
    # value: uninstrumented frames over the frame queues. Then the same K frames on one queue
    # (one frame in flight: the per-frame latency), and again with HIP events bound to the
    # kernels' dispatch packets for the stage times (each event-bound dispatch leaves a 5-10 us
    # bubble on the stream, so the instrumented frame is slower; all three are reported).
    r = main_run.run(a.steps, a.warmup, timing=False, queues=a.queues)
    r1 = main_run.run(a.steps, a.warmup, timing=False) if r["queues"] > 1 else r
    rt = main_run.run(a.steps, 0, timing=True)
    main_run.close()
    for k in ("prepare_ms", "bin_ms", "trace_ms", "launches"):
        r[k] = rt[k]
    r["ms_per_step_instrumented"] = rt["ms_per_step"]
    other = None
    if world > 1:  # the other multi-GPU mode, same steps (secondary: a failure is reported, not fatal)
        om = "bands" if a.mode == "frames" else "frames"
        try:
            orun = Frames(torch, dist, srt, scene, a, om, world, rank, dev, a.variant, a.queues)
            other = (om, orun.run(a.steps, a.warmup, timing=False, queues=a.queues))
            ot = orun.run(a.steps, 0, timing=True)
            orun.close()
            for k in ("prepare_ms", "bin_ms", "trace_ms"):
                other[1][k] = ot[k]
        except Exception as e:  # noqa: BLE001 -- the primary line must still be printed
            other = (om, {"error": f"{type(e).__name__}: {e}"})
    brute = None
    if world == 1 and a.brute_steps > 0 and a.variant != "lds":
        brute = Frames(torch, dist, srt, scene, a, "frames", 1, 0, dev, "lds").run(a.brute_steps, 1, timing=True)
    alt = {}
    if world == 1 and a.brute_steps > 0:  # the other exact accelerator, same frame
        for v in ("cull", "bvh"):
            if v != a.variant:
                fr = Frames(torch, dist, srt, scene, a, "frames", 1, 0, dev, v, a.queues)
                alt[v] = fr.run(a.steps, a.warmup, timing=False, queues=a.queues)
                t = fr.run(a.steps, 0, timing=True)
                fr.close()
                alt[v].update({k: t[k] for k in ("prepare_ms", "bin_ms", "trace_ms")})

    if rank == 0:
        launch_rays = main_run.row_count * W
        rays_tests = launch_rays * n_tri
        alg_bytes = launch_rays * (EDGE_BYTES_PER_TRI * n_tri + PIXEL_IO_BYTES)
        kernel_s = r["trace_ms"] * 1e-3
        achieved_gbs = alg_bytes / kernel_s / 1e9
        io_gbs = launch_rays * PIXEL_IO_BYTES / kernel_s / 1e9
        achieved_tf = rays_tests * FLOPS_PER_TEST / kernel_s / 1e12
        line = {
            "metric": "Mrays/s at 1920x1080 on 100k-tri synthetic mesh",
            "value": round(r["mrays"], 4),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(r["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": "weak" if a.mode == "frames" else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (PCG32 triangle soup, seed 0x5EED; uniform sample offsets resident in HBM)",
            "config": {
                "workload": wl,
                "triangles": int(n_tri),
                "width": W,
                "height": H,
                "spp": 1,
                "parallelism": (f"{a.mode} x{world}" + (" + RCCL gather" if a.mode == "bands" and world > 1 else "")),
                "trace_variant": a.variant,
                "frame_queues": r["queues"],
                "cull_bins": os.environ.get("SRT_CULL_BIN", "1") != "0" if a.variant == "cull" else None,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": pmc_traffic(wl, a.variant),
                "kernel": KERNEL_NAMES[a.variant],
                "kernel_ms": round(r["trace_ms"], 5),
                "bytes_per_launch": alg_bytes,
                "note": "north_star HBM roofline (SURVEY 8d): 36 B per ray-triangle test + 24 B per ray, over the "
                        "trace kernel's HIP-event time (bin kernels excluded). frac > 1: the kernel skips "
                        "(record, tile) pairs that provably miss and re-uses records through LDS (DESIGN.md 6)",
            },
            "pixel_io_roofline": {
                "achieved": round(io_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(io_gbs / HBM_PEAK_GBS, 4),
                "note": "offsets in + RGBA out (24 B/ray) over the trace kernel time: the bytes no design avoids",
            },
            "compute_roofline": {
                "bound": "valu-fp32",
                "achieved": round(achieved_tf, 2),
                "peak": FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved_tf / FP32_PEAK_TFLOPS, 4),
                "flops_per_test": FLOPS_PER_TEST,
                "note": "brute-force-equivalent flops (every ray x every triangle)",
            },
            "stages_ms": {"prepare": round(r["prepare_ms"], 5), "bin": round(r["bin_ms"], 5),
                          "trace_kernel": round(r["trace_ms"], 5), "frame": round(r["ms_per_step"], 5),
                          "frame_instrumented": round(r["ms_per_step_instrumented"], 5),
                          "timed_launches": r["launches"],
                          "note": "cull variant: prepare = PrepareInfoKernel (edge records + per-tile info, one "
                                  "launch), bin = BinTrianglesKernel + TileOrderKernel, trace_kernel "
                                  "= TraceCullKernel; frame = uninstrumented, frame_instrumented = with the events"},
        }
        line["single_queue"] = {
            "mrays_per_s": round(r1["mrays"], 4), "ms_per_step": round(r1["ms_per_step"], 5),
            "note": "the same frames with one frame in flight per GPU (per-frame latency); value keeps "
                    "config.frame_queues frames in flight, each queue with its own scene buffers and HIP stream",
        }
        if brute is not None:
            bs = brute["trace_ms"] * 1e-3
            tf = rays_tests * FLOPS_PER_TEST / bs / 1e12
            line["brute_force"] = {
                "variant": "lds", "kernel": "TraceLdsKernel", "mrays_per_s": round(brute["mrays"], 3),
                "kernel_ms": round(brute["trace_ms"], 4), "steps": a.brute_steps,
                "hbm_roofline_frac": round(alg_bytes / bs / 1e9 / HBM_PEAK_GBS, 4),
                "valu_tflops": round(tf, 2), "valu_frac": round(tf / FP32_PEAK_TFLOPS, 4),
                "note": "north_star design taken literally: every ray tests every triangle, records tiled through LDS",
            }
        for v, o in alt.items():
            line[f"variant_{v}"] = {"kernel": KERNEL_NAMES[v], "mrays_per_s": round(o["mrays"], 3),
                                    "ms_per_step": round(o["ms_per_step"], 5),
                                    "stages_ms": {"prepare": round(o["prepare_ms"], 5), "bin": round(o["bin_ms"], 5),
                                                  "trace_kernel": round(o["trace_ms"], 5)},
                                    "note": "bit-identical frame (tests/test_gpu_parity.py); uninstrumented rate"}
        if other is not None and "error" in other[1]:
            line[other[0]] = other[1]
        elif other is not None:
            om, o = other
            line[om] = {"mrays_per_s": round(o["mrays"], 4), "ms_per_step": round(o["ms_per_step"], 4),
                        "scaling": "weak" if om == "frames" else "strong", "queues": o["queues"],
                        "trace_kernel_ms": round(o["trace_ms"], 5), "bin_ms": round(o["bin_ms"], 5),
                        "prepare_ms": round(o["prepare_ms"], 5)}
        if world == 1 and not a.no_e2e:
            line["e2e_ml_api"] = e2e_ml_api(scene_path, W, H)
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(scene_path, a)
        print(json.dumps(line), flush=True)
    scene.close()
    if world > 1:
        dist.destroy_process_group()
    tmp.cleanup()


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
