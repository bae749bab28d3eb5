#!/usr/bin/env python3
"""Headline benchmark: Mrays/s rendering the 100k-triangle synthetic soup at 1920x1080, 1 spp.

    python bench.py [--gpus N --steps K --warmup W]        (N > 1: launched by torch.distributed.run)

One step = one frame of the hot path on device-resident inputs: edge setup (prepare kernel)
+ brute-force closest hit + shade (trace kernel) for this rank's row band, and for N > 1 the
band gather to rank 0 over RCCL (strong scaling: the frame is fixed, N GPUs split its rows).
Prints ONE JSON line on rank 0 (contract in the task statement; fields in DESIGN.md "Bench").
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
FP32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md chip table (spec, vector fp32)
EDGE_BYTES_PER_TRI = 36      # 9 fp32 edge-function coefficients read per ray-triangle test
PIXEL_IO_BYTES = 8 + 16      # sample offsets in + RGBA out per ray
FLOPS_PER_TEST = 12          # 3 edge functions x 2 FMA (DESIGN.md "Roofline")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--scene", default="soup", choices=["soup", "cornell", "triangle"])
    p.add_argument("--triangles", type=int, default=100_000)
    p.add_argument("--variant", default=os.environ.get("SRT_BENCH_VARIANT", "cull"), choices=["lds", "scalar", "cull"])
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample length")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive ml* API measurement")
    return p.parse_args()


def workload_name(a):
    if a.scene == "soup":
        tri = f"{a.triangles // 1000}k" if a.triangles % 1000 == 0 else str(a.triangles)
        return f"soup-{tri} {a.width}x{a.height} 1spp"
    return f"{a.scene} {a.width}x{a.height} 1spp"


def cpu_baseline(scene_path, a, rank_rows):
    """The oracle ('port') on this host's cores over a bounded, evenly spaced row sample."""
    from oracle import srt_oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    sc = srt_oracle.OracleScene(scene_path)
    h = a.height
    # calibration: one row per thread
    step = max(1, h // threads)
    t0 = time.perf_counter()
    n0 = sc.render(a.width, h, row_begin=0, row_count=h, row_step=step, threads=threads)
    cal = time.perf_counter() - t0
    rows_cal = (h + step - 1) // step
    per_row = cal / rows_cal
    want_rows = max(rows_cal, min(h, int(a.cpu_seconds / max(per_row, 1e-9))))
    step = max(1, h // want_rows)
    t0 = time.perf_counter()
    sc.render(a.width, h, row_begin=0, row_count=h, row_step=step, threads=threads)
    dt = time.perf_counter() - t0
    rows = (h + step - 1) // step
    del n0
    return {
        "value": round(rows * a.width / dt / 1e6, 6),
        "unit": "Mrays/s",
        "cores": srt_oracle.threads(threads),
        "kind": "port",
        "sample": f"{rows} of {h} rows (every {step}th, all {a.width} columns) of {workload_name(a)}; "
                  f"{dt:.1f} s; OpenMP scalar C oracle (oracle/srt_oracle.c)",
    }


def pmc_traffic(workload, variant):
    """HBM bytes per trace launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    f = REPO / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        e = d.get(f"{workload}|{variant}")
        return None if e is None else float(e["hbm_bytes_per_launch"])
    except Exception:
        return None


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    import simpleraytracer_amd as srt
    from simpleraytracer_amd.bands import band_range, band_rows, gather_bands

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    tmp = tempfile.TemporaryDirectory()
    scene_path = os.path.join(tmp.name, f"scene_rank{rank}.srt")
    if a.scene == "soup":
        srt.write_scene(scene_path, "soup", a.triangles)
    else:
        srt.write_scene(scene_path, a.scene)
    scene = srt.DeviceScene(scene_path, local)
    n_tri = scene.triangles

    W, H = a.width, a.height
    row_begin, row_count = band_range(H, world, rank)
    B = band_rows(H, world)
    offsets = torch.full((B, W, 2), 0.5, dtype=torch.float32, device=dev)
    band = torch.zeros((B, W, 4), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]

    def step(i=None):
        e = ev[i] if i is not None else None
        if e:
            e[0].record(stream)
        scene.prepare(W, H, stream)
        if e:
            e[1].record(stream)
        scene.trace(offsets[:row_count], band[:row_count], row_begin, row_count, variant=a.variant, stream=stream)
        if e:
            e[2].record(stream)
        if world > 1:
            gather_bands(band, H, dst=0)

    for _ in range(a.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    prep_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / a.steps
    trace_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / a.steps
    rays_total = W * H * a.steps
    value = rays_total / elapsed / 1e6

    if rank == 0:
        launch_rays = row_count * W
        wl = workload_name(a)
        alg_bytes = launch_rays * (EDGE_BYTES_PER_TRI * n_tri + PIXEL_IO_BYTES)
        achieved_gbs = alg_bytes / (trace_ms * 1e-3) / 1e9
        achieved_tf = launch_rays * n_tri * FLOPS_PER_TEST / (trace_ms * 1e-3) / 1e12
        line = {
            "metric": "Mrays/s at 1920x1080 on 100k-tri synthetic mesh",
            "value": round(value, 4),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (PCG32 triangle soup, seed 0x5EED; sample offsets 0.5 resident in HBM)",
            "config": {
                "workload": wl,
                "triangles": int(n_tri),
                "width": W,
                "height": H,
                "spp": 1,
                "parallelism": f"row-bands x{world}" + (" + RCCL gather" if world > 1 else ""),
                "trace_variant": a.variant,
                "cull_bins": os.environ.get("SRT_CULL_BIN", "1") != "0" if a.variant == "cull" else None,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": pmc_traffic(wl, a.variant),
                "kernel": {"lds": "TraceLdsKernel", "scalar": "TraceScalarKernel", "cull": "TraceCullKernel"}[a.variant],
                "kernel_ms": round(trace_ms, 4),
                "bytes_per_launch": alg_bytes,
                "note": "north_star HBM roofline: 36 B/triangle/ray + 24 B/ray; LDS tiling re-uses each "
                        "record across 2048 rays, so frac > 1 (see DESIGN.md Roofline)",
            },
            "compute_roofline": {
                "bound": "valu-fp32",
                "achieved": round(achieved_tf, 2),
                "peak": FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved_tf / FP32_PEAK_TFLOPS, 4),
                "flops_per_test": FLOPS_PER_TEST,
            },
            "prepare_ms": round(prep_ms, 4),
        }
        if world == 1 and not a.no_e2e:
            line["e2e_ml_api"] = e2e_ml_api(scene_path, W, H)
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(scene_path, a, (row_begin, row_count))
        print(json.dumps(line), flush=True)
    scene.close()
    if world > 1:
        dist.destroy_process_group()
    tmp.cleanup()


def e2e_ml_api(scene_path, W, H, reps=3):
    """PCIe-inclusive rate through the ml* API (host images in, host framebuffer out)."""
    import numpy as np

    import simpleraytracer_amd as srt

    ctx = srt.Context()
    model = ctx.create_model(scene_path)
    model.set_input_info(W, H)
    (idt, iw, ih, ic), (odt, ow, oh, oc) = model.info()
    inp = ctx.create_image(idt, iw, ih, ic)
    out = ctx.create_image(odt, ow, oh, oc)
    inp.array()[...] = np.float32(0.5)
    model.infer(inp, out)
    t0 = time.perf_counter()
    for _ in range(reps):
        model.infer(inp, out)
    dt = (time.perf_counter() - t0) / reps
    inp.close()
    out.close()
    model.close()
    ctx.close()
    return {"mrays_per_s": round(W * H / dt / 1e6, 4), "ms_per_frame": round(dt * 1e3, 3),
            "path": "mlInfer: H2D offsets + prepare + trace + D2H framebuffer (pinned host images)"}


if __name__ == "__main__":
    main()
