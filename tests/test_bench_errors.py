"""bench.py ends a failed run with a JSON error record and a non-zero exit (never a hang or a bare
traceback): on this CPU-only container the engine cannot find a HIP device; on the GPU box an injected
worker failure (SRT_ENGINE_INJECT) stops the run."""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


def run_bench(env_extra, *args, timeout=300):
    env = dict(os.environ, **env_extra)
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, str(REPO / "bench.py"), *args], cwd=REPO, env=env, capture_output=True,
                          text=True, timeout=timeout)


def last_json(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert lines, stdout
    return json.loads(lines[-1])


def test_bench_without_gpu_prints_error_record():
    from conftest import gpu_available

    if gpu_available():
        pytest.skip("a GPU is visible: the no-device path is not reachable")
    r = run_bench({}, "--steps", "1", "--warmup", "0", "--no-extras", "--width", "64", "--height", "32",
                  "--triangles", "1000")
    assert r.returncode == 1, r.stderr[-2000:]
    rec = last_json(r.stdout)
    assert rec["value"] is None and rec["unit"] == "Mrays/s"
    assert "HIP" in rec["error"] or "device" in rec["error"], rec


@pytest.mark.gpu
def test_bench_injected_failure_prints_error_record(gpu):
    r = run_bench({"SRT_ENGINE_INJECT": "fail:0:1", "SRT_COMM_TIMEOUT_S": "5"}, "--steps", "3", "--warmup", "0",
                  "--no-extras", "--width", "320", "--height", "200", "--triangles", "2000", "--frames-per-step", "8")
    assert r.returncode == 1, r.stderr[-2000:]
    rec = last_json(r.stdout)
    assert rec["value"] is None and "injected failure" in rec["error"], rec


@pytest.mark.gpu
def test_bench_ml_multi_child_process(gpu, scenes):
    """The N > 1 line's ml_multi in a one-rank-per-GPU job runs in a child process of rank 0 under a time
    limit (bench.ml_multi_child): here over two fake devices -- both the gather (device copies) and the
    direct per-device D2H produce a rate, and a child that outlives its limit is reported, not waited for."""
    sys.path.insert(0, str(REPO))
    import bench

    out = bench.ml_multi_child(scenes["soup2k"], 320, 200, [0, 0], timeout_s=240)
    assert set(out) == {"copy", "direct"}, out
    for mode in ("copy", "direct"):
        assert out[mode]["mrays_per_s"] > 0 and out[mode]["devices"] == [0, 0], out
    late = bench.ml_multi_child(scenes["soup2k"], 320, 200, [0, 0], timeout_s=0.01)
    assert "did not finish" in late["error"], late


def test_cpu_baseline_times_the_binned_cpu_path_beside_the_oracle(tmp_path):
    """bench.cpu_baseline (every line, N = 1 and N > 1): the brute-force oracle over a row sample and,
    beside it, the product's own CPU render path (ML_VISIBLE_DEVICES=cpu: screen-box binning, the exact
    test) over whole frames, its ids checked against the oracle's rows; cores / model / host CPUs stated.
    The environment it sets for the binned path is restored afterwards."""
    import types

    sys.path.insert(0, str(REPO))
    import bench
    import simpleraytracer_amd as srt

    path = srt.write_scene(str(tmp_path / "soup.srt"), "soup", 3000, seed=7)
    a = types.SimpleNamespace(width=96, height=48, scene="soup", triangles=3000, cpu_seconds=0.5)
    before = {k: os.environ.get(k) for k in ("ML_VISIBLE_DEVICES", "SRT_CPU_THREADS")}
    out = bench.cpu_baseline(path, a)
    assert {k: os.environ.get(k) for k in before} == before
    b = out["binned"]
    assert "error" not in b, b
    assert b["value"] > 0 and b["cores"] >= 1 and b["frames"] >= 1 and b["parity_vs_oracle"] is True, b
    assert out["value"] > 0 and out["cores"] >= 1 and out["kind"] == "port" and out["host_cpus"] >= 1
    assert b["value"] > out["value"]  # binning against brute force on the same rows
