"""Shared fixtures. `-m gpu` tests need an MI355X; everything else runs on CPU.

The product library (simpleraytracer_amd/lib/libModelRunner.so) and the oracle
(oracle/build/libsrt_oracle.so) are built once per session with `make` if missing.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))

# Sanitizer runs (tools/asan_tests.sh): this process has the ASan runtime preloaded and binds the
# sanitized libraries (SRT_LIB / SRT_ORACLE_LIB, read when the bindings are imported); child
# processes (the CLIs, bench.py) are not instrumented and run the normal build without the preload.
if os.environ.get("SRT_ASAN_RUN"):
    import oracle.srt_oracle  # noqa: E402,F401
    import simpleraytracer_amd._native  # noqa: E402,F401

    for _v in ("LD_PRELOAD", "SRT_LIB", "SRT_ORACLE_LIB", "SRT_ASAN_RUN"):
        os.environ.pop(_v, None)

LIB = REPO / "simpleraytracer_amd" / "lib" / "libModelRunner.so"
ORACLE_LIB = REPO / "oracle" / "build" / "libsrt_oracle.so"
REFERENCE = Path("/root/reference/model_runner")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


def _make(*targets):
    subprocess.run(["make", "-s", "-C", str(REPO), *targets], check=True)


@pytest.fixture(scope="session", autouse=True)
def built():
    if not LIB.exists():
        _make("all")
    if not ORACLE_LIB.exists():
        _make("oracle")
    return True


@pytest.fixture(scope="session")
def scenes(tmp_path_factory, built):
    """Scene files of every config: triangle (C1), cornell (C2), soup-100k (C3/C4), small soups."""
    import simpleraytracer_amd as srt

    d = tmp_path_factory.mktemp("scenes")
    out = {
        "triangle": srt.write_scene(str(d / "triangle.srt"), "triangle"),
        "cornell": srt.write_scene(str(d / "cornell.srt"), "cornell"),
        "soup100k": srt.write_scene(str(d / "soup100k.srt"), "soup", 100_000),
        "soup2k": srt.write_scene(str(d / "soup2k.srt"), "soup", 2_000, seed=7),
        "soup300": srt.write_scene(str(d / "soup300.srt"), "soup", 300, seed=11, size=0.2),
    }
    return out


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    return 0


def env_without(*names):
    env = dict(os.environ)
    for n in names:
        env.pop(n, None)
    return env
