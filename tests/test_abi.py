"""C-ABI boundary on CPU: exports, struct layouts, validation order and messages.

The reference behaviours pinned here come from /root/reference/model_runner/{context,image,
model}.cpp (cited per test). Deliberate deviations (DESIGN.md "Boundary deviations") are
asserted as such.
"""
from __future__ import annotations

import ctypes
import re
import subprocess
from pathlib import Path

import pytest

from conftest import REFERENCE, REPO, gpu_available

from simpleraytracer_amd import _native
from simpleraytracer_amd._native import ML_FAIL, ML_FLOAT16, ML_FLOAT32, ML_OK, ImageInfo, ModelParams


@pytest.fixture(scope="module")
def L():
    return _native.lib()


@pytest.fixture
def ctx(L):
    c = L.mlCreateContext()
    assert c
    yield c
    L.mlReleaseContext(c)


def cerr(L, ctx):
    buf = ctypes.create_string_buffer(256)
    return L.mlGetContextError(ctx, buf, 256).decode()


def merr(L, model):
    buf = ctypes.create_string_buffer(256)
    return L.mlGetModelError(model, buf, 256).decode()


def header_symbols():
    names = []
    for h in (REPO / "include").glob("*.h"):
        names += re.findall(r"ML_API_ENTRY\s+[\w\s\*]+?\b(\w+)\s*\(", h.read_text())
    return sorted(set(names))


def test_every_header_symbol_is_exported(L):
    syms = header_symbols()
    assert len(syms) == 14 + 38  # the reference ABI + the srt* extension (include/srt_render.h)
    out = subprocess.run(["nm", "-D", "--defined-only", str(_native.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(syms) <= exported
    for s in syms:
        assert getattr(L, s) is not None
    # nothing else leaks out of the hidden-visibility build
    assert {s for s in exported if s.startswith(("ml", "srt"))} == set(syms)


def test_batch_limit_matches_header():
    import re

    import simpleraytracer_amd as srt

    hdr = (REPO / "include" / "srt_render.h").read_text()
    assert int(re.search(r"#define SRT_MAX_BATCH (\d+)", hdr).group(1)) == srt.MAX_BATCH == 8


def test_reference_entry_points_are_the_ml_family():
    ml = [s for s in header_symbols() if s.startswith("ml")]
    assert ml == sorted([
        "mlCreateContext", "mlGetContextError", "mlReleaseContext", "mlCreateImage", "mlGetImageInfo",
        "mlMapImage", "mlUnmapImage", "mlReleaseImage", "mlCreateModel", "mlGetModelError", "mlGetModelInfo",
        "mlSetModelInputInfo", "mlInfer", "mlReleaseModel"])


LAYOUT_PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "model_runner.h"
int main(void) {
    printf("%zu %zu %zu %zu %zu %d %d %d %d\n", sizeof(ml_model_params), sizeof(ml_image_info),
           offsetof(ml_image_info, dtype), offsetof(ml_image_info, width), offsetof(ml_image_info, channels),
           (int)ML_OK, (int)ML_FAIL, (int)ML_FLOAT32, (int)ML_FLOAT16);
    return 0;
}
"""


def _probe(tmp_path, compiler, lang, include_dir):
    src = tmp_path / f"probe.{lang}"
    src.write_text(LAYOUT_PROBE)
    exe = tmp_path / f"probe_{lang}"
    args = [compiler, "-x", "c" if lang == "c" else "c++", "-Wall", "-Werror", f"-I{include_dir}", str(src),
            "-o", str(exe)]
    if lang == "c":
        args[1:1] = ["-std=c99", "-pedantic"]
    subprocess.run(args, check=True, capture_output=True)
    return subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()


def test_header_is_valid_c_with_reference_layout(tmp_path):
    ours = _probe(tmp_path, "gcc", "c", REPO / "include")
    assert ours == ["24", "32", "0", "8", "24", "0", "1", "0", "1"]
    assert ctypes.sizeof(ImageInfo) == 32 and ctypes.sizeof(ModelParams) == 24
    if REFERENCE.exists():  # the reference header only compiles as C++ (model_runner.h:102)
        ref = _probe(tmp_path, "g++", "cpp", REFERENCE)
        assert ours == ref


def test_context_error_messages(L, ctx):
    # context.cpp:71-79 "Bad context handle"; FillBuffer deviation: the full text, no lost char
    buf = ctypes.create_string_buffer(64)
    assert L.mlGetContextError(None, buf, 64) == b"Bad context handle"
    assert L.mlGetContextError(None, buf, 4) == b"Bad"
    # empty cache: "" (the reference throws std::out_of_range here)
    assert L.mlGetContextError(ctx, buf, 64) == b""
    # buffer_size 0 leaves the buffer untouched (the reference throws)
    buf.value = b"keep"
    L.mlGetContextError(None, buf, 0)
    assert buf.value == b"keep"
    assert L.mlCreateImage(None, ctypes.byref(ImageInfo(0, 1, 1, 1))) is None
    assert L.mlCreateModel(None, ctypes.byref(ModelParams(b"x", None, None))) is None


@pytest.mark.parametrize("info,msg", [
    (None, "Bad image information argument"),                        # image.cpp:24-27
    (ImageInfo(7, 4, 4, 4), "Unsupported image data type: 7"),        # dtype.h:50-51
    (ImageInfo(ML_FLOAT32, 0, 0, 0), "Unspecified image width dimension"),
    (ImageInfo(ML_FLOAT32, 4, 0, 0), "Unspecified image height dimension"),
    (ImageInfo(ML_FLOAT32, 4, 4, 0), "Unspecified image channels dimension"),
])
def test_create_image_validation(L, ctx, info, msg):
    img = L.mlCreateImage(ctx, ctypes.byref(info) if info is not None else None)
    assert img is None
    assert cerr(L, ctx) == msg


@pytest.mark.parametrize("dtype,item", [(ML_FLOAT32, 4), (ML_FLOAT16, 2)])
def test_image_map_contract(L, ctx, dtype, item):
    info = ImageInfo(dtype, 5, 3, 4)
    img = L.mlCreateImage(ctx, ctypes.byref(info))
    assert img and cerr(L, ctx) == ""
    size = ctypes.c_size_t()
    p = L.mlMapImage(img, ctypes.byref(size))
    assert size.value == 5 * 3 * 4 * item
    assert bytes((ctypes.c_char * size.value).from_address(p)) == b"\0" * size.value  # zero-filled
    assert L.mlMapImage(img, None) == p
    assert L.mlUnmapImage(img, p) == ML_OK
    assert L.mlUnmapImage(img, p + 1) == ML_FAIL  # image.cpp:67-75 pointer identity
    got = ImageInfo()
    assert L.mlGetImageInfo(img, ctypes.byref(got)) == ML_OK and got.as_tuple() == (dtype, 5, 3, 4)
    assert L.mlGetImageInfo(img, None) == ML_FAIL
    L.mlReleaseImage(img)
    assert L.mlMapImage(None, None) is None
    assert L.mlUnmapImage(None, None) == ML_FAIL
    assert L.mlGetImageInfo(None, ctypes.byref(got)) == ML_FAIL
    L.mlReleaseImage(None)  # delete nullptr is a no-op


def test_create_model_validation(L, ctx, tmp_path):
    assert L.mlCreateModel(ctx, None) is None
    assert cerr(L, ctx) == "Bad parameters argument"                 # model.cpp:75-78
    assert L.mlCreateModel(ctx, ctypes.byref(ModelParams(None, None, None))) is None
    assert cerr(L, ctx) == "Bad model_path model parameter value"    # model.cpp:80-83
    missing = str(tmp_path / "nope.srt").encode()
    assert L.mlCreateModel(ctx, ctypes.byref(ModelParams(missing, None, None))) is None
    assert cerr(L, ctx) == f"Error reading scene file: {missing.decode()}: cannot open"
    bad = tmp_path / "bad.srt"
    bad.write_bytes(b"NOTASCENE" + b"\0" * 100)
    assert L.mlCreateModel(ctx, ctypes.byref(ModelParams(str(bad).encode(), None, None))) is None
    assert cerr(L, ctx).endswith("bad magic")


def test_model_info_and_set_input_validation(L, ctx, scenes):
    m = L.mlCreateModel(ctx, ctypes.byref(ModelParams(scenes["triangle"].encode(), b"in", b"out")))
    assert m and cerr(L, ctx) == ""
    i, o = ImageInfo(), ImageInfo()
    assert L.mlGetModelInfo(m, ctypes.byref(i), ctypes.byref(o)) == ML_OK
    assert i.as_tuple() == (ML_FLOAT32, 0, 0, 2) and o.as_tuple() == (ML_FLOAT32, 0, 0, 4)
    assert L.mlGetModelInfo(m, None, None) == ML_OK
    assert L.mlSetModelInputInfo(m, None) == ML_FAIL and merr(L, m) == "Bad info parameter"
    assert L.mlSetModelInputInfo(m, ctypes.byref(ImageInfo(ML_FLOAT16, 4, 4, 2))) == ML_FAIL
    assert merr(L, m) == "Overriding data type 0 with 1"            # model.cpp:171-176
    assert L.mlSetModelInputInfo(m, ctypes.byref(ImageInfo(ML_FLOAT32, 4, 4, 3))) == ML_FAIL
    assert merr(L, m) == "Overriding channels dimension 2 with 3"    # model.cpp:178-192
    assert L.mlSetModelInputInfo(m, ctypes.byref(ImageInfo(ML_FLOAT32, 0, 4, 2))) == ML_FAIL
    assert merr(L, m) == "Input image width dimension is not specified"
    # failed calls left the model unchanged
    assert L.mlGetModelInfo(m, ctypes.byref(i), ctypes.byref(o)) == ML_OK and i.width == 0 and o.width == 0
    L.mlReleaseModel(m)


def test_infer_validation_before_render(L, ctx, scenes):
    m = L.mlCreateModel(ctx, ctypes.byref(ModelParams(scenes["triangle"].encode(), None, None)))
    img = L.mlCreateImage(ctx, ctypes.byref(ImageInfo(ML_FLOAT32, 4, 4, 4)))
    assert L.mlInfer(m, None, img) == ML_FAIL and merr(L, m) == "Bad input image handle"
    assert L.mlInfer(m, img, None) == ML_FAIL and merr(L, m) == "Bad output image handle"
    assert L.mlInfer(m, img, img) == ML_FAIL
    assert merr(L, m) == "Output image width dimension 4 does not match 0"   # model.cpp:256-270
    L.mlReleaseImage(img)
    L.mlReleaseModel(m)


def test_null_model_handle(L):
    buf = ctypes.create_string_buffer(64)
    assert L.mlGetModelError(None, buf, 64) == b"Bad model handle"
    assert L.mlGetModelInfo(None, None, None) == ML_FAIL
    assert L.mlSetModelInputInfo(None, None) == ML_FAIL
    assert L.mlInfer(None, None, None) == ML_FAIL
    L.mlReleaseModel(None)


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure path")
def test_no_gpu_fails_loudly(L, ctx, scenes):
    """No CPU fallback: without a HIP device, the render path reports the HIP error."""
    m = L.mlCreateModel(ctx, ctypes.byref(ModelParams(scenes["triangle"].encode(), None, None)))
    assert L.mlSetModelInputInfo(m, ctypes.byref(ImageInfo(ML_FLOAT32, 8, 8, 2))) == ML_FAIL
    assert merr(L, m).startswith("HIP error: no HIP device available")
    assert L.srtDeviceSceneCreate(scenes["triangle"].encode(), 0) is None
    assert "no CPU path" in _native.last_error()
    L.mlReleaseModel(m)


def test_device_stage_argument_errors(L):
    assert L.srtPrepareAsync(None, 8, 8, None) == -1 and _native.last_error() == "Bad scene handle"
    assert L.srtTraceAsync(None, None, None, 0, 1, 0, None) == -1
    assert L.srtDeviceSceneTriangles(None) == 0
    L.srtDeviceSceneRelease(None)


def test_python_mirror_raises_with_reference_messages(scenes):
    import simpleraytracer_amd as srt

    ctx = srt.Context()
    with pytest.raises(srt.MLError, match="cannot open"):
        ctx.create_model("/nonexistent/scene.srt")
    with pytest.raises(srt.MLError, match="Unspecified image height dimension"):
        ctx.create_image(ML_FLOAT32, 3, 0, 1)
    model = ctx.create_model(scenes["cornell"])
    assert model.info() == ((ML_FLOAT32, 0, 0, 2), (ML_FLOAT32, 0, 0, 4))
    with pytest.raises(srt.MLError, match="Overriding channels dimension 2 with 4"):
        model.set_input_info(8, 8, channels=4)
    model.close()
    ctx.close()
