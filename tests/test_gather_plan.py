"""The multi-device band gather of mlInfer on CPU ("fake devices").

srtGatherBandsHost runs Renderer's gather arithmetic (csrc/renderer.cpp GatherPlan: equal padded
bands, ncclGather's receive offsets, the frame as the gather buffer's first rows) on host
memory. Bands rendered separately by the oracle, gathered through it, must equal the oracle's
single-band frame bit for bit, for P in {2, 3, 8} (3 and 8 leave a padded last band, 8 an empty
one on short frames), in float and half images. The same plan drives the RCCL and device-copy
gathers on the GPU (tests/test_gpu_parity.py::test_ml_gather_modes_bitwise).
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from simpleraytracer_amd import _native


def gather_host(bands, w, h, elem):
    L = _native.lib()
    arr = (ctypes.c_void_p * len(bands))(*[b.ctypes.data for b in bands])
    out = np.full((h, w, 4), np.nan, np.float32 if elem == 4 else np.float16)
    rc = L.srtGatherBandsHost(arr, len(bands), w, h, elem, out.ctypes.data)
    assert rc == 0, _native.last_error()
    return out


@pytest.mark.parametrize("p", [1, 2, 3, 8])
@pytest.mark.parametrize("wh", [(24, 37), (16, 100), (9, 5)])
@pytest.mark.parametrize("elem", [4, 2])
def test_host_gather_equals_single_band(scenes, p, wh, elem):
    from oracle.srt_oracle import OracleScene

    from simpleraytracer_amd.bands import band_range, band_rows

    w, h = wh
    rng = np.random.default_rng(p * 100 + h)
    offs = rng.random((h, w, 2), dtype=np.float32)
    oracle = OracleScene(scenes["soup300"])
    ref = oracle.render(w, h, offs)
    b = band_rows(h, p)
    dtype = np.float32 if elem == 4 else np.float16
    bands = []
    for r in range(p):
        r0, cnt = band_range(h, p, r)
        band = np.full((b, w, 4), 7.0, dtype)  # padding rows: never part of the frame
        if cnt:
            band[:cnt] = oracle.render(w, h, offs, row_begin=r0, row_count=cnt)[r0:r0 + cnt].astype(dtype)
        bands.append(np.ascontiguousarray(band))
    got = gather_host(bands, w, h, elem)
    want = ref.astype(dtype)
    assert np.array_equal(got.view(np.uint16 if elem == 2 else np.uint32), want.view(np.uint16 if elem == 2 else np.uint32))


def test_host_gather_rejects_bad_arguments():
    L = _native.lib()
    out = np.zeros(16, np.float32)
    assert L.srtGatherBandsHost(None, 1, 2, 2, 4, out.ctypes.data) == -1
    arr = (ctypes.c_void_p * 1)(out.ctypes.data)
    assert L.srtGatherBandsHost(arr, 1, 2, 2, 3, out.ctypes.data) == -1
    assert "Bad argument" in _native.last_error()


def test_image_size_overflow_is_rejected():
    """mlCreateImage refuses dimensions whose byte size overflows size_t; the
    model refuses frames the kernels cannot index before touching any device."""
    from simpleraytracer_amd._native import ML_FAIL, ML_FLOAT32, ImageInfo, ModelParams

    L = _native.lib()
    ctx = L.mlCreateContext()
    info = ImageInfo(ML_FLOAT32, 1 << 31, 1 << 31, 1 << 20)
    assert not L.mlCreateImage(ctx, ctypes.byref(info))
    buf = ctypes.create_string_buffer(256)
    assert "overflows" in L.mlGetContextError(ctx, buf, 256).decode()
    L.mlReleaseContext(ctx)


def test_frame_side_limit(scenes):
    from simpleraytracer_amd._native import ML_FAIL, ML_FLOAT32, ImageInfo, ModelParams

    L = _native.lib()
    ctx = L.mlCreateContext()
    params = ModelParams(scenes["triangle"].encode(), None, None)
    model = L.mlCreateModel(ctx, ctypes.byref(params))
    assert model
    info = ImageInfo(ML_FLOAT32, (1 << 30) + 1, 16, 2)
    assert L.mlSetModelInputInfo(model, ctypes.byref(info)) == ML_FAIL
    buf = ctypes.create_string_buffer(256)
    assert "exceeds the supported maximum" in L.mlGetModelError(model, buf, 256).decode()
    L.mlReleaseModel(model)
    L.mlReleaseContext(ctx)
