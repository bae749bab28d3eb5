"""Scene files and the device-level render stages (include/srt_render.h).

``DeviceScene`` keeps a scene resident on one GPU and launches the two stages on a caller's
HIP stream with caller-owned device buffers (torch tensors or raw pointers):

    scene = DeviceScene(path, device=0)
    scene.prepare(W, H, stream)                                  # edge records
    scene.trace(offsets, rgba, row_begin, row_count, stream=s)   # closest hit + shade

This is the path bench.py times (inputs resident in HBM) and the one-process-per-GPU
band renderer uses; ``runner.render`` is the host-image ml* path.
"""
from __future__ import annotations

import ctypes
import os

from . import _native
from ._native import (SRT_MAX_BATCH, SRT_SCENE_CORNELL, SRT_SCENE_SOUP, SRT_SCENE_TRIANGLE, SRT_TRACE_BVH,
                      SRT_TRACE_CULL, SRT_TRACE_LDS, SRT_TRACE_SCALAR)

SCENE_KINDS = {"triangle": SRT_SCENE_TRIANGLE, "cornell": SRT_SCENE_CORNELL, "soup": SRT_SCENE_SOUP}
TRACE_VARIANTS = {"lds": SRT_TRACE_LDS, "scalar": SRT_TRACE_SCALAR, "cull": SRT_TRACE_CULL, "bvh": SRT_TRACE_BVH}
MAX_BATCH = SRT_MAX_BATCH
SOUP_SEED = 0x5EED  # 100k soup seed; the 1M soup uses SOUP_SEED + 1


class SrtError(RuntimeError):
    pass


def _check(rc: int):
    if rc != 0:
        raise SrtError(_native.last_error())


def write_scene(path: str, kind: str = "soup", triangles: int = 100_000, seed: int | None = None,
                size: float = 0.0) -> str:
    """Write a generated scene file; returns ``path``."""
    if seed is None:
        seed = SOUP_SEED + (1 if triangles >= 1_000_000 else 0)
    _check(_native.lib().srtWriteScene(os.fsencode(path), SCENE_KINDS[kind], triangles, seed, size))
    return path


def scene_triangles(path: str) -> int:
    n = ctypes.c_ulonglong()
    _check(_native.lib().srtSceneTriangles(os.fsencode(path), ctypes.byref(n)))
    return n.value


def read_scene(path: str):
    """Load a scene file (binary or .obj) through the library: dict of numpy arrays."""
    import numpy as np

    n = ctypes.c_ulonglong()
    _check(_native.lib().srtReadScene(os.fsencode(path), 0, ctypes.byref(n), None, None, None, None, None))
    v = np.empty((n.value, 9), np.float32)
    a = np.empty((n.value, 3), np.float32)
    cam = np.empty(10, np.float32)
    bg = np.empty(3, np.float32)
    flags = ctypes.c_uint()
    _check(_native.lib().srtReadScene(os.fsencode(path), n.value, ctypes.byref(n), v.ctypes.data, a.ctypes.data,
                                      cam.ctypes.data, bg.ctypes.data, ctypes.byref(flags)))
    return {"vertices": v, "albedo": a, "camera": cam, "background": bg, "flags": flags.value}


def convert_scene(src: str, dst: str, input_dtype: int = -1, output_dtype: int = -1) -> str:
    """Write src (binary or .obj) as a binary scene file with the given image data types."""
    _check(_native.lib().srtConvertScene(os.fsencode(src), os.fsencode(dst), input_dtype, output_dtype))
    return dst


def scene_frame(path: str, width: int, height: int):
    """(origin, base, du, dv) float32 triples of the affine primary-ray frame."""
    out = (ctypes.c_float * 12)()
    _check(_native.lib().srtSceneFrame(os.fsencode(path), width, height, out))
    vals = list(out)
    return tuple(tuple(vals[3 * k:3 * k + 3]) for k in range(4))


def _ptr(x) -> int:
    if x is None:
        return 0
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    return int(x)


def _stream(s) -> int:
    if s is None:
        return 0
    if hasattr(s, "cuda_stream"):
        return s.cuda_stream
    return int(s)


class DeviceScene:
    """A scene resident on one HIP device."""

    def __init__(self, path: str, device: int = 0):
        self._lib = _native.lib()
        self.handle = self._lib.srtDeviceSceneCreate(os.fsencode(path), device)
        if not self.handle:
            raise SrtError(_native.last_error())
        self.device = device
        self.path = path
        self.triangles = self._lib.srtDeviceSceneTriangles(self.handle)
        self.width = 0
        self.height = 0

    def prepare(self, width: int, height: int, stream=None):
        _check(self._lib.srtPrepareAsync(self.handle, width, height, _stream(stream)))
        self.width, self.height = width, height

    def _check_buffer(self, name, buf, rows, channels, dtype):
        """Shape / contiguity, and for torch tensors dtype and device: the kernels read and write
        raw pointers on self.device with these element types."""
        want = (rows, self.width) + ((channels,) if channels else ())
        if hasattr(buf, "shape") and tuple(buf.shape) != want:
            raise ValueError(f"{name} must be {want}, got {tuple(buf.shape)}")
        self._check_tensor(name, buf, dtype)

    def _check_tensor(self, name, buf, dtype):
        if hasattr(buf, "is_contiguous") and not buf.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
        if hasattr(buf, "is_cuda"):
            import torch

            want_dtype = {"f32": torch.float32, "i32": torch.int32}[dtype]
            if buf.dtype != want_dtype:
                raise ValueError(f"{name} must be {want_dtype}, got {buf.dtype}")
            if not buf.is_cuda or buf.device.index != self.device:
                raise ValueError(f"{name} must live on cuda:{self.device}, got {buf.device}")

    def trace(self, offsets, rgba, row_begin: int = 0, row_count: int | None = None, variant: str = "cull",
              stream=None):
        """offsets: (rows, W, 2) float32 device buffer; rgba: (rows, W, 4) float32 device buffer."""
        if row_count is None:
            row_count = self.height - row_begin
        self._check_buffer("offsets", offsets, row_count, 2, "f32")
        self._check_buffer("rgba", rgba, row_count, 4, "f32")
        _check(self._lib.srtTraceAsync(self.handle, _ptr(offsets), _ptr(rgba), row_begin, row_count,
                                       TRACE_VARIANTS[variant], _stream(stream)))

    def trace_ids(self, offsets, ids, row_begin: int = 0, row_count: int | None = None, variant: str = "cull",
                  stream=None):
        """Hit ids only (deferred shading): offsets (rows, W, 2) float32, ids (rows, W) int32."""
        if row_count is None:
            row_count = self.height - row_begin
        self._check_buffer("offsets", offsets, row_count, 2, "f32")
        self._check_buffer("ids", ids, row_count, 0, "i32")
        _check(self._lib.srtTraceIdsAsync(self.handle, _ptr(offsets), _ptr(ids), row_begin, row_count,
                                          TRACE_VARIANTS[variant], _stream(stream)))

    def bind_trace_ids(self, offsets, ids, row_begin: int = 0, row_count: int | None = None, variant: str = "cull",
                       stream=None):
        """prepare + trace_ids of this band as a zero-argument callable: the buffers are checked
        once here, each call is then just the two C-ABI calls (a frame loop's host cost is the
        HIP launches, not Python checks). The buffers must stay alive while it is used."""
        if row_count is None:
            row_count = self.height - row_begin
        self._check_buffer("offsets", offsets, row_count, 2, "f32")
        self._check_buffer("ids", ids, row_count, 0, "i32")
        lib, h, w, hh = self._lib, self.handle, self.width, self.height
        op, ip, s, v = _ptr(offsets), _ptr(ids), _stream(stream), TRACE_VARIANTS[variant]

        def run():
            _check(lib.srtPrepareAsync(h, w, hh, s))
            _check(lib.srtTraceIdsAsync(h, op, ip, row_begin, row_count, v, s))

        return run

    def bind_trace_batch(self, offsets, outs, row_begin: int = 0, row_count: int | None = None, variant: str = "cull",
                         stream=None, ids: bool = False, row_interleave: int = 1):
        """prepare + trace of len(outs) (<= MAX_BATCH) frames of this band as a zero-argument
        callable (srtTraceBatchAsync): frame f's sample offsets offsets[f] ((rows, W, 2) float32)
        and its output outs[f] ((rows, W) int32 hit ids with ids=True, else (rows, W, 4) float32
        RGBA). Every frame gets the whole per-frame work; the cull variant launches each stage
        once for the batch. row_interleave P > 1: the band is tile rows row_begin / 16 + k P of
        the frame (bands.interleaved_range). Checked once here; the buffers must stay alive
        while it is used."""
        if row_count is None:
            row_count = self.height - row_begin
        frames = len(outs)
        if frames > MAX_BATCH or len(offsets) != frames:
            raise ValueError(f"1 to {MAX_BATCH} frames, one offsets buffer per output")
        for f in range(frames):
            self._check_buffer(f"offsets[{f}]", offsets[f], row_count, 2, "f32")
            self._check_buffer(f"outs[{f}]", outs[f], row_count, 0 if ids else 4, "i32" if ids else "f32")
        arr = ctypes.c_void_p * max(1, frames)
        offs = arr(*[_ptr(o) for o in offsets])
        out = arr(*[_ptr(o) for o in outs])
        rgba, idp = (None, out) if ids else (out, None)
        lib, h, w, hh = self._lib, self.handle, self.width, self.height
        s, v = _stream(stream), TRACE_VARIANTS[variant]

        def run():
            _check(lib.srtPrepareAsync(h, w, hh, s))
            _check(lib.srtTraceBatchAsync(h, offs, rgba, idp, frames, row_begin, row_count, row_interleave, v, s))

        run.keep = (offsets, outs, offs, out)  # the pointer arrays live as long as the callable
        return run

    def trace_batch(self, offsets, outs, row_begin: int = 0, row_count: int | None = None, variant: str = "cull",
                    stream=None, ids: bool = False, row_interleave: int = 1):
        """One batched call (bind_trace_batch) run once."""
        self.bind_trace_batch(offsets, outs, row_begin, row_count, variant, stream, ids, row_interleave)()

    def shade(self, offsets, ids, rgba, row_begin: int = 0, row_count: int | None = None, stream=None):
        """Deferred shading of the prepared frame's rows from hit ids: the RGBA trace() stores."""
        if row_count is None:
            row_count = self.height - row_begin
        self._check_buffer("offsets", offsets, row_count, 2, "f32")
        self._check_buffer("ids", ids, row_count, 0, "i32")
        self._check_buffer("rgba", rgba, row_count, 4, "f32")
        _check(self._lib.srtShadeAsync(self.handle, _ptr(offsets), _ptr(ids), _ptr(rgba), row_begin, row_count,
                                       _stream(stream)))

    def shade_bands(self, offsets, ids, rgba, band_rows: int, stream=None, interleaved: int = 0):
        """Deferred shading of a batch of frames whose ids were gathered band-major:
        ids (bands, frames, band_rows, W) int32 (bands = ceil(H / band_rows) contiguous bands, or
        `interleaved` bands dealt the frame's tile rows round-robin), offsets (H, W, 2),
        rgba (frames, H, W, 4); one launch (srtShadeBandsAsync)."""
        if band_rows <= 0:
            raise ValueError("band_rows must be positive")
        bands = interleaved if interleaved else (self.height + band_rows - 1) // band_rows
        frames = ids.shape[1] if hasattr(ids, "shape") and len(ids.shape) == 4 else 0
        self._check_buffer("offsets", offsets, self.height, 2, "f32")
        # contiguous bands: a gather over P ranks may carry more (empty, trailing) bands than the
        # ceil(H / band_rows) that hold rows; the kernel never reads them
        if hasattr(ids, "shape") and (len(ids.shape) != 4 or tuple(ids.shape[2:]) != (band_rows, self.width) or
                                      (ids.shape[0] != bands if interleaved else ids.shape[0] < bands)):
            raise ValueError(f"ids must be {(bands, 'frames', band_rows, self.width)}, got {tuple(ids.shape)}")
        if hasattr(rgba, "shape") and tuple(rgba.shape) != (frames, self.height, self.width, 4):
            raise ValueError(f"rgba must be {(frames, self.height, self.width, 4)}, got {tuple(rgba.shape)}")
        for name, buf, dtype in (("ids", ids, "i32"), ("rgba", rgba, "f32")):
            self._check_tensor(name, buf, dtype)
        _check(self._lib.srtShadeBandsAsync(self.handle, _ptr(offsets), _ptr(ids), _ptr(rgba), frames, band_rows,
                                            interleaved, _stream(stream)))

    def spatial_order(self):
        """(order, build_ms): the record ids in spatial order (numpy uint32), built on the device
        at load, and the build's device time."""
        import numpy as np

        out = np.empty(max(1, self.triangles), np.uint32)
        ms = ctypes.c_double()
        _check(self._lib.srtDeviceSceneOrder(self.handle, out.ctypes.data, out.size, ctypes.byref(ms)))
        return out[:self.triangles], ms.value

    def set_stage_timing(self, enable: bool = True):
        """Bind HIP events to the prepare, bin and trace kernels' dispatches (no extra packets)."""
        _check(self._lib.srtSetStageTiming(self.handle, 1 if enable else 0))

    def take_stage_times(self):
        """(timed trace calls, mean prepare ms, mean bin-stage ms, mean trace-kernel ms) since the
        last take; waits for the events."""
        n, p, b, t = ctypes.c_uint(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        _check(self._lib.srtTakeStageTimes(self.handle, ctypes.byref(n), ctypes.byref(p), ctypes.byref(b),
                                           ctypes.byref(t)))
        return n.value, p.value, b.value, t.value

    def close(self):
        if self.handle:
            self._lib.srtDeviceSceneRelease(self.handle)
            self.handle = None

    def __del__(self):
        self.close()
