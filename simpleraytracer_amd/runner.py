"""Python mirror of the ml* C API (reference: /root/reference/model_runner/model_runner.h).

Same objects, call order and error behaviour as the C API, with Python ownership:

    ctx = Context()
    model = ctx.create_model("scene.srt")            # mlCreateModel
    inp, out = model.info()                          # mlGetModelInfo
    model.set_input_info(width=W, height=H)          # mlSetModelInputInfo
    inp_img = ctx.create_image(*model.info()[0])     # mlCreateImage
    ...
    model.infer(inp_img, out_img)                    # mlInfer (renders)

Failures raise MLError carrying the message from mlGetContextError / mlGetModelError.
``render()`` wraps the whole sequence for numpy callers.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _native
from ._native import ML_FLOAT32, ML_OK, ImageInfo, ModelParams


class MLError(RuntimeError):
    """An ml* call returned ML_FAIL / ML_INVALID_HANDLE."""


def _err_text(getter, handle) -> str:
    buf = ctypes.create_string_buffer(1024)
    out = getter(handle, buf, len(buf))
    return (out or b"").decode(errors="replace")


class Image:
    """ml_image: host HWC buffer. ``array()`` is a numpy view of the mapped memory."""

    def __init__(self, ctx: "Context", dtype: int, width: int, height: int, channels: int):
        self._lib = _native.lib()
        info = ImageInfo(dtype, width, height, channels)
        self._ctx = ctx  # keep the context's error cache reachable while the image lives
        self.handle = self._lib.mlCreateImage(ctx.handle, ctypes.byref(info))
        if not self.handle:
            raise MLError(ctx.error())

    def info(self):
        info = ImageInfo()
        if self._lib.mlGetImageInfo(self.handle, ctypes.byref(info)) != ML_OK:
            raise MLError("mlGetImageInfo failed")
        return info.as_tuple()

    def array(self) -> np.ndarray:
        dtype, w, h, c = self.info()
        size = ctypes.c_size_t()
        ptr = self._lib.mlMapImage(self.handle, ctypes.byref(size))
        np_dtype = np.float32 if dtype == ML_FLOAT32 else np.float16
        buf = (ctypes.c_char * size.value).from_address(ptr)
        arr = np.frombuffer(buf, dtype=np_dtype).reshape(h, w, c)
        self._lib.mlUnmapImage(self.handle, ptr)
        return arr

    def close(self):
        if self.handle:
            self._lib.mlReleaseImage(self.handle)
            self.handle = None

    def __del__(self):
        self.close()


class Model:
    """ml_model: a triangle scene; ``infer`` renders one frame."""

    def __init__(self, ctx: "Context", path: str):
        self._lib = _native.lib()
        self._path = os.fsencode(path)
        params = ModelParams(self._path, None, None)
        self.handle = self._lib.mlCreateModel(ctx.handle, ctypes.byref(params))
        if not self.handle:
            raise MLError(ctx.error())

    def error(self) -> str:
        return _err_text(self._lib.mlGetModelError, self.handle)

    def info(self):
        i, o = ImageInfo(), ImageInfo()
        if self._lib.mlGetModelInfo(self.handle, ctypes.byref(i), ctypes.byref(o)) != ML_OK:
            raise MLError(self.error())
        return i.as_tuple(), o.as_tuple()

    def set_input_info(self, width: int, height: int, channels: int = 2, dtype: int = ML_FLOAT32):
        info = ImageInfo(dtype, width, height, channels)
        if self._lib.mlSetModelInputInfo(self.handle, ctypes.byref(info)) != ML_OK:
            raise MLError(self.error())

    def infer(self, inp: Image, out: Image):
        if self._lib.mlInfer(self.handle, inp.handle, out.handle) != ML_OK:
            raise MLError(self.error())

    def close(self):
        if self.handle:
            self._lib.mlReleaseModel(self.handle)
            self.handle = None

    def __del__(self):
        self.close()


class Context:
    """ml_context."""

    def __init__(self):
        self._lib = _native.lib()
        self.handle = self._lib.mlCreateContext()
        if not self.handle:
            raise MLError("Error creating context")

    def error(self) -> str:
        return _err_text(self._lib.mlGetContextError, self.handle)

    def create_model(self, path: str) -> Model:
        return Model(self, path)

    def create_image(self, dtype: int, width: int, height: int, channels: int) -> Image:
        return Image(self, dtype, width, height, channels)

    def close(self):
        if self.handle:
            self._lib.mlReleaseContext(self.handle)
            self.handle = None

    def __del__(self):
        self.close()


def default_offsets(width: int, height: int) -> np.ndarray:
    """Pixel-centre sample offsets (0.5, 0.5): H x W x 2 float32."""
    return np.full((height, width, 2), 0.5, dtype=np.float32)


def render(scene_path: str, width: int, height: int, offsets: np.ndarray | None = None) -> np.ndarray:
    """Render one frame through the ml* API; returns an H x W x 4 copy (float32, or float16
    for a scene whose output data type is ML_FLOAT16; FLOAT16 input scenes take the offsets
    rounded to float16)."""
    ctx = Context()
    model = ctx.create_model(scene_path)
    try:
        (idt0, _, _, _), _ = model.info()
        model.set_input_info(width, height, dtype=idt0)
        (idt, iw, ih, ic), (odt, ow, oh, oc) = model.info()
        inp = ctx.create_image(idt, iw, ih, ic)
        out = ctx.create_image(odt, ow, oh, oc)
        try:
            src = default_offsets(width, height) if offsets is None else np.asarray(offsets, np.float32)
            if src.shape != (height, width, 2):
                raise ValueError(f"offsets must be {(height, width, 2)}, got {src.shape}")
            inp.array()[...] = src
            model.infer(inp, out)
            return out.array().copy()
        finally:
            inp.close()
            out.close()
    finally:
        model.close()
        ctx.close()
