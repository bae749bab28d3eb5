"""ctypes binding of the CPU oracle (oracle/build/libsrt_oracle.so). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / the timed CPU baseline. Parity status: see srt_oracle.h.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "build" / "libsrt_oracle.so"
if os.environ.get("SRT_ORACLE_LIB"):  # the sanitizer build (make asan; tools/asan_tests.sh)
    LIB_PATH = Path(os.environ["SRT_ORACLE_LIB"])


class Scene(ctypes.Structure):
    _fields_ = [
        ("camera", ctypes.c_float * 10),
        ("background", ctypes.c_float * 3),
        ("n", ctypes.c_size_t),
        ("vertices", ctypes.POINTER(ctypes.c_float)),
        ("albedo", ctypes.POINTER(ctypes.c_float)),
    ]


_lib = None
_F = ctypes.POINTER(ctypes.c_float)


def build():
    subprocess.run(["make", "-s", "-C", os.fspath(ORACLE_DIR)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        h = ctypes.CDLL(os.fspath(LIB_PATH))
        h.srto_scene_load.argtypes = [ctypes.c_char_p, ctypes.POINTER(Scene)]
        h.srto_scene_load.restype = ctypes.c_int
        h.srto_scene_free.argtypes = [ctypes.POINTER(Scene)]
        h.srto_scene_free.restype = None
        h.srto_frame.argtypes = [_F, ctypes.c_size_t, ctypes.c_size_t, _F]
        h.srto_frame.restype = None
        h.srto_prepare.argtypes = [_F, ctypes.c_size_t, _F, _F]
        h.srto_prepare.restype = None
        h.srto_closest_hit.argtypes = [_F, ctypes.c_size_t, ctypes.c_float, ctypes.c_float, _F, _F]
        h.srto_closest_hit.restype = ctypes.c_long
        h.srto_pixel_position.argtypes = [ctypes.c_size_t, ctypes.c_size_t, ctypes.c_float, ctypes.c_float,
                                          ctypes.c_size_t, ctypes.c_size_t, _F, _F]
        h.srto_pixel_position.restype = None
        h.srto_render.argtypes = [ctypes.POINTER(Scene), _F, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                  ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, _F]
        h.srto_render.restype = ctypes.c_size_t
        h.srto_shade.argtypes = [ctypes.POINTER(Scene), _F, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                 ctypes.c_size_t, ctypes.c_size_t, _F]
        h.srto_shade.restype = None
        h.srto_threads.argtypes = [ctypes.c_int]
        h.srto_threads.restype = ctypes.c_int
        _lib = h
    return _lib


def _fp(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(_F)


class OracleScene:
    def __init__(self, path: str):
        self._s = Scene()
        rc = lib().srto_scene_load(os.fsencode(path), ctypes.byref(self._s))
        if rc != 0:
            raise RuntimeError(f"oracle could not read scene {path} (code {rc})")
        n = self._s.n
        self.n = n
        self.camera = np.array(self._s.camera[:], np.float32)
        self.background = np.array(self._s.background[:], np.float32)
        self.vertices = np.ctypeslib.as_array(self._s.vertices, shape=(n * 9,)).reshape(n, 9).copy()
        self.albedo = np.ctypeslib.as_array(self._s.albedo, shape=(n * 3,)).reshape(n, 3).copy()

    def frame(self, width: int, height: int) -> np.ndarray:
        out = np.zeros(12, np.float32)
        lib().srto_frame(_fp(self.camera), width, height, _fp(out))
        return out

    def edges(self, width: int, height: int) -> np.ndarray:
        out = np.zeros((self.n, 12), np.float32)
        v = np.ascontiguousarray(self.vertices)
        lib().srto_prepare(_fp(v), self.n, _fp(self.frame(width, height)), _fp(out))
        return out

    def render(self, width: int, height: int, offsets: np.ndarray | None = None, row_begin: int = 0,
               row_count: int | None = None, row_step: int = 1, threads: int = 0) -> np.ndarray:
        """Full-frame H x W x 4 buffer; rows outside the rendered set are NaN."""
        if offsets is None:
            offsets = np.full((height, width, 2), 0.5, np.float32)
        offsets = np.ascontiguousarray(offsets, np.float32)
        assert offsets.shape == (height, width, 2)
        if row_count is None:
            row_count = height - row_begin
        out = np.full((height, width, 4), np.nan, np.float32)
        lib().srto_render(ctypes.byref(self._s), _fp(offsets), width, height, row_begin, row_count, row_step,
                          threads, _fp(out))
        return out

    def shade(self, width: int, height: int, ids: np.ndarray, offsets: np.ndarray | None = None) -> np.ndarray:
        """Deferred shading of a whole frame from hit ids (H x W int32, -1 = miss)."""
        if offsets is None:
            offsets = np.full((height, width, 2), 0.5, np.float32)
        offsets = np.ascontiguousarray(offsets, np.float32)
        ids = np.ascontiguousarray(ids, np.int32)
        assert offsets.shape == (height, width, 2) and ids.shape == (height, width)
        out = np.full((height, width, 4), np.nan, np.float32)
        lib().srto_shade(ctypes.byref(self._s), _fp(offsets), ids.ctypes.data_as(ctypes.c_void_p), width, height, 0,
                         height, _fp(out))
        return out

    def close(self):
        if self._s.vertices:
            lib().srto_scene_free(ctypes.byref(self._s))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def closest_hit(edges: np.ndarray, fx: float, fy: float):
    """(id, t, det) of the oracle's closest-hit scan at image position (fx, fy)."""
    e = np.ascontiguousarray(edges, np.float32)
    t = ctypes.c_float(np.nan)
    d = ctypes.c_float(np.nan)
    i = lib().srto_closest_hit(_fp(e), e.shape[0], fx, fy, ctypes.byref(t), ctypes.byref(d))
    return i, t.value, d.value


def pixel_position(x: int, y: int, sx: float, sy: float, width: int, height: int):
    fx, fy = ctypes.c_float(), ctypes.c_float()
    lib().srto_pixel_position(x, y, sx, sy, width, height, ctypes.byref(fx), ctypes.byref(fy))
    return fx.value, fy.value


def threads(n: int = 0) -> int:
    return lib().srto_threads(n)
