"""ctypes binding of libModelRunner.so (include/model_runner.h + include/srt_render.h).

The shared library is built in-tree by ``make`` (or ``__graft_entry__.build()``) into
``simpleraytracer_amd/lib/libModelRunner.so``. There is no fallback: importing the renderer
without the library raises immediately.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

PACKAGE_DIR = Path(__file__).resolve().parent
LIB_PATH = PACKAGE_DIR / "lib" / "libModelRunner.so"
# Diagnostic runs only (tools/diag_cull.py): SRT_LIB points at the `make diag` build.
if os.environ.get("SRT_LIB"):
    LIB_PATH = Path(os.environ["SRT_LIB"])

ML_OK = 0
ML_FAIL = 1
ML_FLOAT32 = 0
ML_FLOAT16 = 1

SRT_SCENE_TRIANGLE = 0
SRT_SCENE_CORNELL = 1
SRT_SCENE_SOUP = 2
SRT_TRACE_LDS = 0
SRT_TRACE_SCALAR = 1
SRT_TRACE_CULL = 2
SRT_TRACE_BVH = 3
SRT_MAX_BATCH = 8  # include/srt_render.h: frames per srtTraceBatchAsync call
SRT_ROWS_INTERLEAVED = 0
SRT_ROWS_CONTIGUOUS = 1
SRT_ROWS_ROTATED = 2  # contiguous bands rotated per compositor (all-to-all)
SRT_EXCHANGE_ALLTOALL = 0
SRT_EXCHANGE_ROTATING = 1
SRT_EXCHANGE_ROOT = 2
SRT_EXCHANGE_SHARE = 3
SRT_SPLIT_BANDS = 0
SRT_SPLIT_FRAMES = 1
SRT_ENGINE_RCCL_SELF = 1  # srt_engine_options.flags
SRT_TILE_ROWS = 16  # include/srt_render.h: rows per tile row (interleaved bands deal these)


class ImageInfo(ctypes.Structure):
    """``ml_image_info`` (model_runner.h:100-106): 32 bytes, dtype at 0, width at 8."""

    _fields_ = [
        ("dtype", ctypes.c_int),
        ("width", ctypes.c_size_t),
        ("height", ctypes.c_size_t),
        ("channels", ctypes.c_size_t),
    ]

    def as_tuple(self):
        return (self.dtype, self.width, self.height, self.channels)


class ModelParams(ctypes.Structure):
    """``ml_model_params`` (model_runner.h:53-60): 24 bytes."""

    _fields_ = [
        ("model_path", ctypes.c_char_p),
        ("input_node", ctypes.c_char_p),
        ("output_node", ctypes.c_char_p),
    ]


class EngineOptions(ctypes.Structure):
    """``srt_engine_options`` (include/srt_render.h)."""

    _fields_ = [
        ("struct_size", ctypes.c_size_t),
        ("variant", ctypes.c_int),
        ("queues", ctypes.c_size_t),
        ("batch", ctypes.c_size_t),
        ("rows", ctypes.c_int),
        ("exchange", ctypes.c_int),
        ("split", ctypes.c_int),
        ("simulate", ctypes.c_int),
        ("launch", ctypes.c_size_t),
        ("flags", ctypes.c_int),
        ("share", ctypes.c_size_t),
        ("own_rows", ctypes.c_size_t),
    ]


_SZ = ctypes.c_size_t
_PSZ = ctypes.POINTER(ctypes.c_size_t)
_PD = ctypes.POINTER(ctypes.c_double)

# name -> (restype, argtypes)
_SIGNATURES = {
    "mlCreateContext": (ctypes.c_void_p, []),
    "mlGetContextError": (ctypes.c_char_p, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]),
    "mlReleaseContext": (None, [ctypes.c_void_p]),
    "mlCreateImage": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.POINTER(ImageInfo)]),
    "mlGetImageInfo": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ImageInfo)]),
    "mlMapImage": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]),
    "mlUnmapImage": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "mlReleaseImage": (None, [ctypes.c_void_p]),
    "mlCreateModel": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.POINTER(ModelParams)]),
    "mlGetModelError": (ctypes.c_char_p, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]),
    "mlGetModelInfo": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ImageInfo), ctypes.POINTER(ImageInfo)]),
    "mlSetModelInputInfo": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ImageInfo)]),
    "mlInfer": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "mlReleaseModel": (None, [ctypes.c_void_p]),
    "srtGetLastError": (ctypes.c_char_p, []),
    "srtWriteScene": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_ulonglong, ctypes.c_ulonglong,
                                     ctypes.c_float]),
    "srtSceneTriangles": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_ulonglong)]),
    "srtReadScene": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_ulonglong, ctypes.POINTER(ctypes.c_ulonglong),
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.POINTER(ctypes.c_uint)]),
    "srtConvertScene": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]),
    "srtSceneFrame": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t,
                                     ctypes.POINTER(ctypes.c_float)]),
    "srtDeviceSceneCreate": (ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_int]),
    "srtDeviceSceneRelease": (None, [ctypes.c_void_p]),
    "srtDeviceSceneTriangles": (ctypes.c_ulonglong, [ctypes.c_void_p]),
    "srtDeviceSceneOrder": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulonglong,
                                           ctypes.POINTER(ctypes.c_double)]),
    "srtPrepareAsync": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]),
    "srtTraceAsync": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]),
    "srtTraceIdsAsync": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]),
    "srtTraceBatchAsync": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                          ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_size_t,
                                          ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]),
    "srtShadeAsync": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]),
    "srtShadeBandsAsync": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]),
    "srtSetStageTiming": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "srtTakeStageTimes": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "srtEngineUniqueId": (ctypes.c_int, [ctypes.c_void_p]),
    "srtEngineCreate": (ctypes.c_void_p, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), _SZ, _SZ, _SZ,
                                          ctypes.POINTER(EngineOptions)]),
    "srtEngineCreateRank": (ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                              _SZ, _SZ, ctypes.POINTER(EngineOptions)]),
    "srtEngineRelease": (None, [ctypes.c_void_p]),
    "srtEngineSetInputs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, _SZ]),
    "srtEngineRun": (ctypes.c_int, [ctypes.c_void_p, _SZ]),
    "srtEngineVerify": (ctypes.c_int, [ctypes.c_void_p, _PSZ, _PSZ]),
    "srtEngineReadFrame": (ctypes.c_int, [ctypes.c_void_p, _SZ, ctypes.c_void_p]),
    "srtEngineStageTimes": (ctypes.c_int, [ctypes.c_void_p, _SZ, _SZ, ctypes.POINTER(ctypes.c_uint), _PD, _PD, _PD]),
    "srtEngineStageTimesBatch": (ctypes.c_int, [ctypes.c_void_p, _SZ, _SZ, _SZ, ctypes.POINTER(ctypes.c_uint), _PD, _PD,
                                                _PD]),
    "srtEnginePoolSelfTest": (ctypes.c_int, [_SZ, _SZ, ctypes.c_int, ctypes.c_double, _PD, ctypes.POINTER(ctypes.c_int),
                                             ctypes.c_char_p, _SZ]),
    "srtShareAuto": (_SZ, [_SZ, _SZ]),
    "srtRotateOwnRows": (_SZ, [_SZ]),
    "srtRotateSplitForLink": (_SZ, [_SZ, _SZ, ctypes.c_double, ctypes.c_double, ctypes.c_double]),
    "srtEngineSplit": (ctypes.c_int, [ctypes.c_void_p, _PSZ, _PSZ, _PD, _PD, ctypes.POINTER(ctypes.c_int)]),
    "srtEngineInfo": (ctypes.c_int, [ctypes.c_void_p, _PSZ, _PSZ, _PSZ, _PSZ, ctypes.POINTER(ctypes.c_int), _PD]),
    "srtExchangeHost": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), _SZ, _SZ, _SZ, ctypes.c_int, ctypes.c_int, _SZ,
                                       _SZ, ctypes.POINTER(ctypes.c_void_p), _PSZ, _PSZ]),
    "srtEngineExchangeStats": (ctypes.c_int, [ctypes.c_void_p, _SZ, _PSZ, _PD, _PD]),
    "srtExchangeHostShare": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), _SZ, _SZ, _SZ, _SZ, _SZ, _SZ,
                                            ctypes.POINTER(ctypes.c_void_p), _PSZ, _PSZ]),
    "srtScreenBoxHost": (ctypes.c_int, [ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.POINTER(ctypes.c_float)]),
}

_lib = None


def _share_torch_hip_runtime():
    """Load torch's HIP runtime first when torch is installed.

    torch ships its own libamdhip64.so / libhsa-runtime64.so / librccl.so with the same
    SONAMEs (libamdhip64.so.7, ...) as /opt/rocm. If torch is imported first, the dynamic
    loader satisfies this library's NEEDED entries with torch's copies, so the process has ONE
    HIP runtime and torch streams/pointers passed to srt* calls belong to it. Loading this
    library first would pull /opt/rocm's copies, and torch would then load a second runtime.
    """
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib() -> ctypes.CDLL:
    """Load libModelRunner.so once; raise loudly if it has not been built."""
    global _lib
    if _lib is None:
        _share_torch_hip_runtime()
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"{LIB_PATH} is missing: build the HIP library first (`make` at the repo root or "
                "`python -c 'import __graft_entry__ as g; g.build()'`); there is no CPU fallback")
        handle = ctypes.CDLL(os.fspath(LIB_PATH))
        for name, (restype, argtypes) in _SIGNATURES.items():
            if os.environ.get("SRT_LIB") and not hasattr(handle, name):
                continue  # an older build under measurement (A/B): bind what it has
            fn = getattr(handle, name)
            fn.restype = restype
            fn.argtypes = argtypes
        _lib = handle
    return _lib


def exported_names():
    return list(_SIGNATURES)


def last_error() -> str:
    msg = lib().srtGetLastError()
    return msg.decode() if msg else ""
