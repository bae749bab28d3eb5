"""The frame engine (include/srt_render.h srtEngine*, csrc/engine.h): a stream of frames over one
or more GPUs, native from the batch loop down. Python only hands over the inputs and asks for
``run(batches)``; the per-frame work (record setup, bins, trace, the band exchange over RCCL,
deferred shading) is issued by the library's C++ worker threads, one per device.

    eng = FrameEngine(scene_path, 1920, 1080, devices=[0, 1, 2, 3])   # one process, 4 GPUs
    eng = FrameEngine.rank(scene_path, 1920, 1080, device, rank, world, uid)  # one rank per GPU
    eng.set_inputs(offsets)          # (count, H, W, 2) float32 sample offsets, kept on the devices
    eng.run(batches)                 # batches x batch frames, synchronous

A repeated device (``devices=[0, 0]``) rehearses the multi-device path on one GPU: the bands are
exchanged by device copies instead of RCCL, everything else is the same code.
"""
from __future__ import annotations

import ctypes
import os

from . import _native
from ._native import (SRT_ENGINE_RCCL_SELF, SRT_EXCHANGE_ALLTOALL, SRT_EXCHANGE_ROOT, SRT_EXCHANGE_ROTATING,
                      SRT_EXCHANGE_SHARE, SRT_ROWS_CONTIGUOUS, SRT_ROWS_INTERLEAVED, SRT_ROWS_ROTATED, SRT_SPLIT_BANDS, SRT_SPLIT_FRAMES, EngineOptions)
from .device import TRACE_VARIANTS, SrtError

EXCHANGES = {"alltoall": SRT_EXCHANGE_ALLTOALL, "rotating": SRT_EXCHANGE_ROTATING, "root": SRT_EXCHANGE_ROOT,
             "share": SRT_EXCHANGE_SHARE}
ROWS = {"interleaved": SRT_ROWS_INTERLEAVED, "contiguous": SRT_ROWS_CONTIGUOUS, "rotated": SRT_ROWS_ROTATED}
SPLITS = {"bands": SRT_SPLIT_BANDS, "frames": SRT_SPLIT_FRAMES}


def _check(rc: int):
    if rc != 0:
        raise SrtError(_native.last_error())


def _options(variant, queues, batch, rows, exchange, split, simulate=False, launch=0, rccl_self=False, share=0,
             own_rows=0):
    return EngineOptions(ctypes.sizeof(EngineOptions), TRACE_VARIANTS[variant], queues, batch, ROWS[rows],
                         EXCHANGES[exchange], SPLITS[split],
                         1 if simulate else 0, launch, SRT_ENGINE_RCCL_SELF if rccl_self else 0, share, own_rows)


SPLIT_SOURCES = {0: "none", 1: "option", 2: "env", 3: "link", 4: "default"}


def unique_id() -> bytes:
    """128-byte RCCL unique id for FrameEngine.rank (one rank makes it, every rank uses it)."""
    buf = ctypes.create_string_buffer(128)
    _check(_native.lib().srtEngineUniqueId(buf))
    return buf.raw


class FrameEngine:
    """Frames of one scene at W x H over `devices` (this process) or one rank of a job."""

    def __init__(self, path: str, width: int, height: int, devices=(0,), variant: str = "cull", queues: int = 2,
                 batch: int = 16, rows: str = "interleaved", exchange: str = "alltoall", split: str = "bands",
                 launch: int = 0, rccl_self: bool = False, share: int = 0, own_rows: int = 0, _handle=None):
        """rccl_self (one device, tests): the bands path with the frame's ids sent to itself over a
        one-rank RCCL communicator -- the real exchange, its waits and its abort path.
        exchange="share": the compositor traces `share` (a power of two; 0: srtShareAuto, 32 at 1080p)
        of every share + P - 1 tile rows itself. own_rows (rotated rows over two devices): rows of the
        compositor's own band (0: env SRT_ROTATE_OWN, else the split derived from the measured link, else
        80 %; split())."""
        self._lib = _native.lib()
        self.width, self.height, self.batch = width, height, batch
        self.options = {"variant": variant, "queues": queues, "batch": batch, "rows": rows, "exchange": exchange,
                        "split": split, "launch": launch, "rccl_self": rccl_self, "share": share,
                        "own_rows": own_rows}
        if _handle is None:
            devs = (ctypes.c_int * len(devices))(*devices)
            opt = _options(variant, queues, batch, rows, exchange, split, launch=launch, rccl_self=rccl_self,
                           share=share, own_rows=own_rows)
            _handle = self._lib.srtEngineCreate(os.fsencode(path), devs, len(devices), width, height, ctypes.byref(opt))
        if not _handle:
            raise SrtError(_native.last_error())
        self.handle = _handle
        self.path = path
        self.inputs = 0

    @classmethod
    def rank(cls, path: str, width: int, height: int, device: int, rank: int, world: int, uid: bytes | None,
             variant: str = "cull", queues: int = 2, batch: int = 16, rows: str = "interleaved",
             exchange: str = "alltoall", split: str = "bands", simulate: bool = False, launch: int = 0,
             share: int = 0, own_rows: int = 0):
        """This process's rank of a `world`-rank job on `device`; every rank calls it concurrently.
        simulate=True (measurement): no peers, no unique id -- the rank's stream without the exchange."""
        lib = _native.lib()
        opt = _options(variant, queues, batch, rows, exchange, split, simulate, launch, share=share, own_rows=own_rows)
        idbuf = ctypes.create_string_buffer(uid, 128) if uid is not None else None
        h = lib.srtEngineCreateRank(os.fsencode(path), device, rank, world, idbuf, width, height, ctypes.byref(opt))
        if not h:
            raise SrtError(_native.last_error())
        return cls(path, width, height, variant=variant, queues=queues, batch=batch, rows=rows, exchange=exchange,
                   split=split, launch=launch, share=share, own_rows=own_rows, _handle=h)

    def set_inputs(self, offsets):
        """offsets: (count, H, W, 2) or (H, W, 2) float32 host array (numpy or CPU tensor)."""
        import numpy as np

        arr = offsets.numpy() if hasattr(offsets, "numpy") else offsets
        arr = np.ascontiguousarray(arr, dtype=np.float32)
        if arr.ndim == 3:
            arr = arr[None]
        if arr.shape[1:] != (self.height, self.width, 2):
            raise ValueError(f"offsets must be (count, {self.height}, {self.width}, 2), got {arr.shape}")
        _check(self._lib.srtEngineSetInputs(self.handle, arr.ctypes.data, arr.shape[0]))
        self.inputs = arr.shape[0]

    def run(self, batches: int):
        _check(self._lib.srtEngineRun(self.handle, batches))

    def verify(self):
        """(mismatching frames, frames checked): the last batches' locally composited frames vs a
        single-device render of their inputs by another trace variant, bit for bit."""
        bad, n = ctypes.c_size_t(), ctypes.c_size_t()
        _check(self._lib.srtEngineVerify(self.handle, ctypes.byref(bad), ctypes.byref(n)))
        return bad.value, n.value

    def read_frame(self, k: int):
        """Frame k as a (H, W, 4) float32 numpy array (must be resident on this process)."""
        import numpy as np

        out = np.empty((self.height, self.width, 4), np.float32)
        _check(self._lib.srtEngineReadFrame(self.handle, k, out.ctypes.data))
        return out

    def stage_times(self, local: int = 0, launches: int = 100, frames: int = 1):
        """(launches, tile info ms, records + bins + work list ms, trace kernel ms) per launch:
        `launches` traces of `frames` frames each (one launch per stage for all of them, one launch
        in flight) of local device `local`'s band, HIP events bound to the kernels' dispatches."""
        n, p, b, t = ctypes.c_uint(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        _check(self._lib.srtEngineStageTimesBatch(self.handle, local, launches, frames, ctypes.byref(n),
                                                  ctypes.byref(p), ctypes.byref(b), ctypes.byref(t)))
        return n.value, p.value, b.value, t.value

    def info(self):
        d, ld, br, bufr = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        rccl, xb = ctypes.c_int(), ctypes.c_double()
        _check(self._lib.srtEngineInfo(self.handle, ctypes.byref(d), ctypes.byref(ld), ctypes.byref(br),
                                       ctypes.byref(bufr), ctypes.byref(rccl), ctypes.byref(xb)))
        return {"devices": d.value, "local_devices": ld.value, "band_rows": br.value, "buffer_rows": bufr.value,
                "rccl": bool(rccl.value), "exchange_bytes_per_frame": xb.value}

    def split(self):
        """The two-device split (srtEngineSplit): own band rows (0 unless rotated rows over two devices),
        band buffer rows, the link measured at creation (GB/s per direction; 0 without RCCL), the one-GPU
        frame time measured for the split (us; 0 when not derived) and where the split came from."""
        own, bufr = ctypes.c_size_t(), ctypes.c_size_t()
        gbs, fus, src = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        _check(self._lib.srtEngineSplit(self.handle, ctypes.byref(own), ctypes.byref(bufr), ctypes.byref(gbs),
                                        ctypes.byref(fus), ctypes.byref(src)))
        return {"own_rows": own.value, "buffer_rows": bufr.value, "link_gbs": round(gbs.value, 3),
                "frame_us": round(fus.value, 3), "source": SPLIT_SOURCES.get(src.value, str(src.value))}

    def exchange_stats(self, local: int = 0):
        """The last run's exchange on local device `local` (srtEngineExchangeStats): groups timed, mean ms
        per group on the device's exchange stream, bytes the device sent per group."""
        g, ms, sent = ctypes.c_size_t(), ctypes.c_double(), ctypes.c_double()
        _check(self._lib.srtEngineExchangeStats(self.handle, local, ctypes.byref(g), ctypes.byref(ms), ctypes.byref(sent)))
        return {"groups": g.value, "ms_mean": ms.value, "bytes_sent": sent.value}

    def close(self):
        if getattr(self, "handle", None):
            self._lib.srtEngineRelease(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        self.close()


def pool_self_test(workers: int, failing: int, mode: str = "fail", timeout_s: float = 1.0):
    """Host self-test of the engine's worker pool failure handling (no device): worker `failing`
    throws ("fail") or stalls ("stall") while the others wait for a release only the abort gives.
    Returns (error message the run ended with, seconds taken, abort hook calls)."""
    lib = _native.lib()
    el, calls = ctypes.c_double(), ctypes.c_int()
    msg = ctypes.create_string_buffer(1024)
    _check(lib.srtEnginePoolSelfTest(workers, failing, {"fail": 1, "stall": 2}[mode], timeout_s, ctypes.byref(el),
                                     ctypes.byref(calls), msg, len(msg)))
    return msg.value.decode(), el.value, calls.value


def exchange_host(band_ids, height: int, rows: str = "interleaved", exchange: str = "alltoall", batch_index: int = 0,
                  share: int = 0):
    """Host self-test of the engine's band exchange (no device): band_ids = list of P arrays
    (batch, buffer_rows, W) int32, band d's ids of a batch's frames (rotated rows: of frame f the band
    bands.rotated_band(P, d, f % P); share: device d's sender class of frame f, share + (d - f % P - 1)
    % P, unused when d composites f). Returns the list of every compositor's receive buffer, (P, frames
    composited there, buffer_rows, W) int32, exactly as the device path lays it out for the shading
    launch. share: the share exchange's tile rows per cycle (0: srtShareAuto)."""
    import numpy as np

    lib = _native.lib()
    P = len(band_ids)
    batch, _, width = band_ids[0].shape
    frames = (ctypes.c_size_t * P)()
    brows = ctypes.c_size_t()

    def call(inp, outp):
        if exchange == "share":
            return lib.srtExchangeHostShare(inp, P, width, height, share, batch, batch_index, outp, frames,
                                            ctypes.byref(brows))
        return lib.srtExchangeHost(inp, P, width, height, ROWS[rows], EXCHANGES[exchange], batch, batch_index, outp,
                                   frames, ctypes.byref(brows))

    _check(call(None, None))
    ins = [np.ascontiguousarray(b, dtype=np.int32) for b in band_ids]
    for b in ins:
        if b.shape != (batch, brows.value, width):
            raise ValueError(f"band ids must be ({batch}, {brows.value}, {width}), got {b.shape}")
    outs = [np.empty((P, frames[c], brows.value, width), np.int32) for c in range(P)]
    inp = (ctypes.c_void_p * P)(*[b.ctypes.data for b in ins])
    outp = (ctypes.c_void_p * P)(*[o.ctypes.data for o in outs])
    _check(call(inp, outp))
    return outs
