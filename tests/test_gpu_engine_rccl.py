"""GPU: the frame engine's RCCL exchange, its failure handling, and the headline launch shapes.

- The exchange over real RCCL communicators: on this one-GPU box through the one-rank self-exchange
  (SRT_ENGINE_RCCL_SELF: every frame's ids leave through ncclSend and come back through ncclRecv,
  nonblocking communicator, polled waits); on a box with two or more GPUs across distinct devices
  (P = 2 and P = all visible, every exchange pattern), skipped here. Every frame against the full C3
  fixture (tests/golden/fullframes.*: ids bit-exact, RGB <= 1e-5 of the oracle's shading).
- Abort, not hang: an injected worker failure or stall (SRT_ENGINE_INJECT) ends the run with an error
  within the deadline (SRT_COMM_TIMEOUT_S), on the RCCL path and on the device-copy path, and the
  engine refuses further work.
- The headline launch shapes (bench.py at N = 1: 64-frame batches, 8 frames per launch, 2 queues)
  at C3 (every resident frame, every pixel) and C5 (every resident frame, the 64 fixture rows).
"""
from __future__ import annotations

import os

import time

import numpy as np
import pytest

from test_golden_full import META, ids, oracle_rgba, offsets_for, paths, rows_of  # noqa: F401 (fixtures)
from test_gpu_parity import torch_render

pytestmark = pytest.mark.gpu

C3 = "c3_soup100k_1080p"
C5 = "c5_soup1m_4k_rows"
RGB_TOL = 1e-5


class Expected:
    """A fixture's stored rows as the frame must show them: id channel bits and oracle RGB."""

    def __init__(self, path, name, stored_ids):
        m = META[name]
        self.rows = rows_of(m)
        self.id_bits = stored_ids.astype(np.float32).view(np.uint32)
        self.rgb = oracle_rgba(path, m, stored_ids)[..., :3]

    def check(self, frame, what):
        got = frame[self.rows]
        bad = np.argwhere(got[..., 3].view(np.uint32) != self.id_bits)
        assert bad.size == 0, f"{what}: {len(bad)} tri_id mismatches, first {bad[:5].tolist()}"
        d = float(np.abs(got[..., :3] - self.rgb).max())
        assert d <= RGB_TOL, f"{what}: max rgb delta {d}"


def engine(path, m, **kw):
    from simpleraytracer_amd.engine import FrameEngine

    return FrameEngine(path, m["width"], m["height"], **kw)


# ---------------------------------------------------------------------------------------------
# The headline launch shapes


def test_engine_headline_shape_full_c3_fixture(gpu, paths, ids):
    """bench.py's N = 1 line as launched: batches of 64 frames, 8 frames per launch, 2 frame
    queues, whole frames traced and shaded in one kernel. Every frame of the two resident batches,
    every pixel, against the fixture."""
    m = META[C3]
    want = Expected(paths[C3], C3, ids[C3])
    with engine(paths[C3], m, devices=[0], batch=64, launch=8, queues=2) as e:
        e.set_inputs(offsets_for(m))
        e.run(3)  # batches 0..2; the queues hold batches 1 and 2 (frames 64..191)
        for k in range(64, 192):
            want.check(e.read_frame(k), f"frame {k}")
        assert e.verify() == (0, 8)


def test_engine_headline_shape_c5_fixture_rows(gpu, paths, ids):
    """The same launch shape at C5 (1M triangles, 3840 x 2160, one GPU): every resident frame, on
    the 64 stored rows of the C5 fixture."""
    m = META[C5]
    want = Expected(paths[C5], C5, ids[C5])
    with engine(paths[C5], m, devices=[0], batch=64, launch=8, queues=2) as e:
        e.set_inputs(offsets_for(m))
        e.run(2)
        for k in range(0, 128):
            want.check(e.read_frame(k), f"frame {k}")


# ---------------------------------------------------------------------------------------------
# RCCL exchange


def test_engine_rccl_self_exchange_full_c3_fixture(gpu, paths, ids):
    """The bands path over a one-rank RCCL communicator: every frame's ids go out through ncclSend
    and come back through ncclRecv (nonblocking communicator, group, settle, polled waits), then the
    compositor shades them. Every frame of the resident batches against the fixture."""
    m = META[C3]
    want = Expected(paths[C3], C3, ids[C3])
    with engine(paths[C3], m, devices=[0], batch=4, queues=2, rccl_self=True) as e:
        assert e.info()["rccl"]
        # the link probe ran over the one-rank communicator (a copy to itself: a rate, no two-device split)
        sp = e.split()
        assert sp["link_gbs"] > 0 and sp["own_rows"] == 0 and sp["source"] == "none", sp
        e.set_inputs(offsets_for(m))
        e.run(3)
        for k in range(4, 12):
            want.check(e.read_frame(k), f"frame {k}")
        assert e.verify() == (0, 8)


def test_ml_rccl_gather_one_rank_full_c3_fixture(gpu, paths, ids, monkeypatch):
    """mlInfer's ncclGather path on one device (SRT_GATHER=rccl: a one-rank communicator, the band
    path, the gather, the root's shading and copy out) against the fixture."""
    import simpleraytracer_amd as srt

    m = META[C3]
    monkeypatch.setenv("SRT_GATHER", "rccl")
    got = srt.render(paths[C3], m["width"], m["height"])
    Expected(paths[C3], C3, ids[C3]).check(got, "mlInfer one-rank gather")


def _gpus():
    import torch

    return torch.cuda.device_count()


@pytest.mark.parametrize("exchange", ["alltoall", "rotating", "root", "share", "rotated"])
@pytest.mark.parametrize("which", ["2", "all"])
def test_engine_rccl_bands_full_c3_fixture(gpu, paths, ids, exchange, which):
    """Distinct GPUs, RCCL between them (BASELINE config C4): P = 2 and P = every visible GPU (at most
    8), every exchange pattern; every frame of the resident batches against the fixture."""
    n = _gpus()
    if n < 2:
        pytest.skip(f"needs 2 or more GPUs for an RCCL exchange between devices (this box has {n}); the "
                    "same exchange code runs over one rank in test_engine_rccl_self_exchange_full_c3_fixture")
    P = 2 if which == "2" else min(8, n)
    m = META[C3]
    want = Expected(paths[C3], C3, ids[C3])
    kw = {"exchange": "alltoall", "rows": "rotated"} if exchange == "rotated" else {"exchange": exchange}
    with engine(paths[C3], m, devices=list(range(P)), batch=2 * P, queues=2, **kw) as e:
        assert e.info()["rccl"] and e.info()["devices"] == P
        sp = e.split()
        assert sp["link_gbs"] > 0, sp
        if exchange == "rotated" and P == 2 and not os.environ.get("SRT_ROTATE_OWN"):
            # the split derived from the measured link (srtRotateSplitForLink)
            assert sp["source"] == "link" and sp["frame_us"] > 0 and sp["own_rows"] >= m["height"] // 2, sp
        e.set_inputs(offsets_for(m))
        e.run(3)
        for k in range(2 * P, 6 * P):
            want.check(e.read_frame(k), f"P={P} {exchange} frame {k}")
        bad, checked = e.verify()
        assert bad == 0 and checked > 0


def test_ml_rccl_gather_two_devices_full_c3_fixture(gpu, paths, ids, monkeypatch):
    n = _gpus()
    if n < 2:
        pytest.skip(f"needs 2 visible GPUs (this box has {n}); the one-rank gather runs in "
                    "test_ml_rccl_gather_one_rank_full_c3_fixture")
    import simpleraytracer_amd as srt

    m = META[C3]
    monkeypatch.setenv("ML_VISIBLE_DEVICES", "0,1")
    monkeypatch.setenv("SRT_GATHER", "rccl")
    Expected(paths[C3], C3, ids[C3]).check(srt.render(paths[C3], m["width"], m["height"]), "mlInfer 2-GPU gather")


# ---------------------------------------------------------------------------------------------
# Abort, not hang


def _abort_run(scene, monkeypatch, inject, devices, match, **kw):
    from simpleraytracer_amd.device import SrtError
    from simpleraytracer_amd.engine import FrameEngine

    monkeypatch.setenv("SRT_ENGINE_INJECT", inject)
    monkeypatch.setenv("SRT_COMM_TIMEOUT_S", "3")
    w, h = 160, 100
    with FrameEngine(scene, w, h, devices=devices, batch=4, queues=2, **kw) as e:
        e.set_inputs(np.full((1, h, w, 2), 0.5, np.float32))
        t0 = time.monotonic()
        with pytest.raises(SrtError, match=match):
            e.run(4)
        elapsed = time.monotonic() - t0
        assert elapsed < 15.0, f"the failed run took {elapsed:.1f} s (deadline 3 s)"
        with pytest.raises(SrtError, match="earlier failure"):
            e.run(1)


@pytest.mark.parametrize("kind,match", [("fail", "injected failure"), ("stall", "no device made progress")])
def test_engine_rccl_self_abort(gpu, scenes, monkeypatch, kind, match):
    """A worker that throws, or stops progressing, on the RCCL path: the run ends with the error
    (communicators aborted) instead of waiting forever."""
    _abort_run(scenes["soup2k"], monkeypatch, f"{kind}:0:2", [0], match, rccl_self=True)


@pytest.mark.parametrize("kind,match", [("fail", "injected failure"), ("stall", "no device made progress")])
def test_engine_fake_devices_abort(gpu, scenes, monkeypatch, kind, match):
    """The same on the device-copy exchange of three fake devices: the others wait at the host
    barrier for the failed one, and are released with the error."""
    _abort_run(scenes["soup2k"], monkeypatch, f"{kind}:1:1", [0, 0, 0], match)


def test_engine_rccl_self_recovers_after_failed_engine(gpu, scenes, monkeypatch):
    """After a failed, aborted engine, a new engine on the same device renders correctly."""
    from simpleraytracer_amd.engine import FrameEngine

    _abort_run(scenes["soup2k"], monkeypatch, "fail:0:1", [0], "injected failure", rccl_self=True)
    monkeypatch.delenv("SRT_ENGINE_INJECT")
    w, h = 160, 100
    inputs = np.random.default_rng(4).random((1, h, w, 2), dtype=np.float32)
    ref = torch_render(scenes["soup2k"], w, h, inputs[0])
    with FrameEngine(scenes["soup2k"], w, h, devices=[0], batch=4, queues=2, rccl_self=True) as e:
        e.set_inputs(inputs)
        e.run(2)
        for k in range(8):
            assert np.array_equal(e.read_frame(k).view(np.uint32), ref.view(np.uint32)), k


# ---------------------------------------------------------------------------------------------
# Parameter tables (more than 8 frames per launch), distinct inputs, table-ring reuse


def test_engine_table_launches_distinct_inputs(gpu, scenes):
    """Launches of 16 frames take their parameters from a device table (a 4-entry ring per scene):
    2 fake devices, 32-frame batches (two table launches per batch), 64 distinct inputs, 6 batches on
    2 queues = 6 table launches per queue scene, so the ring wraps and its pinned host buffers are
    reused. Every resident frame equals the one-device render of its own input, bit for bit."""
    from simpleraytracer_amd.engine import FrameEngine

    w, h, F = 96, 64, 32
    inputs = np.random.default_rng(31).random((2 * F, h, w, 2), dtype=np.float32)
    refs = [torch_render(scenes["soup2k"], w, h, inputs[i]) for i in range(2 * F)]
    with FrameEngine(scenes["soup2k"], w, h, devices=[0, 0], batch=F, launch=16, queues=2) as e:
        e.set_inputs(inputs)
        e.run(6)
        for k in range(4 * F, 6 * F):
            assert np.array_equal(e.read_frame(k).view(np.uint32), refs[k % (2 * F)].view(np.uint32)), k


def test_engine_frames_split_distinct_frames(gpu, scenes):
    """Split frames: each device renders frames of its own (device d's batch b = frames
    (b * P + d) * F + f), so every frame of the sequence is rendered once and is readable."""
    from simpleraytracer_amd.engine import FrameEngine

    w, h, F, P = 64, 48, 2, 3
    inputs = np.random.default_rng(8).random((2 * F * P, h, w, 2), dtype=np.float32)
    with FrameEngine(scenes["soup300"], w, h, devices=[0] * P, split="frames", batch=F, queues=2) as e:
        e.set_inputs(inputs)
        e.run(2)  # frames 0 .. 2 * F * P - 1, all resident
        for k in range(2 * F * P):
            ref = torch_render(scenes["soup300"], w, h, inputs[k])
            assert np.array_equal(e.read_frame(k).view(np.uint32), ref.view(np.uint32)), k
        assert e.verify() == (0, P * 2 * F)


# ---------------------------------------------------------------------------------------------
# Packed ids (render.h PackedIds): the exchange payload, 16 + k bits per pixel


def collision_scene(path, n=70_000, seed=5):
    """n triangles where triangles k and k + 65536 share their low 16 bits and overlap on screen
    (k < n - 65536): large triangles in front of the camera -- sometimes k nearer, sometimes k +
    65536, sometimes coplanar and identical (a depth tie: the lower id must win) -- so the bit plane
    above the low 16 bits decides every one of their pixels; the rest are small triangles scattered
    over the view."""
    from scenefile import write_custom_scene

    rng = np.random.default_rng(seed)
    v = np.zeros((n, 3, 3), np.float32)
    cen = np.stack([rng.uniform(-1.2, 1.2, n), rng.uniform(-0.7, 0.7, n), rng.uniform(3.0, 6.0, n)], 1)
    v[:] = cen[:, None, :] + rng.uniform(-0.03, 0.03, (n, 3, 3))
    pairs = n - 65536
    for k in range(pairs):
        c = np.array([rng.uniform(-1.0, 1.0), rng.uniform(-0.5, 0.5), 0.0])
        z_a, z_b = rng.uniform(1.5, 2.5), rng.uniform(1.5, 2.5)
        if k % 7 == 0:
            z_b = z_a  # coplanar and identical: equal t, the lower id wins
        tri = np.array([[-0.25, -0.2, 0.0], [0.3, -0.15, 0.0], [0.0, 0.3, 0.0]]) + c
        a, b = tri.copy(), tri.copy()
        if k % 7 != 0:
            b[:, :2] = b[:, :2] * 0.9 + 0.05  # overlapping, not identical
        a[:, 2] += z_a
        b[:, 2] += z_b
        v[k], v[k + 65536] = a, b
    return write_custom_scene(path, v, rng.uniform(0.2, 1.0, (n, 3)))


def test_packed_ids_exchange_bitwise(gpu, tmp_path, monkeypatch):
    """70 000 triangles (one bit plane): ids that differ only above bit 15 cover the same pixels.
    Packed ids through the fake-device exchange (P = 2 and 3) and the one-rank RCCL exchange, and
    int32 ids (SRT_EXCHANGE_IDS=32), give the one-device frame bit for bit; random offsets, uniform in
    some tiles (whose offset the packed ids carry: their shading reads no per-pixel offsets)."""
    from simpleraytracer_amd.engine import FrameEngine

    path = collision_scene(tmp_path / "collide.srt")
    w, h = 256, 144
    inputs = np.random.default_rng(9).random((1, h, w, 2), dtype=np.float32)
    inputs[0, :48] = 0.5  # regular tiles: three tile rows, and one tile column below them
    inputs[0, 48:, 128:192] = 0.25
    ref = torch_render(path, w, h, inputs[0])
    ids = ref[..., 3].astype(np.int64)
    assert (ids >= 65536).sum() > 1000 and ((ids >= 0) & (ids < 70_000 - 65536)).sum() > 1000, \
        "the scene must put both members of the sharing pairs on screen"
    for ids32 in (False, True):
        if ids32:
            monkeypatch.setenv("SRT_EXCHANGE_IDS", "32")
        for kw in ({"devices": [0, 0]}, {"devices": [0, 0, 0]}, {"devices": [0], "rccl_self": True}):
            with FrameEngine(path, w, h, batch=6, queues=2, **kw) as e:
                xb = e.info()["exchange_bytes_per_frame"]
                e.set_inputs(inputs)
                e.run(2)
                for k in range(12):
                    assert np.array_equal(e.read_frame(k).view(np.uint32), ref.view(np.uint32)), (ids32, kw, k)
            if len(kw["devices"]) == 2:  # bands of 16-row tile rows: 5 and 4 of the 9, buffers of 80 rows
                # 4 B or 2.125 B a pixel, plus (packed) one 8-B tile offset per tile, padded to 256 B
                packed = (80 * (256 * 2 + 4 * 8) + 5 * 4 * 8 + 255) // 256 * 256
                assert xb == (80 * 256 * 4 if ids32 else packed), xb


def test_packed_ids_mlinfer_gather_bitwise(gpu, tmp_path, monkeypatch):
    """The mlInfer gather (fake devices, device copies) with packed and with int32 ids."""
    import simpleraytracer_amd as srt

    path = collision_scene(tmp_path / "collide.srt")
    w, h = 200, 120
    ref = srt.render(path, w, h)
    monkeypatch.setenv("ML_VISIBLE_DEVICES", "0,0,0")
    got = srt.render(path, w, h)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    monkeypatch.setenv("SRT_EXCHANGE_IDS", "32")
    got32 = srt.render(path, w, h)
    assert np.array_equal(got32.view(np.uint32), ref.view(np.uint32))


def test_engine_c5_bands_packed_ids(gpu, paths, ids):
    """C5 (1M triangles: four bit planes) split over 2 fake devices, every frame on the 64 stored rows."""
    from simpleraytracer_amd.engine import FrameEngine

    m = META[C5]
    want = Expected(paths[C5], C5, ids[C5])
    with FrameEngine(paths[C5], m["width"], m["height"], devices=[0, 0], batch=2, queues=1) as e:
        e.set_inputs(offsets_for(m))
        e.run(1)
        for k in range(2):
            want.check(e.read_frame(k), f"frame {k}")
