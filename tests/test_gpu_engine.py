"""GPU: the frame engine (csrc/engine.cpp) -- the native path bench.py times at every N.

Frames rendered by the engine, wherever they were composited, are compared with the oracle
(tri_id bit-exact, RGB <= 1e-5) and with a single-device render, bit for bit. Multi-device runs use
"fake devices" (device 0 repeated: the bands are exchanged by device copies, everything else is
the multi-GPU code path), since this box has one GPU.
"""
from __future__ import annotations

import numpy as np
import pytest

from test_gpu_parity import assert_parity, oracle_render, torch_render

pytestmark = pytest.mark.gpu


def engine(path, w, h, devices=(0,), **kw):
    from simpleraytracer_amd.engine import FrameEngine

    return FrameEngine(path, w, h, devices=list(devices), **kw)


def random_inputs(n, h, w, seed=77):
    return np.random.default_rng(seed).random((n, h, w, 2), dtype=np.float32)


@pytest.mark.parametrize("variant", ["cull", "lds"])
def test_engine_one_device_matches_oracle(gpu, scenes, variant):
    w, h, F = 97, 61, 3
    inputs = random_inputs(F, h, w)
    with engine(scenes["soup2k"], w, h, variant=variant, queues=2, batch=F) as e:
        e.set_inputs(inputs)
        e.run(3)  # batches 0..2: frames 0..8; queues hold batches 1 and 2
        for k in range(3, 9):
            assert_parity(e.read_frame(k), oracle_render(scenes["soup2k"], w, h, inputs[k % F]))
        bad, checked = e.verify()
        assert bad == 0 and checked == 2 * F
        with pytest.raises(Exception):
            e.read_frame(0)  # no longer resident


@pytest.mark.parametrize("p", [2, 3, 8])
@pytest.mark.parametrize("rows", ["interleaved", "contiguous"])
@pytest.mark.parametrize("exchange", ["alltoall", "rotating", "root"])
def test_engine_fake_devices_bitwise(gpu, scenes, p, rows, exchange):
    """P fake devices: every frame of the last batches equals a one-device render bit for bit."""
    w, h, F = 130, 100, 4
    inputs = random_inputs(1, h, w, seed=p)
    ref = torch_render(scenes["soup2k"], w, h, inputs[0])
    assert_parity(ref, oracle_render(scenes["soup2k"], w, h, inputs[0]))
    with engine(scenes["soup2k"], w, h, devices=[0] * p, rows=rows, exchange=exchange, queues=2, batch=F) as e:
        assert e.info()["devices"] == p and not e.info()["rccl"]
        e.set_inputs(inputs)
        e.run(3)
        for k in range(F, 3 * F):
            got = e.read_frame(k)
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), k
        bad, checked = e.verify()
        assert bad == 0 and checked == 2 * F


@pytest.mark.parametrize("p,share,queues", [(2, 4, 2), (2, 1, 2), (2, 8, 3), (3, 2, 2), (8, 2, 4), (4, 8, 2),
                                             (2, 16, 2), (2, 0, 2), (8, 0, 2)])
def test_engine_fake_devices_share_bitwise(gpu, scenes, p, share, queues):
    """The share exchange (the compositor of a batch traces `share` of every share + P - 1 tile rows
    itself, straight into its frames; every other device one tile row per cycle, sent as ids and
    shaded there): distinct inputs per frame, every frame of the last batches equal to a one-device
    render of its input, bit for bit -- also with a queue count that makes a queue change roles
    (and so band shapes) from batch to batch. share = 16 at P = 2: a cycle of 17 tile rows is longer
    than the frame, so the sender's band is empty; share = 0: the library's choice (srtShareAuto)."""
    w, h = 150, 230  # 15 tile rows: cycles of share + P - 1 end in a partial one
    F = 4 if 4 % p == 0 else 2 * p  # frames dealt to compositors round-robin: a batch of whole rounds
    inputs = random_inputs(2 * F, h, w, seed=11 + p)
    refs = [torch_render(scenes["soup2k"], w, h, inputs[k]) for k in range(2 * F)]
    with engine(scenes["soup2k"], w, h, devices=[0] * p, exchange="share", share=share, queues=queues,
                batch=F) as e:
        e.set_inputs(inputs)
        e.run(queues + 1)
        for k in range(F, (queues + 1) * F):
            got = e.read_frame(k)
            assert np.array_equal(got.view(np.uint32), refs[k % (2 * F)].view(np.uint32)), k
        bad, checked = e.verify()
        assert bad == 0 and checked == queues * F
        assert e.info()["exchange_bytes_per_frame"] > 0


@pytest.mark.parametrize("p,h", [(2, 100), (3, 100), (8, 230), (4, 61)])
def test_engine_fake_devices_rotated_bitwise(gpu, scenes, p, h):
    """Rotated contiguous bands (device d traces band (d + c) % P of a frame composited on device c;
    the band record pass skipping the record blocks that cannot reach the band): distinct inputs per
    frame, every frame of the resident batches equal to a one-device render, bit for bit. h = 100 at
    P = 3: bands of 34, 34 and 32 rows (two launch groups); h = 61 at P = 4: 16, 16, 16, 13."""
    w, F = 130, 2 * p
    inputs = random_inputs(2 * F, h, w, seed=31 + p)
    refs = [torch_render(scenes["soup2k"], w, h, inputs[k]) for k in range(2 * F)]
    with engine(scenes["soup2k"], w, h, devices=[0] * p, rows="rotated", exchange="alltoall", queues=2,
                batch=F) as e:
        e.set_inputs(inputs)
        e.run(3)
        for k in range(F, 3 * F):
            got = e.read_frame(k)
            assert np.array_equal(got.view(np.uint32), refs[k % (2 * F)].view(np.uint32)), k
        assert e.verify() == (0, 2 * F)


@pytest.mark.parametrize("own,h", [("", 100), ("50", 100), ("90", 100), ("1", 100), ("75", 1080), ("99", 61)])
def test_engine_fake_devices_rotated_two_device_split(gpu, scenes, monkeypatch, own, h):
    """Two devices, rotated all-to-all: the compositor's own band 0 takes SRT_ROTATE_OWN per cent of the
    frame (default 80, rounded to tile rows; engine.cpp RotateOwnRows), band 1 -- the one that crosses
    the link and is shaded from ids -- the rest: every frame bit for bit against a one-device render, and
    the engine's band-0 rows equal to the restatement (bands.rotate_own_rows)."""
    from simpleraytracer_amd.bands import rotate_own_rows

    if own:
        monkeypatch.setenv("SRT_ROTATE_OWN", own)
    else:
        monkeypatch.delenv("SRT_ROTATE_OWN", raising=False)
    p, F = 2, 4
    w = 130 if h < 1000 else 64
    inputs = random_inputs(2 * F, h, w, seed=77)
    refs = [torch_render(scenes["soup2k"], w, h, inputs[k]) for k in range(2 * F)]
    with engine(scenes["soup2k"], w, h, devices=[0] * p, rows="rotated", exchange="alltoall", queues=2,
                batch=F) as e:
        info, split = e.info(), e.split()
        # band_rows: the band stage timing traces, a sent one (band 1); the own band is the split's
        assert info["band_rows"] == h - rotate_own_rows(h) and info["buffer_rows"] == h - rotate_own_rows(h)
        assert split["own_rows"] == rotate_own_rows(h) and split["buffer_rows"] == info["buffer_rows"]
        assert split["source"] == ("env" if own else "default") and split["link_gbs"] == 0.0  # fake devices
        e.set_inputs(inputs)
        e.run(3)
        for k in range(F, 3 * F):
            got = e.read_frame(k)
            assert np.array_equal(got.view(np.uint32), refs[k % (2 * F)].view(np.uint32)), (own, k)
        assert e.verify() == (0, 2 * F)


def test_engine_rotated_two_device_options_split(gpu, scenes, monkeypatch):
    """srt_engine_options.own_rows sets the two-device split (over SRT_ROTATE_OWN), bit for bit; an
    invalid SRT_ROTATE_OWN refuses the engine instead of silently sending 99 % of every frame."""
    from simpleraytracer_amd.device import SrtError

    monkeypatch.setenv("SRT_ROTATE_OWN", "60")
    h, w, F = 100, 130, 4
    inputs = random_inputs(2 * F, h, w, seed=78)
    refs = [torch_render(scenes["soup2k"], w, h, inputs[k]) for k in range(2 * F)]
    with engine(scenes["soup2k"], w, h, devices=[0, 0], rows="rotated", exchange="alltoall", batch=F,
                own_rows=48) as e:
        assert e.split()["own_rows"] == 48 and e.split()["source"] == "option" and e.info()["buffer_rows"] == 52
        e.set_inputs(inputs)
        e.run(2)
        for k in range(F, 2 * F):
            assert np.array_equal(e.read_frame(k).view(np.uint32), refs[k].view(np.uint32)), k
    monkeypatch.setenv("SRT_ROTATE_OWN", "abc")
    with pytest.raises(SrtError, match="SRT_ROTATE_OWN must be an integer"):
        engine(scenes["soup2k"], w, h, devices=[0, 0], rows="rotated", exchange="alltoall", batch=F)


def test_engine_rotated_two_device_stage_times_whole_batch(gpu, scenes, monkeypatch):
    """stage timing and the rank simulation's priming traced device 0's own band (864
    of 1080 rows under the 4/5 split) into send slots sized for the 216-row band 1 -- past the end of the
    send buffer when a launch took the whole batch. They now trace a sender band: a 1080-row frame, the
    batch in one launch, then a run that must still be bit-exact; the rank simulation primes likewise."""
    from simpleraytracer_amd.engine import FrameEngine

    monkeypatch.delenv("SRT_ROTATE_OWN", raising=False)
    h, w, F = 1080, 64, 4
    inputs = random_inputs(F, h, w, seed=79)
    refs = [torch_render(scenes["soup2k"], w, h, inputs[k]) for k in range(F)]
    with engine(scenes["soup2k"], w, h, devices=[0, 0], rows="rotated", exchange="alltoall", batch=F,
                launch=F) as e:
        e.set_inputs(inputs)
        for local in (0, 1):
            n, _, binned, trace = e.stage_times(local, 3, F)
            assert n == 3 and binned > 0 and trace > 0
        assert e.info()["band_rows"] == e.info()["buffer_rows"] == 216
        e.run(2)
        for k in range(F, 2 * F):
            assert np.array_equal(e.read_frame(k).view(np.uint32), refs[k % F].view(np.uint32)), k
    for rank in (0, 1):
        with FrameEngine.rank(scenes["soup2k"], w, h, 0, rank, 2, None, rows="rotated", exchange="alltoall",
                              batch=2, simulate=True) as e:
            e.set_inputs(inputs[:2])
            e.run(2)
            n, _, _, trace = e.stage_times(0, 2, 2)
            assert n == 2 and trace > 0


@pytest.mark.parametrize("queues", [1, 2, 3])
def test_engine_exchange_timing_counts_every_group(gpu, scenes, queues):
    """srtEngineExchangeStats: every batch's exchange group is timed, through a bounded ring of 2 Q + 2
    event pairs (a new pair per batch, kept until release) -- a run of more batches than the
    ring reports one group per batch, a positive mean and the bytes a device sends per batch; a second
    run reports its own groups only."""
    w, h, F = 130, 100, 4
    with engine(scenes["soup2k"], w, h, devices=[0, 0], rows="rotated", exchange="alltoall", queues=queues,
                batch=F) as e:
        e.set_inputs(random_inputs(F, h, w, seed=83))
        for batches in (2 * queues + 7, 3):
            e.run(batches)
            for local in (0, 1):
                st = e.exchange_stats(local)
                assert st["groups"] == batches and st["ms_mean"] > 0 and st["bytes_sent"] > 0, (batches, st)
        assert e.verify()[0] == 0


def test_engine_rotated_needs_alltoall(gpu, scenes):
    from simpleraytracer_amd.device import SrtError

    with pytest.raises(SrtError, match="rotated bands"):
        engine(scenes["soup300"], 40, 40, devices=[0, 0], rows="rotated", exchange="rotating")
    with pytest.raises(SrtError, match="interleaved rows"):  # share deals tile rows: interleaved only
        engine(scenes["soup300"], 40, 40, devices=[0, 0], rows="rotated", exchange="share")


def test_engine_fake_devices_rotating_inputs(gpu, scenes):
    """Distinct inputs per frame through the all-to-all exchange (the compositors' strided offsets)."""
    w, h, p, F = 70, 90, 2, 4
    inputs = random_inputs(2 * F, h, w, seed=5)
    with engine(scenes["soup2k"], w, h, devices=[0] * p, queues=2, batch=F) as e:
        e.set_inputs(inputs)
        e.run(3)
        for k in range(F, 3 * F):
            assert_parity(e.read_frame(k), oracle_render(scenes["soup2k"], w, h, inputs[k % (2 * F)]))
        assert e.verify() == (0, 2 * F)


def test_engine_inputs_must_stride_evenly(gpu, scenes):
    from simpleraytracer_amd.device import SrtError

    with engine(scenes["soup300"], 40, 40, devices=[0, 0], batch=4) as e:
        with pytest.raises(SrtError, match="multiple of the batch"):
            e.set_inputs(random_inputs(3, 40, 40))


def test_engine_frames_split(gpu, scenes):
    w, h, F = 64, 48, 2
    inputs = random_inputs(1, h, w, seed=9)
    ref = oracle_render(scenes["soup300"], w, h, inputs[0])
    with engine(scenes["soup300"], w, h, devices=[0, 0, 0], split="frames", batch=F) as e:
        e.set_inputs(inputs)
        e.run(2)
        assert_parity(e.read_frame(2), ref)
        assert e.verify() == (0, 3 * 2 * F)  # every device's two queues


def test_engine_c3_bands_of_8_bitwise(gpu, scenes):
    """The headline frame (1080p, 100k triangles) as 8 interleaved bands exchanged all-to-all over
    fake devices: every frame equals the one-device frame, which matches the oracle on rows."""
    w, h = 1920, 1080
    inputs = np.full((1, h, w, 2), 0.5, np.float32)
    with engine(scenes["soup100k"], w, h, devices=[0] * 8, batch=16, queues=2) as e:
        e.set_inputs(inputs)
        e.run(2)
        assert e.verify() == (0, 32)
        got = e.read_frame(17)
    rows = np.arange(5, 1080, 90)
    ref = oracle_render(scenes["soup100k"], w, h, row_begin=5, row_count=1075, row_step=90)
    assert_parity(got, ref, rows=rows)


def test_engine_c3_rotated_bands_of_8_bitwise(gpu, scenes):
    """The headline frame as 8 rotated contiguous bands of 135 rows (all-to-all; each device skips
    the record blocks that cannot reach its band): every frame equals the one-device frame."""
    w, h = 1920, 1080
    inputs = np.full((1, h, w, 2), 0.5, np.float32)
    with engine(scenes["soup100k"], w, h, devices=[0] * 8, batch=16, queues=2, rows="rotated") as e:
        e.set_inputs(inputs)
        e.run(2)
        assert e.verify() == (0, 32)
        got = e.read_frame(19)
    rows = np.arange(5, 1080, 90)
    ref = oracle_render(scenes["soup100k"], w, h, row_begin=5, row_count=1075, row_step=90)
    assert_parity(got, ref, rows=rows)


@pytest.mark.parametrize("p", [2, 8])
def test_engine_c3_share_bitwise(gpu, scenes, p):
    """The headline frame over P fake devices with the share exchange at the library's k (32 at 1080p:
    each compositor traces 32 of every 32 + P - 1 tile rows itself, every other device one): every
    frame equals the one-device frame, and P - 1 of every 32 + P - 1 tile rows cross the exchange."""
    w, h = 1920, 1080
    inputs = np.full((1, h, w, 2), 0.5, np.float32)
    with engine(scenes["soup100k"], w, h, devices=[0] * p, batch=16, queues=2, exchange="share") as e:
        e.set_inputs(inputs)
        e.run(p + 1)
        assert e.verify()[0] == 0
        got = e.read_frame(16 * p + 3)  # a frame of the last batch (resident on its compositor)
        xb = e.info()["exchange_bytes_per_frame"]
    classes = 32 + p - 1
    # the senders' band buffers: their largest class's tile rows (P = 2: tile rows 32 and 65 of class
    # 32; P = 8: one) -- not class 0's (2 at P = 8: the padding of round 4)
    per = max(len(range(k, 68, classes)) for k in range(32, classes))
    sent = (p - 1) * per
    assert xb <= sent * 16 * w * 2.2, xb
    rows = np.arange(5, 1080, 90)
    ref = oracle_render(scenes["soup100k"], w, h, row_begin=5, row_count=1075, row_step=90)
    assert_parity(got, ref, rows=rows)


def test_engine_c3_share_of_2_bitwise(gpu, scenes):
    """The headline frame over 2 fake devices with the share exchange at k = 4 (each compositor traces
    4 of every 5 tile rows itself, the other device the fifth): every frame equals the one-device
    frame, and a fifth of the frame's ids cross the exchange."""
    w, h = 1920, 1080
    inputs = np.full((1, h, w, 2), 0.5, np.float32)
    with engine(scenes["soup100k"], w, h, devices=[0, 0], batch=16, queues=2, exchange="share", share=4) as e:
        e.set_inputs(inputs)
        e.run(3)
        assert e.verify() == (0, 16)  # every device composites half of every batch: 4 frames per queue each
        got = e.read_frame(40)
        xb = e.info()["exchange_bytes_per_frame"]
    assert xb < 0.22 * h * w * 2.125, xb  # one sender, 14 of the 68 tile rows
    rows = np.arange(5, 1080, 90)
    ref = oracle_render(scenes["soup100k"], w, h, row_begin=5, row_count=1075, row_step=90)
    assert_parity(got, ref, rows=rows)


def test_engine_stage_times(gpu, scenes):
    w, h = 320, 200
    with engine(scenes["soup2k"], w, h, devices=[0, 0]) as e:
        e.set_inputs(np.full((1, h, w, 2), 0.5, np.float32))
        n, prep, binned, trace = e.stage_times(1, 5)
        assert n == 5 and prep > 0 and binned > 0 and trace > 0
        e.run(1)
        assert e.verify()[0] == 0
