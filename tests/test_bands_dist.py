"""Row-band partition (simpleraytracer_amd.bands, the Python restatement of csrc/engine.cpp
BandSplit), the shading kernel's unscrambling of gathered bands, bench.py's multi-rank control
plane on CPU with gloo (world size 2 and 3: the RCCL unique id shared from rank 0, max-over-ranks
timing and the per-rank report gather), and the band data plane over gloo (world sizes 2 and 3):
real band ids moved between processes in the engine's all-to-all and share layouts, the oracle
standing in for the GPU stages, checked against the library's layout and the single-process frame.
The product data path is native (tests/test_exchange_plan.py on host memory, tests/test_gpu_engine.py
on the GPU).
"""
from __future__ import annotations

import os
import socket
import sys
from types import SimpleNamespace

import numpy as np
import pytest

from simpleraytracer_amd.bands import TILE_ROWS, band_range, band_rows

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("h", [1, 2, 7, 37, 135, 1080, 2160])
@pytest.mark.parametrize("p", [1, 2, 3, 4, 7, 8])
def test_band_partition_covers_frame_once(h, p):
    rows = []
    for r in range(p):
        b, c = band_range(h, p, r)
        assert 0 <= c <= band_rows(h, p)
        rows += list(range(b, b + c))
    assert rows == list(range(h))


def band_major_frame(ids, g, height):
    """Frame g of a band-major batch ids[band][frame][band_rows][width], by ShadeIdsKernel's
    index expression (render.hip): at = ((band * frames + g) * band_rows + y % band_rows) * W + x."""
    bands, frames, b, w = ids.shape
    flat = np.asarray(ids).reshape(-1)
    y = np.arange(height)[:, None]
    x = np.arange(w)[None, :]
    band = y // b
    at = ((band * frames + g) * b + (y - band * b)) * w + x
    return flat[at]


def test_band_major_layout_matches_concatenation():
    ids = np.arange(3 * 4 * 5 * 6).reshape(3, 4, 5, 6)  # 3 bands x 4 frames x 5 rows x 6 cols
    for g in range(4):
        want = np.concatenate([ids[p, g] for p in range(3)])[:13]
        assert np.array_equal(band_major_frame(ids, g, 13), want)


@pytest.mark.parametrize("h", [1, 31, 32, 33, 170, 1080, 2160])
@pytest.mark.parametrize("p", [1, 2, 3, 4, 8, 40])
def test_interleaved_partition_covers_frame_once(h, p):
    from simpleraytracer_amd.bands import interleaved_band_rows, interleaved_frame_rows, interleaved_range

    rows = np.concatenate([interleaved_frame_rows(h, p, r) for r in range(p)])
    assert np.array_equal(np.sort(rows), np.arange(h))
    for r in range(p):
        begin, count = interleaved_range(h, p, r)
        fr = interleaved_frame_rows(h, p, r)
        assert count == len(fr) <= interleaved_band_rows(h, p)
        if count:
            assert begin == r * TILE_ROWS == fr[0]
            local = np.arange(count)  # the kernels' FrameRow(row_begin, P, local)
            assert np.array_equal(begin + local + local // TILE_ROWS * TILE_ROWS * (p - 1), fr)


@pytest.mark.parametrize("h", [1, 16, 17, 100, 230, 500, 1080, 2160])
@pytest.mark.parametrize("p", [1, 2, 3, 4, 8, 16])
def test_share_auto_matches_library(h, p):
    """The default k of the share exchange (engine.cpp ShareAuto through srtShareAuto; no device) is
    the largest power of two <= 32 whose cycle of k + P - 1 tile rows fits the frame (at least 1),
    and the Python restatement (bands.share_auto) agrees."""
    from simpleraytracer_amd import _native
    from simpleraytracer_amd.bands import share_auto

    k = _native.lib().srtShareAuto(h, p)
    tiles = -(-h // TILE_ROWS)
    assert k == share_auto(h, p)
    assert k in (1, 2, 4, 8, 16, 32)
    assert k == 1 or k + p - 1 <= tiles
    assert k == 32 or 2 * k + p - 1 > tiles
    if (h, p) in ((1080, 2), (1080, 8), (2160, 8)):
        assert k == 32


@pytest.mark.parametrize("h", [1, 31, 230, 1080, 2160])
@pytest.mark.parametrize("p,share", [(2, 1), (2, 4), (2, 8), (3, 2), (8, 2), (3, 4), (2, 32), (8, 32), (4, 16)])
def test_share_partition_covers_frame_once(h, p, share):
    """The share exchange (engine.h kShare): for every compositor the ranks' rows partition the frame;
    the compositor's rows follow the grouped row pattern the kernels use (render.h BandFrameRow with
    RowPattern(share + P - 1, share)), each sender's a plain interleave of share + P - 1."""
    from simpleraytracer_amd.bands import share_frame_rows

    classes = share + p - 1
    for c in range(p):
        parts = [share_frame_rows(h, p, share, r, c) for r in range(p)]
        assert np.array_equal(np.sort(np.concatenate(parts)), np.arange(h))
        local = np.arange(len(parts[c]))
        lt, g = local // TILE_ROWS, share.bit_length() - 1  # the kernels' shift and mask (share = 2^g)
        assert np.array_equal(((lt >> g) * classes + (lt & (share - 1))) * TILE_ROWS + local % TILE_ROWS, parts[c])
        for r in range(p):
            if r != c and len(parts[r]):
                cls = share + (r - c - 1) % p
                lr = np.arange(len(parts[r]))
                begin = cls * TILE_ROWS
                assert np.array_equal(begin + lr + lr // TILE_ROWS * TILE_ROWS * (classes - 1), parts[r])


def interleaved_frame(ids, g, height):
    """Frame g of a band-major batch of interleaved bands, by ShadeIdsKernel's interleaved index
    expression (render.hip): t = y / T, band = t % P, local = (t / P) * T + y % T (T = TILE_ROWS)."""
    bands, frames, b, w = ids.shape
    y = np.arange(height)
    t = y // TILE_ROWS
    band, local = t % bands, t // bands * TILE_ROWS + y % TILE_ROWS
    return np.asarray(ids)[band, g, local]


def test_interleaved_layout_matches_partition():
    from simpleraytracer_amd.bands import interleaved_band_rows, interleaved_frame_rows

    h, w, p, frames = 170, 5, 3, 2
    frame = np.arange(frames * h * w).reshape(frames, h, w)
    b = interleaved_band_rows(h, p)
    ids = np.full((p, frames, b, w), -1)
    for r in range(p):
        fr = interleaved_frame_rows(h, p, r)
        ids[r, :, :len(fr)] = frame[:, fr]
    for g in range(frames):
        assert np.array_equal(interleaved_frame(ids, g, h), frame[g])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _job_worker(rank, world, port, out_dir):
    """bench.py's Job as torch.distributed.run starts it (env://, one rank per GPU): gloo control
    plane, the unique id from rank 0, max-over-ranks and the report gather."""
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import bench

    job = bench.Job(SimpleNamespace(gpus=world))
    assert job.ranked and job.launch == "torchrun" and job.world == world and job.devices == [rank]
    uid = job.share_uid(lambda: bytes(range(128)))
    assert uid == bytes(range(128))
    assert job.max_over_ranks(float(rank) + 0.5) == world - 0.5
    assert job.gather([rank, 10 * rank]) == [[r, 10 * r] for r in range(world)]
    job.barrier()
    open(os.path.join(out_dir, f"ok{rank}"), "w").close()
    job.close()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_job_control_plane_gloo(tmp_path, world):
    import torch.multiprocessing as mp

    mp.start_processes(_job_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    assert sorted(os.listdir(tmp_path)) == [f"ok{r}" for r in range(world)]


def test_bench_job_single_process(monkeypatch):
    """No launcher: one process for every GPU (devices 0..N-1, or GPU 0 repeated for the one-GPU
    rehearsal); a WORLD_SIZE that contradicts --gpus is refused."""
    sys.path.insert(0, REPO)
    import bench

    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "SRT_BENCH_ONE_DEVICE"):
        monkeypatch.delenv(k, raising=False)
    job = bench.Job(SimpleNamespace(gpus=4))
    assert not job.ranked and job.launch == "single-process" and job.devices == [0, 1, 2, 3]
    assert job.max_over_ranks(1.5) == 1.5 and job.gather([1]) == [[1]]
    job.close()
    monkeypatch.setenv("SRT_BENCH_ONE_DEVICE", "1")
    job = bench.Job(SimpleNamespace(gpus=3))
    assert job.devices == [0, 0, 0]
    job.close()
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit):
        bench.Job(SimpleNamespace(gpus=4))


def _rows_ids(oracle, w, h, offs, rows):
    """The oracle standing in for a rank's trace: hit ids of `rows` (band order), rendering only them
    (one oracle call per run of consecutive rows)."""
    out = np.full((len(rows), w), -3, np.int32)
    i = 0
    while i < len(rows):
        j = i
        while j + 1 < len(rows) and rows[j + 1] == rows[j] + 1:
            j += 1
        fr = oracle.render(w, h, offs, row_begin=int(rows[i]), row_count=j - i + 1, threads=1)
        out[i:j + 1] = fr[rows[i]:rows[j] + 1, :, 3].astype(np.int32)
        i = j + 1
    return out


def _data_plane_worker(rank, world, port, out_dir, scene, exchange, rows_mode, share):
    """One rank of a world-size job moving real band ids over gloo in the engine's layout (the
    restated ExchangePlan: send regions per compositor, receive slots per sender), the oracle standing
    in for the GPU trace and the deferred shading. Checks: the receive buffer equals the library's
    own layout of every rank's bands (srtExchangeHost / srtExchangeHostShare), and every frame this
    rank composites equals the single-process render bit for bit."""
    sys.path.insert(0, REPO)
    import torch
    import torch.distributed as dist

    from oracle.srt_oracle import OracleScene
    from simpleraytracer_amd.bands import ExchangePlan, rotate_own_rows, share_auto, traced_rows
    from simpleraytracer_amd.engine import exchange_host

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w, h, F = 21, 70, 2 * world
    k = (share or share_auto(h, world)) if exchange == "share" else 0
    plan = ExchangePlan(world, F, exchange, rows_mode)
    oracle = OracleScene(scene)
    offs = [np.random.default_rng(900 + f).random((h, w, 2), dtype=np.float32) for f in range(F)]
    # rotated over two devices: the compositor's band 0 takes the engine's default split (4/5 of the frame,
    # srtExchangeHost's layout; ADVICE r05: this test used to trace even halves there)
    first = rotate_own_rows(h) if rows_mode == "rotated" and world == 2 else 0
    rows = {(d, c): traced_rows(h, world, exchange, rows_mode, d, c, k, first) for d in range(world)
            for c in range(world)}
    # the compositor's own rows travel (to itself) only where its band fits the buffers: not under share, nor
    # rotated over two devices (band 0 is larger than the band buffer, first_sent = 1)
    own_sent = exchange != "share" and not first
    senders = [(d, c) for d in range(world) for c in range(world) if d != c or own_sent]
    brows = max(1, max(len(rows[d, c]) for d, c in senders))
    # this rank's traces of the batch, frame-major (the engine's trace phase; its own frames too)
    mine = np.full((F, brows, w), -7, np.int32)
    for f in range(F):
        c = plan.compositor(f)
        if c != rank or own_sent:
            r = rows[rank, c]
            mine[f, :len(r)] = _rows_ids(oracle, w, h, offs[f], r)
    send = np.full((world * plan.max_frames(), brows, w), -7, np.int32)
    for f in range(F):
        send[plan.send_frame(plan.compositor(f), plan.slot(f))] = mine[f]
    n = plan.frames_for(rank)
    recv = np.full((world, n, brows, w), -1, np.int32)
    # the exchange: one send / receive pair per peer (the engine's ncclSend / ncclRecv group)
    reqs, bufs = [], {}
    for p in range(world):
        if p == rank:
            if exchange != "share":
                recv[plan.recv_slot(rank, rank)] = send[plan.send_frame(rank, 0):plan.send_frame(rank, 0) + n]
            continue
        n_p = plan.frames_for(p)
        s0 = plan.send_frame(p, 0)
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(send[s0:s0 + n_p])), dst=p))
        bufs[p] = torch.empty((n, brows, w), dtype=torch.int32)
        reqs.append(dist.irecv(bufs[p], src=p))
    for q in reqs:
        q.wait()
    for p, t in bufs.items():
        recv[plan.recv_slot(rank, p)] = t.numpy()
    # the library's layout of every rank's bands must be what arrived
    every = [None] * world
    dist.all_gather_object(every, mine)
    lib = exchange_host(every, h, rows_mode if exchange != "share" else "interleaved", exchange, share=k)
    if exchange == "share":  # the slot of the compositor itself is not a sender's: not compared
        assert np.array_equal(lib[rank][:world - 1], recv[:world - 1])
    else:
        assert np.array_equal(lib[rank], recv)
    # deferred shading of this rank's frames from the received ids (and its own rows)
    for f in range(rank, F, world):
        ref = oracle.render(w, h, offs[f], threads=1)
        ids = np.full((h, w), -5, np.int32)
        for d in range(world):
            r = rows[d, rank]
            if d == rank:
                ids[r] = ref[r, :, 3].astype(np.int32)  # the compositor's own rows, traced to RGBA
            else:
                ids[r] = recv[plan.recv_slot(rank, d), plan.slot(f), :len(r)]
        got = oracle.shade(w, h, ids, offs[f])
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (rank, f)
    dist.barrier()
    open(os.path.join(out_dir, f"ok{rank}"), "w").close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("exchange,rows,share", [("alltoall", "interleaved", 0), ("alltoall", "rotated", 0),
                                                 ("alltoall", "contiguous", 0), ("share", "interleaved", 0),
                                                 ("share", "interleaved", 1)])
def test_band_data_plane_over_gloo(tmp_path, scenes, world, exchange, rows, share):
    """The multi-process band data plane on CPU (world sizes 2 and 3): real band ids move between
    processes over gloo in the engine's all-to-all (interleaved, contiguous, rotated) and share
    layouts, the oracle standing in for the GPU stages; every composited frame equals the
    single-process render (the device path of the same layout: tests/test_gpu_engine.py)."""
    import torch.multiprocessing as mp

    mp.start_processes(_data_plane_worker,
                       args=(world, _free_port(), str(tmp_path), scenes["soup300"], exchange, rows, share),
                       nprocs=world, join=True, start_method="spawn")
    assert sorted(os.listdir(tmp_path)) == [f"ok{r}" for r in range(world)]
