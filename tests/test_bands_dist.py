"""Row-band partition and the one-process-per-GPU band gather, on CPU with gloo.

Each rank renders its band with the CPU oracle (a test stand-in for the GPU stage) into a
padded band buffer; simpleraytracer_amd.bands.gather_bands assembles the frame on rank 0, which
must equal the single-process frame bit for bit. world_size 2 and 3 (3 exercises the padded
last band, 1080 / 3 is exact but 37 / 3 is not).
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

from simpleraytracer_amd.bands import TILE_ROWS, band_range, band_rows


@pytest.mark.parametrize("h", [1, 2, 7, 37, 135, 1080, 2160])
@pytest.mark.parametrize("p", [1, 2, 3, 4, 7, 8])
def test_band_partition_covers_frame_once(h, p):
    rows = []
    for r in range(p):
        b, c = band_range(h, p, r)
        assert 0 <= c <= band_rows(h, p)
        rows += list(range(b, b + c))
    assert rows == list(range(h))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, scene_path, w, h, out_path):
    import torch
    import torch.distributed as dist

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    from oracle.srt_oracle import OracleScene
    from simpleraytracer_amd.bands import band_range, band_rows, gather_bands

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b0, cnt = band_range(h, world, rank)
    band = torch.zeros((band_rows(h, world), w, 4), dtype=torch.float32)
    if cnt:
        img = OracleScene(scene_path).render(w, h, row_begin=b0, row_count=cnt, threads=1)
        band[:cnt] = torch.from_numpy(img[b0:b0 + cnt])
    frame = gather_bands(band, h, dst=0)
    if rank == 0:
        np.save(out_path, frame.numpy())
    else:
        assert frame is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,wh", [(2, (48, 37)), (3, (40, 37)), (2, (16, 1))])
def test_gloo_band_gather_equals_single_process(scenes, tmp_path, world, wh):
    import torch.multiprocessing as mp

    from oracle.srt_oracle import OracleScene

    w, h = wh
    out = tmp_path / "frame.npy"
    mp.start_processes(_worker, args=(world, _free_port(), scenes["soup300"], w, h, str(out)), nprocs=world,
                       join=True, start_method="spawn")
    got = np.load(out)
    ref = OracleScene(scenes["soup300"]).render(w, h)
    assert got.shape == (h, w, 4)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def _ids_worker(rank, world, port, scene_path, w, h, frames, queues, out_dir):
    """bench.py's multi-GPU band pipeline with CPU stand-ins for the device stages: rank r
    traces band r of every frame (the oracle's ids), the id bands of frame k are gathered on
    process group k % queues to the compositing rank k % world, which shades the frame from the
    ids (the oracle's stage 3, as srtShadeAsync does on the GPU)."""
    import torch
    import torch.distributed as dist

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    from oracle.srt_oracle import OracleScene
    from simpleraytracer_amd.bands import band_range, band_rows, compositor, gather_band_ids

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    groups = [dist.new_group(list(range(world))) for _ in range(queues)]
    oracle = OracleScene(scene_path)
    b0, cnt = band_range(h, world, rank)
    outs = [torch.empty((world * band_rows(h, world), w), dtype=torch.int32) for _ in range(queues)]
    for k in range(frames):
        offs = np.random.default_rng(1000 + k).random((h, w, 2), dtype=np.float32)
        band = torch.full((band_rows(h, world), w), -5, dtype=torch.int32)
        if cnt:
            img = oracle.render(w, h, offs, row_begin=b0, row_count=cnt, threads=1)
            band[:cnt] = torch.from_numpy(img[b0:b0 + cnt, :, 3].astype(np.int32))
        root = compositor(k, world)
        ids, work = gather_band_ids(band, h, dst=root, group=groups[k % queues], out=outs[k % queues],
                                    async_op=True)
        work.wait()
        if rank == root:
            assert ids.shape == (h, w)
            np.save(os.path.join(out_dir, f"frame{k}.npy"), oracle.shade(w, h, ids.numpy(), offs))
        else:
            assert ids is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,wh", [(2, (40, 37)), (3, (33, 29))])
def test_gloo_id_gather_rotating_compositor(scenes, tmp_path, world, wh):
    """Deferred-shading band pipeline (hit-id gather, rotating compositor, one process group per
    frame queue): every frame, wherever it was composited, equals the single-process frame bit
    for bit."""
    import torch.multiprocessing as mp

    from oracle.srt_oracle import OracleScene

    w, h = wh
    frames = 2 * world + 1
    mp.start_processes(_ids_worker, args=(world, _free_port(), scenes["soup300"], w, h, frames, 2, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    oracle = OracleScene(scenes["soup300"])
    for k in range(frames):
        offs = np.random.default_rng(1000 + k).random((h, w, 2), dtype=np.float32)
        got = np.load(tmp_path / f"frame{k}.npy")
        ref = oracle.render(w, h, offs)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), k


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


def _batch_worker(rank, world, port, scene_path, w, h, batches, out_dir):
    """bench.py's batched band path with CPU stand-ins: rank r traces band r of F frames into an
    (F, B, W) batch, ONE gather per batch (gather_band_batch) to the rotating compositor, which
    shades every frame of the batch from the band-major ids."""
    import torch
    import torch.distributed as dist

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    from oracle.srt_oracle import OracleScene
    from simpleraytracer_amd.bands import band_range, band_rows, compositor, gather_band_batch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    oracle = OracleScene(scene_path)
    b0, cnt = band_range(h, world, rank)
    B = band_rows(h, world)
    out = torch.empty(world * max(batches) * B * w, dtype=torch.int32)
    k = 0
    for bi, frames in enumerate(batches):
        batch = torch.full((frames, B, w), -5, dtype=torch.int32)
        offs = [np.random.default_rng(2000 + k + f).random((h, w, 2), dtype=np.float32) for f in range(frames)]
        for f in range(frames):
            if cnt:
                img = oracle.render(w, h, offs[f], row_begin=b0, row_count=cnt, threads=1)
                batch[f, :cnt] = torch.from_numpy(img[b0:b0 + cnt, :, 3].astype(np.int32))
        root = compositor(bi, world)
        ids, work = gather_band_batch(batch, h, dst=root, out=out, async_op=True)
        work.wait()
        if rank == root:
            assert ids.shape == (world, frames, B, w)
            for f in range(frames):
                np.save(os.path.join(out_dir, f"frame{k + f}.npy"),
                        oracle.shade(w, h, band_major_frame(ids.numpy(), f, h), offs[f]))
        else:
            assert ids is None
        k += frames
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,wh", [(2, (40, 37)), (3, (33, 29))])
def test_gloo_batched_id_gather(scenes, tmp_path, world, wh):
    """One collective per batch of frames (full and partial batches): every frame shaded from the
    band-major gather layout equals the single-process frame bit for bit."""
    import torch.multiprocessing as mp

    from oracle.srt_oracle import OracleScene

    w, h = wh
    batches = [3, 1, 2]
    mp.start_processes(_batch_worker, args=(world, _free_port(), scenes["soup300"], w, h, batches, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    oracle = OracleScene(scenes["soup300"])
    k = 0
    for frames in batches:
        for f in range(frames):
            offs = np.random.default_rng(2000 + k + f).random((h, w, 2), dtype=np.float32)
            got = np.load(tmp_path / f"frame{k + f}.npy")
            ref = oracle.render(w, h, offs)
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (k, f)
        k += frames


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


def _interleaved_worker(rank, world, port, scene_path, w, h, frames, out_dir):
    """Interleaved bands over gloo: rank r renders its tile rows (oracle, tile row by tile row)
    of `frames` frames into an (F, B, W) id batch; one gather; rank 0 shades every frame from the
    band-major interleaved layout."""
    import torch
    import torch.distributed as dist

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    from oracle.srt_oracle import OracleScene
    from simpleraytracer_amd.bands import gather_band_batch, interleaved_band_rows, interleaved_frame_rows

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    oracle = OracleScene(scene_path)
    fr = interleaved_frame_rows(h, world, rank)
    B = interleaved_band_rows(h, world)
    batch = torch.full((frames, B, w), -5, dtype=torch.int32)
    offs = [np.random.default_rng(3000 + f).random((h, w, 2), dtype=np.float32) for f in range(frames)]
    for f in range(frames):
        for k in range(0, len(fr), TILE_ROWS):  # one tile row (contiguous frame rows) at a time
            r0, n = int(fr[k]), min(TILE_ROWS, len(fr) - k)
            img = oracle.render(w, h, offs[f], row_begin=r0, row_count=n, threads=1)
            batch[f, k:k + n] = torch.from_numpy(img[r0:r0 + n, :, 3].astype(np.int32))
    ids, work = gather_band_batch(batch, h, dst=0, async_op=True, interleaved=True)
    work.wait()
    if rank == 0:
        for f in range(frames):
            np.save(os.path.join(out_dir, f"frame{f}.npy"),
                    oracle.shade(w, h, interleaved_frame(ids.numpy(), f, h).astype(np.int32), offs[f]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,wh", [(2, (40, 70)), (3, (33, 100))])
def test_gloo_interleaved_batch(scenes, tmp_path, world, wh):
    """Interleaved bands (tile rows dealt round-robin), one gather per batch: every frame shaded
    from the gathered layout equals the single-process frame bit for bit."""
    import torch.multiprocessing as mp

    from oracle.srt_oracle import OracleScene

    w, h = wh
    mp.start_processes(_interleaved_worker, args=(world, _free_port(), scenes["soup300"], w, h, 2, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    oracle = OracleScene(scenes["soup300"])
    for f in range(2):
        offs = np.random.default_rng(3000 + f).random((h, w, 2), dtype=np.float32)
        got = np.load(tmp_path / f"frame{f}.npy")
        assert np.array_equal(got.view(np.uint32), oracle.render(w, h, offs).view(np.uint32)), f


def test_compositor_rotation():
    from simpleraytracer_amd.bands import compositor

    assert [compositor(k, 3) for k in range(7)] == [0, 1, 2, 0, 1, 2, 0]
    assert [compositor(k, 3, rotate=False) for k in range(4)] == [0, 0, 0, 0]
