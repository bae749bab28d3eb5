"""Row-band partition of a frame over ranks, and the band gathers to one rank.

Multi-GPU layout (DESIGN.md "Multi-GPU"): rank r of P renders frame rows
[r*B, min(H, (r+1)*B)) with B = ceil(H / P); every rank holds a band buffer of exactly B rows
(the last one padded) so the gather has equal counts; the destination receives the bands in
place into one (P*B)-row buffer and keeps the first H rows. Interleaved bands
(``interleaved_range``) deal the frame's 16-row tile rows round-robin instead, so every rank gets
a share of the dense centre; the gathered layout is then unscrambled by the shading kernel. Inside one process, Renderer
(csrc/renderer.cpp) does the same with ncclGather; across processes (one rank per GPU,
torch.distributed over RCCL/xGMI, or gloo on CPU for tests) this module does it with
``dist.gather``.

Two payloads:
  * ``gather_bands``: the band's RGBA framebuffer rows (16 B per pixel);
  * ``gather_band_ids``: the band's hit ids only (int32, 4 B per pixel), for deferred shading:
    the compositing rank shades the whole frame from the ids (srtShadeAsync), bit-identical to
    shading in the trace, with a quarter of the gather bytes.

Frame k of a stream is composited on ``compositor(k, P)`` (rotating: every rank receives and
shades 1/P of the frames, so every xGMI link carries traffic in both directions) or on rank 0.
"""
from __future__ import annotations


def band_rows(height: int, world: int) -> int:
    return (height + world - 1) // world


def band_range(height: int, world: int, rank: int) -> tuple[int, int]:
    """(row_begin, row_count) of ``rank``'s band; row_count may be 0 for trailing ranks."""
    b = band_rows(height, world)
    begin = min(height, rank * b)
    end = min(height, (rank + 1) * b)
    return begin, end - begin


TILE_ROWS = 16  # include/srt_render.h SRT_TILE_ROWS: interleaved bands deal whole tile rows


def interleaved_range(height: int, world: int, rank: int) -> tuple[int, int]:
    """(row_begin, row_count) of ``rank``'s interleaved band: the frame's 16-row tile rows dealt
    round-robin, rank r holding tile rows r, r + P, r + 2P, ... (srtTraceBatchAsync
    row_interleave = P); row_count may be 0. Balances the work of a frame whose centre is denser
    than its edges, which contiguous bands do not."""
    tiles = (height + TILE_ROWS - 1) // TILE_ROWS
    rows = sum(min(TILE_ROWS, height - t * TILE_ROWS) for t in range(rank, tiles, world))
    return min(height, rank * TILE_ROWS), rows


def interleaved_band_rows(height: int, world: int) -> int:
    """Rows of the largest interleaved band (rank 0's): the gather's per-rank buffer height."""
    return interleaved_range(height, world, 0)[1]


def interleaved_frame_rows(height: int, world: int, rank: int):
    """The frame rows of ``rank``'s interleaved band, in band order (numpy int64)."""
    import numpy as np

    tiles = (height + TILE_ROWS - 1) // TILE_ROWS
    return np.concatenate([np.arange(t * TILE_ROWS, min(height, (t + 1) * TILE_ROWS))
                           for t in range(rank, tiles, world)] or [np.zeros(0, np.int64)]).astype(np.int64)


def compositor(frame: int, world: int, rotate: bool = True) -> int:
    """Rank that gathers and shades frame ``frame``: frame % world when rotating, else 0."""
    return frame % world if rotate else 0


def _gather_into(band, height: int, dst: int, group, out, async_op: bool):
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    b = band_rows(height, world)
    if band.shape[0] != b:
        raise ValueError(f"band buffer must have {b} rows, got {band.shape[0]}")
    # dst is a group rank; torch.distributed wants the global rank
    dst_global = dst if group is None else dist.get_global_rank(group, dst)
    if rank == dst:
        shape = (world * b,) + tuple(band.shape[1:])
        if out is None:
            out = torch.empty(shape, dtype=band.dtype, device=band.device)
        elif tuple(out.shape) != shape or not out.is_contiguous() or out.dtype != band.dtype:
            raise ValueError(f"out must be a contiguous {shape} {band.dtype} buffer")
        parts = [out[r * b:(r + 1) * b] for r in range(world)]
        work = dist.gather(band, gather_list=parts, dst=dst_global, group=group, async_op=async_op)
        return out[:height], work
    work = dist.gather(band, gather_list=None, dst=dst_global, group=group, async_op=async_op)
    return None, work


def gather_bands(band, height: int, dst: int = 0, group=None, out=None):
    """Gather every rank's (B, W, C) band to ``dst``; returns the (H, W, C) frame on dst, else None.

    ``out`` (dst only, optional): a (P * B, W, C) buffer the bands are received into in place
    (its row slices are the gather list, so no concatenation copy); allocated when omitted.
    """
    frame, _ = _gather_into(band, height, dst, group, out, async_op=False)
    return frame


def gather_band_ids(band_ids, height: int, dst: int = 0, group=None, out=None, async_op: bool = False):
    """Gather every rank's (B, W) int32 hit-id band to ``dst`` (deferred shading payload).

    Returns (frame_ids or None, work): the (H, W) id frame on dst (a view of ``out``, received
    in place), and the async work handle (None when synchronous). With ``async_op`` the caller
    must ``work.wait()`` (on the stream that consumes the ids) before using them, and before
    overwriting ``band_ids``.
    """
    import torch

    if band_ids.dtype != torch.int32 or band_ids.dim() != 2:
        raise ValueError("band_ids must be a (B, W) int32 tensor")
    return _gather_into(band_ids, height, dst, group, out, async_op)


def gather_band_batch(batch, height: int, dst: int = 0, group=None, out=None, async_op: bool = False,
                      interleaved: bool = False):
    """Gather F frames' bands in ONE collective: every rank's (F, B, W) int32 hit-id batch
    (frame f's band in batch[f]) to ``dst``, received band-major into (P, F, B, W) — the layout
    srtShadeBandsAsync (DeviceScene.shade_bands) shades in one launch. ``interleaved``: the bands
    are interleaved (interleaved_range), each batch band interleaved_band_rows rows.

    One collective per F frames: a torch-RCCL gather costs ~44 us of host time per call
    (tools/host_probe_bands.py), more than a band's trace, so the band path gathers batches.
    ``out`` (dst only): a buffer of at least P*F*B*W int32 elements (viewed, not copied).
    Returns (ids (P, F, B, W) on dst else None, work)."""
    import torch
    import torch.distributed as dist

    if batch.dtype != torch.int32 or batch.dim() != 3 or not batch.is_contiguous():
        raise ValueError("batch must be a contiguous (F, B, W) int32 tensor")
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    frames, b, width = batch.shape
    want = interleaved_band_rows(height, world) if interleaved else band_rows(height, world)
    if b != want:
        raise ValueError(f"batch bands must have {want} rows, got {b}")
    dst_global = dst if group is None else dist.get_global_rank(group, dst)
    if rank != dst:
        return None, dist.gather(batch, gather_list=None, dst=dst_global, group=group, async_op=async_op)
    need = world * frames * b * width
    if out is None:
        out = torch.empty(need, dtype=batch.dtype, device=batch.device)
    elif out.dtype != batch.dtype or not out.is_contiguous() or out.numel() < need:
        raise ValueError(f"out must be a contiguous int32 buffer of at least {need} elements")
    ids = out.view(-1)[:need].view(world, frames, b, width)
    work = dist.gather(batch, gather_list=list(ids.unbind(0)), dst=dst_global, group=group, async_op=async_op)
    return ids, work
