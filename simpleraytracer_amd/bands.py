"""Row-band partition of a frame over ranks, and the band gather to one rank.

Multi-GPU layout (DESIGN.md "Multi-GPU"): rank r of P renders frame rows
[r*B, min(H, (r+1)*B)) with B = ceil(H / P); every rank holds a band buffer of exactly B rows
(the last one padded) so the gather has equal counts; the destination concatenates the bands
and keeps the first H rows. Inside one process, Renderer (csrc/renderer.cpp) does the same
with ncclGather; across processes (one rank per GPU, torch.distributed over RCCL/xGMI, or
gloo on CPU for tests) this module does it with ``dist.gather``.
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


def gather_bands(band, height: int, dst: int = 0, group=None, out=None):
    """Gather every rank's (B, W, C) band to ``dst``; returns the (H, W, C) frame on dst, else None.

    ``out`` (dst only, optional): a (P * B, W, C) buffer the bands are received into in place
    (its row slices are the gather list, so no concatenation copy); allocated when omitted.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    b = band_rows(height, world)
    if band.shape[0] != b:
        raise ValueError(f"band buffer must have {b} rows, got {band.shape[0]}")
    if rank == dst:
        if out is None:
            out = torch.empty((world * b,) + tuple(band.shape[1:]), dtype=band.dtype, device=band.device)
        elif tuple(out.shape) != (world * b,) + tuple(band.shape[1:]) or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous {(world * b,) + tuple(band.shape[1:])} buffer")
        parts = [out[r * b:(r + 1) * b] for r in range(world)]
        dist.gather(band, gather_list=parts, dst=dst, group=group)
        return out[:height]
    dist.gather(band, gather_list=None, dst=dst, group=group)
    return None
