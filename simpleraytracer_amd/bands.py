"""Row-band partition of a frame over P devices (Python restatement of csrc/engine.cpp BandSplit,
for callers and tests).

Contiguous bands: device r renders frame rows [r*B, min(H, (r+1)*B)) with B = ceil(H / P).
Interleaved bands (the engine's default): the frame's 16-row tile rows are dealt round-robin, so
every device gets a share of the dense centre. Either way every device's band buffer has the same
number of rows (the largest band's), so the exchange moves equal counts; the shading kernel
unscrambles the gathered layout (render.hip ShadeIdsKernel). The exchange itself is native
(the frame engine's RCCL send / receive, or ncclGather in Renderer) -- no Python on the data path.
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


def rotated_band(world: int, device: int, compositor: int) -> int:
    """The contiguous band ``device`` traces of a frame composited on ``compositor`` under the
    rotated all-to-all (csrc/engine.h ExchangePlan::BandOf): (device + compositor) % P, so every
    device traces every band once over P consecutive frames; the compositor's receive buffer holds
    device p's ids at slot (p + c) % P = the band (RecvSlot), i.e. band-major in band order."""
    return (device + compositor) % world


def rotate_own_rows(height: int, pct: int | None = None) -> int:
    """Rows of the compositor's own band (band 0) under the rotated all-to-all over two devices without
    a measured link (csrc/engine.cpp RotateOwnRows): ``pct`` per cent of the frame (env SRT_ROTATE_OWN,
    an integer in 1..99 -- anything else raises ValueError, as the library refuses it --, default 80),
    rounded to whole 16-row tile rows, kept inside [1, H - 1]; the other band takes the rest."""
    import os

    if pct is None:
        v = os.environ.get("SRT_ROTATE_OWN", "")
        if v == "":
            pct = 80
        elif not v.lstrip("+-").isdigit() or not 1 <= int(v) <= 99 or v != v.strip():
            raise ValueError(f"SRT_ROTATE_OWN must be an integer per cent in 1..99, got {v!r}")
        else:
            pct = int(v)
    pct = max(1, min(99, pct))
    rows = (height * pct + 50) // 100
    if height > 2 * TILE_ROWS:
        rows = (rows + TILE_ROWS // 2) // TILE_ROWS * TILE_ROWS
    return max(1, min(rows, height - 1 if height > 1 else 1))


def rotate_split_for_link(height: int, width: int, link_gbs: float, frame_us: float,
                          bytes_per_pixel: float) -> int:
    """The two-device split an engine derives from its measured link (csrc/engine.cpp
    RotateSplitForLink): the smallest own band -- whole tile rows, at least half the frame -- whose
    link time per frame of the job, (H - r) W b / 2 / rate, stays within 80 % of the GPUs' time per
    frame of the job, frame_us (0.553 + 0.25 (H - r) / H) (the rank simulation's P = 2 times over the
    own share); the largest own band (one tile row sent) when none does."""
    t = TILE_ROWS
    if height < 2:
        return 1
    tiled = height > 2 * t
    hi = (height - 1) // t * t if tiled else height - 1
    if not (link_gbs > 0 and frame_us > 0 and bytes_per_pixel > 0):
        return hi
    r = (height + 1) // 2
    if tiled:
        r = (r + t - 1) // t * t
    while r <= hi:
        sent = height - r
        link_us = sent * width * bytes_per_pixel / 2.0 / (link_gbs * 1e3)
        gpu_us = frame_us * (0.553 + 0.25 * sent / height)
        if link_us <= 0.8 * gpu_us:
            return min(r, hi)
        r += t if tiled else 1
    return hi


def rotated_range(height: int, world: int, band: int, first_rows: int = 0) -> tuple[int, int]:
    """(row_begin, row_count) of contiguous band ``band`` when band 0 has ``first_rows`` rows (0: the
    even split of band_range) and the later bands split the rest evenly (csrc/engine.cpp BandSplit
    with first_rows; the engine sets it to rotate_own_rows(H) for two devices)."""
    if first_rows == 0 or world == 1:
        return band_range(height, world, band)
    first = min(first_rows, height)
    step = (height - first + world - 2) // (world - 1)
    begin = 0 if band == 0 else min(height, first + (band - 1) * step)
    return begin, min(height, first + band * step) - begin


def share_auto(height: int, world: int) -> int:
    """The share exchange's default tile rows per cycle (csrc/engine.cpp ShareAuto, srtShareAuto): the
    largest power of two <= 32 whose cycle of share + P - 1 tile rows fits the frame."""
    tiles = (height + TILE_ROWS - 1) // TILE_ROWS
    k = 32
    while k > 1 and k + world - 1 > tiles:
        k //= 2
    return k


def share_frame_rows(height: int, world: int, share: int, rank: int, compositor: int):
    """The frame rows ``rank`` traces, in band order, for a frame composited on ``compositor`` under
    the share exchange (csrc/engine.h kShare): the frame's tile rows in cycles of share + P - 1
    classes; the compositor takes the first ``share`` of every cycle (render.h RowPattern(share +
    P - 1, share)), each other rank one class, in rank order after the compositor (numpy int64)."""
    import numpy as np

    classes = share + world - 1
    tiles = (height + TILE_ROWS - 1) // TILE_ROWS
    if rank == compositor:
        mine = [t for t in range(tiles) if t % classes < share]
    else:
        cls = share + (rank - compositor - 1) % world
        mine = list(range(cls, tiles, classes))
    return np.concatenate([np.arange(t * TILE_ROWS, min(height, (t + 1) * TILE_ROWS)) for t in mine]
                          or [np.zeros(0, np.int64)]).astype(np.int64)


class ExchangePlan:
    """Python restatement of csrc/engine.h ExchangePlan for the per-frame exchanges (all-to-all over
    interleaved, contiguous or rotated bands, and share): which device composites frame f of a batch,
    the frame's slot there, and where a device's ids sit in its send and receive buffers. The tests
    move real band ids between processes with it (tests/test_bands_dist.py) and compare the result
    with the library's own layout (srtExchangeHost / srtExchangeHostShare)."""

    def __init__(self, world: int, batch: int, exchange: str = "alltoall", rows: str = "interleaved"):
        if exchange not in ("alltoall", "share"):
            raise ValueError("per-frame exchanges only: alltoall, share")
        self.world, self.batch, self.exchange = world, batch, exchange
        self.rotate = rows == "rotated" and world > 1

    def compositor(self, f: int) -> int:
        return f % self.world

    def slot(self, f: int) -> int:
        return f // self.world

    def frames_for(self, c: int) -> int:
        return (self.batch - c + self.world - 1) // self.world if c < self.batch else 0

    def max_frames(self) -> int:
        return (self.batch + self.world - 1) // self.world

    def send_frame(self, c: int, j: int) -> int:
        """Band frame index of compositor c's j-th frame in a device's send buffer (SendFrames)."""
        return c * self.max_frames() + j

    def recv_slot(self, c: int, p: int) -> int:
        """Slot of device p's ids in compositor c's receive buffer (RecvSlot)."""
        if self.rotate:
            return rotated_band(self.world, p, c)
        if self.exchange == "share":
            return (p + self.world - c - 1) % self.world
        return p


def traced_rows(height: int, world: int, exchange: str, rows: str, device: int, compositor: int, share: int = 0,
                first_rows: int = 0):
    """The frame rows ``device`` traces, in band order, of a frame composited on ``compositor``
    (rotated: band 0 of ``first_rows`` rows when nonzero -- the engine's two-device split,
    rotate_own_rows -- else even bands)."""
    import numpy as np

    if exchange == "share":
        return share_frame_rows(height, world, share, device, compositor)
    if rows == "interleaved":
        return interleaved_frame_rows(height, world, device)
    band = rotated_band(world, device, compositor) if rows == "rotated" else device
    b, c = rotated_range(height, world, band, first_rows if rows == "rotated" else 0)
    return np.arange(b, b + c, dtype=np.int64)
