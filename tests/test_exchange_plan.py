"""The frame engine's band exchange (csrc/engine.cpp ExchangePlan / BandSplit), on host memory.

srtExchangeHost runs the engine's send / receive layout with copies instead of RCCL: every band's
traced ids of a batch land in each compositor's receive buffer exactly where the device path puts
them ([band][frame of the compositor][buffer rows][W]). Here the receive buffers are unscrambled
with ShadeIdsKernel's index expression (render.hip) restated in numpy, and -- with the oracle
standing in for the GPU trace and shade -- every frame composited anywhere must equal the
single-process frame bit for bit.
"""
from __future__ import annotations

import numpy as np
import pytest

from simpleraytracer_amd.bands import (TILE_ROWS, band_range, band_rows, interleaved_frame_rows, interleaved_range,
                                      rotated_band)
from simpleraytracer_amd.engine import exchange_host


def split_rows(h, p, rows):
    """Frame rows of every band (band order), and the bands' buffer rows."""
    if rows == "interleaved" and p > 1:
        fr = [interleaved_frame_rows(h, p, r) for r in range(p)]
        return fr, max(1, max(len(f) for f in fr)) if p > 1 else h
    fr = []
    for r in range(p):
        b, c = band_range(h, p, r)
        fr.append(np.arange(b, b + c))
    return fr, band_rows(h, p)


def unscramble(recv, g, h, rows):
    """Frame g of a compositor's receive buffer (P, frames, B, W), ShadeIdsKernel's mapping:
    interleaved t = y / 16, band = t % P, local = (t / P) * 16 + y % 16; contiguous band = y / B."""
    p, frames, b, w = recv.shape
    y = np.arange(h)
    if rows == "interleaved" and p > 1:
        t = y // TILE_ROWS
        band, local = t % p, t // p * TILE_ROWS + y % TILE_ROWS
    else:
        band, local = y // b, y % b
    return recv[band, g, local]


def compositor(exchange, p, b, f):
    return {"alltoall": f % p, "rotating": b % p, "root": 0}[exchange]


def slot(exchange, p, f):
    return f // p if exchange == "alltoall" else f


def traced_band(rows, exchange, p, b, d, f):
    """The band device d traces of frame f of batch b (rotated: by the frame's compositor)."""
    return rotated_band(p, d, compositor(exchange, p, b, f)) if rows == "rotated" and p > 1 else d


@pytest.mark.parametrize("rows", ["interleaved", "contiguous", "rotated"])
@pytest.mark.parametrize("exchange", ["alltoall", "rotating", "root"])
@pytest.mark.parametrize("p,h,frames,b", [(1, 37, 3, 0), (2, 70, 4, 1), (3, 37, 8, 2), (4, 170, 3, 5),
                                          (8, 170, 16, 3), (8, 10, 5, 1), (3, 33, 1, 4)])
def test_exchange_layout_reassembles_every_frame(rows, exchange, p, h, frames, b):
    if rows == "rotated" and exchange != "alltoall":
        pytest.skip("rotated bands are an all-to-all layout")
    if rows == "rotated" and p == 2:
        pytest.skip("two devices: the compositor's own band is larger than the buffers "
                    "(test_exchange_host_rotated_two_devices_is_the_engines_split)")
    w = 7
    fr, brows = split_rows(h, p, rows)
    # frame f's "ids": a unique value per (frame, row, column)
    truth = np.arange(frames * h * w, dtype=np.int32).reshape(frames, h, w)
    bands = []
    for r in range(p):
        buf = np.full((frames, brows, w), -7, np.int32)
        for f in range(frames):
            j = traced_band(rows, exchange, p, b, r, f)
            buf[f, :len(fr[j])] = truth[f, fr[j]]
        bands.append(buf)
    recv = exchange_host(bands, h, rows, exchange, batch_index=b)
    seen = set()
    for c in range(p):
        assert recv[c].shape[0] == p and recv[c].shape[2:] == (brows, w)
        for f in range(frames):
            if compositor(exchange, p, b, f) != c:
                continue
            seen.add(f)
            got = unscramble(recv[c], slot(exchange, p, f), h, rows)
            assert np.array_equal(got, truth[f]), (c, f)
    assert seen == set(range(frames))


def test_buffer_rows_match_the_partition_helpers():
    for h in (1, 16, 17, 1080, 2160):
        for p in (1, 2, 3, 8):
            for rows in ("interleaved", "contiguous"):
                want = split_rows(h, p, rows)[1]
                bands = [np.zeros((1, want, 3), np.int32) for _ in range(p)]
                out = exchange_host(bands, h, rows, "root")  # raises if the buffer rows disagree
                assert out[0].shape[2] == want
    for p in (2, 3, 8):
        assert interleaved_range(1080, p, 0)[1] == split_rows(1080, p, "interleaved")[1]


def test_exchange_rejects_wrong_buffers():
    with pytest.raises(ValueError):  # contiguous bands of a 10-row frame over 2 devices have 5 rows
        exchange_host([np.zeros((2, 4, 4), np.int32)] * 2, 10, "contiguous", "alltoall")
    with pytest.raises(KeyError):
        exchange_host([np.zeros((2, 5, 4), np.int32)] * 2, 10, "contiguous", "nope")


@pytest.mark.parametrize("p,rows,exchange", [(2, "interleaved", "alltoall"), (3, "contiguous", "alltoall"),
                                             (4, "interleaved", "rotating"), (3, "interleaved", "root"),
                                             (3, "rotated", "alltoall"), (4, "rotated", "alltoall")])
def test_oracle_batch_through_the_exchange(scenes, p, rows, exchange):
    """The engine's band path with CPU stand-ins: band r of every frame traced by the oracle (hit
    ids), exchanged by srtExchangeHost, each compositor shading its frames from the unscrambled ids
    (the oracle's stage 3, as ShadeIdsKernel does): every frame equals the single-process render."""
    from oracle.srt_oracle import OracleScene

    w, h, frames = 24, 53, 5
    oracle = OracleScene(scenes["soup300"])
    offs = [np.random.default_rng(500 + f).random((h, w, 2), dtype=np.float32) for f in range(frames)]
    refs = [oracle.render(w, h, o, threads=1) for o in offs]
    fr, brows = split_rows(h, p, rows)
    bands = []
    for r in range(p):
        buf = np.full((frames, brows, w), -5, np.int32)
        for f in range(frames):
            j = traced_band(rows, exchange, p, 1, r, f)
            buf[f, :len(fr[j])] = refs[f][fr[j], :, 3].astype(np.int32)
        bands.append(buf)
    recv = exchange_host(bands, h, rows, exchange, batch_index=1)
    for f in range(frames):
        c = compositor(exchange, p, 1, f)
        ids = unscramble(recv[c], slot(exchange, p, f), h, rows)
        got = oracle.shade(w, h, ids, offs[f])
        assert np.array_equal(got.view(np.uint32), refs[f].view(np.uint32)), f


def unscramble_share(recv, g, h, share, own_rows):
    """Frame g of a share compositor's receive buffer (P, frames, B, W), ShadeIdsKernel's mapping
    (ShadeRowOf with own_bands = share over share + P - 1 interleaved classes): row y in tile row
    t = y / 16 is class t % classes; classes below `share` are the compositor's own (traced to RGBA,
    taken from own_rows here), class k >= share is at slot k - share, local row (t / classes) * 16 +
    y % 16."""
    p, frames, b, w = recv.shape
    classes = share + p - 1
    out = np.array(own_rows, copy=True)
    for y in range(h):
        t = y // TILE_ROWS
        k = t % classes
        if k >= share:
            out[y] = recv[k - share, g, (t // classes) * TILE_ROWS + y % TILE_ROWS]
    return out


@pytest.mark.parametrize("p,h,share,frames,b", [(2, 230, 4, 4, 0), (2, 230, 1, 2, 3), (3, 230, 2, 6, 1),
                                                (4, 170, 8, 8, 2), (8, 1080, 32, 16, 0), (8, 230, 2, 8, 5),
                                                (2, 230, 16, 4, 1), (3, 100, 0, 3, 0)])
def test_share_exchange_layout_reassembles_every_frame(p, h, share, frames, b):
    """The share exchange on host memory (srtExchangeHostShare: the engine's ExchangePlan with its
    SendFrames / RecvSlot, the same functions ExchangePhase's ncclSend / ncclRecv offsets and
    CopyPhase's copies take): every sender's class rows of every frame land where the compositor's
    deferred shading reads them; with the compositor's own classes, every frame is whole. share = 16
    at P = 2: a cycle of 17 tile rows is longer than the 15-row frame, so the sender's band is empty;
    share = 0: srtShareAuto."""
    from simpleraytracer_amd.bands import share_auto, share_frame_rows

    w = 5
    k = share or share_auto(h, p)
    truth = np.arange(frames * h * w, dtype=np.int32).reshape(frames, h, w)
    rows = {(d, c): share_frame_rows(h, p, k, d, c) for d in range(p) for c in range(p)}
    brows = max(1, max(len(rows[d, c]) for d in range(p) for c in range(p) if d != c))  # sender classes only
    bands = []
    for d in range(p):
        buf = np.full((frames, brows, w), -7, np.int32)
        for f in range(frames):
            c = f % p
            if d != c:
                buf[f, :len(rows[d, c])] = truth[f, rows[d, c]]
        bands.append(buf)
    recv = exchange_host(bands, h, "interleaved", "share", batch_index=b, share=share)
    for f in range(frames):
        c = f % p
        own = np.full((h, w), -9, np.int32)
        own[rows[c, c]] = truth[f, rows[c, c]]
        got = unscramble_share(recv[c], f // p, h, k, own)
        assert np.array_equal(got, truth[f]), (c, f)


@pytest.mark.parametrize("own", ["", "50", "80", "1", "99", "07"])
def test_rotate_own_rows_matches_library(monkeypatch, own):
    """bands.rotate_own_rows (the Python restatement the bench and the tests use) against the engine's
    RotateOwnRows (srtRotateOwnRows) over frame heights from 1 row to 4K, default and overridden splits."""
    from simpleraytracer_amd import _native
    from simpleraytracer_amd.bands import rotate_own_rows

    if own:
        monkeypatch.setenv("SRT_ROTATE_OWN", own)
    else:
        monkeypatch.delenv("SRT_ROTATE_OWN", raising=False)
    lib = _native.lib()
    for h in list(range(1, 70)) + [100, 135, 1079, 1080, 2160, 4321]:
        assert lib.srtRotateOwnRows(h) == rotate_own_rows(h), (own, h)
        assert 1 <= rotate_own_rows(h) <= max(1, h - 1)


@pytest.mark.parametrize("own", ["150", "-5", "0", "abc", "80%", " 80", "8e1"])
def test_rotate_own_rows_rejects_junk(monkeypatch, own):
    """SRT_ROTATE_OWN is parsed strictly (strtol turned junk into 0, clamped to 1 %, so about
    99 % of every frame silently crossed the link): the library returns 0 with the reason in
    srtGetLastError, the restatement raises -- and an engine refuses to start with it."""
    from simpleraytracer_amd import _native
    from simpleraytracer_amd.bands import rotate_own_rows

    monkeypatch.setenv("SRT_ROTATE_OWN", own)
    lib = _native.lib()
    assert lib.srtRotateOwnRows(1080) == 0
    assert "SRT_ROTATE_OWN must be an integer per cent in 1..99" in _native.last_error()
    with pytest.raises(ValueError):
        rotate_own_rows(1080)


@pytest.mark.parametrize("h", [1080, 2160, 100, 61])
def test_exchange_host_rotated_two_devices_is_the_engines_split(monkeypatch, h):
    """srtExchangeHost over two devices with rotated rows lays out the engine's split (it
    reported even halves while the engine used the 4/5 split): buffer rows = the sent band 1 = H -
    rotate_own_rows(H), and every frame reassembles from the compositor's own band plus the received
    band 1 with the shading kernel's index expressions."""
    from simpleraytracer_amd.bands import rotate_own_rows, rotated_range

    monkeypatch.delenv("SRT_ROTATE_OWN", raising=False)
    p, frames, w = 2, 4, 3
    own = rotate_own_rows(h)
    truth = np.arange(frames * h * w, dtype=np.int32).reshape(frames, h, w)
    brows = h - own
    bands = []
    for d in range(p):
        buf = np.full((frames, brows, w), -7, np.int32)
        for f in range(frames):
            c = f % p
            if d != c:  # band 1 of a frame composited on the other device
                b0, n = rotated_range(h, p, 1, own)
                assert (b0, n) == (own, brows)
                buf[f] = truth[f, b0:b0 + n]
        bands.append(buf)
    recv = exchange_host(bands, h, "rotated", "alltoall")
    for c in range(p):
        assert recv[c].shape == (p, frames // p, brows, w)
    for f in range(frames):
        c = f % p
        got = np.full((h, w), -9, np.int32)
        got[:own] = truth[f, :own]                       # the compositor's band 0, traced to RGBA in place
        got[own:] = recv[c][1, f // p]                   # band 1 at RecvSlot(c, other) = BandOf = 1
        assert np.array_equal(got, truth[f]), f


def test_rotate_split_for_link_matches_restatement_and_keeps_the_link_off_the_bound():
    """The two-device split from a measured link (srtRotateSplitForLink, the engine's choice when neither
    an option nor SRT_ROTATE_OWN sets it) over link rates 20 .. 150 GB/s: equal to the Python
    restatement, whole tile rows, at least half the frame, more of the frame kept as the link slows, and
    at the chosen split the modelled link time within 80 % of the GPU time (unless even one tile row sent
    is too much). 1080p C3 figures: one-GPU frame 16.96 us, packed ids 2.125 B per pixel."""
    from simpleraytracer_amd import _native
    from simpleraytracer_amd.bands import TILE_ROWS, rotate_split_for_link

    lib = _native.lib()
    for h, w, frame_us, bpp in ((1080, 1920, 16.96, 2.125), (2160, 3840, 144.7, 2.5), (100, 130, 3.0, 4.0),
                                (61, 64, 1.0, 2.125), (1, 8, 1.0, 4.0)):
        prev = None
        for gbs in list(range(20, 151, 5)) + [0.0, -1.0, 1e9]:
            r = lib.srtRotateSplitForLink(h, w, float(gbs), frame_us, bpp)
            assert r == rotate_split_for_link(h, w, float(gbs), frame_us, bpp), (h, gbs)
            assert 1 <= r <= max(1, h - 1)
            if h > 2 * TILE_ROWS:
                assert r % TILE_ROWS == 0 and r >= h // 2
            if 0 < gbs < 1e9:
                sent = h - r
                link = sent * w * bpp / 2 / (gbs * 1e3)
                gpu = frame_us * (0.553 + 0.25 * sent / h)
                hi = (h - 1) // TILE_ROWS * TILE_ROWS if h > 2 * TILE_ROWS else h - 1
                assert link <= 0.8 * gpu or r == hi, (h, gbs, r)
                if prev is not None:
                    assert r <= prev, (h, gbs)  # a faster link never keeps more of the frame
                prev = r
    # the 1080p soup: the split the engine would pick on a link of 64 GB/s (the DESIGN.md assumption), on
    # the RCCL point-to-point peak of a link (~130 GB/s) and on a slow 20 GB/s one
    assert [rotate_split_for_link(1080, 1920, g, 16.96, 2.125) for g in (20, 64, 130)] == [1008, 832, 544]
