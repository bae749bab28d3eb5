"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the same inputs.

Bar (DESIGN.md "Parity"): triangle ids (alpha channel, float(tri_id)) bit-exact; RGB
per-channel |delta| <= 1e-5. Sizes are chosen so the oracle finishes in seconds; the full
1080p headline frame is checked on a row sample plus size-independent properties.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from scenefile import write_custom_scene

pytestmark = pytest.mark.gpu

RGB_TOL = 1e-5
VARIANTS = ("lds", "scalar", "cull", "bvh")
# cull variant modes: (SRT_CULL_BIN, SRT_CULL_CHUNK, SRT_CULL_BIN_CAP): bin lists on / off,
# candidates per trace work item (64: heavy tiles split into many items), forced list overflow
CULL_MODES = (("1", "", ""), ("1", "64", ""), ("0", "", ""), ("1", "", "8"), ("1", "64", "8"), ("1", "128", ""))


def set_cull_mode(monkeypatch, mode):
    binning, chunk, cap = mode
    monkeypatch.setenv("SRT_CULL_BIN", binning)
    monkeypatch.setenv("SRT_CULL_CHUNK", chunk)
    if cap:
        monkeypatch.setenv("SRT_CULL_BIN_CAP", cap)
    else:
        monkeypatch.delenv("SRT_CULL_BIN_CAP", raising=False)


def oracle_render(path, w, h, offsets=None, **kw):
    from oracle.srt_oracle import OracleScene

    return OracleScene(path).render(w, h, offsets, **kw)


def assert_parity(got, ref, rows=None):
    if rows is not None:
        got, ref = got[rows], ref[rows]
    ids_got = got[..., 3].view(np.uint32)
    ids_ref = ref[..., 3].view(np.uint32)
    bad = np.argwhere(ids_got != ids_ref)
    assert bad.size == 0, f"{len(bad)} tri_id mismatches, first at {bad[:5].tolist()}: " \
                          f"gpu {got[..., 3][tuple(bad[0])]} oracle {ref[..., 3][tuple(bad[0])]}"
    nan_got, nan_ref = np.isnan(got[..., :3]), np.isnan(ref[..., :3])
    assert np.array_equal(nan_got, nan_ref), "NaN rgb positions differ"
    d = np.abs(np.where(nan_ref, 0.0, got[..., :3] - ref[..., :3]))
    assert float(d.max(initial=0.0)) <= RGB_TOL, f"max rgb delta {d.max()}"


def torch_render(path, w, h, offsets=None, variant="cull", bands=None):
    """DeviceScene path (srtPrepareAsync + srtTraceAsync) on device-resident torch buffers."""
    import torch

    import simpleraytracer_amd as srt

    scene = srt.DeviceScene(path, 0)
    stream = torch.cuda.current_stream()
    scene.prepare(w, h, stream)
    off = torch.full((h, w, 2), 0.5, dtype=torch.float32, device="cuda") if offsets is None else \
        torch.from_numpy(np.ascontiguousarray(offsets, np.float32)).cuda()
    out = torch.full((h, w, 4), float("nan"), dtype=torch.float32, device="cuda")
    if bands is None:
        scene.trace(off, out, 0, h, variant=variant, stream=stream)
    else:
        start = 0
        for rows in bands:
            rows = min(rows, h - start)
            o_band = off[start:start + rows].contiguous()
            r_band = torch.empty((rows, w, 4), dtype=torch.float32, device="cuda")
            scene.trace(o_band, r_band, start, rows, variant=variant, stream=stream)
            out[start:start + rows] = r_band
            start += rows
            if start >= h:
                break
    torch.cuda.synchronize()
    res = out.cpu().numpy()
    scene.close()
    return res


def test_c1_single_triangle_256_ml_api(gpu, scenes):
    import simpleraytracer_amd as srt

    got = srt.render(scenes["triangle"], 256, 256)
    ref = oracle_render(scenes["triangle"], 256, 256)
    assert_parity(got, ref)
    assert (got[..., 3] == 0).sum() > 1000 and (got[..., 3] == -1).sum() > 1000


def test_c2_cornell_1080p_ml_api(gpu, scenes):
    import simpleraytracer_amd as srt

    got = srt.render(scenes["cornell"], 1920, 1080)
    ref = oracle_render(scenes["cornell"], 1920, 1080)
    assert_parity(got, ref)
    assert set(np.unique(got[..., 3]).astype(int)) >= set(range(12))


@pytest.mark.parametrize("variant", VARIANTS)
def test_c3_soup100k_1080p_row_sample(gpu, scenes, variant):
    """Headline config: full 1920x1080 frame on the GPU, checked on 24 rows spread over it."""
    got = torch_render(scenes["soup100k"], 1920, 1080, variant=variant)
    rows = np.arange(3, 1080, 45)
    ref = oracle_render(scenes["soup100k"], 1920, 1080, row_begin=3, row_count=1077, row_step=45)
    assert_parity(got, ref, rows=rows)
    ids = got[..., 3]
    assert np.all((ids >= -1) & (ids < 100_000)) and np.all(ids == np.round(ids))
    hit = ids >= 0
    assert 0.05 < hit.mean() < 0.9
    assert np.all(got[hit][:, :3] >= 0) and np.all(got[hit][:, :3] <= 1.0)


@pytest.mark.parametrize("variant", VARIANTS)
def test_soup_random_offsets_full_frame(gpu, scenes, variant):
    rng = np.random.default_rng(1234)
    w, h = 331, 187  # not multiples of the 64-column / 8- and 32-row tiles
    offsets = rng.random((h, w, 2), dtype=np.float32)
    got = torch_render(scenes["soup2k"], w, h, offsets, variant=variant)
    ref = oracle_render(scenes["soup2k"], w, h, offsets)
    assert_parity(got, ref)


def test_mixed_offsets_exercise_both_loop_bodies(gpu, scenes):
    """Offsets constant in some columns, random in others: blocks take both the shared-fx and
    the general loop body; both must agree with the oracle."""
    rng = np.random.default_rng(99)
    w, h = 256, 96
    offsets = np.full((h, w, 2), 0.5, np.float32)
    offsets[:, 64:128, 0] = rng.random((h, 64), dtype=np.float32)
    offsets[:48, 192:, 1] = rng.random((48, 64), dtype=np.float32)
    for variant in VARIANTS:
        got = torch_render(scenes["soup300"], w, h, offsets, variant=variant)
        ref = oracle_render(scenes["soup300"], w, h, offsets)
        assert_parity(got, ref)


@pytest.mark.parametrize("wh", [(1, 1), (1, 300), (300, 1), (65, 33), (64, 32), (97, 61)])
def test_odd_sizes(gpu, scenes, wh):
    w, h = wh
    for variant in VARIANTS:
        got = torch_render(scenes["soup300"], w, h, variant=variant)
        ref = oracle_render(scenes["soup300"], w, h)
        assert_parity(got, ref)


@pytest.mark.parametrize("variant", VARIANTS)
def test_band_split_is_bitwise_identical(gpu, scenes, variant):
    full = torch_render(scenes["soup2k"], 320, 240, variant=variant)
    banded = torch_render(scenes["soup2k"], 320, 240, bands=[7, 33, 1, 64, 200], variant=variant)
    assert np.array_equal(full.view(np.uint32), banded.view(np.uint32))


def test_variants_bitwise_identical_1080p(gpu, scenes):
    """The three trace kernels produce the same frame, bit for bit (headline config)."""
    frames = [torch_render(scenes["soup100k"], 1920, 1080, variant=v) for v in VARIANTS]
    for f in frames[1:]:
        assert np.array_equal(frames[0].view(np.uint32), f.view(np.uint32))


@pytest.mark.parametrize("mode", CULL_MODES)
def test_cull_modes(gpu, scenes, monkeypatch, mode):
    """Every cull mode (bin lists on/off, split work items, forced bin-list overflow) against
    the oracle, with uniform and random offsets, on a frame that leaves partial tiles; and the
    same frame traced as uneven row bands (a band's bin pass writes only the cull records that
    can reach its rows; with forced overflow its tiles stream every record) bit for bit."""
    set_cull_mode(monkeypatch, mode)
    rng = np.random.default_rng(5)
    w, h = 200, 150
    for offsets in (None, rng.random((h, w, 2), dtype=np.float32)):
        got = torch_render(scenes["soup2k"], w, h, offsets, variant="cull")
        assert_parity(got, oracle_render(scenes["soup2k"], w, h, offsets))
        banded = torch_render(scenes["soup2k"], w, h, offsets, variant="cull", bands=[37, 1, 50, 62])
        assert np.array_equal(banded.view(np.uint32), got.view(np.uint32))


def test_cull_setup_state_across_frames(gpu, scenes):
    """The per-frame setup hands off between blocks through self-resetting state (tile-box
    accumulators and the last tile block's bounds, the bin blocks' arrival count and the last
    bin block's work list): one scene over frames whose band shape (one cull arena per shape, at
    most four: seven shapes re-carve the least recently used ones) and offsets (uniform, random,
    far outside the frame, NaN) change, each frame bit-identical to a fresh brute-force render,
    twice in a row."""
    import torch

    import simpleraytracer_amd as srt

    w, h = 333, 170
    rng = np.random.default_rng(29)
    far = np.full((h, w, 2), -3.25, np.float32)
    nan = rng.random((h, w, 2), dtype=np.float32)
    nan[5:40, 70:90] = np.nan
    cases = [(0, h, None), (40, 77, rng.random((h, w, 2), dtype=np.float32)), (0, h, far), (17, 1, None),
             (0, h, nan), (5, 33, None), (60, 100, rng.random((h, w, 2), dtype=np.float32)), (100, 16, None),
             (3, 150, far), (40, 77, None), (0, h, None)]
    scene = srt.DeviceScene(scenes["soup2k"], 0)
    stream = torch.cuda.current_stream()
    for rep in range(2):
        for k, (r0, rows, offs) in enumerate(cases):
            o = np.full((h, w, 2), 0.5, np.float32) if offs is None else offs
            ref = torch_render(scenes["soup2k"], w, h, o, variant="lds")[r0:r0 + rows]
            off = torch.from_numpy(np.ascontiguousarray(o[r0:r0 + rows])).cuda()
            out = torch.full((rows, w, 4), float("nan"), dtype=torch.float32, device="cuda")
            scene.prepare(w, h, stream)
            scene.trace(off, out, r0, rows, variant="cull", stream=stream)
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32)), (rep, k)
    scene.close()


@pytest.mark.parametrize("mode", CULL_MODES[:4])
@pytest.mark.parametrize("offset", [0.5, 0.0, 0.999, -3.25, 7.5])
def test_cull_uniform_offsets(gpu, scenes, monkeypatch, mode, offset):
    """Uniform (per-frame constant) sample offsets, including ones that push rays outside
    the frame and outside the screen-box range (|fx| > 4: no box culling)."""
    set_cull_mode(monkeypatch, mode)
    w, h = 211, 97
    offsets = np.full((h, w, 2), offset, np.float32)
    ref = oracle_render(scenes["soup2k"], w, h, offsets)
    assert_parity(torch_render(scenes["soup2k"], w, h, offsets, variant="cull"), ref)


def test_cull_survivor_overflow_and_ties(gpu, tmp_path, monkeypatch):
    """Every record survives the block cull (large overlapping triangles, many exact
    duplicates spread over several cull steps): survivor lists fill and flush repeatedly,
    and equal-t ties across lists must still resolve to the lowest id."""
    rng = np.random.default_rng(17)
    big = [-2, -2, 3, 2, -2, 3, 0, 2, 3]
    tris = []
    for i in range(5000):
        if i % 7 == 3:
            tris.append(big)  # exact duplicates: ids 3, 10, 17, ... tie everywhere
        else:
            c = rng.uniform([-1, -1, 3.9], [1, 1, 6])
            tris.append(list((c + rng.uniform(-0.8, 0.8, (3, 3))).ravel()))
    albedo = rng.uniform(0.2, 1.0, (len(tris), 3))
    path = write_custom_scene(tmp_path / "dense.srt", tris, albedo)
    ref = oracle_render(path, 96, 80)
    assert (ref[..., 3] == 3).mean() > 0.3
    for mode in CULL_MODES:
        set_cull_mode(monkeypatch, mode)
        assert_parity(torch_render(path, 96, 80, variant="cull"), ref)
    # 3 super-tiles per row, every record in each: the bin kernel's LDS pair buffer overflows
    # (pairs then go straight to the global lists) and the lists exceed small capacities.
    ref = oracle_render(path, 300, 40)
    for mode in CULL_MODES:
        set_cull_mode(monkeypatch, mode)
        assert_parity(torch_render(path, 300, 40, variant="cull"), ref)
    assert_parity(torch_render(path, 300, 40, variant="bvh"), ref)


def nasty_scene(tmp_path):
    """Triangles around and behind the eye, crossing the camera plane, slivers, needles, huge and tiny
    ones, near edge-on (test_cull_nasty_geometry; also the band skip tests)."""
    rng = np.random.default_rng(23)
    tris = []
    for _ in range(600):  # crossing / behind / around the eye
        tris.append(list(rng.uniform(-3, 3, 9)))
    for _ in range(600):  # slivers and needles in front
        a = rng.uniform([-1, -1, 1], [1, 1, 4])
        d = rng.normal(size=3)
        b = a + d * rng.uniform(0.01, 2.0)
        c = a + d * rng.uniform(0.01, 2.0) + rng.normal(size=3) * 10.0 ** rng.uniform(-6, -2)
        tris.append(list(np.concatenate([a, b, c])))
    for _ in range(300):  # tiny, far and near
        a = rng.uniform([-1, -1, 0.05], [1, 1, 50])
        tris.append(list(np.concatenate([a, a + rng.normal(size=3) * 1e-3, a + rng.normal(size=3) * 1e-3])))
    albedo = rng.uniform(0.2, 1.0, (len(tris), 3))
    return write_custom_scene(tmp_path / "nasty.srt", tris, albedo)


def test_cull_nasty_geometry(gpu, tmp_path, monkeypatch):
    """Triangles around and behind the eye, crossing the camera plane, slivers, needles, huge
    and tiny ones, near edge-on: the screen boxes (bounded-region case) and the unbounded
    fallback must never drop a record some ray hits."""
    path = nasty_scene(tmp_path)
    rng2 = np.random.default_rng(8)
    offsets = rng2.random((90, 120, 2), dtype=np.float32)
    for off in (None, offsets):
        ref = oracle_render(path, 120, 90, off)
        for mode in CULL_MODES:
            set_cull_mode(monkeypatch, mode)
            assert_parity(torch_render(path, 120, 90, off, variant="cull"), ref)
        assert_parity(torch_render(path, 120, 90, off, variant="bvh"), ref)


@pytest.mark.parametrize("records", ["stored", "recompute"])
def test_record_modes_bitwise(gpu, scenes, tmp_path, monkeypatch, records):
    """Both record sources of the binned trace (render.h RecordMode, env SRT_TRACE_RECORDS): the 64-B
    cull records the bin kernel stores, or records the trace recomputes from the scene's 48-B spatial
    inputs and the bin kernel's screen boxes. Single frames of the nasty-geometry scene -- plain, with
    list overflow (FULL tiles stream every position) and with offsets outside [0, 1] (range-tagged:
    every tile streams) -- against the oracle, and a batched launch against the LDS brute force, bit
    for bit."""
    import torch

    import simpleraytracer_amd as srt

    monkeypatch.setenv("SRT_TRACE_RECORDS", records)
    path = nasty_scene(tmp_path)
    w, h = 120, 90
    rng = np.random.default_rng(19)
    offsets = rng.random((h, w, 2), dtype=np.float32)
    wild = offsets.copy()
    wild[::7] *= 3.0
    for off in (None, offsets, wild):
        ref = oracle_render(path, w, h, off)
        for mode in (("1", "", ""), ("1", "", "8")):
            set_cull_mode(monkeypatch, mode)
            assert_parity(torch_render(path, w, h, off, variant="cull"), ref)
    monkeypatch.delenv("SRT_CULL_BIN_CAP", raising=False)
    w, h, frames = 200, 120, 3
    offs = [rng.random((h, w, 2), dtype=np.float32) for _ in range(frames)]
    refs = [torch_render(scenes["soup2k"], w, h, o, variant="lds") for o in offs]
    scene = srt.DeviceScene(scenes["soup2k"], 0)
    stream = torch.cuda.current_stream()
    scene.prepare(w, h, stream)
    off = [torch.from_numpy(o).cuda() for o in offs]
    rgba = [torch.full((h, w, 4), float("nan"), dtype=torch.float32, device="cuda") for _ in range(frames)]
    scene.trace_batch(off, rgba, 0, h, variant="cull", stream=stream)
    torch.cuda.synchronize()
    for f in range(frames):
        assert np.array_equal(rgba[f].cpu().numpy().view(np.uint32), refs[f].view(np.uint32)), f
    scene.close()


def test_extreme_offsets(gpu, scenes):
    """Sample offsets far outside [0,1), negative, huge, +-inf and NaN: the box cull must stay
    conservative (monotone fma bounds, NaN never rejects) and match the oracle bit for bit."""
    rng = np.random.default_rng(3)
    w, h = 130, 70
    offsets = rng.uniform(-40, 40, (h, w, 2)).astype(np.float32)
    offsets[5, :, 0] = np.inf
    offsets[6, :, 1] = -np.inf
    offsets[7, ::3, :] = np.nan
    offsets[:, 9, 0] = 1e30
    offsets[:, 10, 1] = -1e30
    ref = oracle_render(scenes["soup300"], w, h, offsets)
    for variant in VARIANTS:
        assert_parity(torch_render(scenes["soup300"], w, h, offsets, variant=variant), ref)


def test_repeat_render_deterministic(gpu, scenes):
    a = torch_render(scenes["soup2k"], 200, 120)
    b = torch_render(scenes["soup2k"], 200, 120)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("devices", ["0,0", "0,0,0", "0,0,0,0,0,0,0,0"])
@pytest.mark.parametrize("mode", ["copy", "direct"])
@pytest.mark.parametrize("rows", ["interleaved", "contiguous"])
def test_ml_gather_modes_bitwise(gpu, scenes, monkeypatch, devices, mode, rows):
    """mlInfer over P row bands on device 0 ("fake devices": one device listed P times): hit-id
    bands gathered to device 0 by device copies at ncclGather's receive offsets, shaded there, one
    D2H -- or every band shaded and copied out by its device ("direct") -- equals the one-band frame
    bit for bit; interleaved 16-row tile rows and contiguous bands (8 bands of 100 rows leave a
    padded last band)."""
    import simpleraytracer_amd as srt

    monkeypatch.delenv("ML_VISIBLE_DEVICES", raising=False)
    ref = srt.render(scenes["soup2k"], 160, 100)
    monkeypatch.setenv("ML_VISIBLE_DEVICES", devices)
    monkeypatch.setenv("SRT_GATHER", mode)
    monkeypatch.setenv("SRT_BAND_ROWS", rows)
    got = srt.render(scenes["soup2k"], 160, 100)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    for variant in ("scalar", "cull", "bvh"):
        monkeypatch.setenv("SRT_TRACE_VARIANT", variant)
        got2 = srt.render(scenes["soup2k"], 160, 100)
        assert np.array_equal(got2.view(np.uint32), ref.view(np.uint32))


def test_ml_rccl_gather_two_devices(gpu, scenes, monkeypatch):
    """The in-process ncclGather path (ML_VISIBLE_DEVICES=0,1: one RCCL communicator per device,
    bands gathered to device 0 over xGMI) equals the one-device frame bit for bit."""
    import torch

    import simpleraytracer_amd as srt

    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 visible GPUs for an RCCL communicator (this box has "
                    f"{torch.cuda.device_count()}); the same gather offsets run in test_ml_gather_modes_bitwise")
    ref = srt.render(scenes["soup2k"], 160, 100)
    monkeypatch.setenv("ML_VISIBLE_DEVICES", "0,1")
    monkeypatch.setenv("SRT_GATHER", "rccl")
    got = srt.render(scenes["soup2k"], 160, 100)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_edge_cases_scene(gpu, tmp_path):
    """Disabled (edge-on / degenerate) triangles, behind-camera, duplicates (tie -> lowest id),
    reversed winding, nested depth order."""
    tris = [
        # 0: far quad-ish triangle at z=3
        [-1, -1, 3, 1, -1, 3, 0, 1, 3],
        # 1: nearer triangle at z=2 (must win over 0 where they overlap)
        [-0.3, -0.3, 2, 0.3, -0.3, 2, 0, 0.3, 2],
        # 2: exact duplicate of 1 (ties lose to id 1)
        [-0.3, -0.3, 2, 0.3, -0.3, 2, 0, 0.3, 2],
        # 3: reversed winding duplicate of 1
        [0.3, -0.3, 2, -0.3, -0.3, 2, 0, 0.3, 2],
        # 4: behind the camera
        [-1, -1, -2, 1, -1, -2, 0, 1, -2],
        # 5: plane through the eye (edge-on): disabled
        [0, -1, 1, 0, 1, 1, 0, 0, 3],
        # 6: zero area
        [0.1, 0.1, 1.5, 0.2, 0.2, 1.5, 0.3, 0.3, 1.5],
        # 7: small triangle in front of everything, off-centre
        [0.5, 0.2, 1.0, 0.7, 0.2, 1.0, 0.6, 0.4, 1.0],
    ]
    path = write_custom_scene(tmp_path / "edge.srt", tris, np.linspace(0.1, 0.9, 24).reshape(8, 3))
    for variant in VARIANTS:
        got = torch_render(path, 257, 129, variant=variant)
        ref = oracle_render(path, 257, 129)
        assert_parity(got, ref)
    ids = set(np.unique(got[..., 3]).astype(int))
    # 3 (reversed winding) and 6 (zero area) are evaluated from other operands / rounding noise,
    # so they may legitimately win a pixel by an ulp; parity above is the contract.
    assert {0, 1, 7, -1} <= ids and not ({2, 4, 5} & ids)


def test_reference_test_app_binary_renders(gpu, scenes, tmp_path):
    """The reference's own test_app.cpp (built from /root/reference by `make ref`, linked to
    this libModelRunner.so) renders C1 end to end; output equals the oracle."""
    import subprocess
    from pathlib import Path

    repo = Path(__file__).resolve().parents[1]
    exe = repo / "oracle" / "_ref" / "ref_test_app"
    if not exe.exists():
        pytest.skip("oracle/_ref/ref_test_app not built (needs /root/reference at build time)")
    inp = tmp_path / "in.bin"
    outp = tmp_path / "out.bin"
    np.full((256, 256, 2), 0.5, np.float32).tofile(inp)
    r = subprocess.run([str(exe), "-m", scenes["triangle"], "-w", "256", "-h", "256", "-i", str(inp), "-o",
                        str(outp)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Output: 256 x 256 x 4" in r.stderr
    got = np.fromfile(outp, np.float32).reshape(256, 256, 4)
    assert_parity(got, oracle_render(scenes["triangle"], 256, 256))


def test_own_test_app_stdin_stdout(gpu, scenes):
    import subprocess
    from pathlib import Path

    exe = Path(__file__).resolve().parents[1] / "bin" / "test_app"
    data = np.full((48, 64, 2), 0.5, np.float32).tobytes()
    r = subprocess.run([str(exe), "-m", scenes["cornell"], "-w", "64", "-h", "48"], input=data,
                       capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    got = np.frombuffer(r.stdout, np.float32).reshape(48, 64, 4)
    assert_parity(got, oracle_render(scenes["cornell"], 64, 48))


def test_no_cpu_fallback_marker(gpu):
    """The product library is the HIP build: its code object targets gfx950."""
    from pathlib import Path

    lib = Path(__file__).resolve().parents[1] / "simpleraytracer_amd" / "lib" / "libModelRunner.so"
    assert b"gfx950" in lib.read_bytes()
    assert os.environ.get("SRT_TRACE_VARIANT") in (None, "lds", "scalar", "cull", "bvh", "0", "1", "2", "3")


@pytest.mark.parametrize("variant", VARIANTS)
def test_stage_timing_does_not_change_the_frame(gpu, scenes, variant):
    """srtSetStageTiming binds events to the kernels' dispatches: same frame, sane times."""
    import torch

    import simpleraytracer_amd as srt

    w, h = 200, 70
    ref = torch_render(scenes["soup300"], w, h, variant=variant)
    scene = srt.DeviceScene(scenes["soup300"], 0)
    stream = torch.cuda.current_stream()
    off = torch.full((h, w, 2), 0.5, dtype=torch.float32, device="cuda")
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    scene.set_stage_timing(True)
    for _ in range(3):
        scene.prepare(w, h, stream)
        scene.trace(off, out, 0, h, variant=variant, stream=stream)
    scene.set_stage_timing(False)
    n, prep, binning, trace = scene.take_stage_times()
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    scene.close()
    assert n == 3
    # a full cull frame computes its tile info inside the bin launch (render.h CullFusedInfo): no
    # separate prepare kernel, the bin stage covers it
    assert (prep == 0.0) if variant == "cull" else (0.0 < prep < 1000.0)
    assert 0.0 < trace < 1000.0
    assert (binning > 0.0) == (variant in ("cull", "bvh"))
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_obj_scene_renders_like_its_binary_conversion(gpu, tmp_path):
    """An OBJ model_path renders through ml* exactly like the oracle on its binary conversion."""
    import simpleraytracer_amd as srt

    rng = np.random.default_rng(5)
    lines = ["mtllib m.mtl", "usemtl a"]
    for i in range(60):
        c = rng.uniform([-1, -1, 2], [1, 1, 4])
        for _ in range(4):
            lines.append("v %.6f %.6f %.6f" % tuple(c + rng.uniform(-0.15, 0.15, 3)))
        lines.append(f"f {4 * i + 1} {4 * i + 2}/1 {4 * i + 3}//2 {4 * i + 4}/3/4")
        if i == 30:
            lines.append("usemtl b")
    (tmp_path / "m.mtl").write_text("newmtl a\nKd 0.9 0.5 0.2\nnewmtl b\nKd 0.2 0.4 0.9\n")
    obj = tmp_path / "quads.obj"
    obj.write_text("\n".join(lines) + "\n")
    binary = srt.convert_scene(str(obj), str(tmp_path / "quads.srt"))
    w, h = 160, 96
    got = srt.render(str(obj), w, h)
    assert_parity(got, oracle_render(binary, w, h))
    assert (got[..., 3] >= 0).sum() > 200  # the quads are in view (auto camera frames the bounding sphere)


@pytest.mark.parametrize("in_dtype,out_dtype", [(0, 1), (1, 0), (1, 1)])
def test_float16_images(gpu, scenes, tmp_path, monkeypatch, in_dtype, out_dtype):
    """ML_FLOAT16 images (scene flags): the frame equals the f32 oracle frame rounded to half
    (rgb within one half ulp of the f32 tolerance, tri_id channel bit-exact after rounding);
    FLOAT16 offsets are the oracle's inputs exactly. One device (chunk pipeline), and two bands
    on device 0 assembled by the band gather (device copies at ncclGather's offsets, padded half
    bands) and by per-band D2H."""
    import simpleraytracer_amd as srt

    path = srt.convert_scene(scenes["soup300"], str(tmp_path / "h.srt"), input_dtype=in_dtype,
                             output_dtype=out_dtype)
    w, h = 96, 63
    rng = np.random.default_rng(3)
    offs = rng.uniform(0, 1, (h, w, 2)).astype(np.float16 if in_dtype else np.float32)
    ref = oracle_render(path, w, h, offs.astype(np.float32))
    for devices, mode in (("0", "direct"), ("0,0", "copy"), ("0,0", "direct")):
        monkeypatch.setenv("ML_VISIBLE_DEVICES", devices)
        monkeypatch.setenv("SRT_GATHER", mode)
        got = srt.render(path, w, h, offs)
        assert got.dtype == (np.float16 if out_dtype else np.float32)
        if out_dtype:
            want = ref.astype(np.float16)
            assert np.array_equal(got[..., 3].view(np.uint16), want[..., 3].view(np.uint16))
            d = np.abs(got[..., :3].astype(np.float32) - want[..., :3].astype(np.float32))
            assert float(d.max()) <= 1e-3
        else:
            assert_parity(got, ref)


@pytest.mark.parametrize("variant", ("cull", "bvh"))
def test_c5_soup1m_4k_row_sample(gpu, tmp_path, variant):
    """Stress config C5 on one GPU: 1M-triangle soup (seed 0x5EED+1, s = 0.01) at 3840x2160,
    checked on 3 rows against the oracle (the full frame would take the CPU hours)."""
    import simpleraytracer_amd as srt

    path = srt.write_scene(str(tmp_path / "soup1m.srt"), "soup", 1_000_000)
    w, h = 3840, 2160
    got = torch_render(path, w, h, variant=variant)
    rows = np.array([700, 1080, 1500])
    ref = np.full((h, w, 4), np.nan, np.float32)
    for r in rows:
        ref[r] = oracle_render(path, w, h, row_begin=int(r), row_count=1)[r]
    assert_parity(got, ref, rows=rows)
    assert 0.05 < (got[..., 3] >= 0).mean() < 0.9


def test_random_cameras_all_variants(gpu, tmp_path):
    """General frames: random eye / look-at / up / vfov (rotated, rolled, wide and narrow views)
    over a random soup around the origin; every variant against the oracle, uniform and random
    offsets."""
    rng = np.random.default_rng(2024)
    for k in range(5):
        c = rng.uniform(-1, 1, (1500, 3))
        tris = (c[:, None, :] + rng.uniform(-0.12, 0.12, (1500, 3, 3))).reshape(-1, 9)
        eye = rng.normal(size=3)
        eye = eye / np.linalg.norm(eye) * rng.uniform(2.5, 6.0)
        look = rng.uniform(-0.3, 0.3, 3)
        up = rng.normal(size=3)
        vfov = float(rng.uniform(15, 110))
        path = write_custom_scene(tmp_path / f"cam{k}.srt", tris, rng.uniform(0.2, 1, (1500, 3)), eye=tuple(eye),
                                  lookat=tuple(look), up=tuple(up), vfov=vfov, background=(0.1, 0.2, 0.3))
        w, h = 173, 111
        offs = rng.random((h, w, 2), dtype=np.float32) if k % 2 else None
        ref = oracle_render(path, w, h, offs)
        assert (ref[..., 3] >= 0).mean() > 0.02, "camera sees the soup"
        for variant in VARIANTS:
            assert_parity(torch_render(path, w, h, offs, variant=variant), ref)


@pytest.mark.parametrize("out_dtype", [0, 1])
def test_ml_pipelined_chunks_bitwise(gpu, scenes, tmp_path, monkeypatch, out_dtype):
    """The single-device mlInfer pipeline (row chunks: H2D / trace / D2H overlapped on three
    streams) gives the unchunked image bit for bit, for chunk counts that do and do not divide
    the height."""
    import simpleraytracer_amd as srt

    path = srt.convert_scene(scenes["soup2k"], str(tmp_path / "s.srt"), output_dtype=out_dtype)
    rng = np.random.default_rng(11)
    w, h = 150, 101
    offs = rng.random((h, w, 2), dtype=np.float32)
    monkeypatch.setenv("SRT_E2E_CHUNKS", "1")
    ref = srt.render(path, w, h, offs)
    for chunks in ("2", "4", "7", "16"):
        monkeypatch.setenv("SRT_E2E_CHUNKS", chunks)
        got = srt.render(path, w, h, offs)
        assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), chunks
    if out_dtype == 0:
        assert_parity(ref, oracle_render(path, w, h, offs))


@pytest.mark.parametrize("variant", ("cull", "bvh"))
def test_concurrent_frame_queues(gpu, scenes, variant):
    """bench.py's frame queues: scenes on their own HIP streams with frames interleaved
    (prepare of one overlapping trace of another) give the single-stream frames bit-for-bit."""
    import torch

    import simpleraytracer_amd as srt

    w, h = 640, 360
    jobs = [(scenes["soup2k"], 0.5), (scenes["soup300"], 0.25), (scenes["soup2k"], 0.8)]
    refs = []
    for path, j in jobs:
        refs.append(torch_render(path, w, h, np.full((h, w, 2), j, np.float32), variant=variant))
    qs = [(srt.DeviceScene(path, 0), torch.cuda.Stream(),
           torch.full((h, w, 2), j, dtype=torch.float32, device="cuda"),
           torch.empty((h, w, 4), dtype=torch.float32, device="cuda")) for path, j in jobs]
    torch.cuda.synchronize()
    for k in range(4 * len(qs)):
        scene, stream, off, out = qs[k % len(qs)]
        scene.prepare(w, h, stream)
        scene.trace(off, out, 0, h, variant=variant, stream=stream)
    torch.cuda.synchronize()
    for (scene, _, _, out), ref in zip(qs, refs):
        assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
        scene.close()


@pytest.mark.parametrize("chunk,chunks", [("64", ""), ("", ""), ("128", "16")])
def test_split_items_across_frames(gpu, scenes, monkeypatch, chunk, chunks):
    """Split work items (a heavy tile part cut into candidate chunks, merged by the last chunk
    through global key slices): frames traced back to back on one scene and stream, each with
    different per-pixel jitter, equal fresh single-frame renders bit for bit -- no key slice or
    arrival counter state leaks from one frame into the next -- and the oracle on a row sample."""
    import torch

    import simpleraytracer_amd as srt

    monkeypatch.setenv("SRT_CULL_CHUNK", chunk)
    monkeypatch.setenv("SRT_CULL_CHUNKS", chunks)
    w, h = 640, 360
    rng = np.random.default_rng(77)
    offs = [rng.random((h, w, 2), dtype=np.float32) for _ in range(3)] + \
           [np.full((h, w, 2), j, np.float32) for j in (0.5, 0.25, 0.75)]
    refs = [torch_render(scenes["soup100k"], w, h, o) for o in offs]
    scene = srt.DeviceScene(scenes["soup100k"], 0)
    stream = torch.cuda.current_stream()
    ins = [torch.from_numpy(o).cuda() for o in offs]
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in offs]
    for rep in range(2):
        for o, out in zip(ins, outs):
            scene.prepare(w, h, stream)
            scene.trace(o, out, 0, h, stream=stream)
    torch.cuda.synchronize()
    for out, ref in zip(outs, refs):
        assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    scene.close()
    rows = np.arange(5, h, 60)
    ref = oracle_render(scenes["soup100k"], w, h, offs[0], row_begin=5, row_count=h - 5, row_step=60)
    assert_parity(refs[0], ref, rows=rows)


@pytest.mark.parametrize("chunk,plan", [("", ""), ("64", ""), ("", "reuse"), ("64", "reuse"), ("64", "order")])
def test_work_plan_is_scheduling_only(gpu, scenes, monkeypatch, chunk, plan):
    """The trace's work plan (tile parts, chunking, split slots, heaviest first) is built once per
    frame slot and trace grid and reused (SRT_WORK_PLAN: auto = by single-frame launches, reuse =
    by every launch, order = none): it decides only which block takes which part, so every frame
    -- whatever frame the plan was made from (the first one here streams every record: offsets
    outside [0, 1]), batched or not, uniform, jittered or NaN offsets -- equals the brute-force
    frame bit for bit."""
    import torch

    import simpleraytracer_amd as srt

    monkeypatch.setenv("SRT_CULL_CHUNK", chunk)
    monkeypatch.setenv("SRT_WORK_PLAN", plan)
    w, h = 640, 360
    rng = np.random.default_rng(81)
    nan = rng.random((h, w, 2), dtype=np.float32)
    nan[100:140, 200:260] = np.nan
    offs = [np.full((h, w, 2), -3.25, np.float32), np.full((h, w, 2), 0.5, np.float32),
            rng.random((h, w, 2), dtype=np.float32), nan, rng.random((h, w, 2), dtype=np.float32)]
    refs = [torch_render(scenes["soup100k"], w, h, o, variant="lds") for o in offs]
    scene = srt.DeviceScene(scenes["soup100k"], 0)
    stream = torch.cuda.current_stream()
    scene.prepare(w, h, stream)
    ins = [torch.from_numpy(o).cuda() for o in offs]
    for rep in range(2):
        outs = [torch.full((h, w, 4), float("nan"), dtype=torch.float32, device="cuda") for _ in offs]
        for o, out in zip(ins, outs):
            scene.trace(o, out, 0, h, stream=stream)
        batch = [torch.full((h, w, 4), float("nan"), dtype=torch.float32, device="cuda") for _ in range(3)]
        scene.trace_batch(ins[2:5], batch, 0, h, stream=stream)  # another trace grid: slots 0-2 re-plan
        again = torch.full((h, w, 4), float("nan"), dtype=torch.float32, device="cuda")
        scene.trace(ins[1], again, 0, h, stream=stream)
        torch.cuda.synchronize()
        for k, (out, ref) in enumerate(zip(outs, refs)):
            assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32)), (rep, k)
        for k, out in enumerate(batch):
            assert np.array_equal(out.cpu().numpy().view(np.uint32), refs[2 + k].view(np.uint32)), (rep, "batch", k)
        assert np.array_equal(again.cpu().numpy().view(np.uint32), refs[1].view(np.uint32)), rep
    scene.close()


@pytest.mark.parametrize("variant", VARIANTS)
def test_deferred_shading_bitwise(gpu, scenes, variant):
    """srtTraceIdsAsync + srtShadeAsync (the multi-GPU band path: hit ids gathered, shaded by the
    compositing GPU) equal the fused srtTraceAsync frame bit for bit, per band, with random
    offsets; the ids are the frame's alpha channel."""
    import torch

    import simpleraytracer_amd as srt

    w, h = 333, 170
    rng = np.random.default_rng(41)
    offs = rng.random((h, w, 2), dtype=np.float32)
    ref = torch_render(scenes["soup2k"], w, h, offs, variant=variant)
    scene = srt.DeviceScene(scenes["soup2k"], 0)
    stream = torch.cuda.current_stream()
    off = torch.from_numpy(offs).cuda()
    ids = torch.full((h, w), -7, dtype=torch.int32, device="cuda")
    rgba = torch.full((h, w, 4), float("nan"), dtype=torch.float32, device="cuda")
    scene.prepare(w, h, stream)
    for r0, rows in ((0, 61), (61, 1), (62, h - 62)):
        scene.trace_ids(off[r0:r0 + rows], ids[r0:r0 + rows], r0, rows, variant=variant, stream=stream)
    # shade the whole frame in two bands on a second scene (its prepare runs inside the shade)
    scene2 = srt.DeviceScene(scenes["soup2k"], 0)
    scene2.prepare(w, h, stream)
    for r0, rows in ((0, 100), (100, h - 100)):
        scene2.shade(off[r0:r0 + rows], ids[r0:r0 + rows], rgba[r0:r0 + rows], r0, rows, stream=stream)
    torch.cuda.synchronize()
    got_ids = ids.cpu().numpy()
    assert np.array_equal(got_ids.astype(np.float32), ref[..., 3])
    assert np.array_equal(rgba.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    scene.close()
    scene2.close()


@pytest.mark.parametrize("bands", [1, 3, 4])
def test_batched_band_shading_bitwise(gpu, scenes, bands):
    """srtShadeBandsAsync (bench.py's batched band gather): the ids of F frames arrive band-major
    ids[band][frame][band_rows][W], the last band padded (170 rows in 3 / 4 bands); one launch
    shades all F frames, each equal to the fused trace bit for bit. Frame f of the batch holds
    the ids of a different frame's band order (the padded rows hold garbage, never read)."""
    import torch

    import simpleraytracer_amd as srt

    w, h, frames = 333, 170, 3
    rng = np.random.default_rng(43)
    offs = rng.random((h, w, 2), dtype=np.float32)
    ref = torch_render(scenes["soup2k"], w, h, offs)
    scene = srt.DeviceScene(scenes["soup2k"], 0)
    stream = torch.cuda.current_stream()
    off = torch.from_numpy(offs).cuda()
    b = (h + bands - 1) // bands
    ids = torch.full((bands, frames, b, w), -7, dtype=torch.int32, device="cuda")
    scene.prepare(w, h, stream)
    for p in range(bands):
        r0, rows = p * b, min(h, (p + 1) * b) - p * b
        for f in range(frames):
            scene.trace_ids(off[r0:r0 + rows], ids[p, f, :rows], r0, rows, stream=stream)
        ids[p, :, rows:] = 2 ** 30  # padding: an id outside the scene, never read
    rgba = torch.full((frames, h, w, 4), float("nan"), dtype=torch.float32, device="cuda")
    scene.shade_bands(off, ids, rgba, b, stream=stream)
    torch.cuda.synchronize()
    got = rgba.cpu().numpy()
    for f in range(frames):
        assert np.array_equal(got[f].view(np.uint32), ref.view(np.uint32)), f
    with pytest.raises(ValueError):
        scene.shade_bands(off, ids, rgba[:2], b, stream=stream)
    scene.close()


@pytest.mark.parametrize("variant", ["cull", "lds"])
def test_trace_batch_bitwise(gpu, scenes, variant):
    """srtTraceBatchAsync: F frames (each with its own random offsets) in one call, RGBA for the
    whole frame and hit ids for a band, equal the frames traced one at a time bit for bit (cull:
    one launch per stage for the batch; other variants: frame by frame). Afterwards the scene's
    single-frame calls (trace, shade from slot 0's records) are still exact."""
    import torch

    import simpleraytracer_amd as srt

    w, h, frames = 333, 170, 3
    rng = np.random.default_rng(47)
    offs = [rng.random((h, w, 2), dtype=np.float32) for _ in range(frames)]
    refs = [torch_render(scenes["soup2k"], w, h, o, variant="lds") for o in offs]
    scene = srt.DeviceScene(scenes["soup2k"], 0)
    stream = torch.cuda.current_stream()
    scene.prepare(w, h, stream)
    off = [torch.from_numpy(o).cuda() for o in offs]
    rgba = [torch.full((h, w, 4), float("nan"), dtype=torch.float32, device="cuda") for _ in range(frames)]
    scene.trace_batch(off, rgba, 0, h, variant=variant, stream=stream)
    r0, rows = 40, 77
    band_off = [o[r0:r0 + rows].contiguous() for o in off] * 3  # 9 > MAX_BATCH: checked below
    ids = [torch.full((rows, w), -7, dtype=torch.int32, device="cuda") for _ in range(srt.MAX_BATCH)]
    scene.trace_batch(band_off[:srt.MAX_BATCH], ids, r0, rows, variant=variant, stream=stream, ids=True)
    torch.cuda.synchronize()
    for f in range(frames):
        assert np.array_equal(rgba[f].cpu().numpy().view(np.uint32), refs[f].view(np.uint32)), f
    for f in range(srt.MAX_BATCH):
        want = refs[f % frames][r0:r0 + rows, :, 3]
        assert np.array_equal(ids[f].cpu().numpy().astype(np.float32), want), f
    # single-frame calls after a batch: a band trace and the deferred shading of ids
    one = torch.empty((rows, w, 4), dtype=torch.float32, device="cuda")
    scene.prepare(w, h, stream)
    scene.trace(band_off[1], one, r0, rows, variant=variant, stream=stream)
    shaded = torch.empty((rows, w, 4), dtype=torch.float32, device="cuda")
    scene.shade(band_off[1], ids[1], shaded, r0, rows, stream=stream)
    torch.cuda.synchronize()
    assert np.array_equal(one.cpu().numpy().view(np.uint32), refs[1][r0:r0 + rows].view(np.uint32))
    assert np.array_equal(shaded.cpu().numpy().view(np.uint32), refs[1][r0:r0 + rows].view(np.uint32))
    with pytest.raises(ValueError):
        scene.trace_batch(band_off, ids + ids[:1], r0, rows, stream=stream, ids=True)
    scene.close()


def test_trace_batch_regular_and_irregular_tiles(gpu, scenes):
    """Ordered (multi-frame) cull launches over frames that mix regular tiles (one sample offset for every
    ray: positions from the column / row tables) and irregular ones (columns and row blocks of jitter, a
    NaN patch), uniform, jittered and FULL-stream regular frames (a uniform offset outside [0, 1]) in one
    batch, and a band of ids: each equal to the brute-force frame bit for bit."""
    import torch

    import simpleraytracer_amd as srt

    w, h = 640, 360
    rng = np.random.default_rng(91)
    mixed = np.full((h, w, 2), 0.5, np.float32)
    mixed[:, 64:128, 0] = rng.random((h, 64), dtype=np.float32)
    mixed[100:180, 300:500] = rng.random((80, 200, 2), dtype=np.float32)
    mixed2 = np.full((h, w, 2), 0.25, np.float32)
    mixed2[:, 600:] = rng.random((h, 40, 2), dtype=np.float32)
    mixed2[200:220, 10:50] = np.nan
    offs = [mixed, np.full((h, w, 2), 0.5, np.float32), rng.random((h, w, 2), dtype=np.float32),
            np.full((h, w, 2), 2.0, np.float32), mixed2]
    refs = [torch_render(scenes["soup100k"], w, h, o, variant="lds") for o in offs]
    scene = srt.DeviceScene(scenes["soup100k"], 0)
    stream = torch.cuda.current_stream()
    scene.prepare(w, h, stream)
    ins = [torch.from_numpy(o).cuda() for o in offs]
    for rep in range(2):
        outs = [torch.full((h, w, 4), float("nan"), dtype=torch.float32, device="cuda") for _ in offs]
        scene.trace_batch(ins, outs, 0, h, stream=stream)
        r0, rows = 37, 200
        ids = [torch.full((rows, w), -7, dtype=torch.int32, device="cuda") for _ in offs]
        scene.trace_batch([o[r0:r0 + rows].contiguous() for o in ins], ids, r0, rows, stream=stream, ids=True)
        torch.cuda.synchronize()
        for k, (out, ref) in enumerate(zip(outs, refs)):
            assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32)), (rep, k)
            assert np.array_equal(ids[k].cpu().numpy().astype(np.float32), ref[r0:r0 + rows, :, 3]), (rep, "ids", k)
    scene.close()


def test_trace_batch_c3_band_of_8(gpu, scenes):
    """The bench's N = 8 band (135 rows of 1080p, C3) batched 8 frames at a time: every frame's
    ids equal a single srtTraceIdsAsync of the band, bit for bit."""
    import torch

    import simpleraytracer_amd as srt

    w, h, r0, rows = 1920, 1080, 405, 135
    scene = srt.DeviceScene(scenes["soup100k"], 0)
    stream = torch.cuda.current_stream()
    scene.prepare(w, h, stream)
    off = torch.full((rows, w, 2), 0.5, dtype=torch.float32, device="cuda")
    ref = torch.empty((rows, w), dtype=torch.int32, device="cuda")
    scene.trace_ids(off, ref, r0, rows, stream=stream)
    ids = [torch.full((rows, w), -7, dtype=torch.int32, device="cuda") for _ in range(srt.MAX_BATCH)]
    run = scene.bind_trace_batch([off] * srt.MAX_BATCH, ids, r0, rows, stream=stream, ids=True)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    for f in range(srt.MAX_BATCH):
        assert torch.equal(ids[f], ref), f
    scene.close()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("mode", [CULL_MODES[0], CULL_MODES[3]])
def test_interleaved_bands_bitwise(gpu, scenes, monkeypatch, world, mode):
    """Interleaved bands (the frame's 16-row tile rows dealt round-robin, row_interleave = P):
    every rank's batched trace of its rows (hit ids and RGBA), then the gathered band-major ids
    shaded with the interleaved layout (srtShadeBandsAsync), equal the brute-force frame bit for
    bit; 170 rows leave a partial last tile row; forced list overflow streams records in a band."""
    import torch

    import simpleraytracer_amd as srt
    from simpleraytracer_amd.bands import interleaved_band_rows, interleaved_frame_rows, interleaved_range

    set_cull_mode(monkeypatch, mode)
    w, h, frames = 333, 170, 2
    offs = np.random.default_rng(53).random((h, w, 2), dtype=np.float32)
    ref = torch_render(scenes["soup2k"], w, h, offs, variant="lds")
    off = torch.from_numpy(offs).cuda()
    stream = torch.cuda.current_stream()
    b = interleaved_band_rows(h, world)
    gathered = torch.full((world, frames, b, w), 2 ** 30, dtype=torch.int32, device="cuda")
    scene = srt.DeviceScene(scenes["soup2k"], 0)
    scene.prepare(w, h, stream)
    for r in range(world):
        r0, rows = interleaved_range(h, world, r)
        fr = interleaved_frame_rows(h, world, r)
        if rows == 0:
            continue
        band_off = off.index_select(0, torch.from_numpy(fr).cuda()).contiguous()
        scene.trace_batch([band_off] * frames, [gathered[r, f, :rows] for f in range(frames)], r0, rows,
                          stream=stream, ids=True, row_interleave=world)
        rgba = torch.empty((rows, w, 4), dtype=torch.float32, device="cuda")
        scene.trace_batch([band_off], [rgba], r0, rows, stream=stream, row_interleave=world)
        torch.cuda.synchronize()
        assert np.array_equal(rgba.cpu().numpy().view(np.uint32), ref[fr].view(np.uint32)), r
    out = torch.full((frames, h, w, 4), float("nan"), dtype=torch.float32, device="cuda")
    scene.shade_bands(off, gathered, out, b, stream=stream, interleaved=world)
    torch.cuda.synchronize()
    for f in range(frames):
        assert np.array_equal(out[f].cpu().numpy().view(np.uint32), ref.view(np.uint32)), f
    with pytest.raises(srt.SrtError):  # an interleaved band must start on a tile row
        scene.trace_batch([off[:1]], [out[0, :1]], 1, 1, stream=stream, row_interleave=2)
    scene.close()


def test_scene_calls_on_two_streams_are_ordered(gpu, scenes):
    """One scene used from two streams (bands on alternating streams, a new prepare in between):
    the library orders the calls, so every frame equals its single-stream render."""
    import torch

    import simpleraytracer_amd as srt

    w, h = 256, 144
    offs = [np.full((h, w, 2), j, np.float32) for j in (0.5, 0.3)]
    refs = [torch_render(scenes["soup2k"], w, h, o) for o in offs]
    scene = srt.DeviceScene(scenes["soup2k"], 0)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in offs]
    torch.cuda.synchronize()
    ins = [torch.from_numpy(o).cuda() for o in offs]  # alive until the end (used on side streams)
    torch.cuda.synchronize()
    for off, out in zip(ins, outs):
        scene.prepare(w, h, streams[0])
        for k, r0 in enumerate(range(0, h, 48)):
            st = streams[k % 2]
            scene.trace(off[r0:r0 + 48], out[r0:r0 + 48], r0, 48, stream=st)
    torch.cuda.synchronize()
    for out, ref in zip(outs, refs):
        assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    scene.close()


def test_device_buffers_are_validated(gpu, scenes):
    """DeviceScene checks dtype and device of torch buffers before passing raw pointers."""
    import torch

    import simpleraytracer_amd as srt

    scene = srt.DeviceScene(scenes["soup300"], 0)
    scene.prepare(64, 32, torch.cuda.current_stream())
    off = torch.full((32, 64, 2), 0.5, dtype=torch.float32, device="cuda")
    with pytest.raises(ValueError, match="float32"):
        scene.trace(off, torch.empty((32, 64, 4), dtype=torch.float16, device="cuda"))
    with pytest.raises(ValueError, match="cuda:0"):
        scene.trace(off, torch.empty((32, 64, 4), dtype=torch.float32))
    with pytest.raises(ValueError, match="int32"):
        scene.trace_ids(off, torch.empty((32, 64), dtype=torch.int64, device="cuda"))
    scene.close()


def morton_order_numpy(path):
    """Independent restatement of spatial.hip MortonKey (float64 numpy, same operation order) and
    the stable sort by (code, id): the checker of the device-built spatial order."""
    import simpleraytracer_amd as srt

    sc = srt.read_scene(path)
    v = sc["vertices"].astype(np.float64)
    cam = sc["camera"]
    eye, look, up, vfov = cam[0:3].astype(np.float64), cam[3:6].astype(np.float64), cam[6:9].astype(np.float64), \
        float(cam[9])
    f = look - eye
    r = np.array([f[1] * up[2] - f[2] * up[1], f[2] * up[0] - f[0] * up[2], f[0] * up[1] - f[1] * up[0]])
    u = np.array([r[1] * f[2] - r[2] * f[1], r[2] * f[0] - r[0] * f[2], r[0] * f[1] - r[1] * f[0]])
    fl = np.sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2])
    rl = np.sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2])
    ul = np.sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2])
    half_h = np.tan(vfov * 3.14159265358979323846 / 360.0)
    d = [(v[:, k] + v[:, 3 + k] + v[:, 6 + k]) / 3.0 - eye[k] for k in range(3)]
    z = (d[0] * f[0] + d[1] * f[1] + d[2] * f[2]) / fl
    with np.errstate(all="ignore"):
        sx = (d[0] * r[0] + d[1] * r[1] + d[2] * r[2]) / rl / z / half_h
        sy = -(d[0] * u[0] + d[1] * u[1] + d[2] * u[2]) / ul / z / half_h

        def cell(w):
            q = (np.fmin(np.fmax(w, -4.0), 4.0) + 4.0) / 8.0 * 65535.0
            return np.where(np.isfinite(q), q, 0.0).astype(np.uint64)

        qx, qy = cell(sx), cell(sy)
    key = np.zeros(len(v), np.uint64)
    for b in range(15, -1, -1):
        key = (key << np.uint64(2)) | (((qy >> np.uint64(b)) & np.uint64(1)) << np.uint64(1)) | \
              ((qx >> np.uint64(b)) & np.uint64(1))
    ok = (z > 0) & np.isfinite(z) & (half_h > 0) & (fl > 0) & (rl > 0) & (ul > 0)
    key = np.where(ok, key, np.uint64(0xFFFFFFFF))
    return np.argsort(key, kind="stable").astype(np.uint32)


@pytest.mark.parametrize("name", ["soup100k", "soup2k", "cornell", "triangle"])
def test_device_spatial_order_matches_host_restatement(gpu, scenes, name):
    """The spatial order built on the GPU at load (Morton codes + rocPRIM radix sort) equals an
    independent float64 numpy restatement with a stable sort, entry for entry; build time > 0."""
    import simpleraytracer_amd as srt

    scene = srt.DeviceScene(scenes[name], 0)
    order, ms = scene.spatial_order()
    scene.close()
    assert np.array_equal(order, morton_order_numpy(scenes[name]))
    assert ms > 0.0


def test_device_spatial_order_edge_scene(gpu, tmp_path):
    """Behind-eye and degenerate centroids take the last key; ties keep id order."""
    import simpleraytracer_amd as srt

    rng = np.random.default_rng(4)
    tris = list(rng.uniform(-3, 3, (500, 9)))
    tris += [[0.1, 0.1, 2, 0.2, 0.1, 2, 0.1, 0.2, 2]] * 50  # exact duplicates (equal codes)
    path = write_custom_scene(tmp_path / "o.srt", tris, rng.uniform(0.2, 1, (len(tris), 3)))
    scene = srt.DeviceScene(str(path), 0)
    order, _ = scene.spatial_order()
    scene.close()
    assert np.array_equal(order, morton_order_numpy(str(path)))


@pytest.mark.parametrize("chunks", ["1", "4", "16"])
def test_split_width_full_frame_bitwise(gpu, scenes, monkeypatch, chunks):
    """The headline frame with every tile part split into up to M candidate chunks (forced M;
    the default M is 1 at 1080p, where the parts alone fill the chip) equals brute force bit for
    bit, uniform and jittered offsets."""
    rng = np.random.default_rng(9)
    for offs in (None, rng.random((1080, 1920, 2), dtype=np.float32)):
        monkeypatch.delenv("SRT_CULL_CHUNKS", raising=False)
        ref = torch_render(scenes["soup100k"], 1920, 1080, offs, variant="lds")
        monkeypatch.setenv("SRT_CULL_CHUNKS", chunks)
        got = torch_render(scenes["soup100k"], 1920, 1080, offs, variant="cull")
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("world,rows,exchange", [(3, "rotated", "alltoall"), (8, "rotated", "alltoall"),
                                                 (4, "interleaved", "alltoall"), (3, "interleaved", "share")])
@pytest.mark.parametrize("kind", ["uniform", "random"])
def test_band_block_skip_nasty_geometry(gpu, tmp_path, world, rows, exchange, kind):
    """The band record pass skips 256-record blocks whose screen-box y extent (render.hip
    LaunchBlockExtents) meets none of the band's rows (BandMayReach): nasty geometry (records around
    and behind the eye with unbounded boxes, slivers whose boxes the float solve pads) and the dense
    soup, in contiguous rotated bands, interleaved bands and the share pattern over fake devices,
    every frame against the oracle. Offsets in [0, 1] (the skip applies) and, in the last frame of
    each batch, outside it (the range tag turns the skip off)."""
    from simpleraytracer_amd.engine import FrameEngine

    w, h = 150, 230
    F = 2 * world
    rng = np.random.default_rng(world)
    inputs = (np.full((F, h, w, 2), 0.5, np.float32) if kind == "uniform"
              else rng.random((F, h, w, 2), dtype=np.float32))
    inputs[F - 1, 3, 7] = (1.5, -0.25)  # one offset outside [0, 1]: that frame's bands are range-tagged
    path = nasty_scene(tmp_path)
    refs = [oracle_render(path, w, h, inputs[k]) for k in range(F)]
    with FrameEngine(path, w, h, devices=[0] * world, rows=rows, exchange=exchange, queues=2, batch=F) as e:
        e.set_inputs(inputs)
        e.run(2)
        for k in range(2 * F):
            assert_parity(e.read_frame(k), refs[k % F])
        assert e.verify() == (0, 2 * F)
