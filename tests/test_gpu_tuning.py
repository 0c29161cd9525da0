"""GPU parity of the TUNING build (lib_tuning/libgolhip.so, -DGOLHIP_TUNING): the stencil variants
measured and rejected for production, the level-split and register-tile kernels and the register-
slab shapes the planner does not pick, selected by the tuning build's environment variables
(GOLHIP_VARIANT / GOLHIP_SPLIT / GOLHIP_TILE / GOLHIP_SLAB), each against the oracle bit for bit.
The production library (lib/libgolhip.so) contains none of these kernels and reads none of these
variables (tests/test_boundary.py checks its strings); tests/test_gpu_parity.py covers it.
"""
import math

import numpy as np
import pytest

from test_gpu_parity import run_engine, tracked_flips_every_depth

from conftest import PKG

# lib_tuning (33 MiB) is built here and pushed to a GPU box only for the runs that load it
# (.gpurunignore); without it this module skips -- the fault library's smoke below still runs
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not (PKG / "lib_tuning" / "libgolhip.so").exists(),
                                 reason="lib_tuning/libgolhip.so not on this box (pushed only for tuning runs)")]


@pytest.fixture(scope="session")
def tuning(golhip):
    return golhip.tuning_library()


@pytest.mark.parametrize("variant", ["driftlds", "drift62", "pre63", "prodmask"])
@pytest.mark.parametrize("k", [1, 2, 6, 12, 16, 32])
@pytest.mark.parametrize("strips", [1, 3])
def test_tracked_flips_every_depth_variants(golhip, tuning, oracle, monkeypatch, variant, k, strips):
    """Flips tracking at every depth for the other drift geometries (half-word halo, 62-word
    chunks, pre-shifted rows everywhere, masked idle lanes)."""
    monkeypatch.setenv("GOLHIP_VARIANT", variant)
    tracked_flips_every_depth(golhip, oracle, k, strips, lib=tuning)


def test_tuning_build_reads_its_selectors(golhip, tuning, monkeypatch):
    """The tuning build's GOLHIP_SLAB selector changes the kernel; the production build ignores it."""
    monkeypatch.setenv("GOLHIP_SLAB", "1608")
    with golhip.Engine(640, 300, k=16, lib=tuning) as e:
        assert e.launch_kind(16) == ("slab", 1608)
    with golhip.Engine(640, 300, k=16) as e:
        assert e.launch_kind(16) != ("slab", 1608)


@pytest.mark.parametrize("variant", ["chainlds", "driftlds", "driftzip", "drift62", "driftnf", "pre63", "skewlds", "chainlds2",
                                     "skewlds2", "chain", "skew", "chain2", "skew2"])
@pytest.mark.parametrize("k", [1, 6, 16])
def test_every_kernel_variant(golhip, tuning, oracle, monkeypatch, variant, k):
    """Every stencil variant (chained/skewed levels, 1 or 2 words per lane, register or LDS-DMA
    prefetch) on the shapes that stress wrap, halo lanes and band seams."""
    monkeypatch.setenv("GOLHIP_VARIANT", variant)
    for (h, w) in [(77, 640), (16, 16), (300, 4160)]:
        rng = np.random.default_rng(h + w + k)
        board = ((rng.random((h, w)) < 0.4) * 255).astype(np.uint8)
        turns = 2 * k + 1
        exp, exp_counts = oracle.packed_run(board, turns)
        for band in (0, 7):
            out, counts, _, _ = run_engine(golhip, board, turns, k=k, counts=True, band_rows=band, lib=tuning)
            assert np.array_equal(out, exp), (variant, k, h, w, band)
            assert np.array_equal(counts.astype(np.int64), exp_counts), (variant, k, h, w, band)


@pytest.mark.parametrize("variant", ["prod", "drift62"])
@pytest.mark.parametrize("k", [20, 24])
def test_tuning_depths_20_24(golhip, tuning, oracle, monkeypatch, variant, k):
    """The tuning build's extra launch depths K = 20 / 24 (62-word drift geometry; measured for the
    driver's 20-turn region as one launch): exactly k deep, counts, wrap, partial chunks."""
    monkeypatch.setenv("GOLHIP_VARIANT", variant)
    for (h, w) in [(64, 4160), (35, 2016), (130, 8192), (20, 1984)]:
        rng = np.random.default_rng(h * 13 + w + k)
        board = ((rng.random((h, w)) < 0.37) * 255).astype(np.uint8)
        turns = 2 * k + 3
        exp, exp_counts = oracle.packed_run(board, turns)
        for band in (0, 40):
            out, counts, cells, count = run_engine(golhip, board, turns, k=k, counts=True, band_rows=band, lib=tuning)
            assert np.array_equal(out, exp), (k, h, w, band)
            assert np.array_equal(counts.astype(np.int64), exp_counts), (k, h, w, band)


@pytest.mark.parametrize("variant", ["driftlds", "driftzip", "drift62", "pre63", "prodmask"])
@pytest.mark.parametrize("k", [2, 4, 6, 8, 10, 12, 14, 16, 32])
def test_drift_variant_every_k(golhip, tuning, oracle, monkeypatch, variant, k):
    """The drifting-sum stencils (rows move one bit east per level, one DPP per level update) --
    half-word-halo chunks (driftlds), 62-word chunks (drift62), 62-word chunks with two steps
    interleaved (driftzip) and 63-word chunks of rows pre-shifted K bits west (pre63, its 65th-word
    DMA and no store realignment): every launch depth, per-turn counts (drifted count windows), multi-
    chunk rows with a partial last chunk and widths that are not a multiple of 128 (replicated
    torus)."""
    monkeypatch.setenv("GOLHIP_VARIANT", variant)
    for (h, w) in [(64, 4160), (35, 2016), (130, 8192), (9, 96), (20, 1984), (24, 3968)]:
        rng = np.random.default_rng(h * 31 + w + k)
        board = ((rng.random((h, w)) < 0.37) * 255).astype(np.uint8)
        turns = 3 * k + 5
        exp, exp_counts = oracle.packed_run(board, turns)
        for band in (0, 3, 40):
            out, counts, cells, count = run_engine(golhip, board, turns, k=k, counts=True, band_rows=band, lib=tuning)
            assert np.array_equal(out, exp), (k, h, w, band)
            assert np.array_equal(counts.astype(np.int64), exp_counts), (k, h, w, band)
            assert count == int((exp == 255).sum())




@pytest.mark.parametrize("split,k", [(s, k) for k in (4, 6, 8, 16, 32) for s in (2, 4, 8)
                                     if k % s == 0])  # levels split evenly over the waves
def test_level_split_kernel(golhip, tuning, oracle, monkeypatch, split, k):
    """The level-split stencil (gol_stencil_split: the K levels of a band over S waves of one
    workgroup, rows handed off through LDS, lockstep barriers) on the shapes that stress wrap,
    half-word halos, short last bands and band seams, with per-turn counts."""
    monkeypatch.setenv("GOLHIP_SPLIT", str(split))
    for (h, w) in [(77, 640), (16, 16), (300, 4160), (129, 200)]:
        rng = np.random.default_rng(h * 7 + w + k + split)
        board = ((rng.random((h, w)) < 0.4) * 255).astype(np.uint8)
        turns = 3 * k + 1
        exp, exp_counts = oracle.packed_run(board, turns)
        for band in (0, 5):
            out, counts, _, _ = run_engine(golhip, board, turns, k=k, counts=True, band_rows=band, lib=tuning)
            assert np.array_equal(out, exp), (split, k, h, w, band)
            assert np.array_equal(counts.astype(np.int64), exp_counts), (split, k, h, w, band)




TILE_CONFIGS = [(2, 16), (4, 8), (4, 16), (4, 32), (6, 16), (8, 8), (8, 16), (8, 32), (10, 16),
                (12, 8), (12, 16), (12, 32), (14, 16), (16, 8), (16, 16), (16, 32)]


@pytest.mark.parametrize("k,tile", TILE_CONFIGS)
def test_register_tile_kernel(golhip, tuning, oracle, monkeypatch, k, tile):
    """The register-tile stencil (gol_tile: T + 2K rows of a 62-word chunk in VGPRs, K
    generations in place) forced at every compiled (K, T): wrap in both directions, boards
    shorter than a tile and than its halo, ragged widths, short last tiles, per-turn counts."""
    monkeypatch.setenv("GOLHIP_TILE", str(tile))
    for (h, w) in [(77, 640), (16, 16), (5, 96), (300, 4160), (129, 200), (40, 8192), (64, 1984)]:
        rng = np.random.default_rng(h * 7 + w + k + tile)
        board = ((rng.random((h, w)) < 0.4) * 255).astype(np.uint8)
        turns = 3 * k + 1
        exp, exp_counts = oracle.packed_run(board, turns)
        out, counts, _, _ = run_engine(golhip, board, turns, k=k, counts=True, lib=tuning)
        assert np.array_equal(out, exp), (k, tile, h, w)
        assert np.array_equal(counts.astype(np.int64), exp_counts), (k, tile, h, w)


@pytest.mark.parametrize("k", [4, 16])
def test_register_tile_tracked_flips(golhip, tuning, oracle, monkeypatch, k):
    """Flips tracking through the tile kernel: the last launch's LD instantiation writes the last
    generation's flips beside its output."""
    monkeypatch.setenv("GOLHIP_TILE", "16")
    h, w = 300, 640
    rng = np.random.default_rng(k)
    board = ((rng.random((h, w)) < 0.4) * 255).astype(np.uint8)
    turns = 2 * k + 1
    before, _ = oracle.packed_run(board, turns - 1)
    exp, _ = oracle.packed_run(board, turns)
    with golhip.Engine(w, h, k=k, lib=tuning) as e:
        e.set_fixed_k(True)
        e.track_flips(True)
        e.load(board)
        e.step(turns)
        assert e.launch_kind(k) == ("tile", 16)
        got = [tuple(c) for c in e.flips().tolist()]
        assert np.array_equal(e.store(), exp)
    assert got == oracle.flips(before, exp)


SLAB_CONFIGS = [(8, 8, 4), (8, 8, 8), (12, 8, 8), (16, 8, 8), (16, 8, 12), (16, 16, 8),
                (16, 8, 12, 2), (16, 12, 8, 2), (16, 12, 8), (16, 12, 7, 2), (16, 10, 8, 2),
                (16, 14, 6, 2),
                # gol_slab2 (NC = 9: the edge hand-off off the critical path)
                (16, 8, 12, 9), (16, 12, 8, 9), (16, 12, 7, 9), (8, 8, 8, 9), (12, 8, 8, 9),
                (16, 16, 5, 9), (16, 8, 8, 9),
                # gol_slab3 (NC = 10: gol_slab2 pipelined across generations)
                (16, 8, 12, 10), (16, 16, 6, 10), (16, 12, 8, 10), (16, 12, 7, 10), (16, 10, 8, 10),
                (16, 8, 10, 10),
                # gol_slab2 with the in-launch count flush whenever S <= K (NC = 11)
                (16, 8, 12, 11), (16, 8, 10, 11), (16, 10, 8, 11), (16, 12, 8, 11),
                # ... and with every generation's counts flushed at the end (NC = 12)
                (16, 12, 7, 12), (16, 12, 8, 12), (16, 16, 6, 12), (16, 16, 5, 12),
                # ... with the younger half of the waves at s_setprio 1 (NC = 13)
                (16, 16, 6, 13), (16, 12, 7, 13), (16, 8, 12, 13),
                # round 5 A/B at 4096^2 with counts: fewer, taller waves (r05t_tune_slab_4096.log)
                (16, 8, 11, 12), (16, 8, 10, 12), (16, 8, 11, 9), (16, 10, 9, 12)]


@pytest.mark.parametrize("cfg", SLAB_CONFIGS)
def test_register_slab_kernel(golhip, tuning, oracle, monkeypatch, cfg):
    """The register-slab stencil (gol_slab: W waves x S rows of a 62-word chunk in VGPRs, edge
    rows swapped through LDS every generation) forced at every compiled (K, W, S): wrap, boards
    shorter than a slab, ragged widths, short last slabs, per-turn counts."""
    k, waves, rows = cfg[:3]
    code = (cfg[3] * 10000 if len(cfg) > 3 else 0) + waves * 100 + rows
    monkeypatch.setenv("GOLHIP_SLAB", str(code))
    for (h, w) in [(77, 640), (16, 16), (5, 96), (300, 4160), (129, 200), (40, 8192), (250, 1984),
                   (100, 4096)]:
        rng = np.random.default_rng(h * 7 + w + k + waves + rows)
        board = ((rng.random((h, w)) < 0.4) * 255).astype(np.uint8)
        turns = 3 * k + 1
        exp, exp_counts = oracle.packed_run(board, turns)
        with golhip.Engine(w, h, k=k, lib=tuning) as e:
            assert e.launch_kind(k) == ("slab", code)
        out, counts, _, _ = run_engine(golhip, board, turns, k=k, counts=True, lib=tuning)
        assert np.array_equal(out, exp), (k, waves, rows, h, w)
        assert np.array_equal(counts.astype(np.int64), exp_counts), (k, waves, rows, h, w)


def test_register_slab_tracked_flips(golhip, tuning, oracle, monkeypatch):
    monkeypatch.setenv("GOLHIP_SLAB", "1608")
    h, w, k = 300, 640, 16
    rng = np.random.default_rng(5)
    board = ((rng.random((h, w)) < 0.4) * 255).astype(np.uint8)
    turns = 2 * k + 1
    before, _ = oracle.packed_run(board, turns - 1)
    exp, _ = oracle.packed_run(board, turns)
    with golhip.Engine(w, h, k=k, lib=tuning) as e:
        e.set_fixed_k(True)
        e.track_flips(True)
        e.load(board)
        e.step(turns)
        got = [tuple(c) for c in e.flips().tolist()]
        assert np.array_equal(e.store(), exp)
    assert got == oracle.flips(before, exp)


@pytest.mark.parametrize("code,k", [(90812, 16), (91208, 16), (91207, 16), (90808, 8), (90808, 12),
                                    (100812, 16), (101208, 16), (101207, 16), (101606, 16), (110812, 16), (121207, 16), (121606, 16), (131606, 16)])
def test_slab2_flips_ring_every_turn(golhip, tuning, oracle, monkeypatch, code, k):
    """gol_slab2 / gol_slab3 writing EVERY generation's flips into the per-turn ring
    (golhip_step_flips) on their production-candidate shapes, with counts: every turn's cells and
    count vs the oracle."""
    monkeypatch.setenv("GOLHIP_SLAB", str(code))
    h, w = 300, 1000
    rng = np.random.default_rng(code)
    board = ((rng.random((h, w)) < 0.4) * 255).astype(np.uint8)
    with golhip.Engine(w, h, k=k, lib=tuning) as e:
        e.load(board)
        prev = oracle.to_cells(board)
        for turns in (k, 2 * k + 3):
            per_turn, alive = e.step_flips(turns, counts=True)
            for t in range(turns):
                cur, _ = oracle.packed_run(prev, 1)
                assert [tuple(c) for c in per_turn[t].tolist()] == oracle.flips(prev, cur), (code, turns, t)
                assert int(alive[t]) == int((cur == 255).sum())
                prev = cur
        assert np.array_equal(e.store(), prev)


PACKED_CONFIGS = [140403, 140404, 140803, 140804, 140806, 141603]


@pytest.mark.parametrize("code", PACKED_CONFIGS)
def test_packed_slab_kernel(golhip, tuning, oracle, monkeypatch, code):
    """gol_slabp (NC = 14): P = 64 / (wd + 2) row segments packed into each wave, for boards of at
    most 62 packed words (1984 cells); P = 10 at 16..128 cells wide, 3 at 512, 1 at 1920 / 1984:
    wrap, short boards, boards shorter than a workgroup, ragged widths, per-turn counts, and the
    last generation's flips (LD = 1)."""
    monkeypatch.setenv("GOLHIP_SLAB", str(code))
    k = 16
    for (h, w) in [(512, 512), (16, 16), (77, 640), (5, 96), (300, 64), (1000, 128), (33, 256),
                   (129, 960), (250, 1984), (40, 1000), (700, 512)]:
        rng = np.random.default_rng(h * 7 + w + code)
        board = ((rng.random((h, w)) < 0.4) * 255).astype(np.uint8)
        turns = 3 * k + 1
        exp, exp_counts = oracle.packed_run(board, turns)
        wd = math.lcm(w, 128) // 32
        waves, rows = code // 100 % 100, code % 100
        packed = waves * (64 // (wd + 2)) * rows - 2 * k >= 1  # else the engine streams
        with golhip.Engine(w, h, k=k, lib=tuning) as e:
            assert (e.launch_kind(k) == ("slab", code)) == packed, (h, w)
        out, counts, _, _ = run_engine(golhip, board, turns, k=k, counts=True, lib=tuning)
        assert np.array_equal(out, exp), (code, h, w)
        assert np.array_equal(counts.astype(np.int64), exp_counts), (code, h, w)
    h, w = 300, 512
    rng = np.random.default_rng(code)
    board = ((rng.random((h, w)) < 0.4) * 255).astype(np.uint8)
    before, _ = oracle.packed_run(board, 2 * k - 1)
    exp, _ = oracle.packed_run(board, 2 * k)
    with golhip.Engine(w, h, k=k, lib=tuning) as e:
        e.set_fixed_k(True)
        e.track_flips(True)
        e.load(board)
        e.step(2 * k)
        assert e.launch_kind(k) == ("slab", code)
        got = [tuple(c) for c in e.flips().tolist()]
        assert np.array_equal(e.store(), exp)
    assert got == oracle.flips(before, exp)


def _stamps(tuning, e):
    """golhip_tuning_stamps_ex: (records, words per wave) of the last stamped launch."""
    import ctypes

    f = tuning.golhip_tuning_stamps_ex
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                  ctypes.POINTER(ctypes.c_int)]
    f.restype = ctypes.c_int
    n, wpw = ctypes.c_size_t(0), ctypes.c_int(0)
    assert f(e._h, None, 0, ctypes.byref(n), ctypes.byref(wpw)) == 0
    out = np.zeros(max(n.value, 8), dtype=np.uint64)
    assert f(e._h, out.ctypes.data, out.size, ctypes.byref(n), ctypes.byref(wpw)) == 0
    return out[: n.value].copy(), wpw.value


def test_stamp_variant_k1_then_deep(golhip, tuning, monkeypatch):
    """Pins the round-4 stamp-variant fix (csrc/tuning/engine_tuning.hip launch_params): only the
    streaming gol_stencil takes the stamp buffer as its p.diff.  Round 4's K = 1 warm-up launch
    (gol_step1) wrote its flips board over the 32 MiB stamp buffer (an illegal memory access,
    profiles/r04/r04d_stamps_fault.log, r04f_stamps_fault.log).  Here, on the bench board (65536^2
    random p = 0.5, seed 3) with GOLHIP_VARIANT=stamp: K = 1, then K = 12 launches, K = 1 again,
    then K = 14 launches; the stamp records are the streaming kernel's (4 words per wave, start <=
    end, shader cycles counted), a K = 1 launch leaves them untouched, and the board digest after
    25 and 1008 turns matches tests/golden/synthetic_golden.json."""
    import bench

    monkeypatch.setenv("GOLHIP_VARIANT", "stamp")
    n = 65536
    d25, d1008 = bench.golden_digest(n, n, 3, 25), bench.golden_digest(n, n, 3, 1008)
    assert d25 and d1008

    def well_formed(st, wpw):
        assert wpw == 4, wpw  # gol_stencil's record; gol_slab2's phase stamps are 8 words
        rec = st.reshape(-1, 4)
        assert len(rec) > 0
        assert (rec[:, 0] > 0).all() and (rec[:, 1] >= rec[:, 0]).all() and (rec[:, 2] > 0).all()

    with golhip.Engine(n, n, k=12, lib=tuning) as e:
        assert e.launch_kind(12) == ("stream", 0)
        e.set_fixed_k(True)
        e.init_random(3)
        e.step(1)  # gol_step1: no stamps
        assert _stamps(tuning, e)[0].size == 0
        e.step(24)  # 12 + 12
        st, wpw = _stamps(tuning, e)
        well_formed(st, wpw)
        assert bench.board_digest(e.store_words(), 1) == d25
        e.step(1)  # K = 1 again: the stamps of the last K = 12 launch stay as they were
        st2, _ = _stamps(tuning, e)
        assert np.array_equal(st, st2)
        e.set_k(14)
        e.step(982)  # 70 x 14 + a 2-deep tail
        well_formed(*_stamps(tuning, e))
        assert bench.board_digest(e.store_words(), 1) == d1008



@pytest.mark.parametrize("code", [151207, 151606, 151204, 151604, 151208, 150812])
def test_slab2_neighbour_flags(golhip, tuning, oracle, monkeypatch, code):
    """gol_slab2 with point-to-point LDS flags between neighbour waves instead of the per-generation
    barrier (NC = 15; the halo waves post their last flag and leave early): boards and counts at
    every turn, calls of K and of a K-tail, short boards (a band shorter than the halo), ragged
    widths, and the last generation's flips (LD = 1), against the oracle."""
    monkeypatch.setenv("GOLHIP_SLAB", str(code))
    k = 16
    for (h, w) in [(300, 1000), (1024, 4096), (77, 640), (33, 2000), (700, 8192), (129, 96)]:
        rng = np.random.default_rng(h * 7 + w + code)
        board = ((rng.random((h, w)) < 0.4) * 255).astype(np.uint8)
        turns = 3 * k + 5
        exp, exp_counts = oracle.packed_run(board, turns)
        with golhip.Engine(w, h, k=k, lib=tuning) as e:
            assert e.launch_kind(k, counts=True) == ("slab", code), (h, w)
        out, counts, _, _ = run_engine(golhip, board, turns, k=k, counts=True, lib=tuning)
        assert np.array_equal(out, exp), (code, h, w)
        assert np.array_equal(counts.astype(np.int64), exp_counts), (code, h, w)
    h, w = 300, 1000
    rng = np.random.default_rng(code)
    board = ((rng.random((h, w)) < 0.4) * 255).astype(np.uint8)
    before, _ = oracle.packed_run(board, 2 * k - 1)
    exp, _ = oracle.packed_run(board, 2 * k)
    with golhip.Engine(w, h, k=k, lib=tuning) as e:
        e.set_fixed_k(True)
        e.track_flips(True)
        e.load(board)
        e.step(2 * k)
        got = [tuple(c) for c in e.flips().tolist()]
        assert np.array_equal(e.store(), exp)
    assert got == oracle.flips(before, exp)
