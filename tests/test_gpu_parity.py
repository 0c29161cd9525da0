"""GPU parity: libgolhip (through its C ABI) against the oracle and the reference's fixtures.

Bit-exact for every board, count and cell list (integer/byte work: no tolerance).
"""
import math

import numpy as np
import pytest

from conftest import REF

pytestmark = pytest.mark.gpu

SIZES = [16, 64, 512]
KS = [1, 2, 4, 8, 16, 32]


def run_engine(golhip, board, turns, k=1, counts=False, band_rows=0, lib=None):
    h, w = board.shape
    with golhip.Engine(w, h, k=k, lib=lib) as e:
        e.set_fixed_k(True)  # launches exactly k deep (the planner would pick its fastest <= k)
        if band_rows:
            e.set_band_rows(band_rows)
        e.load(board)
        c = e.step(turns, counts=counts)
        return e.store(), c, e.alive_cells(), e.alive_count()


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("turns", [0, 1, 100])
def test_check_images(golhip, oracle, n, turns):
    """TestGol / TestPgm (gol_test.go:15-47, pgm_test.go:10-42): final board == check image."""
    _, _, board = oracle.read_pgm(REF / f"images/{n}x{n}.pgm")
    expected_pgm = (REF / f"check/images/{n}x{n}x{turns}.pgm").read_bytes()
    _, _, expected = oracle.read_pgm(REF / f"check/images/{n}x{n}x{turns}.pgm")
    for k in (1, 8, 32):
        out, _, cells, count = run_engine(golhip, board, turns, k=k)
        assert oracle.pgm_bytes(out) == expected_pgm, (n, turns, k)
        exp_cells = oracle.alive_cells(expected)
        assert [tuple(c) for c in cells.tolist()] == exp_cells
        assert count == len(exp_cells)


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("k", [1, 8, 16])
def test_alive_csv_every_turn(golhip, oracle, n, k):
    """check/alive/NxN.csv: the count after every one of 10000 turns (count_test.go, sdl_test.go)."""
    _, _, board = oracle.read_pgm(REF / f"images/{n}x{n}.pgm")
    expected = oracle.read_alive_csv(REF / f"check/alive/{n}x{n}.csv")
    _, counts, _, _ = run_engine(golhip, board, 10000, k=k, counts=True)
    assert [int(c) for c in counts] == [expected[t] for t in range(1, 10001)]


@pytest.mark.parametrize("shape", [(128, 128), (96, 200), (300, 128), (1000, 640), (257, 4096),
                                   (2048, 2048), (40, 8192), (33, 12800)])
@pytest.mark.parametrize("k", KS)
def test_random_boards_vs_oracle(golhip, oracle, shape, k):
    h, w = shape
    rng = np.random.default_rng(h * 7919 + w)
    board = ((rng.random(shape) < 0.45) * 255).astype(np.uint8)
    turns = 2 * k + 3
    exp, exp_counts = oracle.packed_run(board, turns)
    for band in (0, 5, 64):
        out, counts, _, _ = run_engine(golhip, board, turns, k=k, counts=True, band_rows=band)
        assert np.array_equal(out, exp), (shape, k, band)
        assert np.array_equal(counts.astype(np.int64), exp_counts), (shape, k, band)


def test_flips_match_oracle(golhip, oracle):
    """CellFlipped per turn (gol/distributor.go:53-59) from the XOR + compaction kernels, after
    one-generation steps and -- with flips tracking -- after k-deep steps (the last launch writes
    the last generation's flips beside its output)."""
    _, _, board = oracle.read_pgm(REF / "images/512x512.pgm")
    with golhip.Engine(512, 512, k=8) as e:
        e.load(board)
        prev = board.copy()
        for t in range(20):
            e.step(1)
            cur = e.store()
            got = [tuple(c) for c in e.flips().tolist()]
            assert got == oracle.flips(prev, cur)
            prev = cur
        e.step(8)  # untracked k-deep step: the previous generation is not held
        with pytest.raises(golhip.GolHipError):
            e.flips()
        e.track_flips(True)
        for n in (8, 13, 1, 16):
            before = e.store()
            e.step(n)
            after = e.store()
            gen_prev, _ = oracle.packed_run(before, n - 1)
            assert [tuple(c) for c in e.flips().tolist()] == oracle.flips(gen_prev, after), n


def tracked_flips_every_depth(golhip, oracle, k, strips, lib=None):
    """Flips tracking at a launch depth on the single-strip and multi-strip (halo) paths:
    golhip_flips after a k-deep step == the oracle's diff of the last two generations."""
    h, w = 111, 4160
    if h // strips < k:
        pytest.skip("strip shorter than k")
    words = oracle.init_random(w, h, seed=k * 10 + strips)
    with golhip.Engine(w, h, ngpus=1, k=k, strips=strips, lib=lib) as e:
        e.set_fixed_k(True)
        e.track_flips(True)
        e.load_words(words)
        for n in (k, 2 * k + 1):
            before = oracle.unpack(e.store_words(), w)
            e.step(n)
            after = oracle.unpack(e.store_words(), w)
            gen_prev, _ = oracle.packed_run(before, n - 1)
            assert [tuple(c) for c in e.flips().tolist()] == oracle.flips(gen_prev, after), n


@pytest.mark.parametrize("k", [1, 2, 6, 12, 16, 32])
@pytest.mark.parametrize("strips", [1, 3])
def test_tracked_flips_every_depth(golhip, oracle, k, strips):
    """The production kernels (the other drift geometries: tests/test_gpu_tuning.py)."""
    tracked_flips_every_depth(golhip, oracle, k, strips)


def test_tracked_flips_small_board_graphs(golhip, oracle):
    """Small boards replay captured graphs; with tracking the last launch stays a plain,
    flips-writing launch."""
    _, _, board = oracle.read_pgm(REF / "images/512x512.pgm")
    gen_prev, _ = oracle.packed_run(board, 299)
    expected, _ = oracle.packed_run(board, 300)
    with golhip.Engine(512, 512, k=16) as e:
        e.set_graphs(1)
        e.track_flips(True)
        e.load(board)
        e.step(300)
        assert np.array_equal(e.store(), expected)
        assert [tuple(c) for c in e.flips().tolist()] == oracle.flips(gen_prev, expected)


@pytest.mark.parametrize("k,counts", [(8, True), (16, True), (16, False), (12, False)])
@pytest.mark.parametrize("shape,strips", [((512, 512), 1), ((96, 640), 1), ((300, 1000), 2),
                                          ((130, 4160), 4), ((16, 16), 1), ((1000, 2000), 1)])
def test_step_flips_ring_every_turn(golhip, oracle, shape, strips, k, counts):
    """golhip_step_flips: every turn's CellFlipped (turn by turn, row-major) and alive count from
    ONE extraction over the device ring of per-turn flips boards -- the TestSdl event stream
    (sdl_test.go:57-74) -- equal to the oracle's per-turn diffs.  Single-strip small boards fill
    the ring with K-deep register-slab launches that write EVERY generation's flips (K = 8/12/16
    slots per launch, the counting and non-counting slab shapes); strips and the tail of a call
    use one-generation launches."""
    h, w = shape
    rng = np.random.default_rng(h * 3 + w + strips)
    board = ((rng.random(shape) < 0.4) * 255).astype(np.uint8)
    with golhip.Engine(w, h, ngpus=1, k=k, strips=strips) as e:
        e.load(board)
        assert e.flips_ring_capacity() >= 40
        prev = oracle.to_cells(board)
        for turns in (1, 17, 40, 33):
            per_turn, alive = e.step_flips(turns, counts=counts)
            assert len(per_turn) == turns
            for t in range(turns):
                cur, _ = oracle.packed_run(prev, 1)
                assert [tuple(c) for c in per_turn[t].tolist()] == oracle.flips(prev, cur), (turns, t)
                if counts:
                    assert int(alive[t]) == int((cur == 255).sum())
                prev = cur
        assert np.array_equal(e.store(), prev)
        assert [tuple(c) for c in e.flips().tolist()] == [tuple(c) for c in per_turn[-1].tolist()]


def test_step_flips_sdl_512_every_count(golhip, oracle):
    """TestSdl (sdl_test.go:57-74,107-116): a shadow board toggled by every CellFlipped of 100
    turns of images/512x512.pgm, its alive count at each TurnComplete equal to check/alive's CSV --
    through 16-deep ring launches (gol_slab writing every generation's flips)."""
    _, _, board = oracle.read_pgm(REF / "images/512x512.pgm")
    csv = oracle.read_alive_csv(REF / "check/alive/512x512.csv")
    shadow = (board == 255)
    with golhip.Engine(512, 512, k=16) as e:
        e.load(board)
        # 512 rows: golhip_step runs this board with the slab kernels (the whole-board kernel is
        # automatic up to 256 rows); the flips ring with slabs
        assert e.launch_kind(16)[0] == "slab"
        t0 = 0
        for turns in (64, 36):
            per_turn, _ = e.step_flips(turns)
            for t, cells in enumerate(per_turn):
                shadow[cells[:, 1], cells[:, 0]] ^= True
                assert int(shadow.sum()) == csv[t0 + t + 1], t0 + t + 1
            t0 += turns
        assert np.array_equal(shadow * 255, e.store())


@pytest.mark.parametrize("shape", [(512, 512), (16, 16), (77, 640), (300, 4160)])
@pytest.mark.parametrize("k", [1, 16])
def test_step_flips_rows_every_turn(golhip, oracle, shape, k):
    """golhip_step_flips_rows: the same per-turn flips as golhip_step_flips in the compact form
    (uint16 x + per-turn-row offsets), expanded and compared with the oracle's per-turn diffs, and
    interleaved with golhip_step_flips on the same engine (the ring is shared)."""
    h, w = shape
    rng = np.random.default_rng(h * 5 + w + k)
    board = ((rng.random(shape) < 0.4) * 255).astype(np.uint8)
    with golhip.Engine(w, h, k=k) as e:
        e.load(board)
        prev = oracle.to_cells(board)
        for turns, rows_api in ((17, True), (5, False), (40, True)):
            if rows_api:
                x, offs, alive = e.step_flips_rows(turns, counts=True)
                assert offs[0] == 0 and int(offs[-1]) == len(x)
                per_turn = e.rows_to_cells(x, offs, h, turns)
            else:
                per_turn, alive = e.step_flips(turns, counts=True)
            for t in range(turns):
                cur, _ = oracle.packed_run(prev, 1)
                assert [tuple(c) for c in per_turn[t].tolist()] == oracle.flips(prev, cur), (turns, t)
                assert int(alive[t]) == int((cur == 255).sum())
                prev = cur
        assert np.array_equal(e.store(), prev)


def test_step_flips_rows_errors(golhip, oracle):
    import ctypes

    _, _, board = oracle.read_pgm(REF / "images/64x64.pgm")
    n = ctypes.c_size_t(0)
    offs = np.zeros(3 * 64 + 1, np.uint64)
    with golhip.Engine(64, 64) as e:
        e.load(board)
        rc = e._L.golhip_step_flips_rows(e._h, 3, None, 0, ctypes.byref(n), offs.ctypes.data, None)
        assert rc == golhip.ERR_CAP and n.value > 0 and int(offs[-1]) == n.value
        x = np.empty(n.value, np.uint16)
        assert e._L.golhip_flips_fetch_rows(e._h, x.ctypes.data, n.value, ctypes.byref(n), offs.ctypes.data) == 0
        assert e.turn == 3
        got = e.rows_to_cells(x, offs, 64, 3)
        cur = oracle.to_cells(board)
        for t in range(3):
            nxt, _ = oracle.packed_run(cur, 1)
            assert [tuple(c) for c in got[t].tolist()] == oracle.flips(cur, nxt)
            cur = nxt
        rc = e._L.golhip_step_flips_rows(e._h, 1, None, 0, ctypes.byref(n), None, None)
        assert rc == golhip.ERR_ARG  # row_offsets is required
    with golhip.Engine(64, 64, strips=2) as e:
        e.load(board)
        rc = e._L.golhip_step_flips_rows(e._h, 1, None, 0, ctypes.byref(n), offs.ctypes.data, None)
        assert rc == golhip.ERR_STATE  # one strip per handle


def test_step_flips_capacity_errors(golhip, oracle):
    import ctypes

    _, _, board = oracle.read_pgm(REF / "images/64x64.pgm")
    with golhip.Engine(64, 64) as e:
        e.load(board)
        cap = e.flips_ring_capacity()
        n = ctypes.c_size_t(0)
        rc = e._L.golhip_step_flips(e._h, cap + 1, None, 0, ctypes.byref(n), None, None)
        assert rc == golhip.ERR_ARG
        rc = e._L.golhip_step_flips(e._h, 3, None, 0, ctypes.byref(n), None, None)
        assert rc == golhip.ERR_CAP and n.value > 0  # turns advanced; fetch returns the cells
        buf = np.empty((n.value, 2), np.int32)
        assert e._L.golhip_flips_fetch(e._h, buf.ctypes.data, n.value, ctypes.byref(n), None) == 0
        assert e.turn == 3


def test_init_random_matches_oracle(golhip, oracle):
    for (w, h, seed, dens) in [(128, 64, 2, golhip.DENSITY_HALF), (192, 50, 3, 1 << 30),
                               (5120, 16, 2, golhip.DENSITY_HALF)]:
        with golhip.Engine(w, h) as e:
            e.init_random(seed, dens)
            assert np.array_equal(e.store_words(), oracle.init_random(w, h, seed, dens))


def test_words_roundtrip_and_steps(golhip, oracle):
    w, h = 5120, 96
    words = oracle.init_random(w, h, seed=5)
    with golhip.Engine(w, h, k=4) as e:
        e.load_words(words)
        assert np.array_equal(e.store_words(), words)
        counts = e.step(9, counts=True)
        ref = words.copy()
        ref_counts = oracle.packed_run_words(ref, 9)
        assert np.array_equal(e.store_words(), ref)
        assert np.array_equal(counts.astype(np.int64), ref_counts)


def test_turn_counter(golhip):
    with golhip.Engine(128, 128, k=8) as e:
        e.init_random(1)
        e.step(13)
        assert e.turn == 13
        e.turn = 100
        assert e.turn == 100


def test_cap_error_reports_required_count(golhip, oracle):
    _, _, board = oracle.read_pgm(REF / "images/64x64.pgm")
    with golhip.Engine(64, 64) as e:
        e.load(board)
        import ctypes
        n = ctypes.c_size_t(0)
        buf = np.empty((10, 2), np.int32)
        rc = e._L.golhip_alive_cells(e._h, buf.ctypes.data, 10, ctypes.byref(n))
        assert rc == golhip.ERR_CAP and n.value == 2819


@pytest.mark.parametrize("strips", [2, 3, 4, 8])
@pytest.mark.parametrize("k", [1, 4, 8, 16])
def test_row_strips_with_halo_exchange(golhip, oracle, strips, k):
    """The multi-strip path (halo rows, interior/boundary launches, exchange, count reduction)
    with several strips on the box's one GPU; must equal the single-board oracle bit for bit."""
    w, h = 640, 37 * strips + 5
    if h // strips < k:
        pytest.skip("strip shorter than k")
    words = oracle.init_random(w, h, seed=strips * 100 + k)
    turns = 3 * k + 1
    with golhip.Engine(w, h, ngpus=1, k=k, strips=strips) as e:
        assert e.info.world_size == strips and e.info.halo_rows == k
        e.load_words(words)
        counts = e.step(turns, counts=True)
        got = e.store_words()
        cells = e.alive_cells()
        n = e.alive_count()
        e.step(1)
        flips = e.flips()
        after = e.store_words()
    ref = words.copy()
    ref_counts = oracle.packed_run_words(ref, turns)
    assert np.array_equal(got, ref)
    assert np.array_equal(counts.astype(np.int64), ref_counts)
    board = oracle.unpack(ref, w)
    assert [tuple(c) for c in cells.tolist()] == oracle.alive_cells(board)
    assert n == len(cells)
    ref2 = ref.copy()
    oracle.packed_run_words(ref2, 1)
    assert np.array_equal(after, ref2)
    assert [tuple(c) for c in flips.tolist()] == oracle.flips(board, oracle.unpack(ref2, w))


@pytest.mark.parametrize("k", [1, 4, 16])
def test_rank_mode_rccl_ring_of_one(golhip, oracle, monkeypatch, k):
    """Rank mode (golhip_create_rank) as a ring of ONE halo'd strip (GOLHIP_RING_SELF test hook):
    the halos go through ncclSend/ncclRecv to itself in one group on the comm stream, the
    interior launch overlaps them, the boundary bands wait for them, and per-turn counts go
    through ncclAllReduce -- the RCCL path bench.py --gpus N uses, on the box's one GPU."""
    monkeypatch.setenv("GOLHIP_RING_SELF", "1")
    w, h = 640, 5 * k + 37
    words = oracle.init_random(w, h, seed=500 + k)
    turns = 3 * k + 2
    with golhip.Engine(w, h, k=k, rank=0, world_size=1, device=0) as e:
        assert e.info.halo_rows == k and e.info.world_size == 1
        e.load_words(words)
        counts = e.step(turns, counts=True)
        got = e.store_words()
        n = e.alive_count()
    ref = words.copy()
    ref_counts = oracle.packed_run_words(ref, turns)
    assert np.array_equal(got, ref)
    assert np.array_equal(counts.astype(np.int64), ref_counts)
    assert n == int(ref_counts[-1])


def test_row_strips_bytes_roundtrip(golhip, oracle):
    _, _, board = oracle.read_pgm(REF / "images/512x512.pgm")
    with golhip.Engine(512, 512, ngpus=1, k=8, strips=4) as e:
        e.load(board)
        assert np.array_equal(e.store(), oracle.to_cells(board))
        e.step(100)
        out = e.store()
    assert oracle.pgm_bytes(out) == (REF / "check/images/512x512x100.pgm").read_bytes()


@pytest.mark.parametrize("k", [1, 8, 32])
def test_graph_replay_matches_launches(golhip, oracle, k):
    """Small boards replay captured graphs of step blocks; both buffer parities, with and
    without per-turn counts, must equal the oracle."""
    w, h = 1000, 300
    words = oracle.init_random(1024, h, seed=k)[:, :]
    board = oracle.unpack(words, w)
    with golhip.Engine(w, h, k=k) as e:
        e.set_graphs(1)
        e.load(board)
        e.step(1)                                  # odd parity before the graphs
        c1 = e.step(300, counts=True)              # graph replays + tail blocks
        e.step(257)                                # graphs without counts
        got = e.store()
        cells = e.alive_cells()
    exp, exp_counts = oracle.packed_run(board, 1 + 300 + 257)
    assert np.array_equal(got, exp)
    assert np.array_equal(c1.astype(np.int64), exp_counts[1:301])
    assert len(cells) == int((exp == 255).sum())


@pytest.mark.parametrize("k", [2, 8, 12, 14, 16])
def test_counting_and_plain_launches_interleaved(golhip, oracle, k):
    """Production picks the column geometry per launch (pre-shifted 63-word chunks without counts,
    62-word chunks with counts below K = 16): steps with and without per-turn counts interleaved
    on one engine, streaming kernel (explicit band height), equal to the oracle after each."""
    for (h, w, band) in [(300, 4160, 40), (97, 2016, 24), (64, 65536, 16)]:
        rng = np.random.default_rng(h + w + k)
        board = ((rng.random((h, w)) < 0.4) * 255).astype(np.uint8)
        with golhip.Engine(w, h, k=k) as e:
            e.set_fixed_k(True)
            e.set_band_rows(band)
            e.load(board)
            cur = oracle.to_cells(board)
            for n, counts in ((2 * k + 1, True), (k + 3, False), (k, True), (3 * k, False)):
                c = e.step(n, counts=counts)
                exp, exp_counts = oracle.packed_run(cur, n)
                assert np.array_equal(e.store(), exp), (k, h, w, n, counts)
                if counts:
                    assert np.array_equal(c.astype(np.int64), exp_counts), (k, h, w, n)
                cur = exp


@pytest.mark.parametrize("k", [1, 2, 8, 12, 16])
def test_graded_tail_bands(golhip, oracle, k):
    """Graded bands (golhip_set_tail_bands): range 0 ends in short bands after the full-height
    ones -- band seams at both heights, a partial last tail band, a tail longer than the rows
    (ignored), on the streaming kernels (explicit band height) with per-turn counts."""
    for (h, w) in [(300, 4160), (131, 2016), (77, 640)]:
        rng = np.random.default_rng(h * 13 + w + k)
        board = ((rng.random((h, w)) < 0.41) * 255).astype(np.uint8)
        turns = 2 * k + 3
        exp, exp_counts = oracle.packed_run(board, turns)
        for band, tail in [(40, (3, 9)), (64, (5, 13)), (24, (1, 8)), (40, (100, 20))]:
            with golhip.Engine(w, h, k=k) as e:
                e.set_fixed_k(True)
                e.set_band_rows(band)
                e.set_tail_bands(*tail)
                e.load(board)
                c = e.step(turns, counts=True)
                assert np.array_equal(e.store(), exp), (k, h, w, band, tail)
                assert np.array_equal(c.astype(np.int64), exp_counts), (k, h, w, band, tail)


def test_small_board_5120x512_vs_oracle(golhip, oracle):
    """A configs[1]-wide short board on the automatic kernel choice, every count vs the oracle."""
    words = oracle.init_random(5120, 512, seed=2)
    with golhip.Engine(5120, 512, k=16) as e:
        e.load_words(words)
        counts = e.step(200, counts=True)
        got = e.store_words()
    ref_counts = oracle.packed_run_words(words, 200)
    assert np.array_equal(got, words)
    assert np.array_equal(counts.astype(np.int64), ref_counts)


@pytest.mark.parametrize("k", [6, 16])
def test_count_window_flushes(golhip, oracle, k):
    """Per-turn counts go through a count window finalized once per window: with the window at
    its 128-generation minimum and graphs off, a 700-turn call flushes it several times (K = 6
    does not divide it); every count must equal the oracle's and the board must match."""
    w, h = 640, 200
    board = oracle.unpack(oracle.init_random(640, h, seed=11), w)
    with golhip.Engine(w, h, k=k) as e:
        e.step(20, counts=True)  # counts through the default window first, then resize it
        e.set_count_window(128)
        e.set_graphs(0)
        e.load(board)
        c = e.step(700, counts=True)
        got = e.store()
    exp, exp_counts = oracle.packed_run(board, 700)
    assert np.array_equal(got, exp)
    assert np.array_equal(c.astype(np.int64), exp_counts)  # exp_counts[i]: after turn i + 1


def test_small_board_picks_register_slab(golhip, oracle):
    """configs[1]-sized boards take the register-slab path automatically (with the planner's own
    depth choice); results unchanged, counts every turn."""
    # the shape model (pick_reg_kernel) over the gol_slab2 shapes: configs[1] 5120^2 takes 16 x 6
    # (240 slabs, 24 rows per SIMD; the measured order breaks the tie with 8 x 12 / 12 x 8), with
    # counts flushed at the end of the launch (NC = 12); configs[4] 4096^2 takes 12 x 7 (237 slabs,
    # 21 rows per SIMD), the same way with counts
    with golhip.Engine(5120, 5120, k=16) as e:
        assert e.launch_kind(16) == ("slab", 91606)
        assert e.launch_kind(16, counts=True) == ("slab", 121606)
        assert e.launch_kind(8) == ("slab", 808)
        assert e.launch_kind(8, counts=True) == ("slab", 808)
    with golhip.Engine(4096, 4096, k=16) as e:
        assert e.launch_kind(16) == ("slab", 91207)
        assert e.launch_kind(16, counts=True) == ("slab", 121207)
    words = oracle.init_random(5120, 512, seed=2)
    with golhip.Engine(5120, 512, k=16) as e:
        assert e.launch_kind(16, counts=True)[0] == "slab"
        e.load_words(words)
        counts = e.step(200, counts=True)
        got = e.store_words()
    ref_counts = oracle.packed_run_words(words, 200)
    assert np.array_equal(got, words)
    assert np.array_equal(counts.astype(np.int64), ref_counts)


def test_two_chunk_board_takes_16x4_slabs(golhip, oracle):
    """A board of two 62-word chunks at 4096 rows (3968 x 4096: 124 packed words) fits 16 x 4 slabs
    (T = 32, 256 slabs) in one round over the CUs, 16 rows per SIMD against 12 x 7's 21
    (pick_reg_kernel, round 5): every count and the board against the oracle through golhip_step
    with and without counts and through golhip_step_persistent."""
    w, h = 3968, 4096
    board = oracle.unpack(oracle.init_random(w, h, seed=7), w)
    ref = board.copy()
    import torch

    if torch.cuda.get_device_properties(0).multi_processor_count < 256:
        pytest.skip("the 16 x 4 choice needs 256 CUs for this board")
    with golhip.Engine(w, h, k=16) as e:
        assert e.launch_kind(16) == ("slab", 91604)
        assert e.launch_kind(16, counts=True) == ("slab", 121604)
        e.load(board)
        c = e.step(300, counts=True)
        ref, exp = oracle.packed_run(ref, 300)
        assert np.array_equal(c.astype(np.int64), exp)
        e.step(133)
        ref, _ = oracle.packed_run(ref, 133)
        assert np.array_equal(e.store(), ref)
        c = e.step_persistent(261)
        ref, exp = oracle.packed_run(ref, 261)
        assert np.array_equal(c.astype(np.int64), exp)
        assert np.array_equal(e.store(), ref)


def test_one_round_board_takes_12x4_slabs(golhip, oracle):
    """2048^2 (two 62-word chunks, 2048 rows) fits 12 x 4 slabs (T = 16, 256 slabs, 12 rows per SIMD
    against 16 x 4's 16) in one round over the CUs (pick_reg_kernel, round 6), with and without
    counts: every count, the board and the every-generation flips ring against the oracle."""
    import torch

    if torch.cuda.get_device_properties(0).multi_processor_count < 256:
        pytest.skip("the 12 x 4 choice needs 256 CUs for this board")
    n = 2048
    board = oracle.unpack(oracle.init_random(n, n, seed=17), n)
    ref = board.copy()
    with golhip.Engine(n, n, k=16) as e:
        assert e.launch_kind(16) == ("slab", 91204)
        assert e.launch_kind(16, counts=True) == ("slab", 121204)
        e.load(board)
        c = e.step(333, counts=True)
        ref, exp = oracle.packed_run(ref, 333)
        assert np.array_equal(c.astype(np.int64), exp)
        e.step(160)
        ref, _ = oracle.packed_run(ref, 160)
        assert np.array_equal(e.store(), ref)
        per_turn, alive = e.step_flips(48, counts=True)
        for t in range(48):
            nxt, cnt = oracle.packed_run(ref, 1)
            ys, xs = np.nonzero(ref != nxt)
            assert np.array_equal(per_turn[t], np.stack([xs, ys], 1).astype(np.int32)), t
            assert int(alive[t]) == int(cnt[0]), t
            ref = nxt
        assert np.array_equal(e.store(), ref)


@pytest.mark.parametrize("stage", [0, 4096])
@pytest.mark.parametrize("shape", [(512, 512), (300, 1000), (96, 640), (40, 6)])
def test_store_interleaved_with_steps(golhip, oracle, monkeypatch, tmp_path, stage, shape):
    """The `s` snapshot path (gol/distributor.go:93-103,118-119): store_bytes / store_words /
    checkpoint save+load between steps, through the shard's preallocated stage (no per-call device
    allocation).  stage = 4096 shrinks the stage (GOLHIP_STAGE_BYTES) so every transfer runs in
    many row chunks; each snapshot must equal the oracle at that turn."""
    if stage:
        monkeypatch.setenv("GOLHIP_STAGE_BYTES", str(stage))
    h, w = shape
    rng = np.random.default_rng(5)
    board = np.where(rng.random((h, w)) < 0.4, 255, 0).astype(np.uint8)
    ref = board.copy()
    with golhip.Engine(w, h, k=16) as e:
        e.load(board)
        for i, n in enumerate([1, 16, 7, 33]):
            e.step(n)
            ref, _ = oracle.packed_run(ref, n)
            assert np.array_equal(e.store(), ref), (i, n)
            if w % 64 == 0:
                assert np.array_equal(e.store_words(), oracle.pack(ref)[:, : w // 64])
                e.load_words(oracle.pack(ref)[:, : w // 64])  # reload: the stage in the other way
        e.checkpoint_save(str(tmp_path / "ckpt.bin"))
        e.step(5)
        e.checkpoint_load(str(tmp_path / "ckpt.bin"))
        assert np.array_equal(e.store(), ref)
        e.step(3)
        ref, _ = oracle.packed_run(ref, 3)
        assert np.array_equal(e.store(), ref)


@pytest.mark.parametrize("width,height,turns", [(65536, 65536, 120), (262144, 32768, 48), (16384, 8192, 333)])
def test_ring_of_one_equals_single_strip_at_scale(golhip, monkeypatch, width, height, turns):
    """The rank-mode halo path (ring of one: the early exchange, the boundary bands on the edge
    stream, the interior on the compute stream) against the single wrapped strip on the bench's own
    strip shapes -- where the interior launch takes hundreds of us, so a missing dependency of the
    boundary bands on the previous interior shows (round 4: the early exchange alone let the bands
    read rows the interior had not written yet; the 1000-turn ring of one diverged).  The single
    strip is pinned to the oracle by the configs tests."""
    res = {}
    for ring in (False, True):
        if ring:
            monkeypatch.setenv("GOLHIP_RING_SELF", "1")
        else:
            monkeypatch.delenv("GOLHIP_RING_SELF", raising=False)
        with golhip.Engine(width, height, k=16, rank=0, world_size=1, device=0) as e:
            assert e.info.halo_rows == (16 if ring else 0)
            e.init_random(3)
            counts = e.step(turns, counts=True)
            e.step(7)  # uncounted launches too (the planner's other kernels)
            res[ring] = (counts.copy(), e.store_words())
    monkeypatch.delenv("GOLHIP_RING_SELF", raising=False)
    assert np.array_equal(res[True][0], res[False][0])
    assert np.array_equal(res[True][1], res[False][1])


@pytest.mark.parametrize("shape", [(12288, 12288, 40), (16384, 8192, 33)])
def test_mid_board_takes_slab(golhip, oracle, shape):
    """Mid-size boards (up to kSlabMaxWaves1PerCu minimal-band waves per CU) run the register
    slab over several rounds of workgroups: the board and every per-turn count against the
    oracle, with counts (end-of-launch flush) and without."""
    w, h, turns = shape
    words = oracle.init_random(w, h, seed=21)
    with golhip.Engine(w, h, k=16) as e:
        assert e.launch_kind(16)[0] == "slab" and e.launch_kind(16, counts=True)[0] == "slab"
        e.load_words(words)
        counts = e.step(turns, counts=True)
        got = e.store_words()
        e.step(turns)
        got2 = e.store_words()
    ref = words.copy()
    ref_counts = oracle.packed_run_words(ref, turns)
    assert np.array_equal(got, ref)
    assert np.array_equal(counts.astype(np.int64), ref_counts)
    oracle.packed_run_words(ref, turns)
    assert np.array_equal(got2, ref)


@pytest.mark.parametrize("shape,code", [((512, 512), 140403), ((512, 4096), 140603), ((640, 640), 140603),
                                        ((256, 16384), 140603), ((128, 2048), 140403), ((64, 64), 140403),
                                        ((384, 384), 140403), ((896, 200), 140603), ((512, 100000), 140803)])
def test_narrow_board_takes_packed_slab(golhip, oracle, shape, code):
    """Narrow boards (at most 30 packed words) run the packed register slab gol_slabp (NC = 14, P =
    64 / (wd + 2) row segments per wave) at the first of 4 / 6 / 8 waves x 3 rows whose workgroups
    fit one round over the CUs: the board and every per-turn count against the oracle, with counts
    and without (the tall 100000-row board only the shape choice)."""
    w, h = shape
    with golhip.Engine(w, h, k=16) as e:
        e.set_board_kernel(False)  # 512^2 and 64^2 fit the whole-board kernel (tests/test_gpu_board.py)
        assert e.launch_kind(16) == ("slab", code)
        assert e.launch_kind(16, counts=True) == ("slab", code)
        if h > 20000:
            return
        words = oracle.init_random(w, h, seed=23)
        e.load_words(words)
        counts = e.step(2 * 16 + 5, counts=True)
        got = e.store_words()
        e.step(48)
        got2 = e.store_words()
    ref = words.copy()
    ref_counts = oracle.packed_run_words(ref, 2 * 16 + 5)
    assert np.array_equal(got, ref)
    assert np.array_equal(counts.astype(np.int64), ref_counts)
    oracle.packed_run_words(ref, 48)
    assert np.array_equal(got2, ref)


def test_counts_pinned_and_device_buffers_interleaved(golhip, oracle):
    """Calls of at most 127 turns return their per-turn counts through pinned host memory, longer
    calls through the device buffer (graph replays): interleaved on one engine, every count and
    the board against the oracle."""
    for k, calls in ((16, (100, 5000, 37, 127, 128, 4096, 1)),
                     # K = 12: a replayed graph is 10 x 12 = 120 generations, so calls of 120-127
                     # turns replay one (device buffer) although they are under 128
                     (12, (119, 120, 121, 127, 5, 240))):
        words = oracle.init_random(512, 512, seed=31 + k)
        ref = words.copy()
        with golhip.Engine(512, 512, k=k) as e:
            e.load_words(words)
            for turns in calls:
                counts = e.step(turns, counts=True)
                assert np.array_equal(counts.astype(np.int64), oracle.packed_run_words(ref, turns)), (k, turns)
            assert np.array_equal(e.store_words(), ref)


def test_short_calls_interleaved_on_a_narrow_board(golhip, oracle):
    """Short calls on a narrow register-slab board (configs[0]'s shape: packed-slab launches of 16
    and the tail depths 12 / 8 / 4 / 2, pinned count return): repeated and interleaved calls with and
    without counts, both buffer parities, a depth change and a count-window change, every count and
    the board against the oracle, and the turn counter."""
    words = oracle.init_random(512, 512, seed=77)
    ref = words.copy()
    with golhip.Engine(512, 512, k=16) as e:
        e.load_words(words)
        turn = 0
        for turns, counts in [(100, True)] * 4 + [(37, True), (100, False), (37, True), (100, True),
                                                   (1, True), (1, True), (3, False), (100, True)]:
            c = e.step(turns, counts=counts)
            exp = oracle.packed_run_words(ref, turns)
            if counts:
                assert np.array_equal(c.astype(np.int64), exp), turns
            turn += turns
            assert e.turn == turn
        e.set_k(12)
        for _ in range(3):
            c = e.step(50, counts=True)
            assert np.array_equal(c.astype(np.int64), oracle.packed_run_words(ref, 50))
        e.set_count_window(128)
        c = e.step(100, counts=True)
        assert np.array_equal(c.astype(np.int64), oracle.packed_run_words(ref, 100))
        assert np.array_equal(e.store_words(), ref)


@pytest.mark.parametrize("handoff", [0, 1])
@pytest.mark.parametrize("case", ["configs4", "configs1"])
def test_persistent_slab_matches_oracle(golhip, oracle, case, handoff):
    """golhip_step_persistent (gol_slabq: a whole count window of 16-generation blocks in ONE
    launch, each slab waiting for its 3 x 3 neighbourhood through device counters instead of a launch
    boundary; both hand-off forms): configs[4]'s board (4096^2 gun + R-pentomino, 12 x 7 slabs, a short last band: 4096 =
    78 x 52 + 40) and configs[1]'s (5120^2 random, 16 x 6); calls of 16 turns, of more than one count
    window (4096 + 512, the count window shrunk to 4096 / 8 for the second engine), a tail under 16
    turns; every count and the board against the oracle; interleaved with golhip_step."""
    from conftest import GOLDEN

    if case == "configs4":
        n = 4096
        board = np.zeros((n, n), dtype=np.uint8)
        golhip.place(board, golhip.parse_rle((GOLDEN / "gosper_gun.rle").read_text()), 64, 64)
        golhip.place(board, golhip.parse_rle((GOLDEN / "r_pentomino.rle").read_text()), 2048, 2048)
        code = 121207
    else:
        n = 5120
        board = oracle.unpack(oracle.init_random(n, n, seed=2), n)
        code = 121606
    ref = board.copy()
    with golhip.Engine(n, n, k=16) as e:
        assert e.launch_kind(16, counts=True) == ("slab", code)
        e.set_persistent_handoff(handoff)  # 0: release/acquire fences (default), 1: sc1 only
        e.load(board)
        if case == "configs1":
            e.set_count_window(512)
        turn = 0
        for turns, persistent in ((16, True), (600, True), (37, False), (1043, True)):
            c = e.step_persistent(turns) if persistent else e.step(turns, counts=True)
            ref, exp = oracle.packed_run(ref, turns)
            assert np.array_equal(c.astype(np.int64), exp), (case, turns)
            turn += turns
            assert e.turn == turn
        assert np.array_equal(e.store(), ref)


def test_persistent_slab_refuses_other_boards(golhip):
    """Boards whose counting launch is not a one-round gol_slab2 slab: GOLHIP_ERR_STATE, no
    device work."""
    for (w, h) in [(512, 512), (65536, 1024), (16384, 16384)]:
        with golhip.Engine(w, h, k=16) as e:
            e.init_random(1)
            with pytest.raises(golhip.GolHipError):
                e.step_persistent(32)
            assert e.turn == 0
    # a board it takes, but with flip tracking on (gol_slabq writes no flips board)
    with golhip.Engine(4096, 4096, k=16) as e:
        e.init_random(1)
        e.track_flips(True)
        with pytest.raises(golhip.GolHipError, match="flip tracking"):
            e.step_persistent(32)
        assert e.turn == 0
        e.track_flips(False)
        e.step_persistent(32)
        assert e.turn == 32


def test_persistent_slab_refuses_without_residency(golhip, oracle):
    """golhip_step_persistent refuses, before any device work, when its slabs cannot all be
    resident: here the caller owns fewer CUs than the board has slabs (golhip_set_persistent_limit,
    e.g. a GPU shared with other work).  GOLHIP_ERR_STATE, the board bit-identical and the turn
    unchanged; with the limit lifted the same call runs and matches the oracle."""
    import hashlib

    n = 4096
    board = oracle.unpack(oracle.init_random(n, n, seed=5), n)
    with golhip.Engine(n, n, k=16) as e:
        e.load(board)
        e.step(16)
        before = hashlib.sha256(e.store_words().tobytes()).hexdigest()
        e.set_persistent_limit(64)  # configs[4]-size boards have 237 slabs
        with pytest.raises(golhip.GolHipError, match="cannot all be resident") as ei:
            e.step_persistent(320)
        assert ei.value.code == -7
        assert e.turn == 16
        assert hashlib.sha256(e.store_words().tobytes()).hexdigest() == before
        e.set_persistent_limit(0)
        c = e.step_persistent(320)
        ref, exp = oracle.packed_run(board, 16 + 320)
        assert np.array_equal(c.astype(np.int64), exp[16:])
        assert np.array_equal(e.store(), ref)
        assert e.turn == 336



def test_persistent_slab_options_validate_and_limit_is_inclusive(golhip, oracle):
    """golhip_set_persistent_handoff takes only GOLHIP_HANDOFF_FENCED / _SC1 and
    golhip_set_persistent_limit only >= 0 (GOLHIP_ERR_ARG otherwise, the setting unchanged); a limit
    equal to the board's slab count (4096^2 at 12 x 7: 237 slabs) admits the call, one fewer refuses it."""
    n = 4096
    board = oracle.unpack(oracle.init_random(n, n, seed=6), n)
    with golhip.Engine(n, n, k=16) as e:
        for bad in (-1, 2, 7):
            with pytest.raises(golhip.GolHipError) as ei:
                e.set_persistent_handoff(bad)
            assert ei.value.code == -1
        with pytest.raises(golhip.GolHipError) as ei:
            e.set_persistent_limit(-3)
        assert ei.value.code == -1
        e.load(board)
        e.set_persistent_limit(236)
        with pytest.raises(golhip.GolHipError, match="cannot all be resident"):
            e.step_persistent(32)
        assert e.turn == 0
        e.set_persistent_limit(237)
        c = e.step_persistent(32)
        ref, exp = oracle.packed_run(board, 32)
        assert np.array_equal(c.astype(np.int64), exp)
        assert np.array_equal(e.store(), ref)


@pytest.mark.parametrize("seed", range(12))
def test_randomized_geometry_sweep(golhip, oracle, seed):
    """Seeded random geometries through the automatic planner (whole-board kernel, packed and
    register slabs, the streaming stencil, whatever it picks): a random width (the torus is
    lcm(width, 128) wide, replicated), height, k, density and 1 or 2 strips, then a random sequence
    of calls (0 to 70 turns, with and without per-turn counts, the odd golhip_step_flips); every
    board, count and flips list against the oracle."""
    rng = np.random.default_rng(1000 + seed)
    for _ in range(3):
        while True:  # the oracle steps the whole lcm(w, 128)-wide torus: keep it <= 64 M cells
            w = int(rng.integers(1, 2500))
            h = int(rng.integers(1, 1500))
            if math.lcm(w, 128) * h <= 1 << 26:
                break
        k = int(rng.integers(1, 33))
        strips = 2 if h // 2 >= k and rng.random() < 0.3 else 1
        board = ((rng.random((h, w)) < rng.uniform(0.05, 0.6)) * 255).astype(np.uint8)
        ref = board.copy()
        with golhip.Engine(w, h, ngpus=1, k=k, strips=strips) as e:
            e.load(board)
            for _ in range(4):
                turns = int(rng.integers(0, 71))
                mode = rng.integers(0, 3)
                if mode == 2 and strips == 1 and w * h <= 1 << 20 and 0 < turns <= 40:
                    per_turn, alive = e.step_flips(turns, counts=True)
                    for t in range(turns):
                        nxt, _ = oracle.packed_run(ref, 1)
                        assert [tuple(c) for c in per_turn[t].tolist()] == oracle.flips(ref, nxt), (w, h, k, t)
                        assert int(alive[t]) == int((nxt == 255).sum())
                        ref = nxt
                    continue
                c = e.step(turns, counts=bool(mode == 1))
                ref, exp = oracle.packed_run(ref, turns)
                if mode == 1:
                    assert np.array_equal(c.astype(np.int64), exp), (w, h, k, strips, turns)
                assert np.array_equal(e.store(), ref), (w, h, k, strips, turns)
