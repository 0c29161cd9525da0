"""Stable-slab skipping (golhip_set_activity, gol_slab2 ACT) is exact: the register-slab launches of
small boards skip every slab whose 3 x 3 neighbourhood did not change in the previous launch's last
generation, and the boards, every per-turn count and the cell lists stay bit-identical to the
oracle and to the same engine with skipping off.

The boards are sparse on purpose (that is where slabs get skipped): gliders that cross slab, band
and chunk seams and wrap the torus, oscillators (period 2 and 15) that keep a slab active for ever,
still lifes, the reference-sized glider gun + R-pentomino of configs[4], and boards whose width is
not a multiple of 128 (the torus replicated horizontally).  Reference semantics: server/server.go:
21-75 (every cell, every turn), gol/distributor.go:153-191 (the alive count of every turn).
"""
import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

GLIDER = np.array([[0, 255, 0], [0, 0, 255], [255, 255, 255]], np.uint8)
BLINKER = np.array([[255, 255, 255]], np.uint8)
BLOCK = np.array([[255, 255], [255, 255]], np.uint8)
# oscillators that keep their slabs active for ever: the period-2 blinker and toad, the period-15
# pentadecathlon
TOAD = np.array([[0, 255, 255, 255], [255, 255, 255, 0]], np.uint8)
PENTADECATHLON = np.array([[0, 0, 255, 0, 0, 0, 0, 255, 0, 0],
                           [255, 255, 0, 255, 255, 255, 255, 0, 255, 255],
                           [0, 0, 255, 0, 0, 0, 0, 255, 0, 0]], np.uint8)


def sparse_board(h, w, seed, n_gliders=6, n_osc=4, n_still=6):
    rng = np.random.default_rng(seed)
    b = np.zeros((h, w), np.uint8)
    import golhip

    def at():
        return int(rng.integers(0, w)), int(rng.integers(0, h))

    for _ in range(n_gliders):  # random orientations: they cross seams and wrap the torus
        g = GLIDER
        for _ in range(int(rng.integers(0, 4))):
            g = np.rot90(g)
        golhip.place(b, np.ascontiguousarray(g), *at())
    for i in range(n_osc):
        golhip.place(b, (BLINKER, TOAD, PENTADECATHLON)[i % 3], *at())
    for _ in range(n_still):
        golhip.place(b, BLOCK, *at())
    return b


def run_engine(golhip, board, k, calls, activity=True, graphs=-1, counts=True):
    h, w = board.shape
    with golhip.Engine(w, h, k=k) as e:
        e.set_activity(activity)
        e.set_graphs(graphs)
        e.load(board)
        cs = [e.step(n, counts=counts) for n in calls]
        out = e.store()
        stats = e.activity_stats()
    return out, (np.concatenate(cs).astype(np.int64) if counts else None), stats


@pytest.mark.parametrize("h,w,calls,graphs", [
    (4096, 4096, [300, 700, 1000], -1),   # configs[4]-sized slabs (12 x 7 with counts)
    (5120, 5120, [640, 640], 1),          # 16 x 6, graph replays of 128-generation blocks
    (2048, 1152, [512, 33, 455], -1),     # 12 x 4 slabs (round 6; 16 x 4 before); tails of other
                                          # depths between
    (1000, 600, [384, 128], 0),           # width not a multiple of 128 (torus replicated 32 times:
                                          # every object is in every chunk of its band, so only 3
                                          # objects), no graphs, a last band of 8 < K rows
                                          # (12 x 4 slabs: 1000 = 62 x 16 + 8)
    (3076, 3072, [512], -1),              # last band 4 rows (16 x 4 slabs: 3076 = 96 x 32 + 4)
    (4164, 4096, [512], -1),              # last band 4 rows (12 x 7 slabs: 4164 = 80 x 52 + 4)
])
def test_sparse_boards_match_oracle(golhip, oracle, h, w, calls, graphs):
    board = sparse_board(h, w, seed=h + w, **({} if w % 128 == 0 else dict(n_gliders=1, n_osc=1, n_still=1)))
    got, counts, (computed, skipped) = run_engine(golhip, board, 16, calls, graphs=graphs)
    ref, ref_counts = oracle.packed_run(board, sum(calls))
    assert np.array_equal(counts, ref_counts), np.nonzero(counts != ref_counts)[0][:10]
    assert np.array_equal(got, ref)
    # the sparse board really skipped slabs (and still computed the active ones)
    assert skipped > 0 and computed > 0, (computed, skipped)


def test_skipping_on_and_off_identical_without_counts_then_with(golhip, oracle):
    """Non-counting and counting launches (their slab kernels differ, same geometry or not) in one
    handle, skipping on vs off: the same board, the same counts."""
    board = sparse_board(3076, 3072, seed=5, n_gliders=12)
    outs = []
    for act in (True, False):
        with golhip.Engine(3072, 3076, k=16) as e:
            e.set_activity(act)
            e.load(board)
            e.step(400)
            c1 = e.step(300, counts=True)
            e.step(129)
            c2 = e.step(271, counts=True)
            outs.append((e.store(), c1, c2, e.activity_stats()))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1], outs[1][1]) and np.array_equal(outs[0][2], outs[1][2])
    assert outs[0][3][1] > 0 and outs[1][3] == (0, 0), (outs[0][3], outs[1][3])  # 3076 = 96 x 32 + 4
    ref, ref_counts = oracle.packed_run(board, 1100)
    assert np.array_equal(outs[0][0], ref)
    assert np.array_equal(outs[0][2].astype(np.int64), ref_counts[-271:])


def test_new_board_and_other_kernels_reset_the_flags(golhip, oracle):
    """Flags of a settled board must not survive a board change: a sparse board runs until most
    slabs are skipped, then a dense random board is loaded and stepped (every slab active again);
    then the per-turn flips ring (slab launches with flips: no skipping) in between.  Every count and
    board against the oracle."""
    w = h = 2048
    sparse = sparse_board(h, w, seed=9)
    dense = oracle.unpack(oracle.init_random(w, h, seed=21), w)
    with golhip.Engine(w, h, k=16) as e:
        e.set_activity(1)  # forced: 80 slabs, automatic skipping needs more slabs than CUs
        e.load(sparse)
        e.step(800, counts=True)
        assert e.activity_stats()[1] > 0
        e.load(dense)
        c = e.step(300, counts=True)
        ref, ref_c = oracle.packed_run(dense, 300)
        assert np.array_equal(c.astype(np.int64), ref_c) and np.array_equal(e.store(), ref)
        per_turn, alive = e.step_flips(32, counts=True)  # ring launches (flips): no skipping
        c2 = e.step(200, counts=True)
        ref2, ref_c2 = oracle.packed_run(ref, 232)
        assert np.array_equal(alive.astype(np.int64), ref_c2[:32])
        assert np.array_equal(c2.astype(np.int64), ref_c2[32:]) and np.array_equal(e.store(), ref2)


def test_configs4_prefix_matches_golden_counts(golhip):
    """configs[4] (4096^2 glider gun at (64, 64) + R-pentomino at (2048, 2048)): the first 20 000
    turns with every count against the committed golden (the board settles and slabs get skipped),
    skipping on; and the same first 4 096 turns with skipping off give the same counts."""
    import json

    gold = json.loads((GOLDEN / "synthetic_golden.json").read_text())
    deltas = np.load(GOLDEN / gold["cfg5"]["counts_1e6_npz"])["deltas"]
    b = np.zeros((4096, 4096), dtype=np.uint8)
    golhip.place(b, golhip.parse_rle((GOLDEN / "gosper_gun.rle").read_text()), 64, 64)
    golhip.place(b, golhip.parse_rle((GOLDEN / "r_pentomino.rle").read_text()), 2048, 2048)
    exp = (int((b == 255).sum()) + np.cumsum(deltas[:20000].astype(np.int64)))
    with golhip.Engine(4096, 4096, k=16) as e:
        e.set_activity(1)  # forced: 237 slabs, automatic skipping needs more slabs than CUs
        e.load(b)
        c = e.step(20000, counts=True)
        computed, skipped = e.activity_stats()
    assert np.array_equal(c.astype(np.int64), exp)
    # the board is still busy early on (the R-pentomino runs ~1 100 generations, the gun emits
    # gliders until its own gliders wrap round the torus and break it up), yet most slabs skip
    assert skipped > computed > 0, (computed, skipped)
    with golhip.Engine(4096, 4096, k=16) as e:
        e.set_activity(False)
        e.load(b)
        c_off = e.step(4096, counts=True)
    assert np.array_equal(c_off.astype(np.int64), exp[:4096])


def test_automatic_policy_by_slab_count(golhip, oracle):
    """Automatic skipping (the default, golhip_set_activity(-1)) runs only on boards with more slabs
    than CUs: at one slab per CU a launch lasts as long as its slowest computed slab, so skipping
    saves nothing there and its flags cost time (profiles/r05/r05l_act_probe.log).  4096^2 (237
    slabs): never skips; 8192^2 sparse (384 slabs): skips, every count against the oracle."""
    b = sparse_board(4096, 4096, seed=3)
    with golhip.Engine(4096, 4096, k=16) as e:
        e.load(b)
        e.step(256, counts=True)
        assert e.activity_stats() == (0, 0)
    b = sparse_board(8192, 8192, seed=4, n_gliders=10)
    with golhip.Engine(8192, 8192, k=16) as e:
        e.load(b)
        c = e.step(320, counts=True)
        computed, skipped = e.activity_stats()
        got = e.store()
    ref, ref_c = oracle.packed_run(b, 320)
    assert np.array_equal(c.astype(np.int64), ref_c) and np.array_equal(got, ref)
    assert skipped > computed > 0, (computed, skipped)


def test_policy_switches_take_minus_one_zero_one(golhip):
    """golhip_set_activity / golhip_set_board_kernel: -1 automatic, 0 off, 1 on; anything else is
    GOLHIP_ERR_ARG and leaves the setting alone."""
    with golhip.Engine(64, 64, k=16) as e:
        assert e.launch_kind(16)[0] == "board"  # automatic: 64 rows
        for bad in (2, -2, 7):
            with pytest.raises(golhip.GolHipError):
                e.set_board_kernel(bad)
            with pytest.raises(golhip.GolHipError):
                e.set_activity(bad)
        assert e.launch_kind(16)[0] == "board"
        e.set_board_kernel(0)
        assert e.launch_kind(16)[0] == "slab"
        e.set_board_kernel(-1)
        assert e.launch_kind(16)[0] == "board"


def test_switching_skipping_recaptures_graphs(golhip, oracle):
    """Replays captured with skipping on must not keep running it after set_activity(0) (and the
    reverse): the switch drops the captured graphs.  Stats count only the skipping launches."""
    b = sparse_board(8192, 8192, seed=11, n_gliders=8)
    with golhip.Engine(8192, 8192, k=16) as e:
        e.set_graphs(1)
        e.set_activity(1)
        e.load(b)
        c1 = e.step(256, counts=True)  # graph replays with skipping
        s1 = e.activity_stats()
        assert s1[1] > 0
        e.set_activity(0)
        c2 = e.step(256, counts=True)  # recaptured without skipping
        assert e.activity_stats() == s1
        e.set_activity(1)
        c3 = e.step(256, counts=True)
        assert e.activity_stats()[0] > s1[0]
        got = e.store()
    ref, ref_c = oracle.packed_run(b, 768)
    assert np.array_equal(np.concatenate([c1, c2, c3]).astype(np.int64), ref_c)
    assert np.array_equal(got, ref)
