"""The whole-board kernel (stencil_board.hip, gol_board): boards of 128 / 256 / 512 torus cells per
row and 4 W R rows run in ONE workgroup for a whole golhip_step call (one launch per 4096
generations); automatic up to 256 rows, forced here (golhip_set_board_kernel(1)) on taller ones.
Bit-exact against the oracle -- every count of every turn, the board, the last generation's flips
-- on every (W, R) shape, widths whose torus is replicated (16, 64 cells), calls of 1 turn (the
flips of a one-generation step), of many generations in one launch, across count windows, and
against the same engine with the kernel off (the multi-workgroup slabs).

Reference: server/server.go:21-75 (the rule on a torus), gol/distributor.go:53-59 (flips),
:153-191 (counts).  The reference's own fixtures (check/images 16/64/512, check/alive CSVs) run
through this kernel in tests/test_gpu_parity.py where those boards fit its automatic range.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("w,h", [(512, 512), (512, 256), (256, 128), (128, 64), (512, 32), (64, 16),
                                 (16, 16), (32, 8), (128, 4)])
def test_board_kernel_matches_oracle(golhip, oracle, w, h):
    board = (np.random.default_rng(w * 7 + h).random((h, w)) < 0.37).astype(np.uint8) * 255
    with golhip.Engine(w, h, k=16) as e:
        # automatic up to 256 rows (kBoardAutoRows); forced here for every shape
        assert (e.launch_kind(16)[0] == "board") == (h <= 256), e.launch_kind(16)
        e.set_board_kernel(1)
        assert e.launch_kind(16)[0] == "board", e.launch_kind(16)
        e.load(board)
        c1 = e.step(1, counts=True)
        f1 = e.flips()  # a one-generation call: XOR of the two buffers
        c2 = e.step(333, counts=True)
        e.track_flips(True)
        c3 = e.step(37, counts=True)
        f3 = e.flips()  # the last generation's flips, written by the board kernel (LD)
        e.track_flips(False)
        e.step(50)
        got = e.store()
    ref = board.copy()
    exp = []
    prev = None
    for n in (1, 333, 37, 50):
        if n == 37:
            r36, c36 = oracle.packed_run(ref, 36)
            ref_last, c_last = oracle.packed_run(r36, 1)
            exp.append(np.concatenate([c36, c_last]))
            prev, ref = r36, ref_last
            continue
        before = ref
        ref, c = oracle.packed_run(ref, n)
        exp.append(c)
        if n == 1:
            prev1 = before
    assert np.array_equal(c1.astype(np.int64), exp[0])
    assert np.array_equal(c2.astype(np.int64), exp[1])
    assert np.array_equal(c3.astype(np.int64), exp[2])
    assert np.array_equal(got, ref)
    after1, _ = oracle.packed_run(prev1, 1)
    ys, xs = np.nonzero(prev1 != after1)
    assert np.array_equal(f1, np.stack([xs, ys], 1).astype(np.int32))
    ys, xs = np.nonzero(prev != oracle.packed_run(prev, 1)[0])
    assert np.array_equal(f3, np.stack([xs, ys], 1).astype(np.int32))


def test_board_kernel_long_calls_across_count_windows(golhip, oracle):
    """10 000 turns of images/512x512.pgm in one call (three launches over the 4096-generation
    count window), every count against check/alive/512x512.csv, then 5565/5567 for turns past
    10000 (count_test.go:45-51) in a call shorter than a window; the count window shrunk to 128 in a
    second engine (a flush between launches)."""
    from conftest import REF

    _, _, board = oracle.read_pgm(REF / "images/512x512.pgm")
    csv = oracle.read_alive_csv(REF / "check/alive/512x512.csv")
    with golhip.Engine(512, 512, k=16) as e:
        e.set_board_kernel(1)  # forced (automatic only up to 256 rows)
        e.load(board)
        c = e.step(10000, counts=True)
        assert [int(x) for x in c] == [csv[t] for t in range(1, 10001)]
        tail = e.step(9, counts=True)
        assert [int(x) for x in tail] == [5565 if t % 2 == 0 else 5567 for t in range(10001, 10010)]
    with golhip.Engine(512, 512, k=16) as e:
        e.set_board_kernel(1)
        e.set_count_window(128)
        e.load(board)
        c = e.step(1000, counts=True)
        assert [int(x) for x in c] == [csv[t] for t in range(1, 1001)]


def test_board_kernel_on_and_off_identical(golhip, oracle):
    words = oracle.init_random(512, 512, seed=41)
    outs = []
    for on in (True, False):
        with golhip.Engine(512, 512, k=16) as e:
            e.set_board_kernel(on)
            assert e.launch_kind(16)[0] == ("board" if on else "slab")
            e.load_words(words)
            c = [e.step(n, counts=True) for n in (100, 4096, 3, 127)]
            outs.append((np.concatenate(c), e.store_words()))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    ref = words.copy()
    exp = oracle.packed_run_words(ref, 100 + 4096 + 3 + 127)
    assert np.array_equal(outs[0][0].astype(np.int64), exp) and np.array_equal(outs[0][1], ref)


def test_board_launch_plan(golhip):
    assert golhip.launch_plan(128, 128, 16, 100) == [100]
    assert golhip.launch_plan(64, 64, 16, 10000) == [4096, 4096, 1808]
    assert golhip.launch_plan(512, 512, 16, 100) != [100]  # 512 rows: the slab kernels (automatic)
    assert golhip.launch_plan(512, 512, 16, 100, strips=2) != [100]  # strips: not the board kernel


def test_fixed_k_turns_the_board_kernel_off(golhip, oracle):
    """golhip_set_fixed_k: every launch exactly k deep, so a depth sweep measures the k-deep stencil
    launches, not the whole-board kernel (which is not bounded by k); same results either way."""
    words = oracle.init_random(256, 128, seed=3)
    with golhip.Engine(256, 128, k=8) as e:
        assert e.launch_kind(8)[0] == "board"
        e.set_fixed_k(True)
        assert e.launch_kind(8)[0] != "board", e.launch_kind(8)
        e.load_words(words)
        c = e.step(40, counts=True)
        got = e.store_words()
    ref = words.copy()
    exp = oracle.packed_run_words(ref, 40)
    assert np.array_equal(c.astype(np.int64), exp) and np.array_equal(got, ref)
