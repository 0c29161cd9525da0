"""The oracle is pinned against the reference's own fixtures before anything is checked against it.

Fixtures (copied verbatim from the reference into tests/golden/reference/):
  images/*.pgm, check/images/WxHxT.pgm (gol_test.go:24-27), check/alive/WxH.csv (count_test.go:78-89).
"""
import hashlib

import numpy as np
import pytest

from conftest import REF

SIZES = [16, 64, 512]
TURNS = [0, 1, 100]

# SHA-256 of the reference's fixtures as shipped.
FIXTURE_SHA = {
    "check/images/16x16x1.pgm": "162c70c7580bf171cf168fafbabd76a53d5d083790040c2256130bc190353527",
    "check/images/16x16x100.pgm": "dd159427a0112c5949115e9e3d54abc82025141cafda8ded0d8fb7ee42a64f9b",
    "check/images/64x64x1.pgm": "6c1259e17879c9f0da6bdfd91693a1949aeb6cb91ef7ccd761acd250397b3978",
    "check/images/64x64x100.pgm": "aa749f7d53df07afca4a58ed285d0137abcdac64664e63834a13d570c1b0d504",
    "check/images/512x512x1.pgm": "3fe3bd73986e369696eb9048c18854e7df322b987a405a3c9ba644e43e509947",
    "check/images/512x512x100.pgm": "2823119001ed0959e5294b2f123deb8af6f38058f6156721b6a2a625edeca690",
    "check/alive/512x512.csv": "a37fa51e01a35c2328cfb82e70ac66b59014f701d1bc5512af3d7fb599aeac9b",
}


def test_fixtures_are_the_reference_files():
    for rel, sha in FIXTURE_SHA.items():
        assert hashlib.sha256((REF / rel).read_bytes()).hexdigest() == sha, rel


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("turns", TURNS)
def test_reference_restatement_matches_check_images(oracle, n, turns):
    """server/server.go:21-107 + broker/broker.go:37-56 restated; output PGM byte-exact."""
    _, _, board = oracle.read_pgm(REF / f"images/{n}x{n}.pgm")
    expected = (REF / f"check/images/{n}x{n}x{turns}.pgm").read_bytes()
    for threads in (1, 3, 16):  # the reference test matrix runs threads 1..16 (gol_test.go:29)
        out, _ = oracle.ref_run(board, turns, threads=threads, servers=4)
        assert oracle.pgm_bytes(out) == expected


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("turns", TURNS)
def test_packed_oracle_matches_check_images(oracle, n, turns):
    _, _, board = oracle.read_pgm(REF / f"images/{n}x{n}.pgm")
    out, _ = oracle.packed_run(board, turns)
    assert oracle.pgm_bytes(out) == (REF / f"check/images/{n}x{n}x{turns}.pgm").read_bytes()


@pytest.mark.parametrize("n", SIZES)
def test_packed_oracle_matches_alive_csv(oracle, n):
    """All 10000 per-turn counts of check/alive/NxN.csv (count_test.go, sdl_test.go:107-116)."""
    _, _, board = oracle.read_pgm(REF / f"images/{n}x{n}.pgm")
    expected = oracle.read_alive_csv(REF / f"check/alive/{n}x{n}.csv")
    assert sorted(expected) == list(range(1, 10001))
    _, counts = oracle.packed_run(board, 10000)
    assert [int(c) for c in counts] == [expected[t] for t in range(1, 10001)]


def test_reference_restatement_matches_alive_csv_prefix(oracle):
    _, _, board = oracle.read_pgm(REF / "images/512x512.pgm")
    expected = oracle.read_alive_csv(REF / "check/alive/512x512.csv")
    _, counts = oracle.ref_run(board, 30, threads=8)
    assert [int(c) for c in counts] == [expected[t] for t in range(1, 31)]


def test_period_two_tail(oracle):
    """count_test.go:45-51: after turn 10000 the 512 board alternates 5565 (even) / 5567 (odd)."""
    _, _, board = oracle.read_pgm(REF / "images/512x512.pgm")
    _, counts = oracle.packed_run(board, 10010)
    for t in range(10001, 10011):
        assert counts[t - 1] == (5565 if t % 2 == 0 else 5567)


@pytest.mark.parametrize("shape", [(32, 32), (48, 48), (100, 100), (64, 128)])
def test_packed_matches_restatement_on_random_boards(oracle, shape):
    rng = np.random.default_rng(shape[0])
    board = (rng.random(shape) < 0.4).astype(np.uint8) * 255
    if shape[0] == shape[1] and shape[0] % 4 == 0:
        ref, ref_counts = oracle.ref_run(board, 25, threads=5)
        out, counts = oracle.packed_run(board, 25)
        assert np.array_equal(ref, out)
        assert np.array_equal(ref_counts, counts)
    else:  # rectangular / non-multiple-of-64 widths: packed vs a direct numpy rule
        cur = board.copy()
        out, _ = oracle.packed_run(board, 7)
        for _ in range(7):
            a = (cur == 255).astype(np.int32)
            nb = sum(np.roll(np.roll(a, dy, 0), dx, 1)
                     for dy in (-1, 0, 1) for dx in (-1, 0, 1) if (dy, dx) != (0, 0))
            cur = np.where((nb == 3) | ((nb == 2) & (a == 1)), 255, 0).astype(np.uint8)
        assert np.array_equal(cur, out)


def test_reference_split_rejects_rows_dropped_sizes(oracle):
    """broker/broker.go:38 + server/server.go:83: N % 4 != 0 drops rows in the reference."""
    board = np.zeros((10, 10), np.uint8)
    with pytest.raises(ValueError):
        oracle.ref_run(board, 1)


def test_init_random_definition(oracle):
    """splitmix64 counter definition used by the device init (golhip.h golhip_init_random)."""
    w = oracle.init_random(128, 4, seed=7)

    def splitmix(z):
        m = (1 << 64) - 1
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9 & m
        z = (z ^ (z >> 27)) * 0x94D049BB133111EB & m
        return z ^ (z >> 31)

    g = 0x9E3779B97F4A7C15
    for i in range(8):
        assert int(w.reshape(-1)[i]) == splitmix((7 + (i + 1) * g) & ((1 << 64) - 1))
    dens = oracle.init_random(64, 64, seed=3, density_q32=int(0.25 * 2**32))
    frac = np.unpackbits(dens.view(np.uint8)).mean()
    assert 0.2 < frac < 0.3


def test_synthetic_golden_vectors_are_the_oracle(oracle):
    """tests/golden/synthetic_golden.json came from scripts/make_golden.py: spot-check prefixes."""
    import json

    from conftest import GOLDEN

    gold = json.loads((GOLDEN / "synthetic_golden.json").read_text())
    expected = oracle.read_alive_csv(GOLDEN / gold["cfg2"]["counts_csv"])
    w = oracle.init_random(5120, 5120, seed=2)
    counts = oracle.packed_run_words(w, 20)
    assert [int(c) for c in counts] == [expected[t] for t in range(1, 21)]
    assert set(gold) >= {"cfg2", "cfg3", "cfg5"}


def test_golden_count_files_match_their_digests():
    """The per-turn count files (cfg3 CSV, cfg4 CSV, cfg5 1e6 npz) hash to the SHA-256s recorded
    beside them by scripts/make_golden.py, so GPU tests and bench.py compare against exactly the
    oracle's counts."""
    import json

    from conftest import GOLDEN

    gold = json.loads((GOLDEN / "synthetic_golden.json").read_text())
    for cfg in ("cfg3", "cfg4"):
        rows = (GOLDEN / gold[cfg]["counts_csv"]).read_text().splitlines()
        assert rows[0] == "completed_turns,alive_cells"
        n = gold[cfg].get("csv_turns", gold[cfg]["turns"])
        counts = np.array([int(r.split(",")[1]) for r in rows[1:]], dtype="<u8")
        assert [int(r.split(",")[0]) for r in rows[1:]] == list(range(1, n + 1))
        counts = counts[: gold[cfg]["turns"]]
        assert hashlib.sha256(counts.tobytes()).hexdigest() == gold[cfg]["counts_sha256"], cfg
    g5 = gold["cfg5"]
    d = np.load(GOLDEN / g5["counts_1e6_npz"])["deltas"].astype(np.int64)
    c5 = g5["initial_alive"] + np.cumsum(d)
    assert len(c5) == g5["turns_full"] == 1000000
    assert hashlib.sha256(c5.astype("<u4").tobytes()).hexdigest() == g5["counts_1e6_u32_sha256"]
    assert hashlib.sha256(c5[:100000].astype("<u4").tobytes()).hexdigest() == g5["counts_u32_sha256"]
    assert all(int(c5[int(t) - 1]) == v for t, v in g5["counts_every_1000"].items())


def test_cfg3_golden_prefix_is_the_oracle(oracle):
    """First turns of configs[2] (65536^2, seed 3) recomputed on a 4096-row slab would differ
    (torus), so recompute the real board for 2 turns (~1 s on 8 cores) against the count CSV."""
    import json

    from conftest import GOLDEN

    gold = json.loads((GOLDEN / "synthetic_golden.json").read_text())
    expected = oracle.read_alive_csv(GOLDEN / gold["cfg3"]["counts_csv"])
    w = oracle.init_random(65536, 65536, seed=3)
    counts = oracle.packed_run_words(w, 2)
    assert [int(c) for c in counts] == [expected[1], expected[2]]


def test_period_two_tail_board(oracle):
    """The 512x512 board itself (not only its count, count_test.go:45-51) repeats with period 2
    from turn 10000: later boards are pinned by turn 10000 or 10001 (tests/test_host.py)."""
    _, _, b = oracle.read_pgm(REF / "images/512x512.pgm")
    w = oracle.pack(b)
    oracle.packed_run_words(w, 10000, threads=1)
    ref = w.copy()
    oracle.packed_run_words(w, 1, threads=1)
    assert not np.array_equal(w, ref)
    oracle.packed_run_words(w, 1, threads=1)
    assert np.array_equal(w, ref)
