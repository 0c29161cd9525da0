"""GPU parity at BASELINE.json's synthetic configs, against golden vectors the pinned oracle made
(tests/golden/synthetic_golden.json + the per-turn count files, scripts/make_golden.py): every
engine result here is compared with the oracle's, never with another engine run."""
import hashlib
import json

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

GOLD = json.loads((GOLDEN / "synthetic_golden.json").read_text())


def test_cfg2_5120_every_turn(golhip, oracle):
    """configs[1]: 5120^2 random p=0.5 (seed 2), 10000 turns, alive count after EVERY turn."""
    g = GOLD["cfg2"]
    expected = oracle.read_alive_csv(GOLDEN / g["counts_csv"])
    for k in (1, 8, 16):
        with golhip.Engine(5120, 5120, k=k) as e:
            e.init_random(2)
            counts = e.step(10000, counts=True)
            assert [int(c) for c in counts] == [expected[t] for t in range(1, 10001)], k
            assert oracle.digest_words(e.store_words()) == g["final_digest"]


CFG3_COUNTS = GOLDEN / "cfg3_65536_seed3_counts.csv"


@pytest.mark.parametrize("k", [1, 2, 4, 8, 10, 12, 14, 16, 32])
def test_cfg3_65536_thousand_turns(golhip, oracle, k):
    """configs[2]: 65536^2 random (seed 3), 1000 turns at every launch depth -- the benchmarked
    kernel (gol_stencil<16>, drifting sums, auto band grid) at the benchmarked size: board digests
    after 8 and 1000 turns and all 1000 per-turn counts against the oracle's golden vectors."""
    g = GOLD["cfg3"]
    with golhip.Engine(65536, 65536, k=k) as e:
        e.set_fixed_k(True)  # every bulk launch exactly k deep
        e.init_random(3)
        c8 = e.step(8, counts=True)
        assert oracle.digest_words(e.store_words()) == g["digest_after_8"], k
        rest = e.step(992, counts=True)
        assert oracle.digest_words(e.store_words()) == g["digest_after_1000"], k
        counts = np.concatenate([c8, rest]).astype("<u8")
        assert hashlib.sha256(counts.tobytes()).hexdigest() == g["counts_sha256"], k
        assert e.alive_count() == int(counts[-1])


@pytest.mark.parametrize("warmup,steps", [(5, 20), (8, 1000), (0, 17), (3, 45), (8, 1192)])
def test_cfg3_bench_splits(golhip, oracle, warmup, steps):
    """bench.py's own call pattern at k = 16 (warm-up call, then the timed call, each split into
    launch depths by the engine's planner): the alive count after each call equals the oracle's
    golden count of that turn (tests/golden/cfg3_65536_seed3_counts.csv)."""
    expected = oracle.read_alive_csv(CFG3_COUNTS)
    with golhip.Engine(65536, 65536, k=16) as e:
        e.init_random(3)
        if warmup:
            e.step(warmup)
            assert e.alive_count() == expected[warmup]
        e.step(steps)
        assert e.alive_count() == expected[warmup + steps]


def cfg5_board(golhip):
    b = np.zeros((4096, 4096), dtype=np.uint8)
    golhip.place(b, golhip.parse_rle((GOLDEN / "gosper_gun.rle").read_text()), 64, 64)
    golhip.place(b, golhip.parse_rle((GOLDEN / "r_pentomino.rle").read_text()), 2048, 2048)
    return b


def cfg5_golden_counts():
    """The oracle's count after each of the 1e6 turns (delta-encoded npz, scripts/make_golden.py)."""
    g = GOLD["cfg5"]
    d = np.load(GOLDEN / g["counts_1e6_npz"])["deltas"].astype(np.int64)
    counts = g["initial_alive"] + np.cumsum(d)
    assert hashlib.sha256(counts.astype("<u4").tobytes()).hexdigest() == g["counts_1e6_u32_sha256"]
    return counts


def test_cfg5_gun_and_r_pentomino(golhip, oracle):
    """configs[4]: 4096^2 Gosper gun + R-pentomino, 1e6 turns: every per-turn count and the final
    board against the oracle (SHA-256 of the uint32 count array of all 1e6 turns)."""
    g = GOLD["cfg5"]
    b = cfg5_board(golhip)
    assert int((b == 255).sum()) == g["initial_alive"]
    golden = cfg5_golden_counts()
    with golhip.Engine(4096, 4096, k=16) as e:
        e.load(b)
        first = e.step(100000, counts=True)
        assert hashlib.sha256(first.astype("<u4").tobytes()).hexdigest() == g["counts_u32_sha256"]
        assert oracle.digest_words(e.store_words()) == g["digest_after_100000"]
        rest = e.step(900000, counts=True)
        counts = np.concatenate([first, rest]).astype(np.int64)
        assert np.array_equal(counts, golden)
        assert oracle.digest_words(e.store_words()) == g["digest_after_1000000"]


@pytest.mark.parametrize("strips", [1, 2])
def test_cfg4_262144_against_oracle(golhip, oracle, strips):
    """configs[3]: the 262144^2 board (seed 4, 8 GiB packed) on one GPU as 1 or 2 row strips (the
    2-strip run exchanges halos across the seam): digests after 16 and 176 turns (the bench leg's
    warm-up launch and its 160 timed turns) and all 176 per-turn counts against the oracle."""
    g = GOLD["cfg4"]
    n = 262144
    with golhip.Engine(n, n, ngpus=1, k=16, strips=strips) as e:
        e.init_random(4)
        c16 = e.step(16, counts=True)
        assert oracle.digest_words(e.store_words()) == g["digest_after_16"]
        rest = e.step(160, counts=True)
        assert oracle.digest_words(e.store_words()) == g["digest_after_176"]
        counts = np.concatenate([c16, rest]).astype("<u8")
        assert hashlib.sha256(counts.tobytes()).hexdigest() == g["counts_sha256"]
        assert e.alive_count() == int(counts[-1])


def test_cfg5_host_run_ticker_and_keys(golhip, oracle, tmp_path):
    """configs[4] through the C++ host (`gol::Run`, the gol.Run mirror): 1e6 turns with the 2 s
    AliveCellsCount ticker and timed keypresses p (pause, held 2.5 s so the ticker fires while
    paused), s (snapshot while paused), p (resume).  Every tick's count must be the count after its
    reported turn (gol/distributor.go:168-191), the snapshot must be the board after its turn
    (:93-103,118-119), and the final alive list / PGM the board after 1e6 turns (:235-253)."""
    import re
    import subprocess
    import time

    from conftest import ROOT

    gol = ROOT / "distributed-gol_amd" / "lib" / "gol"
    assert gol.exists(), "host binary missing: run __graft_entry__.build()"
    b = cfg5_board(golhip)
    turns = 1000000
    counts = [int(c) for c in cfg5_golden_counts()]  # the oracle's, not the engine's
    initial = int((b == 255).sum())

    def count_after(t):
        return initial if t == 0 else counts[t - 1]

    (tmp_path / "images").mkdir()
    (tmp_path / "images" / "4096x4096.pgm").write_bytes(oracle.pgm_bytes(b))
    out = tmp_path / "out"
    p = subprocess.Popen([str(gol), "-w", "4096", "-h", "4096", "-turns", str(turns), "-k", "16",
                          "-images", str(tmp_path / "images"), "-out", str(out)],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    time.sleep(0.8)
    p.stdin.write("p\n")
    p.stdin.flush()
    time.sleep(2.5)
    p.stdin.write("s\n")
    p.stdin.flush()
    time.sleep(0.3)
    p.stdin.write("p\n")
    p.stdin.flush()
    stdout, _ = p.communicate(timeout=90)  # closes stdin: the key reader sees EOF
    assert p.returncode == 0, stdout[-2000:]
    lines = [re.match(r"Completed Turns (\d+)\s+(.*)$", ln) for ln in stdout.splitlines()]
    events = [(int(m.group(1)), m.group(2)) for m in lines if m]
    ticks = [(t, int(s.split()[-1])) for t, s in events if s.startswith("Alive Cells")]
    assert ticks, stdout[-2000:]
    for t, c in ticks:
        assert c == count_after(t), (t, c)
    states = [s for _, s in events]
    assert "Paused" in states and "Executing" in states, states
    snaps = [s.split()[1] for _, s in events if s.startswith("File ") and s.split()[1] != "4096x4096x%d" % turns]
    assert len(snaps) == 1, states
    t_snap = int(snaps[0].rsplit("x", 1)[1])
    _, _, snap = oracle.read_pgm(out / (snaps[0] + ".pgm"))
    # the paused snapshot is the board after its turn: its count is the golden count of that
    # turn, and advanced to turn 1e6 it reaches the oracle's final board
    assert int((snap == 255).sum()) == count_after(t_snap), t_snap
    with golhip.Engine(4096, 4096, k=16) as e:
        e.load(snap)
        e.step(turns - t_snap)
        assert oracle.digest_words(e.store_words()) == GOLD["cfg5"]["digest_after_1000000"], t_snap
    assert events[-1] == (turns, "Quitting"), events[-3:]
    final = re.search(r"Final turn (\d+): (\d+) alive cells", stdout)
    assert final and int(final.group(1)) == turns and int(final.group(2)) == counts[-1]
    _, _, last = oracle.read_pgm(out / ("4096x4096x%d.pgm" % turns))
    assert int((last == 255).sum()) == counts[-1]
    assert oracle.digest_words(oracle.pack(last)) == GOLD["cfg5"]["digest_after_1000000"]
