"""GPU parity at BASELINE.json's synthetic configs, against golden vectors the pinned oracle made
(tests/golden/synthetic_golden.json, scripts/make_golden.py) and size-independent properties
where the oracle cannot follow (262144^2)."""
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


def test_cfg3_65536_thousand_turns(golhip, oracle):
    """configs[2]: 65536^2 random (seed 3), 1000 turns: board digests and all 1000 counts."""
    g = GOLD["cfg3"]
    with golhip.Engine(65536, 65536, k=8) as e:
        e.init_random(3)
        c8 = e.step(8, counts=True)
        assert oracle.digest_words(e.store_words()) == g["digest_after_8"]
        rest = e.step(992, counts=True)
        assert oracle.digest_words(e.store_words()) == g["digest_after_1000"]
        counts = np.concatenate([c8, rest]).astype("<u8")
        assert hashlib.sha256(counts.tobytes()).hexdigest() == g["counts_sha256"]
        assert e.alive_count() == int(counts[-1])


def test_cfg5_gun_and_r_pentomino(golhip, oracle):
    """configs[4]: 4096^2 Gosper gun + R-pentomino; counts of the first 100000 turns."""
    g = GOLD["cfg5"]
    b = np.zeros((4096, 4096), dtype=np.uint8)
    golhip.place(b, golhip.parse_rle((GOLDEN / "gosper_gun.rle").read_text()), 64, 64)
    golhip.place(b, golhip.parse_rle((GOLDEN / "r_pentomino.rle").read_text()), 2048, 2048)
    assert int((b == 255).sum()) == g["initial_alive"]
    with golhip.Engine(4096, 4096, k=16) as e:
        e.load(b)
        counts = e.step(100000, counts=True)
        assert hashlib.sha256(counts.astype("<u4").tobytes()).hexdigest() == g["counts_u32_sha256"]
        assert oracle.digest_words(e.store_words()) == g["digest_after_100000"]


@pytest.mark.parametrize("strips", [1, 2])
def test_cfg4_262144_window_locality(golhip, oracle, strips):
    """configs[3]: the 262144^2 board (8 GiB packed) is beyond the oracle, so check locality:
    after t turns the cells of a window shrunk by t on every side depend only on the initial
    window.  Windows straddle the torus wrap and (strips=2) the strip boundary."""
    n, t = 262144, 24
    with golhip.Engine(n, n, ngpus=1, k=8, strips=strips) as e:
        e.init_random(4)
        counts = e.step(t, counts=True)
        words = e.store_words()  # 8 GiB host copy: fine on the GPU box (>= 256 GiB host RAM)
        # bottom 128 rows + top 128 rows (torus wrap) and rows around the middle (strip seam)
        for y0 in (n - 128, n // 2 - 128):
            rows = [(y0 + i) % n for i in range(256)]
            init = np.concatenate([oracle.init_random(n, n, seed=4, y0=r, y1=r + 1) for r in rows])
            win = init.copy()
            # the window rows as their own torus: full width, so only the top/bottom t rows can
            # differ from the real board
            oracle.packed_run_words(win, t)
            got = words[rows]
            assert np.array_equal(got[t:-t], win[t:-t]), y0
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
    b = np.zeros((4096, 4096), dtype=np.uint8)
    golhip.place(b, golhip.parse_rle((GOLDEN / "gosper_gun.rle").read_text()), 64, 64)
    golhip.place(b, golhip.parse_rle((GOLDEN / "r_pentomino.rle").read_text()), 2048, 2048)
    turns = 1000000
    with golhip.Engine(4096, 4096, k=16) as e:
        e.load(b)
        counts = [int(c) for c in e.step(turns, counts=True)]
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
    with golhip.Engine(4096, 4096, k=16) as e:
        e.load(b)
        e.step(t_snap)
        assert np.array_equal(snap, e.store()), t_snap
    assert events[-1] == (turns, "Quitting"), events[-3:]
    final = re.search(r"Final turn (\d+): (\d+) alive cells", stdout)
    assert final and int(final.group(1)) == turns and int(final.group(2)) == counts[-1]
    _, _, last = oracle.read_pgm(out / ("4096x4096x%d.pgm" % turns))
    assert int((last == 255).sum()) == counts[-1]
