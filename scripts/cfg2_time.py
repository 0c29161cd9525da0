#!/usr/bin/env python3
"""configs[1] timing for A/B builds (GOLHIP_LIB): 5120^2 seed 2, 10 000 turns, with every count
(median of 5 after a graph-capturing first run) and without counts; counts checked vs the golden
CSV (reported, not asserted: experimental builds may drop counts on purpose)."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402,F401
import numpy as np  # noqa: E402

import golhip  # noqa: E402

GOLDEN = ROOT / "tests" / "golden"
gold = json.loads((GOLDEN / "synthetic_golden.json").read_text())
lines = (GOLDEN / gold["cfg2"]["counts_csv"]).read_text().split()[1:]
exp = np.array([int(ln.split(",")[1]) for ln in lines], dtype=np.uint64)
res = {}
if len(sys.argv) > 1 and sys.argv[1] == "cfg5":
    # configs[4]: 4096^2 glider gun + R-pentomino, the first 200 000 turns with every count
    b = np.zeros((4096, 4096), dtype=np.uint8)
    golhip.place(b, golhip.parse_rle((GOLDEN / "gosper_gun.rle").read_text()), 64, 64)
    golhip.place(b, golhip.parse_rle((GOLDEN / "r_pentomino.rle").read_text()), 2048, 2048)
    deltas = np.load(GOLDEN / gold["cfg5"]["counts_1e6_npz"])["deltas"]
    n = 200000
    exp5 = (int((b == 255).sum()) + np.cumsum(deltas[:n].astype(np.int64))).astype(np.uint64)
    with golhip.Engine(4096, 4096, k=16) as e:
        runs, ok = [], True
        for _ in range(4):
            e.load(b)
            e.sync()
            t = time.perf_counter()
            c = e.step(n, counts=True)
            runs.append(time.perf_counter() - t)
            ok = ok and bool(np.array_equal(c.astype(np.uint64), exp5))
    r = sorted(runs[1:])
    print(json.dumps({"cfg5_counts": {"us_per_turn": round(r[len(r) // 2] / n * 1e6, 4), "ok": ok}}))
    sys.exit(0)
with golhip.Engine(5120, 5120, k=16) as e:
    for counts in (True, False):
        runs, ok = [], True
        for _ in range(6):
            e.init_random(2)
            e.sync()
            t = time.perf_counter()
            c = e.step(10000, counts=counts)
            e.sync()
            runs.append(time.perf_counter() - t)
            if counts:
                ok = ok and bool(np.array_equal(c.astype(np.uint64), exp))
        r = sorted(runs[1:])
        res["counts" if counts else "nocounts"] = {"us_per_turn": round(r[len(r) // 2] / 1e4 * 1e6, 4),
                                                   "best": round(r[0] / 1e4 * 1e6, 4), "ok": ok if counts else None}
print(json.dumps(res))
