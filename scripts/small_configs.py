#!/usr/bin/env python3
"""configs[1] and configs[4] latency on one GPU, through the production path (default planner,
automatic kernel choice): us per turn of golhip_step WITH the alive count of every turn, checked
against the committed goldens (cfg2 CSV: all 10000 counts; cfg5 npz: all 1e6 counts).
Prints one JSON object.  Run on the GPU box from the repo root."""
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
res = {}

# configs[1]: 5120^2 random seed 2, 10000 turns, every count
lines = (GOLDEN / gold["cfg2"]["counts_csv"]).read_text().split()[1:]
exp2 = np.array([int(ln.split(",")[1]) for ln in lines], dtype=np.uint64)
with golhip.Engine(5120, 5120, k=16) as e:
    kind = e.launch_kind(16, counts=True)
    runs = []
    for _ in range(3):
        e.init_random(2)
        e.sync()
        t = time.perf_counter()
        c = e.step(10000, counts=True)
        dt = time.perf_counter() - t
        runs.append(dt)
        ok = bool(np.array_equal(c.astype(np.uint64), exp2))
    dt = min(runs)
    res["cfg2"] = {"us_per_turn": round(dt / 10000 * 1e6, 3), "runs_s": [round(r, 4) for r in runs],
                   "gcups": round(5120 * 5120 * 10000 / dt / 1e9, 1), "counts_match_all_10000": ok,
                   "kernel": f"{kind[0]}{kind[1] or ''}"}

# configs[4]: 4096^2 gun + R-pentomino, 1e6 turns, every count
b = np.zeros((4096, 4096), dtype=np.uint8)
golhip.place(b, golhip.parse_rle((GOLDEN / "gosper_gun.rle").read_text()), 64, 64)
golhip.place(b, golhip.parse_rle((GOLDEN / "r_pentomino.rle").read_text()), 2048, 2048)
deltas = np.load(GOLDEN / gold["cfg5"]["counts_1e6_npz"])["deltas"]
exp5 = (int((b == 255).sum()) + np.cumsum(deltas.astype(np.int64))).astype(np.uint64)
with golhip.Engine(4096, 4096, k=16) as e:
    kind = e.launch_kind(16, counts=True)
    e.load(b)
    e.sync()
    t = time.perf_counter()
    c = e.step(1000000, counts=True)
    dt = time.perf_counter() - t
    res["cfg5"] = {"us_per_turn": round(dt, 3), "gcups": round(4096 * 4096 * 1e6 / dt / 1e9, 1),
                   "counts_match_all_1e6": bool(np.array_equal(c.astype(np.uint64), exp5)),
                   "kernel": f"{kind[0]}{kind[1] or ''}"}
print(json.dumps(res))
