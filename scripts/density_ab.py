#!/usr/bin/env python3
"""The stencil's speed against the board's bit activity: the same fixed-depth launches (the
instruction stream is data-independent: bit-sliced, no branches on cells) on an empty board, a
sparse one and the random p = 0.5 start, pre-heated, alternating; TCUPS per board.
Usage: density_ab.py [size] [k] [rounds]"""
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402,F401

import golhip  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
k = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 7
boards = {"empty": 0, "p0.05": int(0.05 * 2**32), "p0.5": golhip.DENSITY_HALF}
e = golhip.Engine(size, size, k=k)
e.set_fixed_k(True)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.4:
    e.init_random(3)
    e.step(4 * k)
    e.sync()
res = {}
n = 2 * k
for r in range(rounds):
    for name, dens in (boards.items() if r % 2 == 0 else reversed(list(boards.items()))):
        e.init_random(3, dens)
        e.sync()
        t = time.perf_counter()
        e.step(n)
        e.sync()
        dt = time.perf_counter() - t
        res.setdefault(name, []).append(size * size * n / dt / 1e9)
out = {b: round(statistics.median(v), 1) for b, v in res.items()}
print(json.dumps({"k": k, "turns": n, "median_tcups": out}))
for b, v in out.items():
    print(f"{b:>6}: {v:9.1f} ({v / out['p0.5'] - 1:+.1%} vs p0.5)")
