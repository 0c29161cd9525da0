#!/usr/bin/env python3
"""Small-board sweep (configs[1] 5120^2 / configs[4] 4096^2): us per turn of golhip_step WITH
per-turn counts, k x band_rows, median of 3 interleaved rounds.
Usage: tune_small.py size ks bands [turns]"""
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402,F401
import golhip  # noqa: E402

size = int(sys.argv[1])
ks = [int(x) for x in sys.argv[2].split(",")]
bands = [int(x) for x in sys.argv[3].split(",")]
turns = int(sys.argv[4]) if len(sys.argv) > 4 else 2048
e = golhip.Engine(size, size, k=max(ks))
res = {}
for rnd in range(3):
    for k in ks:
        for b in bands:
            e.set_k(k)
            e.set_band_rows(b)
            e.init_random(2)
            e.step(256, counts=True)
            e.sync()
            t = time.perf_counter()
            e.step(turns, counts=True)
            dt = time.perf_counter() - t
            res.setdefault(f"k{k}_b{b}", []).append(dt / turns * 1e6)
out = {key: round(statistics.median(v), 3) for key, v in res.items()}
print(json.dumps({"size": size, "us_per_turn_with_counts": out}))
best = min(out, key=out.get)
print("best", best, out[best])
