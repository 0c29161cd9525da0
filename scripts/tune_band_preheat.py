#!/usr/bin/env python3
"""Band rows x depth at 65536^2 on a pre-heated chip (production variant, fixed depth, interleaved
rounds in one process, median of 3): does the auto band still sit on the best point now that the
clock is steady?  Usage: tune_band_preheat.py [ks] [bands]"""
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402,F401
import golhip  # noqa: E402

ks = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "12,14,16").split(",")]
bands = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,176,220,264,308,352,440,528").split(",")]
N = 65536
e = golhip.Engine(N, N, k=max(ks))
e.set_fixed_k(True)
e.init_random(3)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:  # pre-heat
    e.step(48)
    e.sync()
res = {}
for rnd in range(3):
    for k in ks:
        for b in bands:
            e.set_k(k)
            e.set_band_rows(b)
            n = 16 * k
            e.step(k)
            e.sync()
            t = time.perf_counter()
            e.step(n)
            e.sync()
            dt = time.perf_counter() - t
            res.setdefault(f"k{k}_b{b}", []).append(N * N * n / dt / 1e9)
out = {key: round(statistics.median(v), 1) for key, v in res.items()}
print(json.dumps(out))
for k in ks:
    best = max((v, key) for key, v in out.items() if key.startswith(f"k{k}_"))
    print(f"k={k}: auto {out[f'k{k}_b0']}, best {best[1]} {best[0]}")
