#!/usr/bin/env python3
"""Graded bands on a pre-heated chip: (band rows, tail bands, tail rows) configurations of the
streaming launch at one depth, interleaved rounds in one process, median TCUPS.
Usage: tune_tail.py [size] [k] [configs "B:n2:b2,..."] [rounds]   (B = 0: automatic band)"""
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402,F401
import golhip  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
k = int(sys.argv[2]) if len(sys.argv) > 2 else 12
cfgs = [tuple(int(x) for x in c.split(":")) for c in
        (sys.argv[3] if len(sys.argv) > 3 else "0:0:0,240:150:64,336:150:96").split(",")]
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
e = golhip.Engine(N, N, k=k)
e.set_fixed_k(True)
e.init_random(3)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.4:  # pre-heat
    e.step(48)
    e.sync()
n = max(int(os.environ.get("TUNE_STEPS", "192")) // k, 2) * k
res = {}
for rnd in range(rounds):
    for c in (cfgs if rnd % 2 == 0 else list(reversed(cfgs))):
        b, n2, b2 = c
        e.set_band_rows(b)
        e.set_tail_bands(n2, b2)
        e.step(k)
        e.sync()
        t = time.perf_counter()
        e.step(n)
        e.sync()
        dt = time.perf_counter() - t
        res.setdefault(f"{b}:{n2}:{b2}", []).append(N * N * n / dt / 1e9)
out = {key: round(statistics.median(v), 1) for key, v in res.items()}
print(json.dumps({"k": k, "median": out}))
base = out[f"{cfgs[0][0]}:{cfgs[0][1]}:{cfgs[0][2]}"]
for key, v in sorted(out.items(), key=lambda kv: -kv[1]):
    print(f"{key:>14} {v:9.1f} {v / base - 1:+.2%}")
