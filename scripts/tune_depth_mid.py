#!/usr/bin/env python3
"""Bulk launch depth on streaming boards below 2^31 cells (the planner's rate tier that still
ranks K = 12 first, from round 2): TCUPS of 1680 turns at exactly K = 10 / 12 / 14 / 16
(set_fixed_k), pre-heated, 5 alternating rounds, same seeded board; alive counts equal.
Usage: tune_depth_mid.py [sizes] [turns]"""
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402,F401

import golhip  # noqa: E402

sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "24576,32768,40960").split(",")]
turns = int(sys.argv[2]) if len(sys.argv) > 2 else 1680
out = {}
for n in sizes:
    e = golhip.Engine(n, n, k=16)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        e.init_random(5)
        e.step(64)
        e.sync()
    res, alive = {}, set()
    ks = [0, 10, 12, 14, 16]  # 0: the planner's own choice
    for r in range(5):
        for K in (ks if r % 2 == 0 else list(reversed(ks))):
            e.set_k(K or 16)
            e.set_fixed_k(bool(K))
            e.init_random(5)
            e.step(8)
            e.sync()
            t = time.perf_counter()
            e.step(turns)
            e.sync()
            dt = time.perf_counter() - t
            res.setdefault(K, []).append(n * n * turns / dt / 1e12)
            alive.add(e.alive_count())
    e.close()
    assert len(alive) == 1, alive
    out[n] = {f"k{K}" if K else "planner": round(statistics.median(v), 2) for K, v in res.items()}
    print(json.dumps({str(n): out[n], "kernel": golhip.launch_plan(n, n, 16, 64)[:4]}), flush=True)
print(json.dumps({"depth_mid_tcups": out}))
