#!/usr/bin/env python3
"""The driver's 20-turn region (seed 3, 5 warmup turns, 20 timed) as 12 + 8 (the planner's) and as
8 + 12: per-launch HIP-event durations (golhip_kernel_time around each call) and the region's wall
time, alternating orders in one pre-heated process.  Is the first launch of the region slower than
the same depth in steady state, whatever its depth?  Usage: ab_order.py [rounds]"""
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402

import golhip  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 11
N = 65536
e = golhip.Engine(N, N, k=16)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.4:
    e.init_random(3)
    e.step(48)
    e.sync()
res = {}
alive = set()
orders = [(12, 8), (8, 12)]
for r in range(rounds):
    for order in (orders if r % 2 == 0 else orders[::-1]):
        e.set_fixed_k(False)
        e.set_k(16)
        e.init_random(3)
        e.step(5)
        e.sync()
        torch.cuda.synchronize()
        e.timing(True)
        t = time.perf_counter()
        spans = []
        for K in order:
            e.set_k(K)
            e.set_fixed_k(True)
            e.step(K)
            e.sync()
            ms, launches, gens = e.kernel_time()
            spans.append(ms * 1e3)
        dt = time.perf_counter() - t
        e.timing(False)
        key = "+".join(map(str, order))
        d = res.setdefault(key, {"wall_us": [], "launch_us": [[] for _ in order]})
        d["wall_us"].append(dt * 1e6)
        for i, s in enumerate(spans):
            d["launch_us"][i].append(s)
        alive.add(e.alive_count())
assert len(alive) == 1, alive
out = {k: {"wall_us_median": round(statistics.median(v["wall_us"]), 1),
           "launch_us_median": [round(statistics.median(x), 1) for x in v["launch_us"]],
           "launch_us_all": [[round(y, 1) for y in x] for x in v["launch_us"]]} for k, v in res.items()}
print(json.dumps({"alive_turn25": alive.pop(), "orders": out}, indent=1))
