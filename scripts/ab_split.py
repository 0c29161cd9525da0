#!/usr/bin/env python3
"""The driver's 20-turn region (warmup 5 from the seeded random board, then 20 timed turns) under
different launch splits, pre-heated, alternating rounds in one process: the planner's choice and
fixed maximum depths (20 = k + k + ... + remainder).  Usage: ab_split.py [variants] [ks] [rounds]"""
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
# the tuning build holds the selectable variants / forced shapes (lib/ has only production)
os.environ.setdefault("GOLHIP_LIB", str(ROOT / "distributed-gol_amd" / "lib_tuning" / "libgolhip.so"))
import torch  # noqa: E402

import golhip  # noqa: E402

variants = (sys.argv[1] if len(sys.argv) > 1 else "prod").split(",")
ks = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,10,12,14,16").split(",")]  # 0: planner
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 9
N = 65536
eng = {}
for v in variants:
    os.environ["GOLHIP_VARIANT"] = v
    eng[v] = golhip.Engine(N, N, k=16)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.4:
    for e in eng.values():
        e.init_random(3)
        e.step(48)
        e.sync()
res, alive = {}, set()
cfgs = [(v, k) for v in variants for k in ks]
for r in range(rounds):
    for v, k in (cfgs if r % 2 == 0 else list(reversed(cfgs))):
        e = eng[v]
        e.set_k(k if k else 16)
        e.set_fixed_k(bool(k))
        e.init_random(3)
        e.step(5)
        e.sync()
        torch.cuda.synchronize()
        t = time.perf_counter()
        e.step(20)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        res.setdefault(f"{v}_k{k}", []).append(N * N * 20 / dt / 1e9)
        alive.add(e.alive_count())
assert len(alive) == 1, alive
out = {key: round(statistics.median(x), 1) for key, x in res.items()}
print(json.dumps({"median_tcups": out, "alive_turn25": alive.pop()}))
base = out[f"{variants[0]}_k{ks[0]}"]
for key, x in sorted(out.items(), key=lambda kv: -kv[1]):
    print(f"{key:>12} {x:9.1f} {x / base - 1:+.2%}")
