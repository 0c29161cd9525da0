#!/usr/bin/env python3
"""Row strips on ONE GPU as a scheduling device: with S strips the engine runs each strip's
K-block on its own streams (interior + boundary bands, halos by device copies), so one strip's
next launch can start while another strip's launch drains -- the tail of a launch overlaps work.
Pre-heated, lockstep on the same seeded board, the driver's 20-turn shape (warmup 5, 20 timed).
Usage: ab_strips.py [size] [strips list] [rounds] [turns]"""
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402

import golhip  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
strips = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,4").split(",")]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 7
turns = int(sys.argv[4]) if len(sys.argv) > 4 else 20
eng = {s: golhip.Engine(size, size, k=16, strips=s) for s in strips}
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.4:  # pre-heat
    for e in eng.values():
        e.init_random(3)
        e.step(48)
        e.sync()
res = {}
alive = {}
for r in range(rounds):
    for s in (strips if r % 2 == 0 else list(reversed(strips))):
        e = eng[s]
        e.init_random(3)
        e.step(5)
        e.sync()
        torch.cuda.synchronize()
        t = time.perf_counter()
        e.step(turns)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        e.sync()
        res.setdefault(s, []).append(size * size * turns / dt / 1e9)
        alive.setdefault(s, set()).add(e.alive_count())
assert all(len(a) == 1 for a in alive.values()) and len({next(iter(a)) for a in alive.values()}) == 1, alive
med = {s: round(statistics.median(v), 1) for s, v in res.items()}
print(json.dumps({"median_tcups": med, "rounds": {s: [round(x) for x in v] for s, v in res.items()},
                  "alive": next(iter(alive[strips[0]]))}))
for s in strips:
    print(f"strips={s}: {med[s]} ({med[s] / med[strips[0]] - 1:+.2%})")
