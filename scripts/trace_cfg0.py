#!/usr/bin/env python3
"""configs[0] call timeline: 20 x golhip_step(100, counts=True) on a 512^2 board (production
library), wall time per call printed; run under rocprofv3 --kernel-trace --memory-copy-trace to
place the launches, the count finalize and the count copy inside each call."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import golhip  # noqa: E402

e = golhip.Engine(512, 512, k=16)
e.init_random(5)
e.step(100, counts=True)
e.sync()
ts = []
for _ in range(20):
    e.sync()
    t = time.perf_counter()
    e.step(100, counts=True)
    ts.append((time.perf_counter() - t) * 1e6)
print("us per call:", [round(x, 1) for x in ts])
e.close()
