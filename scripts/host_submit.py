#!/usr/bin/env python3
"""Host side of the driver's 20-turn region: how long golhip_step(20) takes to RETURN (planning,
parameter set-up, timing events and the two launches submitted) against the whole region (through
torch.cuda.synchronize), pre-heated, timing events on and off.  Usage: host_submit.py [reps]"""
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402

import golhip  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 15
N = 65536
e = golhip.Engine(N, N, k=16)
e.init_random(3)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    e.step(48)
    e.sync()
out = {}
for timing in (True, False):
    e.timing(timing)
    ret, tot = [], []
    for _ in range(reps):
        e.init_random(3)
        e.step(5)
        e.sync()
        torch.cuda.synchronize()
        a = time.perf_counter()
        e.step(20)
        b = time.perf_counter()
        torch.cuda.synchronize()
        c = time.perf_counter()
        ret.append((b - a) * 1e6)
        tot.append((c - a) * 1e6)
    out["timing_on" if timing else "timing_off"] = {"step_return_us": round(statistics.median(ret), 1),
                                                    "region_us": round(statistics.median(tot), 1)}
print(json.dumps(out))
