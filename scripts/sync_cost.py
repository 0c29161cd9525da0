#!/usr/bin/env python3
"""Host share of a 20-turn timed region at 65536^2 by how its end is synchronised: A = engine
streams (golhip_sync) then torch.cuda.synchronize (bench.py), B = torch.cuda.synchronize only
(hipDeviceSynchronize waits for every stream of the device, the engine's included).  Alternating
in one process after a pre-heat; wall vs the HIP-event span of the golhip_step call."""
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402
import golhip  # noqa: E402

e = golhip.Engine(65536, 65536, k=16)
e.init_random(3)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    e.step(48)
    e.sync()
res = {"A": [], "B": []}
for rep in range(8):
    for mode in ("A", "B"):
        e.init_random(3)
        e.step(5)
        e.sync()
        e.timing(True)
        torch.cuda.synchronize()
        e.sync()
        t = time.perf_counter()
        e.step(20)
        if mode == "A":
            e.sync()
        torch.cuda.synchronize()
        w = (time.perf_counter() - t) * 1e6
        ms, launches, gens = e.kernel_time()
        e.timing(False)
        res[mode].append((w, ms * 1e3))
for mode, v in res.items():
    wall = statistics.median(x[0] for x in v)
    kern = statistics.median(x[1] for x in v)
    print(mode, "wall_us", round(wall, 1), "kernel_us", round(kern, 1), "host_us", round(wall - kern, 1),
          "min wall-kernel", round(min(x[0] - x[1] for x in v), 1))
