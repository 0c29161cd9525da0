#!/usr/bin/env python3
"""configs[0] calls (512^2, golhip_step(100, counts)): wall time per call vs the HIP-event span of
its stencil launches on the compute stream (golhip_timing), to split a call's time into device
work and host-side latency."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import golhip  # noqa: E402

e = golhip.Engine(512, 512, k=16)
e.init_random(5)
e.step(100, counts=True)
e.timing(True)
walls, spans = [], []
for _ in range(30):
    e.sync()
    ms0, _, _ = e.kernel_time()
    t = time.perf_counter()
    e.step(100, counts=True)
    walls.append((time.perf_counter() - t) * 1e6)
    ms1, _, _ = e.kernel_time()
    spans.append((ms1 - ms0) * 1e3)
walls.sort()
spans.sort()
print("wall us p10/p50/p90:", [round(walls[i], 1) for i in (3, 15, 27)])
print("span us p10/p50/p90:", [round(spans[i], 1) for i in (3, 15, 27)])
e.close()
