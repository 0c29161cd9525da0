#!/usr/bin/env python3
"""Small-board steady state (configs[1]): 5120^2, k from argv, 2000 turns with and without
per-turn counts.  Meant to run under rocprofv3 --kernel-trace."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402,F401
import golhip  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5120
for k in [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "4,8").split(",")]:
    with golhip.Engine(n, n, k=k) as e:
        e.init_random(2)
        e.step(256, counts=True)
        for counts in (True, False):
            e.sync()
            t = time.perf_counter()
            e.step(2000, counts=counts)
            e.sync()
            dt = time.perf_counter() - t
            print(f"n={n} k={k} counts={counts}: {dt / 2000 * 1e6:.3f} us/turn", flush=True)
