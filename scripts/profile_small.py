#!/usr/bin/env python3
"""One small-board run for rocprofv3 (kernel durations vs. gaps): size k turns [counts]."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402,F401
import golhip  # noqa: E402

size, k, turns = (int(x) for x in sys.argv[1:4])
counts = len(sys.argv) > 4 and sys.argv[4] == "counts"
with golhip.Engine(size, size, k=k) as e:
    e.init_random(2)
    e.step(256, counts=counts)
    e.sync()
    e.step(turns, counts=counts)
    e.sync()
