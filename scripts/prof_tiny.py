#!/usr/bin/env python3
"""Kernel-trace driver for the tiny boards: 1600 turns with every count at n x n for each
GOLHIP_SLAB code given (tuning build; "auto" = the automatic choice), one engine at a time, so
that rocprofv3 --kernel-trace --stats separates each variant's kernel durations from the
per-launch gaps.  Usage: prof_tiny.py n code[,code...]"""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
os.environ.setdefault("GOLHIP_LIB", str(ROOT / "distributed-gol_amd" / "lib_tuning" / "libgolhip.so"))
import golhip  # noqa: E402

n = int(sys.argv[1])
for code in sys.argv[2].split(","):
    os.environ.pop("GOLHIP_SLAB", None)
    if code != "auto":
        os.environ["GOLHIP_SLAB"] = code
    e = golhip.Engine(n, n, k=16)
    os.environ.pop("GOLHIP_SLAB", None)
    e.set_fixed_k(True)
    e.init_random(5)
    e.step(32, counts=True)
    e.sync()
    t = time.perf_counter()
    e.step(1600, counts=True)
    e.sync()
    print(code, e.launch_kind(16, counts=True), round((time.perf_counter() - t) * 1e6 / 1600, 3), "us/turn",
          flush=True)
    e.close()
