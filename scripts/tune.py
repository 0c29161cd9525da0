#!/usr/bin/env python3
"""Sweep variant x k x band_rows on one GPU (interleaved rounds in one process, median of 3).
Usage: tune.py [size] [ks] [bands] [variants]"""
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
import torch  # noqa: E402,F401
import golhip  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
ks = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,4,8,16").split(",")]
bands = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "0,128,256,363,512").split(",")]
variants = (sys.argv[4] if len(sys.argv) > 4 else "skew,chain,lds").split(",")
engines = {}
for v in variants:
    os.environ["GOLHIP_VARIANT"] = v
    e = golhip.Engine(size, size, k=max(ks))
    e.set_fixed_k(True)  # every launch exactly k deep
    e.init_random(3)
    engines[v] = e
res = {}
for rnd in range(3):
    for v, e in engines.items():
        for k in ks:
            for b in bands:
                e.set_k(k)
                e.set_band_rows(b)
                n = max(int(os.environ.get("TUNE_STEPS", "32")), 4 * k)
                e.step(k)
                e.sync()
                t = time.perf_counter()
                e.step(n)
                e.sync()
                dt = time.perf_counter() - t
                res.setdefault(f"{v}_k{k}_b{b}", []).append(size * size * n / dt / 1e9)
out = {key: round(statistics.median(v), 1) for key, v in res.items()}
print(json.dumps(out))
best = max(out, key=out.get)
print("best", best, out[best])
