#!/usr/bin/env python3
"""Cost of per-turn alive counts on large boards (the COUNT stencil instantiation) by variant:
GCUPS of golhip_step with and without counts.  Usage: count_cost.py [size] [turns] [variants] [ks]"""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
# the tuning build holds the selectable variants / forced shapes (lib/ has only production)
os.environ.setdefault("GOLHIP_LIB", str(ROOT / "distributed-gol_amd" / "lib_tuning" / "libgolhip.so"))
import torch  # noqa: E402,F401
import golhip  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
turns = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
variants = (sys.argv[3] if len(sys.argv) > 3 else "chainlds,driftlds").split(",")
ks = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "16").split(",")]
res = {}
for v in variants:
  for k in ks:
    os.environ["GOLHIP_VARIANT"] = v
    with golhip.Engine(size, size, k=k) as e:
        e.init_random(3)
        for counts in (False, True, False, True):
            e.step(64, counts=counts)
            e.sync()
            t = time.perf_counter()
            e.step(turns, counts=counts)
            e.sync()
            dt = time.perf_counter() - t
            res.setdefault(f"{v}_k{k}_{'counts' if counts else 'plain'}", []).append(
                round(size * size * turns / dt / 1e9, 1))
print(json.dumps({"size": size, "turns": turns, "gcups": res}))
