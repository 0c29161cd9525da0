#!/usr/bin/env python3
"""Same-process A/B of stencil variants on a pre-heated chip: one engine per variant on the same
seeded board, advanced in lockstep (same turns, so the same density), rounds alternating the
variant order; per (variant, k) the median and every round's TCUPS.  A variant may carry a band
schedule: "pre63@184:364:176" = bands of 184 rows, the last 364 of 176 (golhip_set_tail_bands).
Usage: ab_variant.py [size] [ks] [variants] [rounds] [band_rows]"""
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
ks = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "12,16").split(",")]
variants = (sys.argv[3] if len(sys.argv) > 3 else "prod,pre63").split(",")
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 7
band = int(sys.argv[5]) if len(sys.argv) > 5 else 0
engines = {}
for v in variants:
    os.environ["GOLHIP_VARIANT"] = v.split("@")[0]
    e = golhip.Engine(size, size, k=max(ks))
    e.set_fixed_k(True)
    e.set_band_rows(band)
    if "@" in v:
        b, n2, b2 = (int(x) for x in v.split("@")[1].split(":"))
        e.set_band_rows(b)
        e.set_tail_bands(n2, b2)
    e.init_random(3)
    engines[v] = e
steps = int(os.environ.get("AB_STEPS", "192"))
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.4:  # pre-heat the chip on every engine
    for e in engines.values():
        e.step(48)
        e.sync()
res = {}
for rnd in range(rounds):
    order = list(engines.items()) if rnd % 2 == 0 else list(reversed(engines.items()))
    for k in ks:
        n = max(steps // k, 2) * k
        for v, e in order:
            e.set_k(k)
            e.step(k)
            e.sync()
            t = time.perf_counter()
            e.step(n)
            e.sync()
            dt = time.perf_counter() - t
            res.setdefault(f"{v}_k{k}", []).append(size * size * n / dt / 1e9)
alive = {v: e.alive_count() for v, e in engines.items()}
assert len(set(alive.values())) == 1, alive  # lockstep: every variant on the same board
out = {key: round(statistics.median(v), 1) for key, v in res.items()}
print(json.dumps({"median": out, "rounds": {k: [round(x, 1) for x in v] for k, v in res.items()},
                  "alive": list(alive.values())[0]}))
for k in ks:
    base = out[f"{variants[0]}_k{k}"]
    print(f"k={k}: " + ", ".join(f"{v} {out[f'{v}_k{k}']} ({out[f'{v}_k{k}'] / base - 1:+.2%})" for v in variants))
