#!/usr/bin/env python3
"""Register kernels vs streaming kernels on small/medium boards: us per turn of golhip_step WITH
per-turn counts (configs[1] / configs[4] style), per (size, kernel spec, launch depth K), fixed
depth, median of 3 interleaved rounds.  Specs: 0 = the streaming kernels (level split where it
picks it), tT = gol_tile with T-row tiles, sWWSS = gol_slab with WW waves x SS rows, a = automatic.
Usage: tune_tile.py sizes specs Ks [turns]     e.g. tune_tile.py 2048,5120 0,t16,s1608 8,16"""
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

sizes = [int(x) for x in sys.argv[1].split(",")]
Ts = sys.argv[2].split(",")
Ks = [int(x) for x in sys.argv[3].split(",")]
turns_arg = int(sys.argv[4]) if len(sys.argv) > 4 else 0
counts = os.environ.get("TUNE_COUNTS", "1") != "0"  # TUNE_COUNTS=0: no per-turn counts
res = {}
for size in sizes:
    turns = turns_arg or max(256, min(4096, int(4e10 / (size * size))))
    engines = {}
    for T in Ts:
        for var in ("GOLHIP_TILE", "GOLHIP_SLAB"):
            os.environ.pop(var, None)
        if T == "0":
            os.environ["GOLHIP_TILE"] = os.environ["GOLHIP_SLAB"] = "0"
        elif T.startswith("t"):
            os.environ["GOLHIP_TILE"] = T[1:]
        elif T.startswith("s"):
            os.environ["GOLHIP_SLAB"] = T[1:]
        e = golhip.Engine(size, size, k=max(Ks))
        e.set_fixed_k(True)
        engines[T] = e
    for rnd in range(3):
        for T, e in engines.items():
            for k in Ks:
                e.set_k(k)
                kind = e.launch_kind(k)
                e.init_random(2)
                e.step(2 * k, counts=counts)
                e.sync()
                t = time.perf_counter()
                e.step(turns, counts=counts)
                e.sync()
                dt = time.perf_counter() - t
                res.setdefault(f"{size}/T{T}/k{k}", {"kind": kind, "us": []})["us"].append(dt / turns * 1e6)
    for e in engines.values():
        e.close()
out = {key: {"kind": f"{v['kind'][0]}{v['kind'][1] or ''}", "us_per_turn": round(statistics.median(v["us"]), 3)}
       for key, v in res.items()}
print(json.dumps({"us_per_turn_with_counts": out}, indent=0))
for size in sizes:
    keys = [k for k in out if k.startswith(f"{size}/")]
    best = min(keys, key=lambda k: out[k]["us_per_turn"])
    print("best", best, out[best])
