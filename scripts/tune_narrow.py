#!/usr/bin/env python3
"""Narrow boards (<= 62 packed words: the reference's test sizes and configs[0] 512^2): us per turn
of long golhip_step runs (so the per-call overhead drops out) for the automatic choice and forced
register slabs (tuning build GOLHIP_SLAB; NC = 14 the packed narrow-board slab gol_slabp), with and
without counts, one engine alive at a time, median of 3 interleaved rounds; every variant's counts
must equal the automatic choice's.  Usage: tune_narrow.py sizes codes [turns]
(sizes: HxW,...; codes: auto,141603,80803@8,...)"""
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
os.environ.setdefault("GOLHIP_LIB", str(ROOT / "distributed-gol_amd" / "lib_tuning" / "libgolhip.so"))
import numpy as np  # noqa: E402

import golhip  # noqa: E402

sizes = [tuple(int(v) for v in s.split("x")) for s in sys.argv[1].split(",")]
codes = sys.argv[2].split(",")
turns = int(sys.argv[3]) if len(sys.argv) > 3 else 1600
res = {}
for (h, w) in sizes:
    for counts in (True, False):
        times, kinds, outs = {}, {}, {}
        for r in range(3):
            for code in (codes if r % 2 == 0 else codes[::-1]):
                os.environ.pop("GOLHIP_SLAB", None)
                name, _, kk = code.partition("@")  # code[@k]: launch depth k (default 16)
                k = int(kk or 16)
                if name != "auto":
                    os.environ["GOLHIP_SLAB"] = name
                e = golhip.Engine(w, h, k=k)
                os.environ.pop("GOLHIP_SLAB", None)
                e.set_fixed_k(True)
                e.init_random(5)
                e.step(32, counts=counts)
                e.sync()
                t = time.perf_counter()
                c = e.step(turns, counts=counts)
                e.sync()
                times.setdefault(code, []).append((time.perf_counter() - t) * 1e6 / turns)
                kinds[code] = list(e.launch_kind(k, counts=counts))
                outs.setdefault(code, []).append(np.asarray(c, dtype=np.int64) if counts else e.alive_count())
                e.close()
        ref = outs["auto"][0] if "auto" in outs else None
        for code in times:
            same = ref is None or all(np.array_equal(x, ref) for x in outs[code])
            key = f"{h}x{w}_{'counts' if counts else 'plain'}_{code}"
            res[key] = {"us_per_turn": round(statistics.median(times[code]), 3), "same": bool(same),
                        "kernel": kinds[code]}
            print(json.dumps({key: res[key]}), flush=True)
print(json.dumps({"narrow": res}))
