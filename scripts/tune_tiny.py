#!/usr/bin/env python3
"""Tiny boards (configs[0] 512^2 x 100 and the reference's test sizes): us per turn of a
100-turn golhip_step with every count, for the automatic choice and forced alternatives (tuning
build selectors, read at create): register slabs (GOLHIP_SLAB), register tiles (GOLHIP_TILE), the
streaming kernel (GOLHIP_SLAB=0, GOLHIP_TILE=0) at k = 8 / 16 / 32.  Median of 7 interleaved
rounds; every variant's counts must equal the automatic choice's.
Usage: tune_tiny.py [sizes] [turns]"""
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
import torch  # noqa: E402,F401

import golhip  # noqa: E402

sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "512,256,128").split(",")]
turns = int(sys.argv[2]) if len(sys.argv) > 2 else 100
VARIANTS = {  # name: (env, k)
    "auto": ({}, 16),
    "slab_121606": ({"GOLHIP_SLAB": "121606"}, 16),
    "slab_90812": ({"GOLHIP_SLAB": "90812"}, 16),
    "slab_121207": ({"GOLHIP_SLAB": "121207"}, 16),
    "slab_808_k8": ({"GOLHIP_SLAB": "808"}, 8),
    "tile16": ({"GOLHIP_TILE": "16", "GOLHIP_SLAB": "0"}, 16),
    "tile32": ({"GOLHIP_TILE": "32", "GOLHIP_SLAB": "0"}, 16),
    "stream_k16": ({"GOLHIP_SLAB": "0", "GOLHIP_TILE": "0"}, 16),
    "stream_k32": ({"GOLHIP_SLAB": "0", "GOLHIP_TILE": "0"}, 32),
    "stream_k8": ({"GOLHIP_SLAB": "0", "GOLHIP_TILE": "0"}, 8),
}
KNOBS = ("GOLHIP_SLAB", "GOLHIP_TILE")
res = {}
for n in sizes:
    engs, ok = {}, {}
    for name, (env, k) in VARIANTS.items():
        for key in KNOBS:
            os.environ.pop(key, None)
        os.environ.update(env)
        try:
            e = golhip.Engine(n, n, k=k)
            e.set_fixed_k(True)
            engs[name] = e
        except golhip.GolHipError as err:
            res[f"{n}_{name}"] = f"unsupported: {err}"
    for key in KNOBS:
        os.environ.pop(key, None)
    times = {name: [] for name in engs}
    ref = None
    for r in range(7):
        for name in (list(engs) if r % 2 == 0 else list(reversed(list(engs)))):
            e = engs[name]
            e.init_random(5)
            e.step(16, counts=True)
            e.sync()
            t = time.perf_counter()
            c = e.step(turns, counts=True)
            e.sync()
            times[name].append((time.perf_counter() - t) * 1e6 / turns)
            c = np.asarray(c, dtype=np.int64)
            if name == "auto":
                ref = c if ref is None else ref
            ok.setdefault(name, []).append(c)
    for name in engs:
        same = all(np.array_equal(x, ref) for x in ok[name])
        kind = engs[name].launch_kind(VARIANTS[name][1], counts=True)
        res[f"{n}_{name}"] = {"us_per_turn": round(statistics.median(times[name]), 3), "counts_ok": same,
                              "kernel": list(kind)}
        print(json.dumps({f"{n}_{name}": res[f"{n}_{name}"]}), flush=True)
        engs[name].close()
print(json.dumps({"tiny": res}))
