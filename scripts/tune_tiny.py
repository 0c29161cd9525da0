#!/usr/bin/env python3
"""Tiny boards (configs[0] 512^2 x 100 and the reference's test sizes): us per turn of a
100-turn golhip_step with every count, for the automatic choice and forced alternatives (tuning
build selectors, read at create): register slabs (GOLHIP_SLAB; NC = 14 the narrow-board packed slab gol_slabp), register tiles (GOLHIP_TILE), the
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
    "packed_141603": ({"GOLHIP_SLAB": "141603"}, 16),
    "packed_140806": ({"GOLHIP_SLAB": "140806"}, 16),
    "packed_140804": ({"GOLHIP_SLAB": "140804"}, 16),
    "packed_140803": ({"GOLHIP_SLAB": "140803"}, 16),
    "packed_140404": ({"GOLHIP_SLAB": "140404"}, 16),
    "tile16": ({"GOLHIP_TILE": "16", "GOLHIP_SLAB": "0"}, 16),
    "tile32": ({"GOLHIP_TILE": "32", "GOLHIP_SLAB": "0"}, 16),
    "stream_k16": ({"GOLHIP_SLAB": "0", "GOLHIP_TILE": "0"}, 16),
    "stream_k32": ({"GOLHIP_SLAB": "0", "GOLHIP_TILE": "0"}, 32),
    "stream_k8": ({"GOLHIP_SLAB": "0", "GOLHIP_TILE": "0"}, 8),
}
KNOBS = ("GOLHIP_SLAB", "GOLHIP_TILE")
res = {}
for n in sizes:
    # one engine alive at a time: engines alive together share the process's hardware queues
    # (GPU_MAX_HW_QUEUES), which slowed the later-created ones (round 4, r04p)
    times, ok, kinds = {}, {}, {}
    ref = None
    names = list(VARIANTS)
    for r in range(7):
        for name in (names if r % 2 == 0 else list(reversed(names))):
            env, k = VARIANTS[name]
            for key in KNOBS:
                os.environ.pop(key, None)
            os.environ.update(env)
            try:
                e = golhip.Engine(n, n, k=k)
            except golhip.GolHipError as err:
                res[f"{n}_{name}"] = f"unsupported: {err}"
                continue
            finally:
                for key in KNOBS:
                    os.environ.pop(key, None)
            e.set_fixed_k(True)
            e.init_random(5)
            e.step(16, counts=True)
            e.sync()
            t = time.perf_counter()
            c = e.step(turns, counts=True)
            e.sync()
            times.setdefault(name, []).append((time.perf_counter() - t) * 1e6 / turns)
            c = np.asarray(c, dtype=np.int64)
            if name == "auto":
                ref = c if ref is None else ref
            ok.setdefault(name, []).append(c)
            kinds[name] = list(e.launch_kind(k, counts=True))
            e.close()
    for name in times:
        same = all(np.array_equal(x, ref) for x in ok[name])
        res[f"{n}_{name}"] = {"us_per_turn": round(statistics.median(times[name]), 3), "counts_ok": same,
                              "kernel": kinds[name]}
        print(json.dumps({f"{n}_{name}": res[f"{n}_{name}"]}), flush=True)
print(json.dumps({"tiny": res}))
