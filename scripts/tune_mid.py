#!/usr/bin/env python3
"""Mid-size boards: where the register slab stops paying against the streaming kernel.  us per
turn of a 512-turn golhip_step (with and without per-turn counts) for the automatic choice, a
forced production slab shape and the streaming kernel (tuning build selectors, read at create),
median of 5 interleaved rounds; every variant's counts must equal the automatic choice's.
Usage: tune_mid.py [sizes] [turns]"""
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

sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "6144,8192,10240,12288,16384").split(",")]
turns = int(sys.argv[2]) if len(sys.argv) > 2 else 512
res = {}
for n in sizes:
    for counts in (False, True):
        variants = {"auto": {}, "slab": {"GOLHIP_SLAB": "121606" if counts else "91606"},
                    "stream": {"GOLHIP_SLAB": "0", "GOLHIP_TILE": "0"}}
        engs = {}
        for name, env in variants.items():
            for key in ("GOLHIP_SLAB", "GOLHIP_TILE"):
                os.environ.pop(key, None)
            os.environ.update(env)
            engs[name] = golhip.Engine(n, n, k=16)
        for key in ("GOLHIP_SLAB", "GOLHIP_TILE"):
            os.environ.pop(key, None)
        times = {name: [] for name in engs}
        ref, ok = None, {}
        for r in range(5):
            for name in (list(engs) if r % 2 == 0 else list(reversed(list(engs)))):
                e = engs[name]
                e.init_random(5)
                e.step(32, counts=counts)
                e.sync()
                t = time.perf_counter()
                c = e.step(turns, counts=counts)
                e.sync()
                times[name].append((time.perf_counter() - t) * 1e6 / turns)
                a = e.alive_count()
                key = np.asarray(c, dtype=np.int64).tobytes() if counts else a
                if name == "auto":
                    ref = key if ref is None else ref
                ok.setdefault(name, []).append(key)
        for name, e in engs.items():
            tag = f"{n}_{'c' if counts else 'n'}_{name}"
            res[tag] = {"us_per_turn": round(statistics.median(times[name]), 3),
                        "same_as_auto": all(x == ref for x in ok[name]),
                        "kernel": list(e.launch_kind(16, counts=counts))}
            print(json.dumps({tag: res[tag]}), flush=True)
            e.close()
print(json.dumps({"mid": res}))
