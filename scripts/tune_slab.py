#!/usr/bin/env python3
"""Slab-shape sweep on small boards through the production step path (graphs, count window):
us per turn of golhip_step for each forced gol_slab shape (GOLHIP_SLAB = NC*10000 + W*100 + S,
K = 16), with and without per-turn counts, median of 3 interleaved rounds.  Every shape's
per-turn counts must equal the golden (5120^2 seed 2: tests/golden cfg2 CSV) or, on other
sizes, the automatic shape's counts.
Usage: tune_slab.py size[,size..] shape[,shape..] [turns]   (shape 0 = automatic choice; a size
is N for N x N or WxH)"""
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
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import golhip  # noqa: E402

sizes = sys.argv[1].split(",")
shapes = [int(x) for x in sys.argv[2].split(",")]
turns = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
gold = json.loads((ROOT / "tests/golden/synthetic_golden.json").read_text())
res, ok = {}, {}
for n in sizes:
    w, h = (int(v) for v in n.split("x")) if "x" in n else (int(n), int(n))
    ref = None
    if n == "5120":
        lines = (ROOT / "tests/golden" / gold["cfg2"]["counts_csv"]).read_text().split()[1:]
        ref = np.array([int(ln.split(",")[1]) for ln in lines[:256 + turns]], dtype=np.uint64)
    engines = {}
    for sh in shapes:
        if sh:
            os.environ["GOLHIP_SLAB"] = str(sh)
        else:
            os.environ.pop("GOLHIP_SLAB", None)
        engines[sh] = golhip.Engine(w, h, k=16)
    os.environ.pop("GOLHIP_SLAB", None)
    for rnd in range(3):
        for sh, e in engines.items():
            for counts in (True, False):
                e.init_random(2)
                c0 = e.step(256, counts=counts)
                e.sync()
                t = time.perf_counter()
                c1 = e.step(turns, counts=counts)
                e.sync()
                dt = time.perf_counter() - t
                key = f"{n}_s{sh}_{'c' if counts else 'n'}"
                res.setdefault(key, []).append(dt / turns * 1e6)
                if counts:
                    got = np.concatenate([c0, c1]).astype(np.uint64)
                    if ref is None and sh == 0:
                        ref = got
                    good = ref is not None and np.array_equal(got, ref[:len(got)])
                    ok[key] = ok.get(key, True) and bool(good)
    for e in engines.values():
        e.close()
out = {k: round(statistics.median(v), 4) for k, v in res.items()}
print(json.dumps({"us_per_turn": out, "counts_ok": ok}))
for n in sizes:
    for c in ("c", "n"):
        ks = {k: v for k, v in out.items() if k.startswith(f"{n}_") and k.endswith(f"_{c}")}
        b = min(ks, key=ks.get)
        print("best", n, c, b, ks[b], flush=True)
