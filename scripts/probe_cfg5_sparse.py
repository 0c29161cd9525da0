#!/usr/bin/env python3
"""configs[4] (4096^2 glider gun + R-pentomino, a sparse board): slab shape x stable-slab skipping.

With one slab per CU a launch lasts as long as its slowest computed slab, so skipping buys nothing at
the automatic 12 x 7 (237 slabs).  With SMALLER slabs (12 x 4: T = 16, 768 slabs, three rounds) most
workgroups are skipped ones that exit after one copy, and the dispatcher hands the freed CUs to the
active ones: the active work may fit about one round of 12-row-per-SIMD slabs instead of 21.  This
A/B measures it through golhip_step with every count (checked against the golden npz), on the fault
library (its GOLHIP_SLAB selector forces production shapes).
Usage: probe_cfg5_sparse.py [turns] [shapes]   (shapes: comma list of GOLHIP_SLAB codes, 0 = auto)"""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import golhip  # noqa: E402

turns = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
shapes = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,121204,121604,121207").split(",")]
G = ROOT / "tests" / "golden"
gold = json.loads((G / "synthetic_golden.json").read_text())
b = np.zeros((4096, 4096), dtype=np.uint8)
golhip.place(b, golhip.parse_rle((G / "gosper_gun.rle").read_text()), 64, 64)
golhip.place(b, golhip.parse_rle((G / "r_pentomino.rle").read_text()), 2048, 2048)
deltas = np.load(G / gold["cfg5"]["counts_1e6_npz"])["deltas"][:turns]
exp = (int((b == 255).sum()) + np.cumsum(deltas.astype(np.int64))).astype(np.uint64)
L = golhip.fault_library()
res = {}
for rnd in range(2):
    for sh in shapes:
        for act in (-1, 1):
            if sh:
                os.environ["GOLHIP_SLAB"] = str(sh)
            else:
                os.environ.pop("GOLHIP_SLAB", None)
            with golhip.Engine(4096, 4096, k=16, lib=L) as e:
                os.environ.pop("GOLHIP_SLAB", None)
                e.set_activity(act)
                kind = e.launch_kind(16, counts=True)
                e.load(b)
                e.step(4096, counts=True)  # capture the count graphs
                e.load(b)
                e.sync()
                s0 = e.activity_stats()
                t = time.perf_counter()
                c = e.step(turns, counts=True)
                dt = time.perf_counter() - t
                s1 = e.activity_stats()
            key = f"s{sh}_act{act}"
            r = res.setdefault(key, {"kernel": f"{kind[0]}{kind[1]}", "us_per_turn": [], "ok": True})
            r["us_per_turn"].append(round(dt / turns * 1e6, 4))
            r["ok"] = r["ok"] and bool(np.array_equal(c.astype(np.uint64), exp))
            r["slabs_computed_skipped"] = [s1[0] - s0[0], s1[1] - s0[1]]
            print(key, r, flush=True)
print(json.dumps({"turns": turns, "results": res}))
