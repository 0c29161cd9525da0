#!/usr/bin/env python3
"""Stable-slab skipping on boards with many rounds of slabs per launch (more slabs than the chip
holds at once): sparse (tests/test_gpu_activity.py sparse_board) and dense random, on / off, us
per turn over calls of 512 turns with counts.
Usage: probe_act_large.py [sizes, comma-separated] [kinds: sparse,dense]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import golhip  # noqa: E402
from test_gpu_activity import sparse_board  # noqa: E402

sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [4096, 8192, 12288, 16384]
kinds = sys.argv[2].split(",") if len(sys.argv) > 2 else ["sparse", "dense"]
out = {}
for n in sizes:
    for kind in kinds:
        b = sparse_board(n, n, seed=n, n_gliders=20, n_osc=10, n_still=10) if kind == "sparse" else None
        row = {}
        for act in (True, False):
            with golhip.Engine(n, n, k=16) as e:
                e.set_activity(act)
                if b is not None:
                    e.load(b)
                else:
                    e.init_random(5)
                e.step(512, counts=True)
                e.sync()
                best = 1e9
                for _ in range(3):
                    t = time.perf_counter()
                    e.step(512, counts=True)
                    e.sync()
                    best = min(best, time.perf_counter() - t)
                row["on" if act else "off"] = {"us_per_turn": round(best / 512 * 1e6, 3),
                                               "kind": e.launch_kind(16, counts=True), "stats": e.activity_stats()}
        out[f"{kind}_{n}"] = row
        print(kind, n, row, flush=True)
print(json.dumps(out))
