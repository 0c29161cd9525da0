#!/usr/bin/env python3
"""A/B of the persistent counting slab (golhip_step_persistent, opt-in: one launch
per 4096-generation count window, neighbour hand-offs instead of launch boundaries) against the
production path (golhip_step: graph replays of 16-generation gol_slab2 launches), on configs[4]
(4096^2 glider gun + R-pentomino) and configs[1]'s board (5120^2 random seed 2).  Same board
and counts required (bit-exact), then us per turn, best of `reps` calls of `turns` turns.
Both hand-off forms of the persistent call (golhip_set_persistent_handoff): "persistent" = the
default agent-scope release/acquire fences, "persistent_sc1" = the sc1-only measured form.
Usage: probe_slabq.py [turns] [reps] [boards]   (boards: N or WxH, comma-separated; default
4096,5120; 4096 is configs[4]'s board, the others random seed 2)"""
import ctypes
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

turns = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
boards = (sys.argv[3] if len(sys.argv) > 3 else "4096,5120").split(",")
L = golhip.load_library()
G = ROOT / "tests" / "golden"


def board(n):
    if n == "4096":
        b = np.zeros((4096, 4096), dtype=np.uint8)
        golhip.place(b, golhip.parse_rle((G / "gosper_gun.rle").read_text()), 64, 64)
        golhip.place(b, golhip.parse_rle((G / "r_pentomino.rle").read_text()), 2048, 2048)
        return b
    return None


out = {}
for n in boards:
    w, h = (int(v) for v in n.split("x")) if "x" in n else (int(n), int(n))
    b = board(n)
    res = {}
    for mode in ("production", "persistent", "persistent_sc1"):
        with golhip.Engine(w, h, k=16) as e:
            shape = e.launch_kind(16, counts=True)[1]
            if mode == "persistent_sc1":
                e.set_persistent_handoff(golhip.HANDOFF_SC1)
            if b is not None:
                e.load(b)
            else:
                e.init_random(2)
            counts_all, best = [], 1e9
            for r in range(reps + 1):
                c = np.zeros(turns, dtype=np.uint64)
                e.sync()
                t = time.perf_counter()
                if mode == "production":
                    c = e.step(turns, counts=True)
                else:
                    c = e.step_persistent(turns)
                e.sync()
                dt = time.perf_counter() - t
                counts_all.append(np.asarray(c, dtype=np.uint64).copy())
                if r > 0:  # the first call captures graphs / warms up
                    best = min(best, dt)
            res[mode] = {"us_per_turn": round(best / turns * 1e6, 4), "counts": np.concatenate(counts_all),
                         "board": e.store_words()}
    same = all(bool(np.array_equal(res["production"]["counts"], res[m]["counts"]) and
                    np.array_equal(res["production"]["board"], res[m]["board"])) for m in ("persistent", "persistent_sc1"))
    out[f"{n}_{shape}"] = {"production_us_per_turn": res["production"]["us_per_turn"],
                           "persistent_fenced_us_per_turn": res["persistent"]["us_per_turn"],
                           "persistent_sc1_us_per_turn": res["persistent_sc1"]["us_per_turn"], "bit_exact": same}
    print(n, shape, out[f"{n}_{shape}"], flush=True)
print(json.dumps(out))
