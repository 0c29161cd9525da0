#!/usr/bin/env python3
"""A/B of the two round-5 small-board paths against the register slabs they replace:
  board  : the whole-board single-workgroup kernel (stencil_board.hip) vs the multi-workgroup
           slab kernels, per square size (us per turn over calls of `turns` turns with counts);
  skip   : stable-slab skipping on / off on a dense board (5120^2 random, every slab active) and on
           configs[4] (4096^2 gun + R-pentomino, after its busy first 20 000 turns), us per turn.
Usage: probe_act_board.py [turns per call] [calls]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import golhip  # noqa: E402

turns = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 5


def timed(e, n, counts=True):
    e.step(n, counts=counts)  # warm (graphs, buffers)
    e.sync()
    best = 1e9
    c = None
    for _ in range(calls):
        t = time.perf_counter()
        c = e.step(n, counts=counts)
        e.sync()
        best = min(best, time.perf_counter() - t)
    return best / n * 1e6, c


out = {"turns_per_call": turns, "calls": calls, "board": {}, "skip": {}}
for size in (16, 64, 128, 256, 512):
    row = {}
    ref = None
    for board_kernel in (True, False):
        with golhip.Engine(size, size, k=16) as e:
            e.set_board_kernel(board_kernel)
            e.load(((np.random.default_rng(size).random((size, size)) < 0.4) * 255).astype(np.uint8))
            kind = e.launch_kind(16, counts=True)
            us, c = timed(e, turns)
            if ref is None:
                ref = c
            row["board" if board_kernel else "slab"] = {"kernel": f"{kind[0]}{kind[1]}", "us_per_turn": round(us, 3)}
            assert np.array_equal(c, ref)
    out["board"][size] = row
    print(size, row, flush=True)

b4 = np.zeros((4096, 4096), dtype=np.uint8)
G = ROOT / "tests" / "golden"
golhip.place(b4, golhip.parse_rle((G / "gosper_gun.rle").read_text()), 64, 64)
golhip.place(b4, golhip.parse_rle((G / "r_pentomino.rle").read_text()), 2048, 2048)
for name, (w, h) in (("dense_5120", (5120, 5120)), ("configs4_4096", (4096, 4096))):
    row = {}
    for act in (True, False):
        with golhip.Engine(w, h, k=16) as e:
            e.set_activity(act)
            if name == "dense_5120":
                e.init_random(2)
            else:
                e.load(b4)
                e.step(20000)  # past the busy start
            us, _ = timed(e, turns)
            row["on" if act else "off"] = {"us_per_turn": round(us, 3), "stats": e.activity_stats()}
    out["skip"][name] = row
    print(name, row, flush=True)
print(json.dumps(out))
