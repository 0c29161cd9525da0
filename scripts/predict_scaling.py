#!/usr/bin/env python3
"""Predicted multi-GPU efficiency from single-GPU measurements of the exact per-GPU strip shapes.

Every rank of a golhip_create_rank board runs the same code on its strip: the K-row halo exchange
(RCCL send/recv on the comm stream), the interior launch overlapped with it, and the two boundary
bands after the halos land.  GOLHIP_RING_SELF=1 runs exactly that on one GPU -- a ring of ONE
halo'd strip whose halos go through ncclSend/ncclRecv to itself -- so the per-GPU time of a
G-GPU run is predicted by the ring-of-one time of its strip (what it leaves out: the xGMI latency
of a real neighbour instead of a self-copy, hidden behind the interior launch as long as the
exchange is shorter than it, and the end-of-region barrier).

  strong (configs[3]): 262144 wide, strips of 262144/G rows, vs the 1-GPU board as one strip
                       (no halos: rows wrap): eff(G) = t1 / t_ring(262144/G rows)... per GPU, i.e.
                       eff(G) = T(1 GPU, whole board) / (G x T_ring(strip of G))
  weak (bench --gpus N): 65536 x 65536 per GPU, vs the N = 1 line's single 65536^2 strip:
                       eff = T(single 65536^2) / T_ring(65536^2 strip)

Each shape: one single-strip and one ring-of-one engine on the same seeded board, pre-heated,
alternating rounds; the alive counts of both must agree.
Usage: predict_scaling.py [rounds] [weak turns list] [strong turns] [strong gpus list]"""
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402

import golhip  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
weak_turns = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "20,1000").split(",")]
strong_turns = int(sys.argv[3]) if len(sys.argv) > 3 else 160
strong_gpus = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "1,2,4,8").split(",")]
assert strong_gpus[0] == 1
K = 16


def make(width, rows, ring):
    if ring:
        os.environ["GOLHIP_RING_SELF"] = "1"
    else:
        os.environ.pop("GOLHIP_RING_SELF", None)
    try:
        return golhip.Engine(width, rows, k=K, rank=0, world_size=1, device=0)
    finally:
        os.environ.pop("GOLHIP_RING_SELF", None)


def timed(e, seed, warmup, turns):
    e.init_random(seed)
    e.step(warmup)
    e.sync()
    torch.cuda.synchronize()
    t = time.perf_counter()
    e.step(turns)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    e.sync()
    return dt, e.alive_count()


def measure(width, rows, seed, warmup, turns):
    engs = {"single": make(width, rows, False), "ring": make(width, rows, True)}
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:  # pre-heat the chip
        for e in engs.values():
            e.init_random(seed)
            e.step(2 * K)
            e.sync()
    times, alive = {n: [] for n in engs}, {n: set() for n in engs}
    for r in range(rounds):
        for n in (list(engs) if r % 2 == 0 else list(reversed(engs))):
            dt, a = timed(engs[n], seed, warmup, turns)
            times[n].append(dt)
            alive[n].add(a)
    for e in engs.values():
        e.close()
    assert len(alive["single"]) == 1 and alive["single"] == alive["ring"], alive
    med = {n: statistics.median(v) for n, v in times.items()}
    cells = width * rows * turns
    return {"shape": f"{width}x{rows}", "turns": turns, "warmup": warmup,
            "ms_single": round(med["single"] * 1e3, 3), "ms_ring": round(med["ring"] * 1e3, 3),
            "tcups_single": round(cells / med["single"] / 1e12, 2),
            "tcups_ring": round(cells / med["ring"] / 1e12, 2),
            "ring_over_single": round(med["ring"] / med["single"], 4),
            "alive": next(iter(alive["single"]))}


out = {"weak": [], "strong": []}
for turns in weak_turns:
    m = measure(65536, 65536, 3, 5 if turns <= 20 else 8, turns)
    m["predicted_weak_eff"] = round(1.0 / m["ring_over_single"], 4)
    out["weak"].append(m)
    print(json.dumps(m), flush=True)
base = None
for G in (strong_gpus if strong_turns > 0 else []):
    rows = 262144 // G
    m = measure(262144, rows, 4, K, strong_turns)
    if G == 1:
        base = m["ms_single"]  # the 1-GPU strong leg: the whole board as one strip
    m["gpus"] = G
    m["predicted_strong_eff"] = round(base / (G * m["ms_ring"]), 4)
    out["strong"].append(m)
    print(json.dumps(m), flush=True)
print(json.dumps(out))
