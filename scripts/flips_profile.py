#!/usr/bin/env python3
"""Profiling driver for the per-turn flips path and the snapshot path (run under rocprofv3):

  * golhip_step_flips at 512^2 and 5120^2 (random p=0.5, seed 7), 128 turns per call, a few calls
    -- the TestSdl event stream (sdl_test.go:57-74) -- wall time per turn printed;
  * `s` snapshots at 5120^2: golhip_store_bytes between steps (gol/distributor.go:93-103), which
    must issue no hipMalloc/hipFree (the per-shard stage is allocated at create).

Usage: python scripts/flips_profile.py [--calls N] [--snapshots N] [--rows]"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa: E402,F401  (one HIP runtime per process)

import golhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--calls", type=int, default=8)
ap.add_argument("--snapshots", type=int, default=8)
ap.add_argument("--rows", action="store_true", help="golhip_step_flips_rows (uint16 x + row offsets)")
a = ap.parse_args()
res = {}
for n in (512, 5120):
    with golhip.Engine(n, n, k=16) as e:
        e.init_random(7)
        T = min(128, e.flips_ring_capacity())
        step = (lambda: len(e.step_flips_rows(T)[0])) if a.rows else \
            (lambda: sum(len(x) for x in e.step_flips(T)[0]))
        step()  # ring + pinned host list allocated, code paths warm
        e.init_random(7)
        cells = 0
        t0 = time.perf_counter()
        for _ in range(a.calls):
            cells += step()
        dt = time.perf_counter() - t0
        res[f"flips_{n}"] = {"us_per_turn": round(dt / (a.calls * T) * 1e6, 2), "turns_per_call": T,
                             "flips_per_turn": round(cells / (a.calls * T), 1),
                             "list_bytes_per_call": int(cells / a.calls * (2 if a.rows else 8)),
                             "launch_kind": e.launch_kind(16)}
with golhip.Engine(5120, 5120, k=16) as e:
    e.init_random(2)
    e.store()  # first call: host pages of the output array
    t0 = time.perf_counter()
    for _ in range(a.snapshots):
        e.step(16)
        e.store()
    res["snapshots_5120"] = {"count": a.snapshots,
                             "ms_per_step16_plus_store": round((time.perf_counter() - t0) / max(a.snapshots, 1) * 1e3, 3)}
print(json.dumps(res), flush=True)
