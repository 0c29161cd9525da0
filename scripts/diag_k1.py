#!/usr/bin/env python3
"""Diagnostic: k = 1 launch time after different preceding engine histories (one process)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import torch  # noqa
import golhip  # noqa


def k1_us(e, n=256):
    e.set_k(1)
    e.step(2)
    e.sync()
    e.timing(True)
    e.step(n)
    e.sync()
    ms, l, _ = e.kernel_time()
    e.timing(False)
    return round(ms * 1e3 / max(l, 1), 1)


def run(name, k0, main, timing, count):
    e = golhip.Engine(65536, 65536, k=k0)
    e.init_random(3)
    e.step(8)
    e.sync()
    r = {"fresh": k1_us(e)}
    e.set_k(k0)
    e.timing(timing)
    e.step(main)
    e.sync()
    e.timing(False)
    if count:
        e.alive_count()
    r["after"] = k1_us(e)
    r["again"] = k1_us(e)
    e.close()
    print(name, r, flush=True)


for rep in range(2):
    run("k16 main1000 timing count", 16, 1000, True, True)
    run("k16 main1000 notiming nocount", 16, 1000, False, False)
    run("k1 main1000 timing count", 1, 1000, True, True)
    run("k16 main0", 16, 0, False, False)
