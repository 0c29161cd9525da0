#!/usr/bin/env python3
"""Measure every BASELINE.json config on one GPU (the headline configs[2] is bench.py's line).

  cfg1  images/512x512.pgm, 100 turns: GPU wall time incl. load/store vs the reference algorithm
        on the host (oracle port, 16 threads); output must equal check/images/512x512x100.pgm
  cfg2  5120^2 random seed 2, 10000 turns with the alive count of EVERY turn (checked vs golden)
  cfg4  262144^2 random seed 4 (8 GiB packed) on 1 GPU, 64 turns (the strong-scaling base)
  cfg5  4096^2 Gosper gun + R-pentomino, 1e6 turns through the C++ host (gol::Run, 2 s ticker,
        TurnComplete every turn), wall time and ticks; plus golhip_step alone
Prints one JSON object.  Run on the GPU box from the repo root.
"""
import json
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import torch  # noqa: E402,F401  (single HIP runtime, see golhip.py)
import numpy as np  # noqa: E402

import golhip  # noqa: E402
import oracle  # noqa: E402  (checker + CPU baseline only)

GOLDEN = ROOT / "tests" / "golden"
REF = GOLDEN / "reference"
res = {}


def sync_time(fn):
    t = time.perf_counter()
    out = fn()
    return time.perf_counter() - t, out


# ---- cfg1
_, _, board = oracle.read_pgm(REF / "images/512x512.pgm")
expected = (REF / "check/images/512x512x100.pgm").read_bytes()


def cfg1_gpu():
    with golhip.Engine(512, 512, k=8) as e:
        e.load(board)
        e.step(100)
        return e.store()


cfg1_gpu()  # warm (module load, code object)
dt, out = sync_time(cfg1_gpu)
dtc, outc = sync_time(lambda: oracle.ref_run(board, 100, threads=4, servers=4)[0])
res["cfg1"] = {"gpu_s": round(dt, 5), "gpu_gcups": round(512 * 512 * 100 / dt / 1e9, 2),
               "cpu_reference_port_s": round(dtc, 3),
               "cpu_gcups": round(512 * 512 * 100 / dtc / 1e9, 3), "cpu_threads": 16,
               "bit_exact": oracle.pgm_bytes(out) == expected and oracle.pgm_bytes(outc) == expected,
               "note": "GPU time includes engine create, PGM load, 100 turns, store"}

# ---- cfg2
gold = json.loads((GOLDEN / "synthetic_golden.json").read_text())
exp2 = oracle.read_alive_csv(GOLDEN / gold["cfg2"]["counts_csv"])
cfg2 = {}
for k in (8, 16, 32):
    with golhip.Engine(5120, 5120, k=k) as e:
        e.init_random(2)
        e.step(64, counts=True)
        e.init_random(2)
        e.sync()
        dt, counts = sync_time(lambda: e.step(10000, counts=True))
        ok = [int(c) for c in counts] == [exp2[t] for t in range(1, 10001)]
        cfg2[f"k{k}"] = {"s": round(dt, 4), "gcups": round(5120 * 5120 * 10000 / dt / 1e9, 1),
                         "us_per_turn": round(dt / 10000 * 1e6, 3), "counts_match": ok}
res["cfg2"] = cfg2

# ---- cfg4 (1 GPU)
with golhip.Engine(262144, 262144, k=8) as e:
    e.init_random(4)
    e.step(8)
    e.sync()
    dt, _ = sync_time(lambda: (e.step(64), e.sync()))
    res["cfg4_1gpu"] = {"turns": 64, "s": round(dt, 4),
                        "gcups": round(262144 ** 2 * 64 / dt / 1e9, 1)}

# ---- cfg5
b = np.zeros((4096, 4096), dtype=np.uint8)
golhip.place(b, golhip.parse_rle((GOLDEN / "gosper_gun.rle").read_text()), 64, 64)
golhip.place(b, golhip.parse_rle((GOLDEN / "r_pentomino.rle").read_text()), 2048, 2048)
cfg5 = {}
for k in (16, 32):
    with golhip.Engine(4096, 4096, k=k) as e:
        e.load(b)
        e.sync()
        dt, counts = sync_time(lambda: e.step(1000000, counts=True))
        cfg5[f"step_k{k}"] = {"s": round(dt, 3), "us_per_turn": round(dt, 3),
                              "gcups": round(4096 * 4096 * 1e6 / dt / 1e9, 1),
                              "count_1e6": int(counts[-1])}
with golhip.Engine(4096, 4096, k=16) as e:
    e.load(b)
    counts5 = [int(c) for c in e.step(1000000, counts=True)]
init5 = int((b == 255).sum())
for keys in (False, True):
    with tempfile.TemporaryDirectory() as d:
        (Path(d) / "images").mkdir()
        (Path(d) / "images" / "4096x4096.pgm").write_bytes(oracle.pgm_bytes(b))
        t = time.perf_counter()
        p = subprocess.Popen([str(ROOT / "distributed-gol_amd/lib/gol"), "-w", "4096", "-h", "4096",
                              "-turns", "1000000", "-k", "16", "-images", f"{d}/images",
                              "-out", f"{d}/out"], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                             text=True)
        if keys:  # p (hold 2.5 s: the 2 s ticker fires while paused), s, p
            for key, wait in (("p", 0.8), ("s", 2.5), ("p", 0.3)):
                time.sleep(wait)
                p.stdin.write(key + "\n")
                p.stdin.flush()
        out, _ = p.communicate(timeout=600)
        wall = time.perf_counter() - t
    ticks = [ln for ln in out.splitlines() if "Alive Cells" in ln]
    tick_ok = all(int(ln.split()[-1]) == (init5 if int(ln.split()[2]) == 0
                                          else counts5[int(ln.split()[2]) - 1]) for ln in ticks)
    cfg5["host_run_keys" if keys else "host_run"] = {
        "wall_s": round(wall, 2), "rc": p.returncode, "ticks": len(ticks),
        "ticks_match_counts": tick_ok, "first_ticks": ticks[:3],
        "states": [ln for ln in out.splitlines() if ln.endswith(("Paused", "Executing"))
                   or "output complete" in ln],
        "final": out.splitlines()[-1:],
        "note": ("gol::Run with TurnComplete per turn + 2 s AliveCellsCount ticker"
                 + (", keys p (2.5 s) s p; wall includes the pause" if keys else
                    "; finishes before the first 2 s tick"))}
res["cfg5"] = cfg5
print(json.dumps(res))
