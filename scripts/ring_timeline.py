#!/usr/bin/env python3
"""Per-block timeline of the split step (ring of one, GOLHIP_RING_SELF=1) from a rocprofv3
--kernel-trace CSV: where the boundary bands, the interior and the RCCL send/recv of each block
run relative to each other, and what the block's wall time is made of.

  run:     ring_timeline.py run [size] [turns] [ring 0/1] [warmup]   (under rocprofv3 --kernel-trace)
  analyse: ring_timeline.py <trace dir> [blocks to print] [last blocks analysed (default 70)]"""
import csv
import glob
import json
import os
import re
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

if sys.argv[1] == "run":
    sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
    import time

    import torch  # noqa: F401

    import golhip
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    turns = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    ring = sys.argv[4] != "0" if len(sys.argv) > 4 else True
    warm = int(sys.argv[5]) if len(sys.argv) > 5 else 8
    if ring:
        os.environ["GOLHIP_RING_SELF"] = "1"
    e = golhip.Engine(size, size, k=16, rank=0, world_size=1, device=0)
    t = time.perf_counter()
    while time.perf_counter() - t < 0.3:
        e.init_random(3)
        e.step(32)
        e.sync()
    e.init_random(3)
    e.step(warm)
    e.sync()
    t = time.perf_counter()
    e.step(turns)
    e.sync()
    print(json.dumps({"size": size, "turns": turns, "ring": ring,
                      "ms": round((time.perf_counter() - t) * 1e3, 3), "alive": e.alive_count()}))
    e.close()
    sys.exit(0)

d = sys.argv[1]
if len(sys.argv) > 2 and sys.argv[2] == "tail":  # the last N dispatches, raw
    n = int(sys.argv[3])
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60],
                         r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Queue_Id", "")))
    rows.sort()
    rows = rows[-n:]
    t0 = rows[0][0]
    for s_, e_, nm, g, q in rows:
        print(f"{(s_ - t0) / 1e3:9.2f} .. {(e_ - t0) / 1e3:9.2f}  ({(e_ - s_) / 1e3:7.2f} us)  q{q} g{g}  {nm}")
    sys.exit(0)
nprint = int(sys.argv[2]) if len(sys.argv) > 2 else 6
nlast = int(sys.argv[3]) if len(sys.argv) > 3 else 70
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        grid = int(r.get("Grid_Size_X", r.get("Grid_Size", "0")) or 0)
        rows.append({"s": int(r["Start_Timestamp"]), "e": int(r["End_Timestamp"]), "name": r["Kernel_Name"],
                     "grid": grid, "q": r.get("Queue_Id", r.get("Stream_Id", ""))})
rows.sort(key=lambda r: r["s"])


def kind(r):
    n = r["name"]
    if "nccl" in n.lower():
        return "rccl"
    if "gol_stencil" in n:
        return "stencil"
    return re.sub(r"\W.*", "", n)[:24]


st = [r for r in rows if kind(r) == "stencil"]
if not st:
    sys.exit("no stencil dispatches")
big = max(r["grid"] for r in st)
t0 = rows[0]["s"]
blocks = []
cur = None
for r in rows:
    k = kind(r)
    if k == "stencil" and r["grid"] >= big // 4:  # an interior (or a single-strip launch)
        cur = {"interior": r, "bands": [], "rccl": [], "other": []}
        blocks.append(cur)
    elif cur is not None:
        (cur["bands"] if k == "stencil" else cur["rccl"] if k == "rccl" else cur["other"]).append(r)


def us(x):
    return round(x / 1e3, 2)


blocks = blocks[-(nlast + 1):]
summ = {"interior_us": [], "block_us": [], "gap_after_interior_us": [], "bands_after_interior_end_us": [],
        "bands_us": [], "rccl_us": []}
for i, b in enumerate(blocks[:-1]):
    nxt = blocks[i + 1]["interior"]
    it = b["interior"]
    summ["interior_us"].append(us(it["e"] - it["s"]))
    summ["block_us"].append(us(nxt["s"] - it["s"]))
    summ["gap_after_interior_us"].append(us(nxt["s"] - it["e"]))
    if b["bands"]:
        summ["bands_us"].append(us(max(x["e"] for x in b["bands"]) - min(x["s"] for x in b["bands"])))
        summ["bands_after_interior_end_us"].append(us(max(x["e"] for x in b["bands"]) - it["e"]))
    if b["rccl"]:
        summ["rccl_us"].append(us(max(x["e"] for x in b["rccl"]) - min(x["s"] for x in b["rccl"])))
    if i < nprint or i >= len(blocks) - 1 - 2:
        ev = [("interior", it)] + [("bands", x) for x in b["bands"]] + [("rccl", x) for x in b["rccl"]] + \
             [(kind(x), x) for x in b["other"]]
        ev.sort(key=lambda kv: kv[1]["s"])
        print(f"block {i}: " + "; ".join(f"{n}[q{x['q']} g{x['grid']}] {us(x['s'] - it['s'])}..{us(x['e'] - it['s'])}"
                                         for n, x in ev))
out = {k: {"mean": round(statistics.mean(v), 2), "median": round(statistics.median(v), 2), "n": len(v)}
       for k, v in summ.items() if v}
out["window_us"] = us(rows[-1]["e"] - t0)
out["dispatches"] = len(rows)
print(json.dumps(out))
