#!/usr/bin/env python3
"""Split a small-board run's time into kernel execution and the gaps between dispatches, from a
rocprofv3 --kernel-trace --output-format csv directory (scripts/profile_small.py under rocprofv3).

Per kernel (short name, grid size): dispatches, mean/median duration, and the mean gap from the
previous dispatch's end to this one's start; then the whole timed window: busy vs idle share.
Usage: launch_timeline.py <trace dir> [last N dispatches (default: all)]"""
import csv
import glob
import re
import statistics
import sys
from collections import defaultdict

d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     r.get("Grid_Size_X", r.get("Grid_Size", ""))))
rows.sort()
if last:
    rows = rows[-last:]


def short(n):
    m = re.search(r"(gol_stencil_split|gol_stencil|gol_step1|\w+_rows|\w+counts?\w*)", n)
    k = re.search(r"ILi(\d+)E", n)
    return (m.group(1) if m else n[:40]) + (f"<{k.group(1)}>" if k else "")


per = defaultdict(lambda: {"dur": [], "gap": []})
prev_end = None
for s, e, n, g in rows:
    key = f"{short(n)} grid {g}"
    per[key]["dur"].append(e - s)
    if prev_end is not None:
        per[key]["gap"].append(s - prev_end)
    prev_end = e
for key, v in sorted(per.items(), key=lambda kv: -sum(kv[1]["dur"])):
    gaps = v["gap"] or [0]
    print(f"{key:50s} n={len(v['dur']):6d} dur mean {statistics.mean(v['dur']) / 1e3:8.2f} us "
          f"median {statistics.median(v['dur']) / 1e3:8.2f} us   gap-before mean "
          f"{statistics.mean(gaps) / 1e3:7.2f} us median {statistics.median(gaps) / 1e3:7.2f} us")
if rows:
    span = rows[-1][1] - rows[0][0]
    busy = sum(e - s for s, e, _, _ in rows)
    print(f"window {span / 1e3:.1f} us, {len(rows)} dispatches, busy {100 * busy / span:.1f} %, "
          f"idle {100 * (1 - busy / span):.1f} %")
