#!/usr/bin/env python3
"""Kernel stats (calls, total/avg/min/max ns, %) from a rocprofv3 --kernel-trace --stats SQLite
database (rocprofv3's default output format in ROCm 7), as CSV like rocprofv3's kernel_stats.csv,
one row per (kernel, grid size): launches of one kernel over different boards stay apart.
Usage: rocpd_stats.py <rp_results.db> [out.csv]"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
grid = "grid_x" if "grid_x" in cols else "0"
rows = db.execute(f"select {name}, {grid}, count(*), sum(end-start), avg(end-start), min(end-start), "
                  f"max(end-start) from kernels group by {name}, {grid} "
                  f"order by sum(end-start) desc").fetchall()
tot = sum(r[3] for r in rows) or 1
out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
w = csv.writer(out)
w.writerow(["Name", "GridX", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
for n, g, c, t, a, mn, mx in rows:
    w.writerow([n, g, c, t, round(a, 1), round(100 * t / tot, 2), mn, mx])
