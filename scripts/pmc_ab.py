#!/usr/bin/env python3
"""Per-dispatch PMC of the timed gol_stencil launches (largest grid) for several pass directories
of one variant: counter averages, duration, effective clock (GRBM_GUI_ACTIVE / 8 / duration) and
derived rates.  Usage: pmc_ab.py <dir prefix> [variants...]   (dirs <prefix>/<variant>_p<i>)"""
import csv
import glob
import json
import sys
from collections import defaultdict

prefix, variants = sys.argv[1], sys.argv[2:] or ["prod", "pre63"]
out = {}
for v in variants:
    cnt, durs, ghz = defaultdict(list), [], []
    for d in sorted(glob.glob(f"{prefix}/{v}_p*")):
        rows = []
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            rows += [r for r in csv.DictReader(open(f)) if "gol_stencil" in r.get("Kernel_Name", "")]
        if not rows:
            continue
        big = max(int(r["Grid_Size"]) for r in rows)
        for r in rows:
            if int(r["Grid_Size"]) != big:
                continue
            ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            cnt[r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                durs.append(ns)
                ghz.append(float(r["Counter_Value"]) / 8 / ns)
    avg = {c: sum(x) / len(x) for c, x in cnt.items()}
    o = {"counters": {c: round(x) for c, x in avg.items()}}
    if durs:
        o["duration_us"] = round(sum(durs) / len(durs) / 1e3, 1)
        o["clock_ghz"] = round(sum(ghz) / len(ghz), 3)
        if "SQ_INSTS_VALU" in avg:
            o["valu_T_per_s"] = round(avg["SQ_INSTS_VALU"] / (o["duration_us"] * 1e-6) / 1e12, 4)
            o["valu_issue_frac_at_clock"] = round(o["valu_T_per_s"] / (1024 * o["clock_ghz"] * 1e9 / 2 / 1e12), 4)
        if "SQ_BUSY_CYCLES" in avg and "SQ_WAVE_CYCLES" in avg:
            o["wave_cycles_per_busy"] = round(avg["SQ_WAVE_CYCLES"] / avg["SQ_BUSY_CYCLES"], 2)
    out[v] = o
print(json.dumps(out, indent=1))
