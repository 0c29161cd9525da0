#!/usr/bin/env python3
"""Summarise scripts/pmc_variants.sh output: per variant, stencil kernel mean duration and the
per-launch mean of every SQ/GRBM counter, plus derived ratios."""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

out = Path(sys.argv[1])
res = {}
for vdir in sorted(p for p in out.iterdir() if p.is_dir()):
    r = {}
    for f in glob.glob(str(vdir / "trace" / "**" / "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "gol_stencil" in row["Name"]:
                r["stencil_avg_us"] = float(row["AverageNs"]) / 1e3
                r["stencil_calls"] = int(row["Calls"])
    acc = defaultdict(list)
    for f in glob.glob(str(vdir / "p*" / "**" / "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "gol_stencil" in row["Kernel_Name"]:
                acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
                r["vgpr"] = int(row["VGPR_Count"])
    for k, v in acc.items():
        r[k] = sum(v) / len(v)
    if "SQ_INSTS_VALU" in r and "SQ_WAVES" in r:
        r["valu_per_wave"] = r["SQ_INSTS_VALU"] / r["SQ_WAVES"]
    if "SQ_BUSY_CYCLES" in r and "SQ_ACTIVE_INST_VALU" in r:
        r["valu_active_frac_of_wave_cycles"] = r["SQ_ACTIVE_INST_VALU"] / max(r.get("SQ_WAVE_CYCLES", 1), 1)
    res[vdir.name] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}
print(json.dumps(res, indent=1))
