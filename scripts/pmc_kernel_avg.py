#!/usr/bin/env python3
"""Per-dispatch averages of rocprofv3 --pmc counters for the kernels matching a pattern, from one or
more --output-format csv directories (one pass each), plus derived shares of the wave cycles
(MI355X_MICROARCH.md: SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~ SQ_WAVE_CYCLES, all in
quad-cycles) and the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration).
Usage: pmc_kernel_avg.py <pattern> <dir> [<dir> ...]"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

pat = re.compile(sys.argv[1])
vals = defaultdict(list)
durs = defaultdict(list)
name_of = {}
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if not pat.search(r["Kernel_Name"]):
                continue
            key = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void golhip::(anonymous namespace)::", "")
            name_of[key] = r["Kernel_Name"]
            vals[(key, r["Counter_Name"])].append(float(r["Counter_Value"]))
            durs[(key, r["Counter_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {}
for (k, c), v in sorted(vals.items()):
    e = out.setdefault(k, {})
    e[c] = sum(v) / len(v)
    e.setdefault("dispatches", len(v))
    if c == "GRBM_GUI_ACTIVE":
        dur = sum(durs[(k, c)]) / len(durs[(k, c)])
        e["duration_us_pmc_pass"] = round(dur / 1e3, 3)
        e["clock_ghz"] = round(e[c] / 8 / dur, 3)
for k, e in out.items():
    wc = e.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_WAIT_INST_LDS"):
            if c in e:
                e[f"{c}_share_of_wave_cycles"] = round(e[c] / wc, 4)
    if e.get("SQ_INSTS_VALU") and e.get("SQ_WAVES"):
        e["valu_per_wave"] = round(e["SQ_INSTS_VALU"] / e["SQ_WAVES"], 1)
print(json.dumps(out, indent=1))
