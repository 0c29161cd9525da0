#!/usr/bin/env python3
"""Per-dispatch averages of rocprofv3 --pmc counters for the kernels matching a pattern, from one or
more --output-format csv directories (one pass each), plus derived shares of the wave cycles
(MI355X_MICROARCH.md: SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~ SQ_WAVE_CYCLES, all in
quad-cycles) and the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration).

Kernels are keyed by their FULL template name (namespaces dropped, the argument list cut at the
parenthesis that closes the template, so "(anonymous namespace)" and template arguments survive):
gol_slab<16, 12, 8, 2, true, false> and count_finalize never share a key.

The effective clock is only reported where it can be read: the GRBM_GUI_ACTIVE quotient reads high
on dispatches shorter than about 0.3 ms (MI355X_MICROARCH.md "DVFS give-back"), so for shorter
dispatches, or any quotient above the 2.4 GHz peak, clock_ghz is null and clock_ghz_raw keeps the
quotient with the reason.
Usage: pmc_kernel_avg.py <pattern> <dir> [<dir> ...]"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

PEAK_GHZ = 2.4
MIN_CLOCK_DISPATCH_US = 300.0


def kernel_key(name: str) -> str:
    """'void golhip::(anonymous namespace)::gol_slab<16, 12, 8, 2, true, false>(unsigned int
    const*, ...)' -> 'gol_slab<16, 12, 8, 2, true, false>'."""
    n = name.strip()
    if n.startswith("void "):
        n = n[5:]
    n = n.replace("(anonymous namespace)::", "")
    depth = 0
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            n = n[:i]
            break
    return re.sub(r"^(\w+::)+", "", n)


def main(argv):
    pat = re.compile(argv[1])
    vals = defaultdict(list)
    durs = defaultdict(list)
    for d in argv[2:]:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if not pat.search(r["Kernel_Name"]):
                    continue
                key = kernel_key(r["Kernel_Name"])
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
            q = e[c] / 8 / dur
            if q > PEAK_GHZ or dur / 1e3 < MIN_CLOCK_DISPATCH_US:
                e["clock_ghz"] = None
                e["clock_ghz_raw"] = round(q, 3)
                e["clock_note"] = (f"GRBM_GUI_ACTIVE/8/duration = {q:.3f} GHz not used: "
                                   + ("above the 2.4 GHz peak" if q > PEAK_GHZ else
                                      f"dispatch {dur / 1e3:.1f} us < {MIN_CLOCK_DISPATCH_US:.0f} us"))
            else:
                e["clock_ghz"] = round(q, 3)
    for k, e in out.items():
        wc = e.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_WAIT_INST_LDS"):
                if c in e:
                    e[f"{c}_share_of_wave_cycles"] = round(e[c] / wc, 4)
        if e.get("SQ_INSTS_VALU") and e.get("SQ_WAVES"):
            e["valu_per_wave"] = round(e["SQ_INSTS_VALU"] / e["SQ_WAVES"], 1)
    return out


if __name__ == "__main__":
    print(json.dumps(main(sys.argv), indent=1))
