#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs of scripts/pmc_passes.sh into per-launch numbers.

HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE under-counts wide streaming reads by 2x and other widths are uncalibrated, so the read
and write scales are CALIBRATED here on two kernels of known traffic that use the stencil's own
access width (4-byte lanes): popcount_rows reads exactly the board once, init_random_rows writes
exactly the board once.
valu_instr_per_launch: SQ_INSTS_VALU of one stencil dispatch (wave64 instructions issued);
clock_ghz: GRBM_GUI_ACTIVE / 8 / the dispatch duration of the same pass's --kernel-trace.
Usage: pmc_summary.py <pmc dir> <k> <board bytes> [<json out> <key>]
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(d):
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def short_name(name):
    return ("stencil" if ("gol_stencil" in name or "gol_step1" in name) else "popcount" if "popcount_rows" in name
            else "init" if "init_random" in name else None)


def grbm_clock(d):
    """Effective clock of the timed stencil dispatches (largest grid): GRBM_GUI_ACTIVE (summed
    over the 8 XCDs) / 8 / the dispatch's duration (MI355X_MICROARCH.md, DVFS give-back)."""
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        rows = [r for r in csv.DictReader(open(f))
                if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and short_name(r.get("Kernel_Name", "")) == "stencil"]
        if not rows:
            continue
        big = max(int(r["Grid_Size"]) for r in rows)
        ghz, durs = [], []
        for r in rows:
            if int(r["Grid_Size"]) != big:
                continue
            ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            durs.append(ns)
            ghz.append(float(r["Counter_Value"]) / 8 / ns)
        if ghz:
            return sum(ghz) / len(ghz), sum(durs) / len(durs)
    return None, None


def main():
    d, k, board = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values per dispatch
    rows = load(d)
    # the timed stencil launches only: the largest grid (the engine also launches every depth's
    # kernel once, empty, to load its code object at create)
    big = max((int(r["Grid_Size"]) for r in rows if short_name(r.get("Kernel_Name", "")) == "stencil"), default=0)
    for r in rows:
        short = short_name(r.get("Kernel_Name", ""))
        if short == "stencil" and int(r["Grid_Size"]) != big:
            continue
        if short:
            per[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {kn: {c: sum(v) / len(v) for c, v in cs.items()} for kn, cs in per.items()}
    out = {"k": k, "board_bytes": board, "avg_per_dispatch": avg}
    try:
        rscale = board / (avg["popcount"]["FETCH_SIZE"] * 1024)
        wscale = board / (avg["init"]["WRITE_SIZE"] * 1024)
        fetch = avg["stencil"]["FETCH_SIZE"] * 1024 * rscale
        write = avg["stencil"]["WRITE_SIZE"] * 1024 * wscale
        out.update({"read_scale": rscale, "write_scale": wscale,
                    "stencil_read_bytes": fetch, "stencil_write_bytes": write,
                    "hbm_bytes_per_launch": fetch + write,
                    "algorithmic_bytes_per_launch": 0.25 * board * 8 * k})
    except KeyError as e:
        out["error"] = f"missing {e}"
    st = avg.get("stencil", {})
    if "SQ_INSTS_VALU" in st:
        out["valu_instr_per_launch"] = st["SQ_INSTS_VALU"]
    clock, dur = grbm_clock(d)
    if clock:
        out["clock_ghz"] = round(clock, 3)
        out["kernel_trace_avg_ns_grbm_pass"] = round(dur)
    if "SQ_LDS_BANK_CONFLICT" in st and st.get("SQ_LDS_IDX_ACTIVE"):
        # extra LDS cycles from bank conflicts over all LDS-array cycles (MI355X_MICROARCH.md)
        out["lds_bank_conflict_cycles"] = st["SQ_LDS_BANK_CONFLICT"]
        out["lds_active_cycles"] = st["SQ_LDS_IDX_ACTIVE"]
        out["lds_bank_conflict_frac"] = st["SQ_LDS_BANK_CONFLICT"] / st["SQ_LDS_IDX_ACTIVE"]
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 5:
        try:
            allj = json.load(open(sys.argv[4]))
        except Exception:
            allj = {}
        allj[sys.argv[5]] = out
        json.dump(allj, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
