#!/usr/bin/env python3
"""Per-kernel VGPRs / spills / occupancy from a -Rpass-analysis=kernel-resource-usage log, with the
gol_stencil template arguments decoded (K, COUNT, SKEW, D, PF, HH, DR, ZIP, FILLU)."""
import re
import sys

NAMES = ["K", "COUNT", "SKEW", "D", "PF", "HH", "DR", "ZIP", "FILLU", "LD"]
txt = open(sys.argv[1]).read()
for b in re.split(r"remark: Function Name: ", txt)[1:]:
    name = b.split()[0]
    m = re.search(r"gol_stencilI(.*?)EEEv", name)
    if not m:
        continue
    args = re.findall(r"L([ib])(\d+)E?", m.group(1))
    desc = " ".join(f"{n}={v}" for n, (_, v) in zip(NAMES, args))
    g = lambda k: (re.search(k + r": (\S+)", b) or [None, "?"])[1]
    vg, sp = g("VGPRs"), g("VGPRs Spill")
    sc, oc = g(r"ScratchSize \[bytes/lane\]"), g(r"Occupancy \[waves/SIMD\]")
    print(f"{desc:60s} VGPR {vg:>4} spill {sp:>3} scratch {sc:>4} occ {oc}")
