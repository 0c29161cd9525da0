#!/usr/bin/env python3
"""Every loop (label ... backward branch) of one kernel in a `hipcc -S` gfx950 listing, with its
instruction mix: VALU (bitop3 / alignbit / DPP / bcnt / other), SALU, LDS, VMEM.
Usage: isa_loops.py <file.s> <symbol prefix>"""
import re
import sys
from collections import Counter

lines = open(sys.argv[1]).read().splitlines()
i0 = next(i for i, ln in enumerate(lines) if ln.startswith(sys.argv[2]) and re.match(r"^\S+:", ln))
body = []
for ln in lines[i0 + 1:]:
    if ln.startswith(".Lfunc_end"):
        break
    body.append(ln)
labels = {ln.split(":")[0]: i for i, ln in enumerate(body) if re.match(r"^\.LBB\w+:", ln)}
print(lines[i0].split(":")[0])
for i, ln in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", ln)
    if not m:
        continue
    t = m.group(1) or m.group(2)
    if t not in labels or labels[t] >= i:
        continue
    a = labels[t]
    ops = [x.strip().split()[0] for x in body[a:i + 1] if x.strip() and not x.strip().startswith((";", "."))]
    cnt = Counter()
    for o in ops:
        if o.startswith("v_bitop3"): cnt["bitop3"] += 1
        elif o.startswith("v_alignbit"): cnt["alignbit"] += 1
        elif o.startswith("v_mov_b32_dpp") or "dpp" in o: cnt["dpp"] += 1
        elif o.startswith("v_bcnt"): cnt["bcnt"] += 1
        elif o.startswith("v_"): cnt["valu_other"] += 1
        elif o.startswith(("s_waitcnt", "s_nop", "s_barrier")): cnt[o] += 1
        elif o.startswith("s_"): cnt["salu"] += 1
        elif o.startswith("ds_"): cnt["lds"] += 1
        elif o.startswith(("buffer_", "global_")): cnt["vmem"] += 1
    valu = sum(cnt[k] for k in ("bitop3", "alignbit", "dpp", "bcnt", "valu_other"))
    print(f"  loop {t} (lines {a}-{i}): VALU {valu} {dict(cnt)}")
