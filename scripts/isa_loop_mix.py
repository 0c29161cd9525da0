#!/usr/bin/env python3
"""Instruction mix of a kernel's steady loop from `make asm` output (hipcc -S, gfx950).

Finds the kernel whose (demangled-ish) symbol contains every given substring, takes its loop
bodies (a label L ... a backward branch to L) and prints, for the largest loop, the count of
each instruction class per loop iteration: v_bitop3, v_alignbit, DPP moves, v_bcnt, other VALU,
SALU, LDS, VMEM (buffer/global), s_waitcnt, s_nop.
Usage: isa_loop_mix.py <file.s> <symbol substring> [...]"""
import re
import sys
from collections import Counter

path, subs = sys.argv[1], sys.argv[2:]
lines = open(path).read().splitlines()
# kernel bodies: "<sym>:" ... ".Lfunc_end"
kernels, cur, name = {}, None, None
for ln in lines:
    m = re.match(r"^(_Z\S+):\s*(;.*)?$", ln)
    if m:
        name, cur = m.group(1), []
        kernels[name] = cur
        continue
    if name and ln.startswith(".Lfunc_end"):
        name = None
        continue
    if name is not None:
        cur.append(ln)
cands = [k for k in kernels if all(s in k for s in subs)]
if not cands:
    sys.exit(f"no kernel matches {subs}")
for k in cands:
    body = kernels[k]
    labels = {ln.split(":")[0]: i for i, ln in enumerate(body) if re.match(r"^\.LBB\w+:", ln)}
    loops = []
    for i, ln in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", ln)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i:
                loops.append((i - labels[tgt], labels[tgt], i))
    if not loops:
        continue
    loops.sort(reverse=True)
    n, a, b = loops[0]
    mix = Counter()
    for ln in body[a:b + 1]:
        t = ln.strip().split()
        if not t or t[0].startswith((";", ".", "//")):
            continue
        op = t[0]
        if op.startswith("v_bitop3"):
            mix["v_bitop3"] += 1
        elif op.startswith("v_alignbit"):
            mix["v_alignbit"] += 1
        elif "dpp" in ln or op.startswith("v_mov_b32_dpp"):
            mix["dpp"] += 1
        elif op.startswith("v_bcnt"):
            mix["v_bcnt"] += 1
        elif op.startswith("v_"):
            mix["valu_other:" + op] += 1
        elif op.startswith("s_waitcnt"):
            mix["s_waitcnt"] += 1
        elif op.startswith("s_nop"):
            mix["s_nop"] += 1
        elif op.startswith("s_"):
            mix["salu"] += 1
        elif op.startswith("ds_"):
            mix["lds:" + op] += 1
        elif op.startswith(("buffer_", "global_")):
            mix["vmem:" + op] += 1
        else:
            mix["other:" + op] += 1
    valu = sum(v for kk, v in mix.items() if kk in ("v_bitop3", "v_alignbit", "dpp", "v_bcnt") or kk.startswith("valu_other"))
    print(f"{k}\n  largest loop: {n} lines (body lines {a}..{b}); VALU {valu}")
    for kk, v in sorted(mix.items(), key=lambda x: -x[1]):
        print(f"    {kk:40s} {v}")
