#!/usr/bin/env python3
"""Build-time guard of the hand-counted vmcnt waits in the LDS-DMA stencils.

gol_stencil (PF = 1) and gol_stencil_split keep their input rows in an LDS ring filled by LDS-DMA
(buffer_load ... lds / global_load_lds).  The compiler does not order those DMAs with the ring's
ds_reads, so each step waits by hand with `s_waitcnt vmcnt(N)`, where N assumes the wave issued a
fixed number of DMAs and stores after the row it is about to read (golhip_stencil.hpp: kWait,
kWait2, the split kernel's PL - 4).  If the compiler emits FEWER vector-memory ops between those
waits than the formula assumed (a store merged or sunk past a wait, a DMA hoisted), vmcnt(N)
returns while the step's row is still in flight and the step reads a stale slot -- silently.

For every such kernel in the given objects this script:
  * models the wave's vmcnt counter in program order (the steady loop unrolled twice: entered from
    the unrolled fill and from its own back edge; every VMEM op counted, compiler waits applied)
    and fails if any hand wait leaves a DMA of the row its step reads outstanding;
  * fails a PRODUCTION kernel (the kVariantProd family, LD or not, and the level-split kernel) that
    uses scratch memory (private segment > 0, scratch_* instructions): a spill in the hot kernel
    puts scratch traffic into the ring's vmcnt stream and costs HBM round trips per step.  Spills
    of experimental variants (GOLHIP_VARIANT) and register-to-register spills (VGPR -> AGPR,
    SGPR -> VGPR lanes) are reported, not failed.

Usage: check_vmcnt.py [--expect-fail | --scratch-only] OBJ...   exit 0 = every kernel passes.
--scratch-only: only the scratch/spill check, on every kernel of the objects (register kernels).
--expect-fail inverts the result: exit 0 only if some kernel FAILS (the Makefile's self-test on guard_selftest.o, the
production K = 16 kernel forced to 8 waves per SIMD, which spills).
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

LLVM = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / "lib" / "llvm" / "bin"
STENCIL_ARGS = ["K", "COUNT", "SKEW", "D", "PF", "HH", "DR", "ZIP", "FILLU", "LD", "WPE", "PRE", "MASK"]
DEFAULTS = {"DR": 0, "ZIP": 1, "FILLU": 1, "LD": 0, "WPE": 0, "PRE": 0, "MASK": 0}
VMEM = re.compile(r"^(buffer_|global_|scratch_|flat_)")


def device_object(obj: Path, tmp: Path) -> Path:
    """Extract the gfx950 code object of a HIP object file: its .hip_fatbin section, unbundled by
    clang-offload-bundler (which also inflates the compressed bundles --offload-compress writes;
    llvm-objdump --offloading hands those out still compressed)."""
    fat = tmp / (obj.name + ".fatbin")
    subprocess.run([str(LLVM / "llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", str(obj), os.devnull],
                   check=True, capture_output=True)
    co = tmp / (obj.name + ".gfx950.co")
    r = subprocess.run([str(LLVM / "clang-offload-bundler"), "--type=o", "--unbundle",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"],
                       capture_output=True, text=True)
    if r.returncode != 0 or not co.exists() or co.stat().st_size == 0:
        raise SystemExit(f"{obj}: no gfx950 code object ({r.stderr.strip()})")
    return co


def kernel_metadata(co: Path) -> dict[str, dict[str, int]]:
    notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], check=True,
                           capture_output=True, text=True).stdout
    meta, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            cur = meta.setdefault(m.group(1), {})
            continue
        m = re.match(r"\s+\.(private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count):\s+(\d+)", line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return meta


def kernel_code(co: Path) -> dict[str, list[tuple[int, str, int | None]]]:
    """Per kernel: (address, instruction, branch target address or None)."""
    dis = subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", str(co)],
                         check=True, capture_output=True, text=True).stdout
    funcs, cur, base = {}, None, 0
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(\S+)>:$", line)
        if m:
            base, cur = int(m.group(1), 16), funcs.setdefault(m.group(2), [])
            continue
        s = line.strip()
        if cur is None or not s or s.startswith(";"):
            continue
        addr = re.search(r"//\s*([0-9A-Fa-f]+):", s)
        tgt = re.search(r"<[^>+]+\+0x([0-9a-f]+)>", s)
        cur.append((int(addr.group(1), 16) if addr else -1, s.split(";")[0].split("//")[0].strip(),
                    base + int(tgt.group(1), 16) if tgt and s.startswith("s_") and "branch" in s else None))
    return funcs


def stencil_args(name: str) -> dict[str, int] | None:
    m = re.search(r"gol_stencilI(.*?)EEEv", name)
    if not m:
        return None
    vals = [int(v) for _, v in re.findall(r"L([ib])(\d+)E?", m.group(1))]
    args = dict(DEFAULTS)
    args.update(dict(zip(STENCIL_ARGS, vals)))
    return args


def expected_schedule(a: dict[str, int]) -> tuple[int, int, int]:
    """(hand wait immediate, DMAs per row, rows per hand wait) of an LDS-DMA gol_stencil, as
    golhip_stencil.hpp derives them (NSTORE, PL, kWait / kWait2)."""
    nstore = (3 if a["HH"] else 1) * (2 if a["LD"] else 1)
    d = a["D"] + a["PRE"]  # PRE: the row's DMA and the single-lane 65th-word DMA
    pl = 16 if (a["K"] <= 2 and nstore + (d + nstore) * 14 - 2 <= 63) else 8
    if a["ZIP"] == 2:
        return 2 * nstore + (2 + 2 * nstore) * (pl // 2 - 2) - 2, d, 2
    return nstore + (d + nstore) * (pl - 2) - 2, d, 1


def is_production(a: dict[str, int]) -> bool:
    """kVariantProd at depth K (golhip_internal.hpp prod_pre / golhip_stencil.hpp): drifting sums,
    one-word lanes, LDS-DMA ring, unrolled fill, whole-word chunks; pre-shifted rows (PRE) at
    K = 16.  The pre-shifted geometry at other depths (kVariantPre63) is held to the same bar.
    Any register budget (WPE) counts: the self-test is the K = 16 kernel forced to spill."""
    return (a["SKEW"] == 0 and a["D"] == 1 and a["PF"] == 1 and a["DR"] == 1 and a["ZIP"] == 1
            and a["FILLU"] == 1 and a["HH"] == 0 and (a["PRE"] == 1 or a["K"] != 16))


def is_dma(ins: str) -> bool:
    """An LDS-DMA: global_load_lds_* or a buffer load with the trailing `lds` operand."""
    return ins.startswith("global_load_lds") or (ins.startswith("buffer_load") and ins.endswith(" lds"))


def vmcnt(ins: str) -> int | None:
    m = re.match(r"s_waitcnt\b.*vmcnt\((\d+)\)", ins)
    return int(m.group(1)) if m else None


LINEARIZE_NOTES: list[str] = []


def linearize(code, hand: set[int]) -> list[int]:
    """Program order with the innermost loop that holds a hand wait unrolled twice (the steady
    loop: its first iteration is entered from the unrolled fill, the second from its own
    back edge).  Other branches are ignored: the ring code is branch-free by construction."""
    index = {a: i for i, (a, _, _) in enumerate(code)}
    best = None
    for i, (a, ins, t) in enumerate(code):
        # s_cbranch_execz skips a lane-masked region when no lane is active.  A BACKWARD execz is
        # skipped only when the fall-through path reaches the same target too (a later branch back
        # to it closes the loop, so the execz is an early exit of a region inside it, never the
        # steady loop's own back edge); otherwise it is kept as a back-edge candidate and reported
        # (LINEARIZE_NOTES), so the guard cannot silently pick a different loop.  The ring code
        # itself has no masked regions since PRE's 65th word became a whole-wave DMA; the
        # prodmask variant's `if (live)` around the whole ring is a FORWARD execz.
        if ins.startswith("s_cbranch_execz"):
            if t is None or t >= a:
                continue
            if any(t2 == t for _, _, t2 in code[i + 1:]):
                continue
            LINEARIZE_NOTES.append(f"backward s_cbranch_execz at {a:#x} -> {t:#x} with no later "
                                   "back edge to its target: kept as a loop back edge")
        if t is not None and t < a and t in index:
            lo = index[t]
            if any(lo <= h <= i for h in hand) and (best is None or i - lo < best[1] - best[0]):
                best = (lo, i)
    order = list(range(len(code)))
    if best:
        lo, hi = best
        order = order[:hi + 1] + order[lo:hi + 1] + order[hi + 1:]
    return order


def simulate(code, wait: int, dmas_per_row: int, rows_per_wait: int, split: bool) -> list[str]:
    """In-order vmcnt model of one wave.  The n-th hand wait must leave none of the DMAs of rows
    [Z n, Z n + Z) outstanding (Z = rows_per_wait): the row DMA'd n-th is read by the n-th step.
    Every VMEM op counts; compiler vmcnt waits are applied too (they only ever wait longer).
    Split kernel: only wave 0 issues DMAs, and the other waves' code is laid out in between, so
    only DMAs and the hand waits are modelled (fewer ops in flight: conservative)."""
    ins = [c[1] for c in code]
    if split:
        hand = {i for i, x in enumerate(ins) if vmcnt(x) == wait}
    else:
        hand = {i for i, x in enumerate(ins[:-1]) if vmcnt(x) == wait and ins[i + 1] == "s_waitcnt lgkmcnt(0)"}
    if not hand:
        return [f"no hand-counted s_waitcnt vmcnt({wait})"]
    errs, out, ndma, nwait = [], [], 0, 0
    for i in linearize(code, hand):
        x = ins[i]
        if is_dma(x):
            out.append(ndma // dmas_per_row)
            ndma += 1
        elif VMEM.match(x):
            if not split:
                out.append(None)
        elif (n := vmcnt(x)) is not None and (i in hand or not split):
            out = out[len(out) - n:] if n < len(out) else out
            if i in hand:
                need = rows_per_wait * (nwait + 1) - 1
                late = sorted({r for r in out if r is not None and r <= need})
                if late:
                    errs.append(f"hand wait #{nwait} (vmcnt({n}) at {code[i][0]:#x}) leaves row(s) "
                                f"{late} of its step in flight")
                    if len(errs) > 4:
                        break
                nwait += 1
    return errs


def check_object(obj: Path) -> tuple[int, list, list]:
    failures, notes, checked = [], [], 0
    with tempfile.TemporaryDirectory() as td:
        co = device_object(obj, Path(td))
        meta, code = kernel_metadata(co), kernel_code(co)
    for name, ins in code.items():
        a = stencil_args(name)
        split = "gol_stencil_split" in name
        if not split and (a is None or a["PF"] != 1):
            continue
        checked += 1
        prod = split or is_production(a)
        md = meta.get(name, {})
        scratch = [f"{k} = {md[k]}" for k in ("private_segment_fixed_size",) if md.get(k, 0)]
        if any(c[1].startswith("scratch_") for c in ins):
            scratch.append("scratch instructions present")
        regs = [f"{k} = {md[k]}" for k in ("vgpr_spill_count", "sgpr_spill_count") if md.get(k, 0)]
        if split:  # wave 0: one DMA per row, s_waitcnt vmcnt(PL - 4), PL = 8
            errs = simulate(ins, 4, 1, 1, split=True)
        else:
            errs = simulate(ins, *expected_schedule(a), split=False)
        if prod:
            errs += scratch
        elif scratch:
            notes.append((obj.name, name, scratch + regs))
        if errs:
            failures.append((obj.name, name, errs + regs))
        elif regs and prod:
            notes.append((obj.name, name, regs))
    return checked, failures, notes


def check_scratch_only(obj: Path) -> tuple[int, list, list]:
    """Register kernels (gol_tile / gol_slab in stencil_tile.o: rows + chains held in VGPRs, no
    LDS-DMA ring): every kernel must be scratch-free -- a spill there goes unnoticed otherwise."""
    failures = []
    with tempfile.TemporaryDirectory() as td:
        co = device_object(obj, Path(td))
        meta, code = kernel_metadata(co), kernel_code(co)
    for name, ins in code.items():
        md = meta.get(name, {})
        errs = [f"{k} = {md[k]}" for k in ("private_segment_fixed_size", "vgpr_spill_count",
                                            "sgpr_spill_count") if md.get(k, 0)]
        if any(c[1].startswith("scratch_") for c in ins):
            errs.append("scratch instructions present")
        if errs:
            failures.append((obj.name, name, errs))
    return len(code), failures, []


def main() -> int:
    args = sys.argv[1:]
    expect_fail = "--expect-fail" in args
    objs = [Path(a) for a in args if not a.startswith("--")]
    if "--scratch-only" in args:
        results = [check_scratch_only(o) for o in objs]
        checked = sum(r[0] for r in results)
        failures = [f for r in results for f in r[1]]
        for obj, name, errs in failures:
            print(f"FAIL {obj} {name}: {'; '.join(errs)}")
        print(f"check_vmcnt --scratch-only: {checked} kernels checked, {len(failures)} use scratch")
        return 1 if failures or checked == 0 else 0
    with ThreadPoolExecutor(max_workers=min(8, len(objs) or 1)) as pool:
        results = list(pool.map(check_object, objs))
    checked = sum(r[0] for r in results)
    failures = [f for r in results for f in r[1]]
    for obj, name, msgs in (n for r in results for n in r[2]):
        print(f"note {obj} {name}: {'; '.join(msgs)}")
    for obj, name, errs in failures:
        print(f"FAIL {obj} {name}")
        for e in errs:
            print(f"     {e}")
    for n in sorted(set(LINEARIZE_NOTES)):
        print(f"warn: {n}")
    print(f"check_vmcnt: {checked} LDS-DMA kernels checked, {len(failures)} failed")
    if expect_fail:
        if failures:
            print("check_vmcnt: the deliberately spilling self-test is rejected, as it must be")
            return 0
        print("check_vmcnt: the self-test was NOT rejected -- the guard is broken")
        return 1
    return 1 if failures or checked == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
