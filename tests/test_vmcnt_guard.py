"""The build-time vmcnt guard (scripts/check_vmcnt.py) on synthetic schedules and on the built
code objects: a correct ring schedule passes, a schedule that issues fewer VMEM ops than the hand
wait assumes fails, and the deliberately spilling self-test object is rejected."""
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "distributed-gol_amd" / "lib"
sys.path.insert(0, str(ROOT / "scripts"))
import check_vmcnt as cv  # noqa: E402


def ring_kernel(K=16, HH=1, LD=0, D=1, nstore=None, wait=None, steady_steps=8, PRE=0):
    """A synthetic LDS-DMA stencil as the disassembler shows it: PL-1 prologue rows (DMA +
    dummy stores), 2K fill steps, a PL-step steady loop with a back edge, then the drain.
    PRE: two DMAs per row (the row and the row one word east)."""
    args = dict(K=K, COUNT=0, SKEW=0, D=D, PF=1, HH=HH, DR=1, ZIP=1, FILLU=1, LD=LD, WPE=0, PRE=PRE)
    w, dmas, _ = cv.expected_schedule(args)
    ns = nstore if nstore is not None else (3 if HH else 1) * (2 if LD else 1)
    code, addr = [], 0x1000

    def emit(ins, tgt=None):
        nonlocal addr
        code.append((addr, ins, tgt))
        addr += 8

    def row():
        for _ in range(D + PRE):
            emit("buffer_load_dword v3, s[0:3], 0 offen lds")

    def stores():
        for _ in range(ns):
            emit("buffer_store_dword v5, v6, s[8:11], 0 offen")

    def step():
        emit(f"s_waitcnt vmcnt({wait if wait is not None else w})")
        emit("s_waitcnt lgkmcnt(0)")
        row()
        emit("ds_read_b32 v7, v8")
        emit("v_bitop3_b32 v9, v10, v11, v12 bitop3:0x96")
        stores()

    pl = 16 if (K <= 2 and ns + (dmas + ns) * 14 - 2 <= 63) else 8  # the kernel's ring depth
    for _ in range(pl - 1):
        row()
        stores()
    for _ in range((2 * K + pl - 1) // pl * pl):
        step()
    top = addr
    for _ in range(max(steady_steps, pl)):
        step()
    emit("s_cmp_lt_i32 s4, s5")
    emit("s_cbranch_scc1 65000", top)
    emit("s_waitcnt vmcnt(0)")
    emit("s_endpgm")
    return code, (w, dmas, 1)


@pytest.mark.parametrize("K,HH,LD,PRE", [(16, 1, 0, 0), (16, 1, 1, 0), (8, 0, 0, 0), (12, 0, 1, 0),
                                         (16, 0, 0, 1), (16, 0, 1, 1), (2, 0, 0, 1)])
def test_correct_schedule_passes(K, HH, LD, PRE):
    code, sched = ring_kernel(K=K, HH=HH, LD=LD, PRE=PRE)
    assert cv.simulate(code, *sched, split=False) == []


def test_pre_wait_without_its_second_dma_fails():
    # a pre-shifted kernel whose hand wait counts two DMAs per row while the code issues one (the
    # second DMA merged away or hoisted out of the step): the wait is too loose for its row
    _, (w_pre, d_pre, _) = ring_kernel(K=16, HH=0, PRE=1)
    assert d_pre == 2
    code, (w, d, z) = ring_kernel(K=16, HH=0, PRE=0, wait=w_pre)
    assert w_pre > w and d == 1
    assert cv.simulate(code, w_pre, d, z, split=False)


def test_masked_region_skip_is_not_a_back_edge():
    # a lane-masked region at the end of the steady loop, closed by an execz skip to the loop top
    # (what the compiler emitted for a lane-0-only DMA): the model follows the fall-through path
    code, sched = ring_kernel(K=8, HH=0)
    top = next(a for a, ins, _ in code if ins.startswith("s_waitcnt vmcnt(") and ins != "s_waitcnt vmcnt(0)")
    i = next(i for i, c in enumerate(code) if c[1].startswith("s_cbranch_scc1"))
    code.insert(i, (code[i][0] - 4, "s_cbranch_execz 65000", top))
    assert cv.simulate(code, *sched, split=False) == []


def test_fewer_stores_than_counted_fails():
    # three half-word stores merged into one: the hand wait no longer covers its row
    code, sched = ring_kernel(K=16, HH=1, nstore=1)
    errs = cv.simulate(code, *sched, split=False)
    assert errs and "in flight" in errs[0]


def test_wait_too_loose_fails():
    code, (w, d, z) = ring_kernel(K=8, HH=0, wait=None)
    code_loose, _ = ring_kernel(K=8, HH=0, wait=w + 3)
    assert cv.simulate(code, w, d, z, split=False) == []
    assert cv.simulate(code_loose, w + 3, d, z, split=False)


def test_extra_compiler_wait_is_accepted():
    # a compiler vmcnt(0) before a step only waits longer: still correct
    code, sched = ring_kernel(K=8, HH=0, nstore=0)
    assert cv.simulate(code, *sched, split=False)
    patched = []
    for c in code:
        if c[1].startswith("s_waitcnt vmcnt(") and c[1] != "s_waitcnt vmcnt(0)":
            patched.append((c[0] - 4, "s_waitcnt vmcnt(0)", None))
        patched.append(c)
    assert cv.simulate(patched, *sched, split=False) == []


def test_missing_hand_wait_fails():
    code, (w, d, z) = ring_kernel(K=8, HH=0)
    assert cv.simulate(code, w + 1, d, z, split=False) == [f"no hand-counted s_waitcnt vmcnt({w + 1})"]


def test_production_classification():
    base = dict(COUNT=0, SKEW=0, D=1, PF=1, DR=1, ZIP=1, FILLU=1, LD=0, WPE=0, PRE=0)
    assert cv.is_production(dict(base, K=16, HH=0, PRE=1))
    assert cv.is_production(dict(base, K=8, HH=0, LD=1))
    assert cv.is_production(dict(base, K=12, HH=0, PRE=1))     # pre63 at K = 12: same bar
    assert not cv.is_production(dict(base, K=16, HH=0))        # drift62 at K = 16: experiment
    assert not cv.is_production(dict(base, K=16, HH=1))        # half-word halo: superseded
    assert cv.is_production(dict(base, K=16, HH=0, PRE=1, WPE=8))  # the self-test: production, spilling
    assert not cv.is_production(dict(base, K=8, HH=0, ZIP=2))


def test_mangled_template_arguments():
    name = ("_ZN6golhip12_GLOBAL__N_111gol_stencilILi16ELb0ELb0ELi1ELi1ELb0ELb1ELi1ELb1ELb0ELi0ELb1EEEvPKjPjNS_"
            "13StencilParamsEPy")
    a = cv.stencil_args(name)
    assert (a["K"], a["HH"], a["DR"], a["LD"], a["WPE"], a["PRE"]) == (16, 0, 1, 0, 0, 1)
    assert cv.is_production(a)
    old = ("_ZN6golhip12_GLOBAL__N_111gol_stencilILi16ELb0ELb0ELi1ELi1ELb1ELb1ELi1ELb1ELb0ELi0EEEvPKjPjNS_"
           "13StencilParamsEPy")  # a name without the trailing PRE argument: PRE defaults to 0
    assert cv.stencil_args(old)["PRE"] == 0


needs_objs = pytest.mark.skipif(not (LIB / "guard_selftest.o").exists() or not (LIB / "stencil_k16.o").exists(),
                                reason="device objects not built (make -C distributed-gol_amd)")


@needs_objs
def test_spilling_selftest_is_rejected():
    r = subprocess.run([sys.executable, str(ROOT / "scripts" / "check_vmcnt.py"), "--expect-fail",
                        str(LIB / "guard_selftest.o")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "scratch" in r.stdout
    # and without --expect-fail the same object fails the build
    r = subprocess.run([sys.executable, str(ROOT / "scripts" / "check_vmcnt.py"),
                        str(LIB / "guard_selftest.o")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 1


@needs_objs
def test_production_k16_object_passes():
    r = subprocess.run([sys.executable, str(ROOT / "scripts" / "check_vmcnt.py"), str(LIB / "stencil_k16.o")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    assert ", 0 failed" in r.stdout


def test_backward_execz_is_skipped_only_when_the_loop_closes_elsewhere():
    """A backward s_cbranch_execz to the steady loop's top is an early exit inside the loop when a
    later branch closes the loop; with no such branch it is kept as the back edge and warned about
    (advice r03: skipping every execz could pick the wrong loop)."""
    code, _ = ring_kernel(K=8, HH=0)
    top = next(t for _, ins, t in code if ins.startswith("s_cbranch_scc1"))
    hand = {i for i, (_, ins, _) in enumerate(code) if cv.vmcnt(ins) not in (None, 0)}
    base = cv.linearize(code, hand)
    # an execz inside the loop, jumping back to its top; the scc1 back edge still closes the loop
    i_exec = next(i for i, (a, ins, t) in enumerate(code) if a > top and ins.startswith("ds_read"))
    a_exec = code[i_exec][0]
    with_inner = code[:i_exec] + [(a_exec, "s_cbranch_execz 65001", top)] + code[i_exec + 1:]
    cv.LINEARIZE_NOTES.clear()
    assert cv.linearize(with_inner, hand) == base
    assert cv.LINEARIZE_NOTES == []
    # the loop closed ONLY by a backward execz (no scc1 back edge): kept as the back edge, warned
    only_exec = [(a, "s_cbranch_execz 65001" if ins.startswith("s_cbranch_scc1") else ins, t)
                 for a, ins, t in code]
    cv.LINEARIZE_NOTES.clear()
    assert cv.linearize(only_exec, hand) == base
    assert len(cv.LINEARIZE_NOTES) == 1 and "kept as a loop back edge" in cv.LINEARIZE_NOTES[0]
