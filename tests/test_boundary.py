"""The drop-in boundary: libgolhip.so loads, exports every symbol include/golhip.h declares, and its
pure host helpers work -- all without a GPU (no compute calls here)."""
import re
import subprocess

import pytest

from conftest import PKG, ROOT


def header_functions():
    text = (ROOT / "include" / "golhip.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(golhip_\w+)\s*\(", text, re.M)))


def test_header_lists_the_required_exports():
    fns = header_functions()
    # SURVEY.md section 8(b) required exports
    for name in ["golhip_create", "golhip_destroy", "golhip_load_bytes", "golhip_init_random",
                 "golhip_step", "golhip_alive_count", "golhip_store_bytes", "golhip_alive_cells",
                 "golhip_flips", "golhip_turn", "golhip_last_error"]:
        assert name in fns


def test_library_exports_every_declared_symbol(golhip):
    so = PKG / "lib" / "libgolhip.so"
    out = subprocess.check_output(["nm", "-D", "--defined-only", str(so)], text=True)
    exported = set(re.findall(r" T (golhip_\w+)", out))
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing
    assert sorted(golhip.EXPORTS) == header_functions()
    lib = golhip.load_library()
    for f in header_functions():
        assert hasattr(lib, f)


def test_library_is_gfx950_code(golhip):
    so = PKG / "lib" / "libgolhip.so"
    data = so.read_bytes()
    assert b"gfx950" in data


# the tuning library's selectors and fault hooks (csrc/tuning/engine_tuning.hip): the production
# library must not even hold their names, so a stray environment variable cannot change its kernels
TUNING_SELECTORS = ["GOLHIP_VARIANT", "GOLHIP_SPLIT", "GOLHIP_TILE", "GOLHIP_SLAB", "GOLHIP_BAND_ROWS",
                    "GOLHIP_FIXED_K", "GOLHIP_LDS_PAD", "GOLHIP_STEP1", "GOLHIP_GRAPHS",
                    "GOLHIP_COUNT_WINDOW", "GOLHIP_FAULT"]


def test_production_sources_never_name_the_tuning_build():
    """Tuning-only code lives in tuning-only translation units (csrc/tuning/), which the production
    library does not link: no production source holds a GOLHIP_TUNING switch, and the production
    library exports no tuning symbol."""
    csrc = PKG / "csrc"
    prod_sources = [p for p in csrc.iterdir() if p.suffix in (".hip", ".hpp")]
    assert len(prod_sources) >= 10
    for p in prod_sources:
        text = p.read_text()
        assert "GOLHIP_TUNING" not in text and "kTuningBuild" not in text, p.name
    make = (PKG / "Makefile").read_text()
    assert "-DGOLHIP_TUNING" not in make
    out = subprocess.check_output(["nm", "-D", "--defined-only", str(PKG / "lib" / "libgolhip.so")], text=True)
    assert "golhip_tuning" not in out


def test_production_library_reads_only_documented_hooks():
    """lib/libgolhip.so holds no tuning selector (the `strings | grep GOLHIP_VARIANT` check) and only
    the two documented test hooks; lib_tuning/libgolhip.so holds the selectors."""
    prod = (PKG / "lib" / "libgolhip.so").read_bytes()
    names = set(re.findall(rb"GOLHIP_[A-Z][A-Z0-9_]+", prod))
    assert names == {b"GOLHIP_RING_SELF", b"GOLHIP_STAGE_BYTES"}, names
    tuning = (PKG / "lib_tuning" / "libgolhip.so").read_bytes()
    for sel in TUNING_SELECTORS:
        assert sel.encode() in tuning, sel
    # the experiment harness stays out of the shipped library: it is several times smaller
    assert len(prod) * 3 < len(tuning), (len(prod), len(tuning))


def test_tuning_library_exports_the_same_abi(golhip):
    out = subprocess.check_output(["nm", "-D", "--defined-only", str(PKG / "lib_tuning" / "libgolhip.so")],
                                  text=True)
    assert set(re.findall(r" T (golhip_\w+)", out)) >= set(header_functions())


def test_version_and_strerror(golhip):
    lib = golhip.load_library()
    assert lib.golhip_version() >= 100
    assert lib.golhip_strerror(golhip.ERR_CAP) == b"output capacity too small"


@pytest.mark.parametrize("height,world", [(65536, 1), (65536, 8), (262144, 8), (10, 3), (512, 4)])
def test_strip_bounds_cover_the_board(golhip, height, world):
    """broker/broker.go:37-56 splits rows into strips; here every row is covered exactly once
    for ANY height (the reference drops rows when N % 4 != 0)."""
    y = 0
    for r in range(world):
        y0, rows = golhip.strip_bounds(height, world, r)
        assert y0 == y and rows >= height // world
        y += rows
    assert y == height


def test_strip_bounds_rejects_bad_args(golhip):
    with pytest.raises(golhip.GolHipError):
        golhip.strip_bounds(100, 4, 4)


def test_engine_without_device_fails_loudly(golhip):
    """No CPU fallback: creating an engine where no gfx950 device exists raises."""
    if golhip.device_count() > 0:
        pytest.skip("a device is present")
    with pytest.raises(golhip.GolHipError):
        golhip.Engine(64, 64)


SUPPORTED_DEPTHS = {1, 2, 4, 6, 8, 10, 12, 14, 16, 32}


@pytest.mark.parametrize("turns", [1, 5, 17, 20, 25, 33, 45, 1000, 1192])
def test_launch_plan_covers_the_turns(golhip, turns):
    """golhip_launch_plan (the sequence golhip_step runs) advances exactly `turns` generations in
    supported depths <= k, every launch depth the stencil is built for."""
    plan = golhip.launch_plan(65536, 65536, 16, turns)
    assert sum(plan) == turns
    assert all(0 < d <= 16 and d in SUPPORTED_DEPTHS for d in plan)


def test_launch_plan_short_runs_are_balanced(golhip):
    """The driver's short run (20 turns) is split into two launches of near-equal depth, not the
    greedy 16 + 4 (a 4-level launch runs at half the rate, profiles/r01_bench.json k sweep)."""
    plan = golhip.launch_plan(65536, 65536, 16, 20)
    assert len(plan) == 2 and min(plan) >= 8, plan
    bulk = golhip.launch_plan(65536, 65536, 16, 1000)
    assert len(bulk) <= 1000 // 10 + 2  # mostly deep launches


def test_launch_plan_small_boards_replay_graphs(golhip):
    """Small (launch-bound) boards replay captured graphs of deep launches (negative entries)."""
    plan = golhip.launch_plan(4096, 4096, 16, 1000000)
    graphs = [-d for d in plan if d < 0]
    assert graphs and sum(graphs) + sum(d for d in plan if d > 0) == 1000000
    assert not any(d < 0 for d in golhip.launch_plan(65536, 65536, 16, 1000))
    assert not any(d < 0 for d in golhip.launch_plan(4096, 4096, 16, 1000000, strips=2))


def test_launch_plan_long_runs_replay_large_graphs(golhip):
    """Long small-board runs replay 4096-generation graphs (one count finalize + copy per replay),
    then 128-generation graphs, then single launches."""
    plan = golhip.launch_plan(5120, 5120, 16, 10000)
    graphs = [-d for d in plan if d < 0]
    assert graphs[:2] == [4096] * 2 and set(graphs[2:]) <= {128}
    assert sum(graphs) + sum(d for d in plan if d > 0) == 10000


def test_launch_plan_bulk_depth_by_board_size(golhip):
    """The bulk depth follows the strip size (profiles/r02/r02ae_depth_by_size.txt and round 3's
    pre-shifted geometry, pre-heated chip): K = 14 on strips of 2^31 .. 2^35 cells (65536^2: 125.6
    vs 124.1 at K = 12), K = 12 below (graph-replayed streaming boards), K = 16 on larger strips
    (262144^2: 139 vs 138 at K = 14); register-slab boards replay graphs of 16-deep launches."""
    from collections import Counter

    assert Counter(golhip.launch_plan(65536, 65536, 16, 1008)) == {14: 72}
    p131 = golhip.launch_plan(131072, 131072, 16, 480)
    assert sum(p131) == 480 and Counter(p131)[14] >= 32
    assert Counter(golhip.launch_plan(262144, 262144, 16, 160)) == {16: 10}
    # per strip: the 262144^2 board over 8 ranks is 2^33 cells per strip -> K = 14 in bulk
    p8 = golhip.launch_plan(262144, 262144, 16, 480, strips=8)
    assert sum(p8) == 480 and Counter(p8)[14] >= 32
    # the driver's 20-turn region stays 12 + 8 (a 6-deep launch runs at ~3/4 the rate)
    assert sorted(golhip.launch_plan(65536, 65536, 16, 20)) == [8, 12]
    assert sorted(golhip.launch_plan(65536, 131072, 16, 20, strips=2)) == [8, 12]
    # 16384^2 takes the register slab since round 4 (at most 40 minimal-band waves per CU): 8
    # launches of K = 16 per replay; 20480^2 still streams: 10 launches of K = 12 per replay
    graphs16k = [-d for d in golhip.launch_plan(16384, 16384, 16, 2000) if d < 0]
    assert graphs16k and set(graphs16k) == {128}
    graphs20k = [-d for d in golhip.launch_plan(20480, 20480, 16, 2000) if d < 0]
    assert graphs20k and set(graphs20k) == {120}
    graphs5k = [-d for d in golhip.launch_plan(5120, 5120, 16, 10000) if d < 0]
    assert graphs5k[:2] == [4096, 4096]  # the register slab keeps K = 16
    # the maximum depth still caps everything
    assert max(golhip.launch_plan(65536, 65536, 8, 1000)) <= 8


@pytest.mark.parametrize("width,height,world", [(262144, 262143, 2), (65536, 65537, 2),
                                                (4096, 4099, 4), (65536, 196607, 3)])
def test_launch_plan_is_rank_independent_on_uneven_strips(golhip, width, height, world):
    """Every launch of a split board exchanges K-row halos, so every rank of a rank-mode board must
    run the same depths.  Strips differ by a row when height % world != 0; the planner ranks depths
    from the largest strip, ceil(height / world) rows, which every rank shares (the engine's
    run_steps and golhip_launch_plan use the same helper).  262143 rows on 2 ranks is the case
    that split 131071 vs 131072 rows across the 2^35-cell bulk-depth switch (K = 12 vs 16)."""
    rows = [golhip.strip_bounds(height, world, r)[1] for r in range(world)]
    assert len(set(rows)) > 1  # the strips really are uneven
    ceil_rows = -(-height // world)
    for turns in (20, 25, 160, 1008):
        plan = golhip.launch_plan(width, height, 16, turns, strips=world)
        # the same plan as a board whose every strip has the largest strip's rows
        assert plan == golhip.launch_plan(width, ceil_rows * world, 16, turns, strips=world)
        assert sum(plan) == turns
    if (width, height) == (262144, 262143):
        assert set(golhip.launch_plan(width, height, 16, 160, strips=2)) == {16}


def test_register_slab_boards_take_the_fewest_launches(golhip):
    """Register-slab boards (latency-bound launches, about the same cost at any depth) plan the tail
    of a call in the fewest launches of the slab depths {16, 12, 8, 4, 2, 1} (slab_first_k): configs[0]
    (512^2 x 100) is 6 x 16 + 4, not 5 x 16 + 12 + 8 (profiles/r05/r05p_cfg0_timeline.log); boards of
    at most 256 rows run the whole-board kernel, one launch per call; streaming boards keep the
    rate-model split (20 turns at 65536^2: 12 + 8)."""
    assert golhip.launch_plan(512, 512, 16, 100) == [16] * 6 + [4]
    assert golhip.launch_plan(512, 512, 16, 37) == [16, 16, 4, 1]
    assert golhip.launch_plan(1000, 600, 16, 46) == [16, 16, 12, 2]
    assert golhip.launch_plan(256, 256, 16, 100) == [100]
    assert golhip.launch_plan(4096, 4096, 16, 20) == [16, 4]
    assert sorted(golhip.launch_plan(65536, 65536, 16, 20)) == [8, 12]
