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
