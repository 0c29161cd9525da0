"""The C++ host mirror of gol.Run (distributed-gol_amd/host) -- the reference's own integration
tests (gol_test.go, pgm_test.go, count_test.go, sdl_test.go) restated in tests/host/*.cpp and run
here as native binaries."""
import subprocess

import pytest

from conftest import PKG, REF

LIB = PKG / "lib"


def run(binary, *args, timeout=300):
    p = subprocess.run([str(LIB / binary), *map(str, args)], cwd=REF, capture_output=True,
                       text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return p.stdout


def test_host_cpu_units(tmp_path):
    """Channel semantics and the PGM codec, no device calls."""
    assert "ok" in run("test_host_cpu", REF, tmp_path)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["TestGol", "TestPgm", "TestSdl", "TestPublish", "TestAlive",
                                  "TestKeys"])
def test_reference_integration_tests(name, tmp_path):
    out = run("test_gol_host", name, tmp_path, timeout=240)
    assert f"{name}: ok" in out
