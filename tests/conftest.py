"""Shared test setup.

Markers: ``gpu`` = needs an MI355X (runs on the GPU box via ``pytest -m gpu``); everything else
runs on CPU.  The oracle (``oracle/``) is imported only here in tests, as the checker.
"""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "distributed-gol_amd"
GOLDEN = ROOT / "tests" / "golden"
REF = GOLDEN / "reference"
for p in (ROOT / "oracle", PKG, ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O

    O.build()
    return O


@pytest.fixture(scope="session")
def golhip():
    import golhip as G

    G.load_library()
    return G
