"""Measurement tooling on CPU: the bench's board digest equals the oracle's definition, and the PMC
summariser keys every kernel by its full template name (round 3's regex cut every engine kernel at
"(anonymous namespace)", averaging gol_slab and count_finalize into one bucket)."""
import importlib.util
import sys

import numpy as np

from conftest import ROOT


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def test_bench_digest_matches_oracle(oracle):
    import bench

    assert bench.DIGEST_CHUNK_ROWS == oracle.DIGEST_CHUNK_ROWS
    words = oracle.init_random(640, 9000, seed=4)
    assert bench.chunk_digests(words) == oracle.chunk_digests(words)
    # strips that start on chunk boundaries hash to the whole board's digest
    parts = bench.chunk_digests(words[:4096]) + bench.chunk_digests(words[4096:8192]) + \
        bench.chunk_digests(words[8192:])
    assert oracle.board_digest(parts) == oracle.board_digest(oracle.chunk_digests(words))
    flipped = words.copy()
    flipped[5000, 3] ^= np.uint64(1 << 17)
    assert oracle.board_digest(oracle.chunk_digests(flipped)) != oracle.board_digest(parts)


def test_golden_board_digests_are_registered():
    """bench.py's parity.digest_ok has goldens for the N = 1 bench board and the weak-scaling
    boards at the driver's (25) and the default (1008) turn."""
    import bench

    for n in (1, 2, 4, 8):
        for turn in (25, 1008):
            d = bench.golden_digest(65536, 65536 * n, 3, turn)
            assert d is not None and len(d) == 64, (n, turn)
    assert bench.golden_digest(65536, 65536, 3, 26) is None


def test_pmc_kernel_key():
    m = _load("pmc_kernel_avg", ROOT / "scripts" / "pmc_kernel_avg.py")
    slab = ("void golhip::(anonymous namespace)::gol_slab<16, 12, 8, true, 0, 2>(unsigned int const*, "
            "unsigned int*, golhip::StencilParams, unsigned long long*)")
    fin = "golhip::(anonymous namespace)::count_finalize(unsigned long long*, unsigned long long*)"
    assert m.kernel_key(slab) == "gol_slab<16, 12, 8, true, 0, 2>"
    assert m.kernel_key(fin) == "count_finalize"
    assert m.kernel_key(slab) != m.kernel_key(slab.replace("12, 8", "8, 12"))
