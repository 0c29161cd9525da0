"""CPU model of the drifting-row-sum stencil geometry (gol_stencil DR, golhip_kernels.hip).

The kernel is checked against the oracle on the GPU (test_gpu_parity.py); this file pins the two
geometric facts it relies on, on the CPU, with a bit-level numpy model of one wave chunk:
  * after d drifted generations, wave position P holds cell P - d of generation d for every
    P in [2d, 2048) -- the west edge goes stale two bits per generation, the east edge never;
  * the count windows (lanes 1..63 in full, lanes past the row end dropped) tile the torus row
    exactly once at every drift d <= 16, for any packed width.
The oracle here is the packed CPU stepper (test infrastructure), used as the checker.
"""
import numpy as np
import pytest

WAVE_BITS = 64 * 32   # one wave: 64 lanes x 32 cells
STRIDE = 63 * 32      # cells owned per chunk (half-word halo geometry, K <= 16)


def life_rows(above, mid, below, west_fill):
    """One drifted level on three rows of wave bits (bool arrays, position-indexed):
    position P gets the next state of the cell at P - 1, from positions P-2..P of the input;
    positions 0, 1 read the (garbage) west word west_fill."""
    def shifted(row, k):
        return np.concatenate([west_fill[len(west_fill) - k:], row[:-k]])

    def sum3(row):
        return row.astype(np.int8) + shifted(row, 1) + shifted(row, 2)

    s9 = sum3(above) + sum3(mid) + sum3(below)
    centre = shifted(mid, 1)
    return (s9 == 3) | ((s9 == 4) & centre)


@pytest.mark.parametrize("d_max", [1, 6, 16])
def test_drifted_levels_match_generations(oracle, d_max):
    rng = np.random.default_rng(d_max)
    h, w = 48, 4096
    board = rng.random((h, w)) < 0.4
    base = 1000  # the wave's first cell (any column; the torus wraps)
    cols = (base + np.arange(WAVE_BITS)) % w
    rows = board[:, cols]
    for d in range(1, d_max + 1):
        garbage = rng.random((h, 2)) < 0.5
        rows = np.stack([life_rows(rows[(y - 1) % h], rows[y], rows[(y + 1) % h], garbage[y])
                         for y in range(h)])
        gen, _ = oracle.packed_run((board * 255).astype(np.uint8), d)
        exp = gen[:, (base + np.arange(WAVE_BITS) - d) % w] == 255
        valid = slice(2 * d, WAVE_BITS)
        assert np.array_equal(rows[:, valid], exp[:, valid]), d


@pytest.mark.parametrize("wd", [4, 20, 63, 64, 128, 160, 2048, 8192])
def test_count_windows_tile_the_row(wd):
    """wd = packed row words (a multiple of 4: L = lcm(width, 128))."""
    L = 32 * wd
    nchunks = -(-wd // 63)
    for d in range(1, 17):
        hits = np.zeros(L, dtype=np.int64)
        for c in range(nchunks):
            for lane in range(1, 64):
                colraw = 63 * c + lane - 1
                if colraw >= wd:  # count_lane: lanes past the row end drop their sums
                    continue
                # position P = 32*lane + b holds cell 32*(63c - 1) + P - d
                first = 32 * (63 * c - 1) + 32 * lane - d
                hits[(first + np.arange(32)) % L] += 1
        assert (hits == 1).all(), (wd, d)
