#!/usr/bin/env python3
"""One engine for PMC / trace runs of the small-board kernels: an n x n random board (p = 0.5),
`turns` turns per call with counts, 3 calls; board kernel mode -1 (automatic) / 1 (forced) / 0.
Usage: profile_board.py n turns board_mode"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import numpy as np  # noqa: E402

import golhip  # noqa: E402

n, turns, mode = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
with golhip.Engine(n, n, k=16) as e:
    e.set_board_kernel(mode)
    e.load(((np.random.default_rng(n).random((n, n)) < 0.5) * 255).astype(np.uint8))
    for _ in range(3):
        e.step(turns, counts=True)
    e.sync()
    print(n, turns, mode, e.launch_kind(16, counts=True))
