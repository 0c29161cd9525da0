#!/usr/bin/env python3
"""The host contract with per-turn CellFlipped events (the SDL consumer's stream, gol/distributor.go:
53-59; sdl_test.go toggles a pixel per event): lib/host_bench -flips, pipelined (delivery thread,
depth 2) against unpipelined (depth 0), on configs[4]'s board (4096^2 gun + R-pentomino) and on the
reference's images/512x512.pgm.  Every run's final count is checked against the goldens
(tests/golden cfg5 npz; check/alive/512x512.csv).  Prints one JSON object.
Usage: host_flips_ab.py [turns_4096] [turns_512]"""
import json
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import numpy as np  # noqa: E402

import golhip  # noqa: E402

t4096 = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
t512 = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
G = ROOT / "tests" / "golden"
EXE = ROOT / "distributed-gol_amd" / "lib" / "host_bench"
gold = json.loads((G / "synthetic_golden.json").read_text())
out = {}
with tempfile.TemporaryDirectory(prefix="golhip_flips_") as d:
    dp = Path(d)
    (dp / "images").mkdir()
    (dp / "out").mkdir()
    b = np.zeros((4096, 4096), dtype=np.uint8)
    golhip.place(b, golhip.parse_rle((G / "gosper_gun.rle").read_text()), 64, 64)
    golhip.place(b, golhip.parse_rle((G / "r_pentomino.rle").read_text()), 2048, 2048)
    (dp / "images" / "4096x4096.pgm").write_bytes(b"P5\n4096 4096\n255\n" + b.tobytes())
    deltas = np.load(G / gold["cfg5"]["counts_1e6_npz"])["deltas"][:t4096]
    c0 = int((b == 255).sum())
    np.concatenate([[c0], c0 + np.cumsum(deltas.astype(np.int64))]).astype("<u4").tofile(dp / "exp4096.u32")
    (dp / "images" / "512x512.pgm").write_bytes((G / "reference" / "images" / "512x512.pgm").read_bytes())
    csv = (G / "reference" / "check" / "alive" / "512x512.csv").read_text().split()[1:]
    counts512 = [6511] + [int(ln.split(",")[1]) for ln in csv][:t512]
    np.array(counts512, dtype="<u4").tofile(dp / "exp512.u32")
    for n, turns, exp in ((4096, t4096, "exp4096.u32"), (512, t512, "exp512.u32")):
        for depth in (2, 0):
            cmd = [str(EXE), "-w", str(n), "-h", str(n), "-turns", str(turns), "-images", str(dp / "images"),
                   "-out", str(dp / "out"), "-expected", str(dp / exp), "-ticker_ms", "2000", "-flips",
                   "-depth", str(depth)]
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            key = f"{n}x{n}_depth{depth}"
            if p.returncode != 0:
                out[key] = {"failed": p.returncode, "stderr": p.stderr[-1500:]}
            else:
                r = json.loads(p.stdout.strip().splitlines()[-1])
                out[key] = {k: r[k] for k in ("turns", "wall_s", "turn_complete_span_s", "us_per_turn_streaming",
                                              "cell_flipped", "turn_complete", "final")}
            print(key, out[key], flush=True)
print(json.dumps(out))
