#!/bin/bash
# round 6 (r): host_bench exactly as bench.py's cfg5_host leg runs it (1e6 turns, 2 s ticker, keys
# p/s/p), directly under rocprofv3 --kernel-trace --stats (not as a child of bench.py), after a
# plain run of the same command: does the r06n SIGSEGV need the python parent?
set -u
O=gpurun_out/r06r
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
python3 - <<'PY'
import json, sys
from pathlib import Path
sys.path.insert(0, "distributed-gol_amd")
import numpy as np, golhip
G = Path("tests/golden"); gold = json.loads((G / "synthetic_golden.json").read_text())
d = Path("/tmp/r06r"); (d / "images").mkdir(parents=True, exist_ok=True); (d / "out").mkdir(exist_ok=True)
b = np.zeros((4096, 4096), dtype=np.uint8)
golhip.place(b, golhip.parse_rle((G / "gosper_gun.rle").read_text()), 64, 64)
golhip.place(b, golhip.parse_rle((G / "r_pentomino.rle").read_text()), 2048, 2048)
(d / "images" / "4096x4096.pgm").write_bytes(b"P5\n4096 4096\n255\n" + b.tobytes())
deltas = np.load(G / gold["cfg5"]["counts_1e6_npz"])["deltas"]
c0 = int((b == 255).sum())
np.concatenate([[c0], c0 + np.cumsum(deltas.astype(np.int64))]).astype("<u4").tofile(d / "exp.u32")
PY
HB="distributed-gol_amd/lib/host_bench -w 4096 -h 4096 -turns 1000000 -images /tmp/r06r/images -out /tmp/r06r/out -expected /tmp/r06r/exp.u32 -ticker_ms 2000 -keys p@0.5,s@0.8,p@2.3 -depth 2"
$G 60 $O/plain.log $HB || exit $?
tail -c 300 $O/plain.log
$G 120 $O/prof.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r06r/p1 -o p -- $HB || exit $?
grep -m3 "SIGSEGV\|^{\|rc=" $O/prof.log | cut -c1-300
exit 0
