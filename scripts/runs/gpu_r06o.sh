#!/bin/bash
# round 6 (o): lib/host_bench SIGSEGVs inside golhip_step when bench.py runs under rocprofv3 (the
# child inherits the tool, r06n).  Bisect: host_bench plain, under the tool, under the tool with
# the engine's graphs off (lib_faults' GOLHIP_GRAPHS selector), and the Python engine on the same
# board under the tool from a worker thread.  (A segfault ends the call: the graphs-off run goes first.)
set -u
O=gpurun_out/r06o
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
python3 - <<'PY'
import json, sys
from pathlib import Path
sys.path.insert(0, "distributed-gol_amd")
import numpy as np, golhip
G = Path("tests/golden"); gold = json.loads((G / "synthetic_golden.json").read_text())
d = Path("/tmp/r06o"); (d / "images").mkdir(parents=True, exist_ok=True); (d / "out").mkdir(exist_ok=True)
b = np.zeros((4096, 4096), dtype=np.uint8)
golhip.place(b, golhip.parse_rle((G / "gosper_gun.rle").read_text()), 64, 64)
golhip.place(b, golhip.parse_rle((G / "r_pentomino.rle").read_text()), 2048, 2048)
(d / "images" / "4096x4096.pgm").write_bytes(b"P5\n4096 4096\n255\n" + b.tobytes())
deltas = np.load(G / gold["cfg5"]["counts_1e6_npz"])["deltas"][:20000]
c0 = int((b == 255).sum())
np.concatenate([[c0], c0 + np.cumsum(deltas.astype(np.int64))]).astype("<u4").tofile(d / "exp.u32")
PY
HB="distributed-gol_amd/lib/host_bench -w 4096 -h 4096 -turns 20000 -images /tmp/r06o/images -out /tmp/r06o/out -expected /tmp/r06o/exp.u32 -ticker_ms 2000 -depth 0"
$G 60 $O/plain.log $HB || exit $?
tail -c 400 $O/plain.log
LD_LIBRARY_PATH=$PWD/distributed-gol_amd/lib_faults GOLHIP_GRAPHS=0 $G 90 $O/prof_nographs.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r06o/p2 -o p -- $HB || exit $?
grep -m3 "SIGSEGV\|^{\|rc=" $O/prof_nographs.log
$G 90 $O/prof.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r06o/p1 -o p -- $HB || exit $?
grep -m3 "SIGSEGV\|^{\|rc=" $O/prof.log
exit 0
