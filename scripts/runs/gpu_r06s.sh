#!/bin/bash
# round 6 (s): device per-turn counts now reach the caller through the shard's pinned count buffer
# (engine_comm.hip reduce_u64) instead of a pageable device-to-host copy.  The count-heavy GPU
# tests, the host contract, then host_bench's 1e6-turn cfg5 run under rocprofv3 (r06r: SIGSEGV).
# Result: 247 passed, the SIGSEGV unchanged (it is in hipGraphLaunch under the tool); change reverted.
set -u
O=gpurun_out/r06s
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 600 $O/tests.log python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_host.py tests/test_gpu_rank_host.py || exit $?
tail -2 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q "FAILED\|[0-9] failed" $O/tests.log || exit 1
python3 - <<'PY'
import json, sys
from pathlib import Path
sys.path.insert(0, "distributed-gol_amd")
import numpy as np, golhip
G = Path("tests/golden"); gold = json.loads((G / "synthetic_golden.json").read_text())
d = Path("/tmp/r06s"); (d / "images").mkdir(parents=True, exist_ok=True); (d / "out").mkdir(exist_ok=True)
b = np.zeros((4096, 4096), dtype=np.uint8)
golhip.place(b, golhip.parse_rle((G / "gosper_gun.rle").read_text()), 64, 64)
golhip.place(b, golhip.parse_rle((G / "r_pentomino.rle").read_text()), 2048, 2048)
(d / "images" / "4096x4096.pgm").write_bytes(b"P5\n4096 4096\n255\n" + b.tobytes())
deltas = np.load(G / gold["cfg5"]["counts_1e6_npz"])["deltas"]
c0 = int((b == 255).sum())
np.concatenate([[c0], c0 + np.cumsum(deltas.astype(np.int64))]).astype("<u4").tofile(d / "exp.u32")
PY
HB="distributed-gol_amd/lib/host_bench -w 4096 -h 4096 -turns 1000000 -images /tmp/r06s/images -out /tmp/r06s/out -expected /tmp/r06s/exp.u32 -ticker_ms 2000 -keys p@0.5,s@0.8,p@2.3 -depth 2"
$G 60 $O/plain.log $HB || exit $?
tail -c 300 $O/plain.log
$G 120 $O/prof.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r06s/p1 -o p -- $HB || exit $?
grep -v "^W2026\|^E2026" $O/prof.log | grep -m3 "SIGSEGV\|^{\|rc=" | cut -c1-400
exit 0
