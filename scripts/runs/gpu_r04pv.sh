#!/bin/bash
# round 4 (pv): the driver-shaped 20/5 line and the rank rehearsal on the final tree
set -u
O=gpurun_out/r04pv
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 200 $O/pinned.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "pinned or narrow_board" --timeout 120 --timeout-method thread || exit $?
tail -2 $O/pinned.log
$G 300 $O/bench20.log python3 bench.py --steps 20 --warmup 5 || exit $?
GOLHIP_RING_SELF=1 $G 200 $O/rehearsal20.log python3 bench.py --steps 20 --warmup 5 --pg-always --no-cpu --no-sweep --no-strong --no-configs --no-flips || exit $?
for f in bench20 rehearsal20; do grep '^{' $O/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$f'", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["parity"]["ok"], d["parity"].get("digest_ok"), d["process"], (d.get("configs") or {}).get("ok"))'; done
