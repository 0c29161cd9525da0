#!/bin/bash
# round 4 (p): full validation after the bench/barrier/stream changes: GPU suite, smoke, the
# default bench line and the driver-shaped 20/5 line, and the rank rehearsal at 20/5
set -u
O=gpurun_out/r04p
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 900 $O/suite.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
tail -3 $O/suite.log
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -2 $O/smoke.log
$G 400 $O/bench.log python3 bench.py || exit $?
$G 300 $O/bench20.log python3 bench.py --steps 20 --warmup 5 || exit $?
GOLHIP_RING_SELF=1 $G 200 $O/rehearsal20.log python3 bench.py --steps 20 --warmup 5 --pg-always --no-cpu --no-sweep --no-strong --no-configs --no-flips || exit $?
for f in bench bench20 rehearsal20; do grep '^{' $O/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$f'", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["parity"]["ok"], d["parity"].get("digest_ok"), d["process"], (d.get("configs") or {}).get("ok"))'; done
