#!/bin/bash
# round 4 (ps): per-turn counts through a pinned host buffer (no device-to-host copy per call):
# configs[0] call time, GPU suite, smoke, default bench line
set -u
O=gpurun_out/r04ps
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 120 $O/cfg0.log python3 -u scripts/trace_cfg0.py || exit $?
cat $O/cfg0.log
$G 900 $O/suite.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
tail -3 $O/suite.log
grep -q " passed" $O/suite.log && ! grep -q "failed" $O/suite.log || exit 1
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -2 $O/smoke.log
$G 400 $O/bench.log python3 bench.py || exit $?
grep '^{' $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["parity"]["ok"], d["parity"].get("digest_ok")); print(json.dumps(d.get("configs")))'
