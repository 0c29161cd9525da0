#!/bin/bash
# round 4 (pfinal2): the last validation after limiting pinned counts to <= 127-turn calls:
# GPU suite, smoke, default bench line (configs leg included)
set -u
O=gpurun_out/r04pfinal2
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 900 $O/suite.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
tail -3 $O/suite.log
grep -q " passed" $O/suite.log && ! grep -q "failed" $O/suite.log || exit 1
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -2 $O/smoke.log
$G 400 $O/bench.log python3 bench.py || exit $?
grep '^{' $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["parity"]["ok"], d["parity"].get("digest_ok")); print(json.dumps(d.get("configs")))'
