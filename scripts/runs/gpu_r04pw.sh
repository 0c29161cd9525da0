#!/bin/bash
# round 4 (pw): pinned counts only below one replayed graph (<= 127 turns): configs[0] call time,
# 1600-turn narrow-board counts, the count tests, the default bench line
set -u
O=gpurun_out/r04pw
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 120 $O/cfg0.log python3 -u scripts/trace_cfg0.py || exit $?
cat $O/cfg0.log
$G 300 $O/narrow.log python3 -u scripts/tune_narrow.py 512x512,4096x512 auto,121207 1600 || exit $?
$G 300 $O/tests.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
tail -2 $O/tests.log
$G 400 $O/bench.log python3 bench.py || exit $?
grep '^{' $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["parity"]["ok"], d["parity"].get("digest_ok")); print(json.dumps(d.get("configs")))'
