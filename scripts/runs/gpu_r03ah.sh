#!/bin/bash
# round 3 (ah): validation of the committed tree: full GPU suite, smoke, the driver's 20/5
# command and the default bench (uninstrumented timed regions)
set -u
O=gpurun_out/r03ah
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 900 $O/gpu_suite.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
tail -3 $O/gpu_suite.log
grep -q " passed" $O/gpu_suite.log && ! grep -q " failed" $O/gpu_suite.log || exit 1
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -1 $O/smoke.log
$G 400 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep "^{" $O/bench20.log | cut -c1-200
$G 500 $O/bench.log python3 bench.py || exit $?
grep "^{" $O/bench.log | cut -c1-200
