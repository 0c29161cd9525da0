#!/bin/bash
# round 3 (q): production K = 16 on the pre-shifted 63-word geometry: full GPU suite, smoke, the
# default bench and the driver's 20/5 command, the lockstep A/B against the half-word halo kept
set -u
O=gpurun_out/r03q
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 900 $O/gpu_suite.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
tail -3 $O/gpu_suite.log
grep -q " passed" $O/gpu_suite.log && ! grep -q " failed" $O/gpu_suite.log || exit 1
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -1 $O/smoke.log
$G 500 $O/bench.log python3 bench.py || exit $?
grep "^{" $O/bench.log | cut -c1-300
$G 400 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep "^{" $O/bench20.log | cut -c1-300
$G 300 $O/tune_tail_k12.log python3 scripts/tune_tail.py 65536 12 0:0:0,168:0:0,264:0:0,240:150:64,240:150:96,336:150:96,336:150:128,336:300:64,432:150:128,432:300:96 5 || exit $?
tail -11 $O/tune_tail_k12.log
$G 300 $O/tune_tail_k16.log python3 scripts/tune_tail.py 65536 16 0:0:0,264:0:0,336:150:96,432:150:128,432:300:96,528:150:128 5 || exit $?
tail -7 $O/tune_tail_k16.log
