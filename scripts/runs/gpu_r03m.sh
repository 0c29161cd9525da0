#!/bin/bash
# round 3 (m): re-validation of HEAD on a fresh container's build: full GPU suite, smoke, the
# driver's bench command, and the 16-wave slab sweep whose results the cut-off session lost
set -u
O=gpurun_out/r03m
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 900 $O/gpu_suite.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
tail -3 $O/gpu_suite.log
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -1 $O/smoke.log
$G 400 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep "^{" $O/bench20.log | cut -c1-300
$G 400 $O/tune_slab.log python3 scripts/tune_slab.py 4096,5120 0,20812,21208,21207,21606,21605 || exit $?
tail -5 $O/tune_slab.log
