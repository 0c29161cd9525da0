#!/bin/bash
# round 5: the GPU suite after 16 x 4 joined the production slab shapes, and the automatic choice
# on the two-chunk board against the forced 12 x 7 (tuning build)
set -u
O=gpurun_out/r05z
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 900 $O/suite.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
tail -3 $O/suite.log
$G 300 $O/tune.log python3 scripts/tune_slab.py 3968x4096,2048,5120x512 0,121207 4096 || exit $?
grep best $O/tune.log
