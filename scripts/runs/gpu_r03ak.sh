#!/bin/bash
# round 3 (ak): the default bench line with every timed depth's PMC entry present (issued rate)
set -u
O=gpurun_out/r03ak
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 500 $O/bench.log python3 bench.py || exit $?
grep "^{" $O/bench.log | cut -c1-200
