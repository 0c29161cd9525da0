#!/bin/bash
# round 4 (p): the narrow-board packed slab gol_slabp (NC = 14, tuning build): parity vs the
# oracle, then tiny-board timings against the production choice
set -u
O=gpurun_out/r04pk
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/parity.log python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q -k packed --timeout 120 --timeout-method thread || exit $?
tail -3 $O/parity.log
$G 400 $O/tiny.log python3 -u scripts/tune_tiny.py 512,256,128,64,960 100 || exit $?
grep -v '^{"tiny' $O/tiny.log
