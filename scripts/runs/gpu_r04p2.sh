#!/bin/bash
# round 4 (p2): gol_slabp parity; tiny-board timings one engine at a time; kernel trace of 512^2
set -u
O=gpurun_out/r04p2
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/parity.log python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q -k packed --timeout 120 --timeout-method thread || exit $?
tail -3 $O/parity.log
$G 300 $O/prof_plain.log python3 -u scripts/prof_tiny.py 512 auto,121207,140803,140804 || exit $?
cat $O/prof_plain.log
$G 300 $O/prof.log rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u scripts/prof_tiny.py 512 auto,121207,140803,140804 || exit $?
find $O/prof -name '*kernel_stats.csv' -exec cat {} \;
$G 500 $O/tiny.log python3 -u scripts/tune_tiny.py 512,64 100 || exit $?
grep -v '^{"tiny' $O/tiny.log
