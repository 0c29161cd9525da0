#!/bin/bash
# round 5: T = 16 slabs (48 rows, 12 rows per SIMD) against the automatic 16 x 4 on 2048^2 and
# 3968 x 4096 (tuning build, forced shapes, 4096 turns)
set -u
O=gpurun_out/r05zc
mkdir -p $O
G=scripts/guard.sh
$G 400 $O/tune.log python3 scripts/tune_slab.py 2048,3968x4096 0,120806,121204 4096 || exit $?
grep best $O/tune.log
