#!/bin/bash
# round 5: A/B of rows per CU at 4096 rows (tuning build).  A 3968-wide board (124 words = exactly
# two 62-word chunks) takes 12 x 6 / 16 x 4 slabs in one round (206 / 256 slabs) where 4096-wide
# needs 3 chunks; us/turn of 12 x 7 (84 rows per CU) vs 12 x 6 (72) vs 16 x 5 (80) vs 16 x 4 (64)
set -u
O=gpurun_out/r05y
mkdir -p $O
G=scripts/guard.sh
$G 400 $O/tune.log python3 scripts/tune_slab.py 3968x4096,4096 0,121207,121206,121605,121604 4096 || exit $?
tail -3 $O/tune.log
