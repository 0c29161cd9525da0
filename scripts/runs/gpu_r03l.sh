#!/bin/bash
# round 3 (l): 16-wave slabs (16 x 6, 16 x 5: finer rows, the pure-halo waves' dead generations
# spread over all four SIMDs) against the current shapes, same call
set -u
O=gpurun_out/r03l
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/tune_slab.log python3 scripts/tune_slab.py 4096,5120 0,20812,21208,21207,21606,21605 || exit $?
tail -5 $O/tune_slab.log
