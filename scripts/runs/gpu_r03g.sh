#!/bin/bash
# round 3 (g): K = 12 band sweep at 65536^2 (the planner's 168-row bands vs taller ones that cut
# the band trapezoid), 384 timed generations per point, 3 interleaved rounds
set -u
O=gpurun_out/r03g
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
TUNE_STEPS=384 $G 500 $O/tune_k12_bands.log python3 scripts/tune.py 65536 12 0,168,184,200,216,224,232 prod || exit $?
tail -3 $O/tune_k12_bands.log
TUNE_STEPS=384 $G 500 $O/tune_k16_bands.log python3 scripts/tune.py 65536 16 0,192,216,240,264 prod || exit $?
tail -3 $O/tune_k16_bands.log
