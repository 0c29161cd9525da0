#!/bin/bash
# round 3 (j): the tail depths of short runs (K = 8 and K = 10 band sweeps at 65536^2: the driver's
# 20 turns run 12 + 8), then the default bench and the driver's bench on the current tree
set -u
O=gpurun_out/r03j
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
TUNE_STEPS=256 $G 500 $O/tune_k8_bands.log python3 scripts/tune.py 65536 8 0,128,160,192,224,256,320 prod || exit $?
tail -2 $O/tune_k8_bands.log
TUNE_STEPS=256 $G 500 $O/tune_k10_bands.log python3 scripts/tune.py 65536 10 0,160,192,224,256 prod || exit $?
tail -2 $O/tune_k10_bands.log
$G 500 $O/bench.log python3 bench.py || exit $?
grep "^{" $O/bench.log | cut -c1-200
$G 400 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep "^{" $O/bench20.log | cut -c1-200
