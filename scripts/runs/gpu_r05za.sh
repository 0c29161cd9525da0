#!/bin/bash
# round 5: the skipping tests after their boards moved to keep short last bands under 16 x 4 / 12 x 7
set -u
O=gpurun_out/r05za
mkdir -p $O
G=scripts/guard.sh
$G 400 $O/act.log python -u -m pytest tests/test_gpu_activity.py -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
tail -2 $O/act.log
