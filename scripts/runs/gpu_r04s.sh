#!/bin/bash
# round 4 (s): tuning-build launch depths 20 / 24 -- parity, then the driver's 20-turn region as ONE
# K = 20 launch against 12 + 8 (density-matched lockstep A/B), and the 1000-turn rate at K = 20
set -u
O=gpurun_out/r04s
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/parity.log python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q -k "depths_20_24" --timeout 240 --timeout-method thread || exit $?
tail -2 $O/parity.log
grep -q " passed" $O/parity.log && ! grep -qE " failed| error" $O/parity.log || exit 1
$G 300 $O/ab_split.log python3 scripts/ab_split.py prod 0,12,20,16 11 || exit $?
tail -6 $O/ab_split.log
