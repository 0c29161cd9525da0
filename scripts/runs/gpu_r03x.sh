#!/bin/bash
# round 3 (x): production with the last chunk's idle lanes exec-masked off (prodmask): parity, then
# the pre-heated lockstep A/B at 65536^2 (K = 8/12/16) and 262144^2 (K = 16)
set -u
O=gpurun_out/r03x
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 600 $O/pytest_mask.log python -u -m pytest tests/test_gpu_parity.py -m gpu -k "prodmask" -x -q --timeout 300 --timeout-method thread || exit $?
tail -2 $O/pytest_mask.log
grep -q " passed" $O/pytest_mask.log && ! grep -q " failed" $O/pytest_mask.log || exit 1
AB_STEPS=480 $G 400 $O/ab_65536.log python3 scripts/ab_variant.py 65536 8,12,16 prod,prodmask 9 || exit $?
tail -3 $O/ab_65536.log
AB_STEPS=96 $G 400 $O/ab_262144.log python3 scripts/ab_variant.py 262144 16 prod,prodmask 5 || exit $?
tail -1 $O/ab_262144.log
