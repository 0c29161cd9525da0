#!/bin/bash
# round 3 (o): pre63 with the 65th word from a second whole-wave DMA (no exec-mask branches):
# parity, then the same-call A/B against the production geometry at 65536^2 and 262144^2
set -u
O=gpurun_out/r03o
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 600 $O/pytest_pre63.log python -u -m pytest tests/test_gpu_parity.py -m gpu -k pre63 -x -q --timeout 300 --timeout-method thread || exit $?
tail -2 $O/pytest_pre63.log
grep -q " passed" $O/pytest_pre63.log && ! grep -q "failed" $O/pytest_pre63.log || exit 1
TUNE_STEPS=256 $G 500 $O/tune_pre63_65536.log python3 scripts/tune.py 65536 8,12,16 0 prod,pre63 || exit $?
tail -2 $O/tune_pre63_65536.log
TUNE_STEPS=64 $G 500 $O/tune_pre63_262144.log python3 scripts/tune.py 262144 12,16 0 prod,pre63 || exit $?
tail -2 $O/tune_pre63_262144.log
TUNE_STEPS=256 $G 500 $O/tune_pre63_bands.log python3 scripts/tune.py 65536 8,12 0,144,168,192,216,240 pre63 || exit $?
tail -2 $O/tune_pre63_bands.log
