#!/bin/bash
# Round-2 GPU session D: launch depth x geometry at 65536^2 (occupancy vs depth).
set -u
O=gpurun_out/r02d
mkdir -p $O
export TMPDIR=/tmp
scripts/guard.sh 300 $O/pytest_k.log python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "drift_variant_every_k" || exit $?
grep -q " failed" $O/pytest_k.log && exit 1
TUNE_STEPS=256 scripts/guard.sh 400 $O/tune.log python -u scripts/tune.py 65536 10,12,14,16 0 driftlds,drift62 || exit $?
TUNE_STEPS=256 scripts/guard.sh 400 $O/tune_b.log python -u scripts/tune.py 65536 12,14 0,200,240,264,300,336 drift62 || exit $?
