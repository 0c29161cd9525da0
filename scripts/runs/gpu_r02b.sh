#!/bin/bash
# Round-2 GPU session B: parity of the new drift variants, then interleaved variant tune at 65536^2.
set -u
O=gpurun_out/r02b
mkdir -p $O
export TMPDIR=/tmp
scripts/guard.sh 600 $O/pytest_variants.log python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "variant" || exit $?
grep -q " failed" $O/pytest_variants.log && exit 1
TUNE_STEPS=256 scripts/guard.sh 300 $O/tune.log python -u scripts/tune.py 65536 8,12,16 0 driftlds,drift62,driftzip || exit $?
TUNE_STEPS=256 scripts/guard.sh 300 $O/tune32.log python -u scripts/tune.py 65536 16,32 0 drift62,driftzip,chainlds || exit $?
