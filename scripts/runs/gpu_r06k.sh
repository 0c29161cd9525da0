#!/bin/bash
# round 6 (k): lib_tuning pushed for this call: the tuning / fail-fast suites against the final
# round-6 kernels (after the batched count flush)
set -u
O=gpurun_out/r06k
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 700 $O/tuning.log python -u -m pytest tests/test_gpu_tuning.py tests/test_gpu_failfast.py -m gpu -x -q --timeout 280 --timeout-method thread || exit $?
tail -3 $O/tuning.log
