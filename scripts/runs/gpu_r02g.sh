#!/bin/bash
set -u
O=gpurun_out/r02g
mkdir -p $O
export TMPDIR=/tmp
scripts/guard.sh 600 $O/pytest_flips.log python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "flips" || exit $?
grep -q " failed" $O/pytest_flips.log && exit 1
scripts/guard.sh 900 $O/pytest.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread || exit $?
scripts/guard.sh 400 $O/bench.log python -u bench.py --no-cpu || exit $?
