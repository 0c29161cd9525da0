#!/bin/bash
# Round-2 GPU session A: short bench (driver's 20/5), full GPU suite, default bench.
set -u
O=gpurun_out/r02a
mkdir -p $O
export TMPDIR=/tmp
scripts/guard.sh 300 $O/bench20.log python -u bench.py --steps 20 --warmup 5 --no-cpu || exit $?
scripts/guard.sh 900 $O/pytest.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit $?
scripts/guard.sh 400 $O/bench.log python -u bench.py || exit $?
