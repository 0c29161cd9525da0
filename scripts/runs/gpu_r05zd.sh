#!/bin/bash
# round 5: the tuning-build tests after the last tuning-library rebuild, and smoke
set -u
O=gpurun_out/r05zd
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 600 $O/tuning.log python -u -m pytest tests/test_gpu_tuning.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
tail -2 $O/tuning.log
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -2 $O/smoke.log
