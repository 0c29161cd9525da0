#!/bin/bash
# round 2 (ap): GPU suite + smoke on the final tree
set -u
O=gpurun_out/r02ap
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
$G 1000 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
tail -1 $O/pytest_gpu.log
