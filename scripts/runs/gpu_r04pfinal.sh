#!/bin/bash
# round 4 (pfinal): the last validation of the final tree: GPU suite and smoke
set -u
O=gpurun_out/r04pfinal
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 900 $O/suite.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
tail -3 $O/suite.log
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -2 $O/smoke.log
