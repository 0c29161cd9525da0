#!/bin/bash
# Full GPU suite + smoke + small configs + default bench (DPP count reduction, slab policy).
set -u
O=gpurun_out/r02o
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
$G 1000 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
tail -3 $O/pytest_gpu.log
$G 300 $O/small_configs.log python3 scripts/small_configs.py || exit $?
$G 400 $O/bench.log python3 bench.py || exit $?
tail -1 $O/bench.log
echo done
