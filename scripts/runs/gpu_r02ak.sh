#!/bin/bash
# round 2 (ak): final full validation of the committed tree: smoke, GPU suite, bench default and 20/5
set -u
O=gpurun_out/r02ak
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
$G 1000 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
tail -2 $O/pytest_gpu.log
$G 400 $O/bench.log python3 bench.py || exit $?
$G 300 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
echo done
