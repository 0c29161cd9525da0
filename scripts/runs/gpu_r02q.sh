#!/bin/bash
# Round-2 validation: smoke, full GPU suite, small configs, bench (default and the driver's
# 20/5), rocprofv3 --kernel-trace --stats of both bench commands.
set -u
O=gpurun_out/r02q
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
$G 1000 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
tail -2 $O/pytest_gpu.log
$G 300 $O/small_configs.log python3 scripts/small_configs.py || exit $?
$G 400 $O/bench.log python3 bench.py || exit $?
$G 300 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
$G 400 $O/prof20.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof20 -o b -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-sweep --no-strong --no-flips || exit $?
$G 400 $O/prof.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b -- python3 bench.py --no-cpu --no-sweep --no-strong --no-flips || exit $?
echo done
