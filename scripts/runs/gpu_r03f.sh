#!/bin/bash
# round 3 (f): slab shape model + sums exchange + RCCL process group in bench: whole GPU suite,
# smoke, the driver's bench command and the default bench, rocprof kernel stats of the 20/5 bench
set -u
O=gpurun_out/r03f
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
$G 1100 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread || exit $?
tail -1 $O/pytest_gpu.log
$G 400 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep "^{" $O/bench20.log | cut -c1-300
$G 300 $O/prof20.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof20 -o b -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-sweep --no-strong --no-flips --no-configs || exit $?
find /tmp/prof20 -name "*kernel_stats.csv" -exec cp {} $O/prof20_kernel_stats.csv \;
grep "^{" $O/prof20.log > $O/prof20_line.json
