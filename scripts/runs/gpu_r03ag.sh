#!/bin/bash
# round 3 (ag): the timed region without per-launch events (value), the roofline from an identical
# instrumented pass: the driver's 20/5 command twice, the default bench, the bench multi-rank path
# through the host transport at world 2
set -u
O=gpurun_out/r03ag
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
for i in 1 2; do
$G 400 $O/bench20_$i.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep "^{" $O/bench20_$i.log | cut -c1-200
done
$G 500 $O/bench.log python3 bench.py || exit $?
grep "^{" $O/bench.log | cut -c1-200
$G 600 $O/pytest_rank.log python -u -m pytest tests/test_gpu_rank_host.py -m gpu -x -q --timeout 500 --timeout-method thread || exit $?
tail -2 $O/pytest_rank.log
