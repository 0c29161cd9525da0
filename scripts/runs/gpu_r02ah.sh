#!/bin/bash
# round 2 (ah): after the K = 10 rate fix: cfg3 plan tests, bench default and 20/5
set -u
O=gpurun_out/r02ah
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 600 $O/pytest.log python -u -m pytest tests/test_gpu_configs.py -k "cfg3" -x -q --timeout 300 --timeout-method thread || exit $?
tail -1 $O/pytest.log
$G 400 $O/bench.log python3 bench.py || exit $?
$G 300 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
echo done
