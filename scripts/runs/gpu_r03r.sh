#!/bin/bash
# round 3 (r): the compact per-turn flips (golhip_step_flips_rows): parity tests, then the bench's
# flips leg (golhip_step_flips vs the rows form at 512^2 and 5120^2)
set -u
O=gpurun_out/r03r
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 600 $O/pytest_flips.log python -u -m pytest tests/test_gpu_parity.py -m gpu -k "flips" -x -q --timeout 300 --timeout-method thread || exit $?
tail -2 $O/pytest_flips.log
grep -q " passed" $O/pytest_flips.log && ! grep -q " failed" $O/pytest_flips.log || exit 1
$G 400 $O/bench_flips.log python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-configs --no-sweep --no-strong || exit $?
grep "^{" $O/bench_flips.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['flips_path']))"
