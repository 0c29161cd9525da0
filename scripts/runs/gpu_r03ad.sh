#!/bin/bash
# round 3 (ad): interleaved counting / plain launches (per-launch geometry) and the driver's 20/5
# line with the refreshed PMC entries
set -u
O=gpurun_out/r03ad
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 600 $O/pytest_interleaved.log python -u -m pytest tests/test_gpu_parity.py -m gpu -k "interleaved or graded or drift_variant" -x -q --timeout 300 --timeout-method thread || exit $?
tail -2 $O/pytest_interleaved.log
grep -q " passed" $O/pytest_interleaved.log && ! grep -q " failed" $O/pytest_interleaved.log || exit 1
$G 400 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep "^{" $O/bench20.log | cut -c1-200
