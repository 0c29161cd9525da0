#!/bin/bash
# round 4 (d): fail-fast modes (unmatched receive, stalled halos, absent peer), the whole GPU suite
# with gol_slab2 in production, smoke, the driver's 20/5 line, strip-shape prediction with the
# early exchange, and per-wave stamps of the streaming launches (tuning build)
set -u
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/failfast.log python -u -m pytest tests/test_gpu_failfast.py -m gpu -v -s --timeout 300 --timeout-method thread || exit $?
grep -E "^\{|PASSED|FAILED|passed|failed" $O/failfast.log | cut -c1-400
$G 1000 $O/gpu_suite.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread || exit $?
tail -4 $O/gpu_suite.log
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -1 $O/smoke.log
$G 400 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu || exit $?
grep "^{" $O/bench20.log | cut -c1-300
$G 400 $O/predict.log python3 scripts/predict_scaling.py 5 20,1000 160 || exit $?
grep "^{" $O/predict.log | cut -c1-250
$G 300 $O/stamps.log python3 scripts/stamp_launch.py 65536 12,8,14,16 4 300 || exit $?
grep '"launch"' $O/stamps.log | cut -c1-330
