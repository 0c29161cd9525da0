#!/bin/bash
# round 4 (g): re-validation after the stamp-buffer fix (r04f fault), then the full GPU suite
# stream): the safe fail-fast tests, the early-exchange race fix (ring of one == single strip at
# scale), the strip-shape prediction, and per-wave stamps of the streaming launches
set -u
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/failfast.log python -u -m pytest tests/test_gpu_failfast.py -m gpu -v -s --timeout 250 --timeout-method thread || exit $?
grep -E "^\{|PASSED|FAILED|passed|failed" $O/failfast.log | cut -c1-500
$G 300 $O/ring_scale.log python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "ring_of_one" --timeout 250 --timeout-method thread || exit $?
tail -6 $O/ring_scale.log
grep -q " passed" $O/ring_scale.log && ! grep -q " failed" $O/ring_scale.log || exit 1
$G 400 $O/predict.log python3 scripts/predict_scaling.py 5 20,1000 160 || exit $?
grep "^{" $O/predict.log | cut -c1-250
$G 300 $O/stamps.log python3 scripts/stamp_launch.py 65536 12,8,14,16 4 300 || exit $?
grep '"launch"' $O/stamps.log | cut -c1-330
$G 900 $O/suite.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
tail -4 $O/suite.log
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
$G 400 $O/bench.log python3 bench.py || exit $?
grep "^{" $O/bench.log | cut -c1-600
