#!/bin/bash
# round 3 (n): the pre-shifted 63-word stencil (kVariantPre63): its parity tests, an A/B against
# the production geometry at 65536^2 and 262144^2, then the full GPU suite, smoke and the driver's
# bench command on the tree, and the 16-wave slab sweep the cut-off session's results were lost for
set -u
O=gpurun_out/r03n
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 600 $O/pytest_pre63.log python -u -m pytest tests/test_gpu_parity.py -m gpu -k pre63 -x -q --timeout 300 --timeout-method thread || exit $?
tail -2 $O/pytest_pre63.log
grep -q " passed" $O/pytest_pre63.log && ! grep -q "failed" $O/pytest_pre63.log || exit 1
TUNE_STEPS=256 $G 500 $O/tune_pre63_65536.log python3 scripts/tune.py 65536 8,12,16 0 prod,pre63 || exit $?
tail -2 $O/tune_pre63_65536.log
TUNE_STEPS=64 $G 500 $O/tune_pre63_262144.log python3 scripts/tune.py 262144 12,16 0 prod,pre63 || exit $?
tail -2 $O/tune_pre63_262144.log
$G 900 $O/gpu_suite.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
tail -3 $O/gpu_suite.log
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -1 $O/smoke.log
$G 400 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep "^{" $O/bench20.log | cut -c1-300
$G 400 $O/tune_slab.log python3 scripts/tune_slab.py 4096,5120 0,20812,21208,21207,21606,21605 || exit $?
tail -5 $O/tune_slab.log
