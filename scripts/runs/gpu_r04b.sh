#!/bin/bash
# round 4 (b): the production/tuning split, RCCL fail-fast, early halo exchange and gol_slab2 on
# hardware: fail-fast tests (fresh processes), slab2 parity, slab2 vs slab A/B on configs[1]/[4],
# the whole GPU suite, smoke, the driver's 20/5 line, the strip-shape prediction again
set -u
O=gpurun_out/r04b
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/failfast.log python -u -m pytest tests/test_gpu_failfast.py -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
tail -5 $O/failfast.log
$G 400 $O/slab2.log python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q -k "slab" --timeout 300 --timeout-method thread || exit $?
tail -3 $O/slab2.log
grep -q " passed" $O/slab2.log && ! grep -q " failed" $O/slab2.log || exit 1
$G 300 $O/tune_slab.log python3 scripts/tune_slab.py 5120,4096 0,20812,90812,91208,91207,91606,91605 4096 || exit $?
tail -6 $O/tune_slab.log
$G 1000 $O/gpu_suite.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
tail -3 $O/gpu_suite.log
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -1 $O/smoke.log
$G 400 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu || exit $?
grep "^{" $O/bench20.log | cut -c1-300
$G 400 $O/predict.log python3 scripts/predict_scaling.py 5 20,1000 160 || exit $?
grep "^{" $O/predict.log | cut -c1-250
