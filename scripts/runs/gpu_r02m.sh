#!/bin/bash
set -u
O=gpurun_out/r02m
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/pytest_slab.log python -u -m pytest tests/test_gpu_parity.py -k "register_slab_kernel" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" $O/pytest_slab.log && ! grep -q "FAILED\|ERROR" $O/pytest_slab.log || { echo "tests failed"; exit 1; }
$G 500 $O/tune_slab.log python3 scripts/tune_tile.py 4096,5120,8192 0,s0808,s0810,s0811,s0812,s0813,s0814,s0816,s0820,s0824,s1604,s1606,s1608,s0416,s0424 16 || exit $?
TUNE_COUNTS=0 $G 500 $O/tune_slab_nc.log python3 scripts/tune_tile.py 5120 0,s0808,s0810,s0811,s0812,s0813,s0814,s0816,s0820,s1606,s0416,s0424 16 || exit $?
echo done
