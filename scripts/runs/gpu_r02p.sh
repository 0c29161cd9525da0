#!/bin/bash
set -u
O=gpurun_out/r02p
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py -k "register_slab or small_board" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" $O/pytest.log && ! grep -q "FAILED\|ERROR" $O/pytest.log || { echo "tests failed"; exit 1; }
$G 300 $O/small_configs.log python3 scripts/small_configs.py || exit $?
$G 400 $O/tune.log python3 scripts/tune_tile.py 4096,5120,8192 s0812,s0811,s0816,s1606,s1608 16 || exit $?
TUNE_COUNTS=0 $G 400 $O/tune_nc.log python3 scripts/tune_tile.py 5120 s0812 16 || exit $?
echo done
