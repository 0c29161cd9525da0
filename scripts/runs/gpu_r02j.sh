#!/bin/bash
# Register tile/slab kernels: parity first, then the small/medium-board sweep against the streaming kernels.
set -u
O=gpurun_out/r02j
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/pytest_tile.log python -u -m pytest tests/test_gpu_parity.py -k "register_ or graph or count_window or alive_csv or small_board" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" $O/pytest_tile.log && ! grep -q "FAILED\|ERROR" $O/pytest_tile.log || { echo "tests failed"; exit 1; }
$G 300 $O/small_configs.log python3 scripts/small_configs.py || exit $?
$G 400 $O/tune_small.log python3 scripts/tune_tile.py 512,4096,5120 0,t16,s0808,s0816,s1608,s1616 8,16 || exit $?
TUNE_COUNTS=0 $G 400 $O/tune_small_nc.log python3 scripts/tune_tile.py 512,5120 0,t16,s0808,s0816,s1608 8,16 || exit $?
echo done
