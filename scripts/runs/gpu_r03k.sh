#!/bin/bash
# round 3 (k): slab micro-optimisations (accumulating v_bcnt chain, branch-free exchange through
# zero neighbour blocks, immediate LDS offsets): slab / flips / configs tests, the shape sweep, the
# configs timings
set -u
O=gpurun_out/r03k
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 700 $O/pytest_slab.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "slab or flips or alive_csv or check_images or cfg5 or cfg2 or small_board" -m gpu -x -v --timeout 600 --timeout-method thread || exit $?
tail -1 $O/pytest_slab.log
$G 400 $O/tune_slab.log python3 scripts/tune_slab.py 4096,5120,512 0,21208,21207,20812 || exit $?
tail -6 $O/tune_slab.log
$G 300 $O/configs.log python3 scripts/small_configs.py || exit $?
tail -2 $O/configs.log
