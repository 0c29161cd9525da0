#!/bin/bash
# round 3 (e): gol_slab exchanging edge-row sums instead of rows; new slab shapes (W x S = 84, 80):
# slab/flips parity tests, then the shape sweep at 5120^2 and 4096^2 with and without counts
set -u
O=gpurun_out/r03e
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 600 $O/pytest_slab.log python -u -m pytest tests/test_gpu_parity.py -k "slab or flips or alive_csv or check_images" -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
tail -1 $O/pytest_slab.log
$G 400 $O/tune_slab.log python3 scripts/tune_slab.py 5120,4096 0,20812,21208,41208,21207,21008,21406 || exit $?
tail -5 $O/tune_slab.log
$G 300 $O/configs.log python3 scripts/small_configs.py || exit $?
tail -2 $O/configs.log
