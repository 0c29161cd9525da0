#!/bin/bash
# round 6 (f): the host Channel without the per-element wake-ups: per-turn CellFlipped through
# gol::Run again (pipelined vs unpipelined), and the host contract tests
set -u
O=gpurun_out/r06f
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/host_tests.log python -u -m pytest tests/test_host.py -m gpu -x -v --timeout 280 --timeout-method thread || exit $?
tail -3 $O/host_tests.log
$G 600 $O/host_flips_ab.log python -u scripts/host_flips_ab.py 100000 10000 || exit $?
tail -1 $O/host_flips_ab.log
