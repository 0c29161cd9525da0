#!/bin/bash
# round 6 (m): gol_slab2 with point-to-point LDS flags between neighbour waves instead of the
# per-generation workgroup barrier (NC = 15, tuning library) against the production barrier form
# (NC = 12 counting, automatic), on configs[4]'s 4096^2, configs[1]'s 5120^2 and 2048^2; every
# per-turn count checked (golden CSV at 5120^2, the automatic shape's counts elsewhere).
set -u
O=gpurun_out/r06m
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tuning.py -k "neighbour_flags" || exit $?
tail -3 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q "FAILED" $O/tests.log || exit 1
$G 400 $O/tune_pf.log python -u scripts/tune_slab.py 4096,5120,2048 0,121207,151207,121606,151606,121204,151204 4096 || exit $?
tail -8 $O/tune_pf.log
