#!/bin/bash
# round 4 (w): gol_slab2 end-flush with the younger half of each workgroup's waves at s_setprio 1
# (NC = 13) against the production end-flush shapes (NC = 12): parity, sweep
set -u
O=gpurun_out/r04w
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/parity.log python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q -k "slab" --timeout 240 --timeout-method thread || exit $?
tail -2 $O/parity.log
grep -q " passed" $O/parity.log && ! grep -qE " failed| error" $O/parity.log || exit 1
$G 400 $O/tune.log python3 scripts/tune_slab.py 5120,4096 0,121606,131606,121207,131207,90812,130812 4096 || exit $?
grep -E "^best|^\{" $O/tune.log | cut -c1-1000
