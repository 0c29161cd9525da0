#!/bin/bash
# round 4 (u): gol_slab2 with every count flushed at the end of the launch (NC = 12) against the
# in-loop flush of the 2S <= K shapes (12 x 7 at 4096^2): parity, sweep, stamps
set -u
O=gpurun_out/r04u
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/parity.log python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q -k "slab" --timeout 240 --timeout-method thread || exit $?
tail -2 $O/parity.log
grep -q " passed" $O/parity.log && ! grep -qE " failed| error" $O/parity.log || exit 1
$G 400 $O/tune.log python3 scripts/tune_slab.py 5120,4096 0,90812,91207,121207,91208,121208,91606,121606,121605 4096 || exit $?
grep -E "^best|^\{" $O/tune.log | cut -c1-1200
GOLHIP_SLAB=121207 $G 120 $O/stamps_4096.log python3 scripts/slab_stamps.py 4096 4 1 || exit $?
grep "\"launch\": 3" $O/stamps_4096.log | cut -c1-600
