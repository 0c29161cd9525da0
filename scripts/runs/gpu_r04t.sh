#!/bin/bash
# round 4 (t): gol_slab2 with the in-launch count flush whenever S <= K (NC = 11): parity, the
# slab sweep against the production shapes, phase stamps
set -u
O=gpurun_out/r04t
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/parity.log python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q -k "slab" --timeout 240 --timeout-method thread || exit $?
tail -2 $O/parity.log
grep -q " passed" $O/parity.log && ! grep -qE " failed| error" $O/parity.log || exit 1
$G 400 $O/tune.log python3 scripts/tune_slab.py 5120,4096 0,90812,110812,91208,111208,110810,111008,91207 4096 || exit $?
grep -E "^best|^\{" $O/tune.log | cut -c1-1200
GOLHIP_SLAB=110812 $G 120 $O/stamps_5120.log python3 scripts/slab_stamps.py 5120 4 1 || exit $?
grep '"launch": 3' $O/stamps_5120.log | cut -c1-600
