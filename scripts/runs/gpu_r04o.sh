#!/bin/bash
# round 4 (o): gol_slab3 (gol_slab2 pipelined across generations): parity on every compiled shape
# (tuning build), the slab-shape sweep against gol_slab2 on configs[1] / configs[4] sizes, and
# its phase stamps
set -u
O=gpurun_out/r04o
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/parity.log python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q -k "slab" --timeout 240 --timeout-method thread || exit $?
tail -3 $O/parity.log
grep -q " passed" $O/parity.log && ! grep -qE " failed| error" $O/parity.log || exit 1
$G 400 $O/tune.log python3 scripts/tune_slab.py 5120,4096 0,90812,91606,91208,91207,100812,101606,101208,101207,101008,100810 4096 || exit $?
grep -E "^best|^\{" $O/tune.log | cut -c1-1500
GOLHIP_SLAB=100812 $G 120 $O/stamps_5120.log python3 scripts/slab_stamps.py 5120 4 1 || exit $?
GOLHIP_SLAB=101207 $G 120 $O/stamps_4096.log python3 scripts/slab_stamps.py 4096 4 1 || exit $?
grep '"launch": 3' $O/stamps_*.log | cut -c1-600
