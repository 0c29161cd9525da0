#!/bin/bash
# round 4 (c): why the ring-of-one create failed in r04b (non-blocking RCCL communicator), then
# the fail-fast tests, slab2 parity (idle-wave publish fix) and the slab2 A/B
set -u
O=gpurun_out/r04c
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 120 $O/ring1.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "ring_of_one" --timeout 100 --timeout-method thread || exit $?
tail -5 $O/ring1.log
NCCL_DEBUG=WARN $G 300 $O/failfast.log python -u -m pytest tests/test_gpu_failfast.py -m gpu -v --timeout 250 --timeout-method thread || exit $?
tail -8 $O/failfast.log
$G 400 $O/slab2.log python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q -k "slab" --timeout 300 --timeout-method thread || exit $?
tail -3 $O/slab2.log
grep -q " passed" $O/slab2.log && ! grep -q " failed" $O/slab2.log || exit 1
$G 300 $O/tune_slab.log python3 scripts/tune_slab.py 5120,4096 0,20812,90812,91208,91207,91606,91605 4096 || exit $?
tail -6 $O/tune_slab.log
