#!/bin/bash
# round 5: the persistent call's tests (incl. the flip-tracking refusal), and rocprofv3 kernel
# stats of the persistent A/B probe (one gol_slabq launch per count window beside gol_slab2)
set -u
O=gpurun_out/r05x
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/tests.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "persistent or interleaved" || exit $?
tail -2 $O/tests.log
$G 300 $O/prof.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05x_prof -o p -- python3 scripts/probe_slabq.py 4096 3 || exit $?
find /tmp/r05x_prof -name "*kernel_stats.csv" -exec cp {} $O/slabq_kernel_stats.csv \;
grep -E "^(4096|5120) " $O/prof.log
